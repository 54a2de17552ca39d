# Round-3 GPU check: the config-shape tests first (own log), then the whole -m gpu suite, then the
# bench at the driver's settings.   gpurun --timeout 1200 -- 'bash tools/gpu/r3.sh <tag>'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > "$out/configs.log" 2>&1
rc=$?
tail -12 "$out/configs.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_configs.py > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --semantics hogwild --no-cpu-baseline > "$out/bench20_hog.log" 2>&1 || { tail -5 "$out/bench20_hog.log"; exit 1; }
grep '^{' "$out/bench20_hog.log"
exit $rc
