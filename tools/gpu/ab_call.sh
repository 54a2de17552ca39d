# -m gpu suite, then ubench_call A/B of environment variants (one process each), then one bench
# line at the driver's settings.
#   gpurun --timeout 900 -- 'bash tools/gpu/ab_call.sh <tag> "ENV=a" "ENV=b" ...'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
  rc=$?
  tail -3 "$out/gpu_tests.log"
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u tools/ubench_call.py --ab "$@" > "$out/ab.log" 2>&1 || { tail -20 "$out/ab.log"; exit 1; }
cat "$out/ab.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log" | cut -c1-400
