# Round 4: the split builder's tag fix (planted stale words), the sharded tests with per-step oracle
# checks, and a K=20 bench line.  gpurun --timeout 900 -- 'bash tools/gpu/r4_tags.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_build_tags.py tests/test_gpu_sharded.py > "$out/tests.log" 2>&1
rc=$?
tail -4 "$out/tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log" | cut -c1-400
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --sharded > "$out/bench20_sharded_w1.log" 2>&1 || { tail -5 "$out/bench20_sharded_w1.log"; exit 1; }
grep '^{' "$out/bench20_sharded_w1.log" | cut -c1-400
