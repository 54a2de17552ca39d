# Round 4 state check: the new tests (planted tags, per-step sharded oracle, atomic step, local
# semantics), benches (exact K=20, --sharded world 1, local, hogwild, atomic) and the C5 tests.
#   gpurun --timeout 1200 -- 'bash tools/gpu/r4_full.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
step() {  # name, timeout, command...
  local name="$1" to="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -3 "$out/$name.log"
  return $rc
}
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step tags 400 $PYT tests/test_gpu_build_tags.py tests/test_gpu_sharded.py &&
step local 400 $PYT tests/test_gpu_hogwild.py tests/test_gpu_parity.py -k "local or atomic or hogwild" &&
step bench20 200 python bench.py --steps 20 --warmup 5 &&
step stamps 200 python tools/ubench_call_stamps.py 8 &&
BPRMF_K2_ITEM_LG=0 step stamps_k2full 200 python tools/ubench_call_stamps.py 8 &&
step bench20_sh 200 python bench.py --steps 20 --warmup 5 --sharded &&
step bench_local20 200 python bench.py --steps 20 --warmup 5 --semantics local --no-cpu-baseline &&
step bench_local 200 python bench.py --semantics local --no-cpu-baseline &&
step bench_hog 200 python bench.py --semantics hogwild --no-cpu-baseline &&
step bench_atomic20 200 python bench.py --steps 20 --warmup 5 --step atomic --no-cpu-baseline &&
step c5 500 $PYT tests/test_gpu_configs.py -k c5
rc=$?
grep -h '^{' "$out"/bench*.log | cut -c1-600
exit $rc
