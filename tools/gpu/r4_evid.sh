# Round 4 evidence: full GPU suite, smoke, rocprofv3 stats of the K=20 bench, fused-step
# per-workgroup stamps, HR@10 of exact vs local, PMC traffic of the fused step.
#   gpurun --timeout 1200 -- 'bash tools/gpu/r4_evid.sh <tag>'
set -o pipefail
tag="$1"
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
step() {  # name, timeout, command...
  local name="$1" to="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -3 "$out/$name.log"
  return $rc
}
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
step step_stamps 200 python tools/ubench_step_stamps.py &&
step stamps 200 python tools/ubench_call_stamps.py 8 &&
BPRMF_SAMPLE_TREE=0 step stamps_bsearch 200 python tools/ubench_call_stamps.py 8 &&
step bench20 200 python bench.py --steps 20 --warmup 5 &&
step hr 400 python tools/hr_modes.py --which f5,ml20m --modes exact,local --seeds 11,12 --epochs 10 &&
cd /tmp && export TMPDIR=/tmp &&
step prof 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
rc=$?
cd "$R"
find "$out/prof" -name "*kernel_stats.csv" | head -3
exit $rc
