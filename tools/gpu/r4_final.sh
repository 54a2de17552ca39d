# Round 4 final evidence: GPU suite, smoke, the driver's bench line three times, the defaults,
# rocprofv3 stats of the K=20 bench.   gpurun --timeout 1200 -- 'bash tools/gpu/r4_final.sh <tag>'
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
  tail -2 "$out/$name.log" | cut -c1-400
  return $rc
}
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench20a 200 python bench.py --steps 20 --warmup 5 &&
step bench20b 200 python bench.py --steps 20 --warmup 5 &&
step bench20c 200 python bench.py --steps 20 --warmup 5 &&
step bench_defaults 300 python bench.py --no-cpu-baseline &&
cd /tmp && export TMPDIR=/tmp &&
step prof 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
rc=$?
cd "$R"
exit $rc
