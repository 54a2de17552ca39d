# State check of a tree: the -m gpu suite, smoke(), then the driver's bench line (K=20, W=5).
#   gpurun --timeout 1100 -- 'bash tools/gpu/check.sh <tag> [pytest -k expression]'
set -o pipefail
tag="$1"; sel="${2:-}"
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
step() {  # name, timeout, command...
  local name="$1" to="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$out/$name.log" | cut -c1-600
  return $rc
}
if [ -n "$sel" ]; then
  step gpu_tests 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$sel"
else
  step gpu_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
fi &&
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench20 240 python bench.py --steps 20 --warmup 5
