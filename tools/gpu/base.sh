# Quick state check of a tree: -m gpu suite, smoke(), K=20 bench exact, builder PMC pass.
#   gpurun --timeout 900 -- 'bash tools/gpu/base.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -5 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log" | cut -c1-300
