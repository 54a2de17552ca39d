# GPU-box check: pytest -m gpu (log under gpurun_out/<tag>/), then bench lines at the driver's
# settings (--steps 20 --warmup 5) and at the defaults.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/round.sh <tag> [pytest -k expr]'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
sel=()
if [ -n "$1" ]; then sel=(-k "$1"); fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${sel[@]}" > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log"
timeout -k 10 240 python bench.py > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log"
