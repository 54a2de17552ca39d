# Round-end evidence: pytest -m gpu, three bench lines at the driver's settings (K=20 / W=5), one
# at the defaults, and rocprofv3 kernel stats of a K=20 run; everything under gpurun_out/<tag>/.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu/final.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20_$r.log" 2>&1 || { tail -5 "$out/bench20_$r.log"; exit 1; }
  grep '^{' "$out/bench20_$r.log" | cut -c1-230
done
timeout -k 10 240 python bench.py > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" | cut -c1-230
bash tools/gpu/prof.sh "$tag/prof20" --steps 20 --warmup 5 > /dev/null
