# The local mode's quality / speed frontier over its merge period (local_steps): HR@10, NDCG@10
# and the final-table loss on the planted ml-20m shape and F5 (seed 11), and bench.py's local
# line at the same period.   gpurun --timeout 1200 -- 'bash tools/gpu/frontier.sh <tag> [periods]'
set -o pipefail
tag="$1"; periods="${2:-16 32 64}"
out="gpurun_out/$tag"
mkdir -p "$out"
for ls in $periods; do
  timeout -k 10 300 python -u tools/hr_modes.py --which planted,f5 --modes local --seeds 11 --epochs 10 \
    --users-eval 20000 --local-steps "$ls" >> "$out/hr_modes.jsonl" 2>> "$out/hr_modes.err" || { tail -n 20 "$out/hr_modes.err"; exit 1; }
  timeout -k 10 200 python bench.py --semantics local --local-steps "$ls" --no-cpu-baseline > "$out/bench_ls$ls.log" 2>&1 || { tail -n 5 "$out/bench_ls$ls.log"; exit 1; }
  python -c "
import json
d=json.loads(open('$out/bench_ls$ls.log').read().strip().splitlines()[-1]); r=d['roofline']
print('local_steps $ls', d['value'], r['avg_us_per_step'], r['frac'])" | tee -a "$out/bench.txt"
done
cut -c80-400 "$out/hr_modes.jsonl"
