# The local mode's in-flight window (BPRMF_HOGWILD_WINDOW, default min(U, I)): quality on the
# planted ml-20m shape and F5 (seed 11) and bench.py's local line at each window.
#   gpurun --timeout 1200 -- 'bash tools/gpu/window.sh <tag> [windows]'
set -o pipefail
tag="$1"; wins="${2:-13372 6686 3343}"
out="gpurun_out/$tag"
mkdir -p "$out"
for w in $wins; do
  export BPRMF_HOGWILD_WINDOW=$w
  timeout -k 10 300 python -u tools/hr_modes.py --which planted,f5 --modes local --seeds 11 --epochs 10 \
    --users-eval 20000 | sed "s/^{/{\"window\": $w, /" >> "$out/hr_modes.jsonl" 2>> "$out/hr_modes.err" || { tail -n 20 "$out/hr_modes.err"; exit 1; }
  timeout -k 10 200 python bench.py --semantics local --no-cpu-baseline > "$out/bench_w$w.log" 2>&1 || { tail -n 5 "$out/bench_w$w.log"; exit 1; }
  python -c "
import json
d=json.loads(open('$out/bench_w$w.log').read().strip().splitlines()[-1]); r=d['roofline']
print('window $w', d['value'], r['avg_us_per_step'], r['frac'])" | tee -a "$out/bench.txt"
done
cut -c1-20,150-420 "$out/hr_modes.jsonl"
