# Environment knobs' effect on the local mode: quality on the planted ml-20m shape and F5 (seed 11)
# and bench.py's local line, for the defaults ("base") and each knob setting given.
#   gpurun --timeout 1200 -- 'bash tools/gpu/knob_quality.sh <tag> "ENV=v ENV2=v" ["ENV=w" ...]'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for knob in "" "$@"; do
  variant=$([ -z "$knob" ] && echo base || echo "k$n")
  n=$((n + 1))
  ( [ -n "$knob" ] && export $knob
    timeout -k 10 300 python -u tools/hr_modes.py --which planted,f5 --modes local --seeds 11 --epochs 10 \
      --users-eval 20000 | sed "s/^{/{\"variant\": \"$variant\", \"knob\": \"$knob\", /" >> "$out/hr_modes.jsonl" 2>> "$out/hr_modes.err" &&
    timeout -k 10 200 python bench.py --semantics local --no-cpu-baseline > "$out/bench_$variant.log" 2>&1 ) ||
    { tail -n 20 "$out/hr_modes.err" "$out/bench_$variant.log"; exit 1; }
  python -c "
import json
d=json.loads(open('$out/bench_$variant.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$variant', '$knob', d['value'], r['avg_us_per_step'], r['frac'])" | tee -a "$out/bench.txt"
done
grep -v popularity "$out/hr_modes.jsonl" | cut -c1-60,190-440
