# bench.py at the driver's settings, N times in a row (each a fresh process), lines appended to
# gpurun_out/<tag>/runs.jsonl; prints value, ms/step and the step launches' us/step per run.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/k20_runs.sh <tag> [N]'
set -o pipefail
tag="$1"; n="${2:-5}"
out="gpurun_out/$tag"
mkdir -p "$out"
for r in $(seq 1 "$n"); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$out/b$r.log" 2>&1 || { tail -5 "$out/b$r.log"; exit 1; }
  grep '^{' "$out/b$r.log" >> "$out/runs.jsonl"
done
python3 - "$out/runs.jsonl" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])
EOF
