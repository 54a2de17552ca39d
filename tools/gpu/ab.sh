# A/B of step-path switches (environment variables) on the default bench workload.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/ab.sh <tag> "ENV=.. ENV2=.." "ENV=.." ...'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for cfg in "$@"; do
  n=$((n + 1))
  env $cfg timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > "$out/ab$n.log" 2>&1 || { tail -5 "$out/ab$n.log"; exit 1; }
  echo "[$cfg] $(grep '^{' "$out/ab$n.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])')"
done
