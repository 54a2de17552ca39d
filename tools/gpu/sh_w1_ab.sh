# A/B of sharded-path switches at world 1 (--sharded), 2000 steps each; prints value, ms/step,
# step-launch us/step per variant.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/sh_w1_ab.sh <tag> "ENV=.." "ENV=.."'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for v in "$@"; do
  n=$((n + 1))
  env $v timeout -k 10 200 python bench.py --sharded --steps 2000 --warmup 100 --no-cpu-baseline > "$out/ab$n.log" 2>&1 || { tail -5 "$out/ab$n.log"; exit 1; }
  echo "[$v] $(grep '^{' "$out/ab$n.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])')"
done
