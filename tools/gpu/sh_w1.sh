# World-1 sharded bench lines at the driver's settings, per environment variant (A/B).
#   gpurun --timeout 900 -- 'bash tools/gpu/sh_w1.sh <tag> "ENV=a" "ENV=b" ...'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for v in "$@"; do
  n=$((n + 1))
  env $v timeout -k 10 200 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > "$out/b$n.log" 2>&1 || { tail -5 "$out/b$n.log"; exit 1; }
  echo "[$v] $(grep '^{' "$out/b$n.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])')"
done
