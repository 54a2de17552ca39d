# A/B of sharded-path switches at world 1 (--sharded) at the driver's settings (K=20, W=5),
# 3 rounds of the variants; prints value and ms/step per run.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/sh_k20_ab.sh <tag> "ENV=.." "ENV=.."'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
for rep in 1 2 3; do
  for v in "$@"; do
    env $v timeout -k 10 200 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > "$out/k20.log" 2>&1 || { tail -5 "$out/k20.log"; exit 1; }
    echo "[$v] $(grep '^{' "$out/k20.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
