# A/B of the IPC runner's exchange forms with 2 ranks on the box's one GPU (gloo process group),
# 1000 steps each: the rates say nothing about xGMI (both ranks share one device) but compare
# what the forms cost on the device itself (uncached landing reads vs receive copies).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/sh_w2_ab.sh <tag> "ENV=.." "ENV=.."'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for v in "$@"; do
  n=$((n + 1))
  env $v timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus 2 --steps 1000 --warmup 100 --pg-backend gloo --no-cpu-baseline > "$out/ab$n.log" 2>&1 || { tail -20 "$out/ab$n.log"; exit 1; }
  echo "[$v] $(grep '^{' "$out/ab$n.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])')"
done
