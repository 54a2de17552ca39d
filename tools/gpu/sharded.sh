# Sharded runner on the box's one GPU: world 1 (--sharded) and world 2 / 4 rehearsals (one
# process per rank on the same device, gloo process group, IPC transport), driver settings.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/sharded.sh <tag> [steps] [warmup]'
set -o pipefail
tag="$1"; steps="${2:-20}"; warm="${3:-5}"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 240 python bench.py --sharded --steps "$steps" --warmup "$warm" --no-cpu-baseline > "$out/w1.log" 2>&1 || { tail -20 "$out/w1.log"; exit 1; }
grep '^{' "$out/w1.log"
for w in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29600 + w)) bench.py --gpus $w --steps "$steps" --warmup "$warm" --pg-backend gloo --no-cpu-baseline > "$out/w$w.log" 2>&1 || { tail -30 "$out/w$w.log"; exit 1; }
  grep '^{' "$out/w$w.log"
done
