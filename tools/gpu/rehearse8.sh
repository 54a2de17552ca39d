# bench.py's N=8 path rehearsed on the box's one GPU: 8 processes (gloo process group, IPC
# transport, every rank on cuda:0), the driver's settings.  Rates mean nothing here (8 ranks share
# one device); the run checks that the N=8 launch, IPC mapping and exchanges complete.
# GPU_MAX_HW_QUEUES=1: 8 processes x 4 queues oversubscribe the device's hardware queues, and a
# rank whose kernel spins on a peer flag can then starve the peer's unmapped queue until the 10 s
# wait gives up (seen at 8 ranks with the default; on an 8-GPU node each device hosts one process).
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/gpu/rehearse8.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
export GPU_MAX_HW_QUEUES=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --steps 20 --warmup 5 --pg-backend gloo --no-cpu-baseline \
  > "$out/w8.log" 2>&1 || { grep -h "Error" "$out/w8.log" | head -5; exit 1; }
grep '^{' "$out/w8.log"
