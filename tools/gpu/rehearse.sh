# bench.py's multi-process path rehearsed on the box's one GPU: W processes (gloo process group,
# every rank on cuda:0).  Rates mean nothing here (the ranks share one device); the run checks
# that the launch, the transport and the exchanges complete.
#   gpurun --timeout 900 -- 'bash tools/gpu/rehearse.sh <tag> <W> [bench.py args...]'
# e.g. exact sharded, IPC:   bash tools/gpu/rehearse.sh r8 8 --steps 20 --warmup 5
#      local, IPC all-reduce: bash tools/gpu/rehearse.sh rdp 4 --semantics local --transport ipc \
#                               --dp-steps 256 --dp-overlap --steps 512 --warmup 128
# GPU_MAX_HW_QUEUES=1: 8 processes x 4 queues oversubscribe the device's hardware queues, and a
# rank whose kernel spins on a peer flag can starve a peer's unmapped queue.
set -o pipefail
tag="$1"; W="$2"; shift 2
out="gpurun_out/$tag"
mkdir -p "$out"
[ "$W" -gt 4 ] && export GPU_MAX_HW_QUEUES=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$W" --master-addr 127.0.0.1 \
  --master-port $((29600 + W)) bench.py --gpus "$W" --pg-backend gloo --no-cpu-baseline "$@" \
  > "$out/w$W.log" 2>&1 || { grep -h "Error" "$out/w$W.log" | head -n 5; exit 1; }
grep -h '^{' "$out/w$W.log" | cut -c1-400
