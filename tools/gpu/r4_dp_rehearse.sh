# semantics "local" across processes on the one GPU (IPC all-reduce, gloo group): tests, then
# bench.py's multi-process path at worlds 2 and 4 (rates meaningless: the ranks share the GPU)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ipc.py tests/test_gpu_local_dp.py > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for w in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29700 + w)) bench.py --gpus $w --semantics local --transport ipc --pg-backend gloo --dp-steps 256 --dp-overlap --no-cpu-baseline --steps 512 --warmup 128 > "$out/w$w.log" 2>&1 || { tail -30 "$out/w$w.log"; exit 1; }
  grep -h '^{' "$out/w$w.log" | cut -c1-200
done
