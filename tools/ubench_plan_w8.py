"""The sharded runner's per-call kernels at the C3 per-rank shape with W in-process shards on the
one GPU (loopback transport, one host thread per shard): ml-20m shape, d=128, B=4096 per rank,
K-step calls.  Run under rocprofv3 --kernel-trace --stats to read k_owner_plan's duration per
rank at world W (each rank's plan kernel does that rank's work; the ranks share the device).

  python tools/ubench_plan_w8.py [W] [K] [calls]
"""
import importlib
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
CALLS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
sh = rl.sharded
U, I, d, B = 138493, 26744, 128, 4096
pos = syn.make_positives(U, I, 10_000_000, 20261015)
grp = sh.ThreadGroup(W)
errs = []


def run(r):
    try:
        m = sh.ShardedBPRMF(U, I, d, batch_size=B, seed=3, device=0, comm=sh.ThreadComm(grp, r))
        S = m.set_train(pos)
        m.attach_runner("loopback", key=77)
        first = 0
        for _ in range(CALLS):
            m.train_steps(0, first, K)
            first += K
            if first + K > S:
                first = 0
    except BaseException as e:  # noqa: BLE001
        errs.append(e)
        grp.barrier.abort()


ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
[t.start() for t in ts]
[t.join(timeout=600) for t in ts]
if errs:
    raise errs[0]
print(f"ok: world {W}, {CALLS} calls of {K} steps per rank")
