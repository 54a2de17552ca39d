"""semantics "local" at world W rehearsed on one GPU (W in-process ranks, threads + the loopback
transport): per-call wall clock of `steps` steps of every rank, and (under
`rocprofv3 --kernel-trace --stats`) the per-launch durations of the merge kernels k_dp_delta /
k_dp_apply / k_dp_sum beside k_hogwild.  The ranks share the GPU, so the wall clock is not what W
GPUs take; the merge kernels' durations are what one GPU's share of a merge costs.

    python tools/ubench_local_dp.py [W] [steps] [dp_steps]"""
import importlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    ov = len(sys.argv) > 4 and sys.argv[4] == "overlap"
    import torch  # noqa: F401  (HIP runtime first)
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, d, B = 138493, 26744, 128, 4096
    pos = syn.make_positives(U, I, 20_000_263, 20261015)
    sh = rl.sharded
    grp = sh.ThreadGroup(W)
    out, errs = [None] * W, []

    def run(r):
        try:
            m = sh.ShardedBPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, seed=5, device=0,
                                comm=sh.ThreadComm(grp, r), semantics="local", dp_steps=dp,
                                dp_overlap=ov)
            m.set_train(pos)
            m.attach_runner("loopback", key=9300 + W)
            m.train_steps(0, 0, dp)  # warm-up: one merge period
            walls = []
            for c in range(3):
                grp.barrier.wait()
                t0 = time.perf_counter()
                st = m.train_steps(0, dp * (1 + c * steps // dp), steps)
                walls.append(time.perf_counter() - t0)
            out[r] = (walls, st)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    if errs:
        raise errs[0]
    walls = [max(o[0][c] for o in out) for c in range(3)]
    print(json.dumps({"world": W, "steps_per_call": steps, "dp_steps": dp, "dp_overlap": ov, "batch_per_rank": B,
                      "wall_s_per_call": [round(w, 5) for w in walls],
                      "us_per_step_all_ranks_on_one_gpu": round(min(walls) / steps * 1e6, 2),
                      "note": "W ranks share one GPU: not the W-GPU time"}), flush=True)


if __name__ == "__main__":
    main()
