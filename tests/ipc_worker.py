"""Worker of tests/test_gpu_ipc.py (not a test module): one rank of a 2-process sharded run on the
box's one GPU, gloo process group for the handle exchange, the library's IPC transport for the
steps.  Writes its shard's weights and stats to OUT (npz)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, mode = sys.argv[1], sys.argv[2]
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    rl = importlib.import_module("recommend-lib_amd")
    sh = rl.sharded
    spec = np.load(os.environ["IPC_SPEC"])
    U, I, D, B = (int(spec[k]) for k in ("U", "I", "D", "B"))
    local = mode == "local"  # semantics "local": the item table replicated, merged by all-reduce
    kw = dict(semantics="local", local_steps=int(spec["period"]), dp_steps=int(spec["dp"]),
              dp_overlap=bool(spec["overlap"])) if local else {}
    if mode in ("stale1", "stale1_auto"):  # the stale-1 step's device-flag form (IPC transport)
        kw = dict(semantics="stale1")
    m = sh.ShardedBPRMF(U, I, D, lr=float(spec["lr"]), wd=float(spec["wd"]), batch_size=B,
                        seed=int(spec["seed"]), device=0, **kw)
    if local:
        m.set_train(spec["pos"])
        m.set_weights(sh.shard_rows(spec["P0"], rank, world), spec["Q0"])
        m.attach_runner("ipc")
        batches = [(spec["u"][k], spec["i"][k], spec["j"][k]) for k in range(spec["u"].shape[0])]
        st = m.train_replay(batches)
        st2 = m.train_replay(batches)
    elif mode in ("replay", "stale1", "stale1_auto"):
        m.set_weights(sh.shard_rows(spec["P0"], rank, world), sh.shard_rows(spec["Q0"], rank, world))
        m.attach_runner("auto" if mode == "stale1_auto" else "ipc")
        batches = [(spec["u"][k], spec["i"][k], spec["j"][k]) for k in range(spec["u"].shape[0])]
        st = m.train_replay(batches)
        st2 = m.train_replay(batches)  # replays the captured step graph
    else:
        S = m.set_train(spec["pos"])
        m.attach_runner("ipc")
        st = m.train_steps(0, 0, S)
        st2 = m.train_steps(1, 0, 5)
    torch.cuda.synchronize()
    P, Q = m.get_weights()
    np.savez(out, P=P, Q=Q, loss=st["loss"] + st2["loss"], triplets=st["triplets"] + st2["triplets"],
             runner=str(m.runner))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
