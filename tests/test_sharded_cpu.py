"""CPU, world_size 2 over gloo: the sharded orchestrator (ShardedBPRMF + TorchComm) exchanges ids,
rows and gradients correctly.  G ranks stepping their users' share of each global batch must equal
one dense reference step on the whole global batch (the oracle)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, load_pkg

U, I, D, LR, WD = 37, 29, 8, 0.05, 0.01
STEPS, GB = 5, 64  # global batch of 64 triplets per step


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    g = np.random.default_rng(5)
    P0 = (0.1 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((I, D))).astype(np.float32)
    batches = []
    for k in range(STEPS):
        u = g.integers(0, U, GB)
        i = g.integers(0, I, GB)
        j = g.integers(0, I, GB)
        if k == 2:
            i[:20] = 3  # a hot item
        batches.append((u, i, j))
    return P0, Q0, batches


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_fake import FakeShard
        sh = load_pkg().sharded
        P0, Q0, batches = _problem()
        fake = FakeShard(U, I, D, LR, WD, GB, rank, world, sh.shard_rows(P0, rank, world),
                         sh.shard_rows(Q0, rank, world))
        m = sh.ShardedBPRMF(U, I, D, lr=LR, wd=WD, batch_size=GB, backend=fake)
        m.plan_replay(batches)
        for k in range(STEPS):
            m.step_replay(k)
        P, Q = m.get_weights()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), P=P, Q=Q)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_equals_global_batch_step(tmp_path, world):
    from oracle import bpr_oracle as O
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    sh = load_pkg().sharded
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    P = sh.unshard_rows([p["P"] for p in parts], U)
    Q = sh.unshard_rows([p["Q"] for p in parts], I)
    P0, Q0, batches = _problem()
    for u, i, j in batches:
        O.bpr_step_dense(P0, Q0, u, i, j, LR, WD)
    np.testing.assert_allclose(P, P0, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(Q, Q0, rtol=1e-5, atol=1e-7)


def test_thread_comm_matches_torch_comm_semantics():
    """ThreadComm (in-process shards) implements the same all-to-all as torch.distributed."""
    import threading
    sh = load_pkg().sharded
    world = 3
    grp = sh.ThreadGroup(world)
    outs = [None] * world

    def run(r):
        c = sh.ThreadComm(grp, r)
        sc = np.array([r + 1, 0, 2])  # rank r sends r+1 rows to 0, none to 1, 2 to 2
        inp = torch.arange(sc.sum(), dtype=torch.float32) + 100 * r
        counts = c.exchange_counts(sc[None, :].astype(np.int32), None)[0]
        out = torch.empty(int(counts.sum()))
        c.all_to_all(out, inp, counts, sc)
        outs[r] = (counts.tolist(), out.tolist())

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert outs[0] == ([1, 2, 3], [0.0, 100.0, 101.0, 200.0, 201.0, 202.0])
    assert outs[1] == ([0, 0, 0], [])
    assert outs[2] == ([2, 2, 2], [1.0, 2.0, 102.0, 103.0, 203.0, 204.0])
