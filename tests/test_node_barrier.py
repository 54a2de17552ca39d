"""The node barrier (include/bprmf.h bprmf_node_barrier_*, csrc/node_barrier.cpp): host only, so
it runs here without a GPU.  Several processes meet many times; no rank may leave a generation
before every rank has entered it, and a missing rank ends in an error, not a hang."""
import multiprocessing as mp
import os
import time

import pytest


def _rank(path, world, rank, iters, start, out):
    import importlib
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    rl = importlib.import_module("recommend-lib_amd")
    start.wait()
    b = rl.sharded.NodeBarrier(path, world, rank, create=False)
    ins, outs = [], []
    for _ in range(iters):
        if rank == (len(ins) % world):
            time.sleep(0.002)  # a late rank, a different one each time
        ins.append(time.monotonic_ns())
        b.wait(30.0)
        outs.append(time.monotonic_ns())
    b.close()
    out.put((rank, ins, outs))


def test_no_rank_leaves_before_all_arrive(rl, tmp_path):
    world, iters = 4, 60
    path = str(tmp_path / "barrier")
    b0 = rl.sharded.NodeBarrier(path, world, 0, create=True)  # made before the ranks open it
    ctx = mp.get_context("spawn")
    start, out = ctx.Barrier(world), ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(path, world, r, iters, start, out)) for r in range(world)]
    [p.start() for p in ps]
    res = {}
    for _ in range(world):
        r, ins, outs = out.get(timeout=240)
        res[r] = (ins, outs)
    [p.join(timeout=60) for p in ps]
    b0.close()
    assert all(p.exitcode == 0 for p in ps)
    for k in range(iters):
        last_in = max(res[r][0][k] for r in range(world))
        first_out = min(res[r][1][k] for r in range(world))
        assert first_out >= last_in, k


def test_missing_rank_times_out(rl, tmp_path):
    path = str(tmp_path / "barrier2")
    b = rl.sharded.NodeBarrier(path, 2, 0, create=True)
    t0 = time.monotonic()
    with pytest.raises(Exception):
        b.wait(0.2)
    assert time.monotonic() - t0 < 10
    # the timed-out arrival is still counted: the barrier is poisoned, so a peer arriving now
    # (which would otherwise complete the generation with one rank short) and every later wait
    # of this rank fail at once
    peer = rl.sharded.NodeBarrier(path, 2, 1, create=False)
    t0 = time.monotonic()
    with pytest.raises(Exception, match="poisoned"):
        peer.wait(30.0)
    with pytest.raises(Exception, match="poisoned"):
        b.wait(30.0)
    assert time.monotonic() - t0 < 5
    peer.close()
    with pytest.raises(Exception):  # a different world size on the same file is refused
        rl.sharded.NodeBarrier(path, 3, 1, create=False)
    b.close()
    assert os.path.exists(path)
