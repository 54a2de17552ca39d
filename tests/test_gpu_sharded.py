"""GPU: the sharded step kernels (bprmf_dist_*) through the real orchestrator, several shards on
the one GPU of the box stepped by threads (ThreadComm in place of RCCL).  G shards stepping their
users' share of each global batch == one single-GPU step on the whole global batch."""
import threading

import numpy as np
import pytest

from oracle import bpr_oracle as O
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

U, I, D = 301, 157, 128


def _run_threads(rl, world, fn):
    grp = rl.sharded.ThreadGroup(world)
    out, errs = [None] * world, []

    def run(r):
        try:
            out[r] = fn(rl.sharded.ThreadComm(grp, r), r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_sharded_replay_equals_single_gpu_global_batch(rl, world):
    g = np.random.default_rng(world)
    P0 = (0.05 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, D))).astype(np.float32)
    GB, steps = 512, 6
    batches = []
    for k in range(steps):
        u, i, j = g.integers(0, U, GB), g.integers(0, I, GB), g.integers(0, I, GB)
        i[:40] = 7  # hot item (> kLongSeg references)
        batches.append((u, i, j))
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=GB, device=0, comm=comm)
        m.set_weights(sh.shard_rows(P0, r, world), sh.shard_rows(Q0, r, world))
        m.plan_replay(batches)
        snaps = []
        for k in range(steps):
            m.step_replay(k)
            snaps.append(m.get_weights())  # every step's state, checked below
        return snaps

    parts = _run_threads(rl, world, fn)
    Pr, Qr = P0.copy(), Q0.copy()
    for k, (u, i, j) in enumerate(batches):
        O.bpr_step_dense(Pr, Qr, u, i, j, 0.05, 0.01)
        for r in range(world):
            for name, got, want in (("P", parts[r][k][0], Pr[r::world]), ("Q", parts[r][k][1], Qr[r::world])):
                bad = ~np.isclose(got, want, rtol=1e-5, atol=1e-6)
                assert not bad.any(), (f"world {world}, step {k}, rank {r}: {name} differs from the "
                                       f"dense oracle in {int(bad.sum())} of {bad.size} elements "
                                       f"(max {np.abs(got - want).max():.3g})")


@pytest.mark.parametrize("Uu,Ii", [(16, 32), (4, 8)])
def test_sharded_replay_power_of_two_shards(rl, Uu, Ii):
    """Two shards whose local user counts are powers of two: each shard's batch has empty slots
    (the other shard's triplets) in the middle, whose sort key must order after every local user
    (regression: with log2(rows) sort bits it collided with the last user and split its segment)."""
    g = np.random.default_rng(Uu)
    world, GB, steps, d = 2, 64, 5, 8
    P0 = (0.1 * g.standard_normal((Uu, d))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((Ii, d))).astype(np.float32)
    batches = [(g.integers(0, Uu, GB), g.integers(0, Ii, GB), g.integers(0, Ii, GB)) for _ in range(steps)]
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(Uu, Ii, d, lr=0.05, wd=0.01, batch_size=GB, device=0, comm=comm)
        m.set_weights(sh.shard_rows(P0, r, world), sh.shard_rows(Q0, r, world))
        m.plan_replay(batches)
        for k in range(steps):
            m.step_replay(k)
        return m.get_weights()

    parts = _run_threads(rl, world, fn)
    P = sh.unshard_rows([p[0] for p in parts], Uu)
    Q = sh.unshard_rows([p[1] for p in parts], Ii)
    Pr, Qr = P0.copy(), Q0.copy()
    for u, i, j in batches:
        O.bpr_step_dense(Pr, Qr, u, i, j, 0.05, 0.01)
    np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)


def test_sharded_sampler_training(rl, golden):
    """Sampler mode over 2 shards: each shard's batches are its own users' triplets, bit-exact with
    the oracle sampler for that shard; training reduces the loss."""
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    Uu, Ii = int(f["U"]), int(f["I"])
    world, B, seed = 2, 2048, 31
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(Uu, Ii, 32, batch_size=B, seed=seed, device=0, comm=comm)
        S = m.set_train(pos)
        losses = []
        for e in range(3):
            tot = 0.0
            for s in range(S):
                tot += m.step(e, s, want_loss=True)
            losses.append(tot)
        return S, losses

    out = _run_threads(rl, world, fn)
    S = out[0][0]
    for r in range(world):
        mine = pos[pos[:, 0] % world == r]
        assert S >= (len(mine) * 4 + B - 1) // B
        l = out[r][1]
        assert l[-1] < l[0], l
    # shard 1's sampler == the oracle's (shard seed = seed + rank * 0x9E3779B97F4A7C15)
    m1 = rl.BPRMF(Uu, Ii, 8, batch_size=B, seed=seed, rank=1, world=world)
    m1.set_train(pos)
    mine = pos[pos[:, 0] % world == 1]
    indptr, indices = O.build_csr(mine[:, 0], mine[:, 1], Uu)
    got = m1.sample(0, 0, 1000)
    want = C.sample(mine[:, 0], mine[:, 1], indptr, indices, Ii, 4,
                    (seed + 0x9E3779B97F4A7C15) & (2**64 - 1), 0, 0, 1000)
    for x, y in zip(got, want):
        assert np.array_equal(x, y)


# ---- the library-driven runner (bprmf_dist_train_*): exchanges issued from C++ ---------------
def _runner_threads(rl, world, key, fn):
    """`world` shards in this process, one thread each, loopback transport group `key`."""
    grp = rl.sharded.ThreadGroup(world)
    out, errs = [None] * world, []

    def run(r):
        try:
            out[r] = fn(rl.sharded.ThreadComm(grp, r), r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    if errs:
        raise errs[0]
    assert all(not t.is_alive() for t in ts), "runner threads did not finish"
    return out


def _batches(g, steps, GB, hot=True):
    out = []
    for _ in range(steps):
        u, i, j = g.integers(0, U, GB), g.integers(0, I, GB), g.integers(0, I, GB)
        if hot:
            i[:40] = 7  # hot item (> kLongSeg references)
        out.append((u, i, j))
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_runner_replay_equals_single_gpu_global_batch(rl, world):
    g = np.random.default_rng(100 + world)
    P0 = (0.05 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, D))).astype(np.float32)
    GB, steps = 512, 7
    batches = _batches(g, steps, GB)
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=GB, device=0, comm=comm)
        m.set_weights(sh.shard_rows(P0, r, world), sh.shard_rows(Q0, r, world))
        m.attach_runner("loopback", key=1000 + world)
        st = m.train_replay(batches)
        return m.get_weights(), st

    parts = _runner_threads(rl, world, 1000 + world, fn)
    P = sh.unshard_rows([p[0][0] for p in parts], U)
    Q = sh.unshard_rows([p[0][1] for p in parts], I)
    Pr, Qr = P0.copy(), Q0.copy()
    loss = 0.0
    for u, i, j in batches:
        loss += O.bpr_step_dense(Pr, Qr, u, i, j, 0.05, 0.01)
    np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)
    assert sum(p[1]["triplets"] for p in parts) == steps * GB
    got_loss = sum(p[1]["loss"] for p in parts)
    assert abs(got_loss - loss) <= 1e-4 * abs(loss), (got_loss, loss)


def test_runner_sampler_matches_python_orchestration_and_is_reproducible(rl, golden):
    """Sampler mode, 2 shards: the C++ runner and the per-step Python orchestration take the same
    steps (same batches, same exchanges); the runner is bitwise reproducible run to run."""
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    Uu, Ii = int(f["U"]), int(f["I"])
    world, B, seed, d = 2, 1024, 5, 64
    sh = rl.sharded

    def runner(comm, r, key):
        m = sh.ShardedBPRMF(Uu, Ii, d, batch_size=B, seed=seed, device=0, comm=comm)
        S = m.set_train(pos)
        m.attach_runner("loopback", key=key)
        m.train_steps(0, 0, S)
        m.train_steps(1, 0, 9)
        return m.get_weights()

    def python_path(comm, r):
        m = sh.ShardedBPRMF(Uu, Ii, d, batch_size=B, seed=seed, device=0, comm=comm)
        S = m.set_train(pos)
        for s in range(S):
            m.step(0, s)
        for s in range(9):
            m.step(1, s)
        return m.get_weights()

    a = _runner_threads(rl, world, 2001, lambda c, r: runner(c, r, 2001))
    b = _runner_threads(rl, world, 2002, lambda c, r: runner(c, r, 2002))
    c = _runner_threads(rl, world, 0, python_path)
    for r in range(world):
        for x, y, z in zip(a[r], b[r], c[r]):
            assert np.array_equal(x, y), "runner not bitwise reproducible"
            np.testing.assert_allclose(x, z, rtol=1e-5, atol=1e-6)


def test_world1_runner_equals_single_gpu_path(rl, golden, monkeypatch):
    """At one rank train_steps runs the single-GPU fused step (nothing to exchange);
    BPRMF_DIST_W1_RUNNER=1 keeps the sharded runner (owner gather, K1 on the gathered rows, K2's
    per-slot gradients, owner apply), which tools/gpu/stale1_parts.sh measures.  Both take the same
    steps from the same sampler stream: equal to fp32 summation-order tolerance, losses too."""
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    Uu, Ii = int(f["U"]), int(f["I"])
    B, seed, d = 1024, 13, 64
    sh = rl.sharded
    outs = []
    for env in ("0", "1"):
        monkeypatch.setenv("BPRMF_DIST_W1_RUNNER", env)

        def runner(comm, r, key):
            m = sh.ShardedBPRMF(Uu, Ii, d, batch_size=B, seed=seed, device=0, comm=comm)
            S = m.set_train(pos)
            m.attach_runner("loopback", key=key)
            a = m.train_steps(0, 0, S)
            b = m.train_steps(1, 3, 9)
            return m.get_weights(), a["loss"] + b["loss"]

        key = 4100 + int(env)
        outs.append(_runner_threads(rl, 1, key, lambda c, r: runner(c, r, key))[0])
    (Pa, Qa), la = outs[0]
    (Pb, Qb), lb = outs[1]
    np.testing.assert_allclose(Pa, Pb, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Qa, Qb, rtol=1e-5, atol=1e-6)
    assert la == pytest.approx(lb, rel=1e-5)


@pytest.mark.parametrize("world", [1, 3, 8])
def test_runner_split_builder_equals_one_workgroup_build(rl, golden, monkeypatch, world):
    """The runner's batches (owner-major item slots, padded per owner) from the split builder (one
    user and eight item-part workgroups per batch) and from the one-workgroup builder give the
    same training bit for bit, sampled chunks of both lengths included."""
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    Uu, Ii = int(f["U"]), int(f["I"])
    B, seed, d = 1024, 9, 32
    sh = rl.sharded
    outs = []
    for env in ("1", "0"):
        monkeypatch.setenv("BPRMF_SPLIT_ITEMS", env)

        def runner(comm, r, key):
            m = sh.ShardedBPRMF(Uu, Ii, d, batch_size=B, seed=seed, device=0, comm=comm)
            S = m.set_train(pos)
            m.attach_runner("loopback", key=key)
            m.train_steps(0, 0, S)
            st = m.train_steps(1, 2, 7)
            return m.get_weights(), st["loss"]

        key = 3000 + 10 * world + int(env)
        outs.append(_runner_threads(rl, world, key, lambda c, r: runner(c, r, key)))
    for r in range(world):
        (Pa, Qa), la = outs[0][r]
        (Pb, Qb), lb = outs[1][r]
        assert np.array_equal(Pa, Pb) and np.array_equal(Qa, Qb)
        assert la == lb


def test_runner_rccl_transport_one_rank(rl):
    """The RCCL transport (library-owned communicator, unique id broadcast by the process group)
    at world 1, graph-captured or eager, with or without RCCL carrying the self blocks, gives the
    loopback transport's result bit for bit."""
    import os
    import torch
    import torch.distributed as dist
    g = np.random.default_rng(7)
    P0 = (0.05 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, D))).astype(np.float32)
    batches = _batches(g, 5, 256)
    sh = rl.sharded
    res = []
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    # rccl: steps replayed from a captured hipGraph; rccl + self exchange: this rank's own blocks
    # go through RCCL send/recv inside the captured graph; loopback: eager, device copies
    cases = [("rccl", {}), ("rccl", {"BPRMF_DIST_SELF_EXCHANGE": "1"}), ("loopback", {}),
             ("rccl", {"BPRMF_NO_GRAPH": "1"})]
    try:
        for transport, env in cases:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=256, device=0)
                m.set_weights(P0, Q0)
                m.attach_runner(transport, key=3001)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k)
                    else:
                        os.environ[k] = v
            m.train_replay(batches)  # first sighting of the chunk shape: eager launches
            m.train_replay(batches)  # second: captured into a hipGraph
            m.train_replay(batches)  # third: the cached graph is replayed
            res.append(m.get_weights())
    finally:
        if own:
            dist.destroy_process_group()
    for r in res[1:]:
        for x, y in zip(res[0], r):
            assert np.array_equal(x, y)


def test_python_orchestrated_steps_over_nccl_world1(rl):
    """The per-step Python path (plan_replay + step_replay over TorchComm on nccl = RCCL) at world
    1 against the dense oracle: the library's kernels and torch's collectives and allocations run
    on one dedicated non-default stream, from torch's default stream and from a side stream."""
    import os
    import torch
    import torch.distributed as dist
    g = np.random.default_rng(17)
    P0 = (0.05 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, D))).astype(np.float32)
    batches = _batches(g, 6, 512)
    sh = rl.sharded
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        outs = []
        for side in (False, True):
            m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=512, device=0)
            m.set_weights(P0, Q0)
            m.plan_replay(batches)
            ctx = torch.cuda.stream(torch.cuda.Stream(0)) if side else torch.cuda.stream(
                torch.cuda.current_stream(0))
            with ctx:
                for k in range(len(batches)):
                    m.step_replay(k)
            torch.cuda.synchronize()
            outs.append(m.get_weights())
    finally:
        if own:
            dist.destroy_process_group()
    Pr, Qr = P0.copy(), Q0.copy()
    for u, i, j in batches:
        O.bpr_step_dense(Pr, Qr, u, i, j, 0.05, 0.01)
    for P, Q in outs:
        np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)
