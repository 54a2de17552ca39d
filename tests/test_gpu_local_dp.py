"""GPU: semantics "local" at world > 1 (csrc/dist.cpp dp_run / dp_merge): users
sharded, the whole item table on every rank, the ranks' tables merged every dp_steps steps and at
every call's end.  Opt-in, NOT the reference step.  Several ranks share the box's one GPU through
the in-process loopback transport (its all-reduce sums the ranks' deltas in rank order).

What is pinned:
  * the arithmetic, by the SERIAL build (BPRMF_HOGWILD_SERIAL=1: one lane group per rank, slot
    order) against oracle/bpr_oracle.py:local_dp_serial, replayed, at worlds 2 and 3, with hot
    items, XCD periods shorter than, equal to and longer than the merge period;
  * the overlapped schedule (dp_overlap: each merge's sum lands one period later) the same way;
  * every rank ends a call with the same item table, bit for bit (across processes with the IPC
    transport's all-reduce: tests/test_gpu_ipc.py);
  * the sampled parallel mode trains (loss falls, weights finite) and its epoch covers each rank's
    own positives once.
Tolerance: the serial GPU against the float64-dot oracle, as tests/test_gpu_hogwild.py (HOG_ATOL),
a few ulp per update; the merge's decays are exp2 of fp32 products on both sides."""
import threading

import numpy as np
import pytest

from oracle import bpr_oracle as O

pytestmark = pytest.mark.gpu

HOG_ATOL = 2e-6


def _threads(rl, world, fn):
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
    assert all(not t.is_alive() for t in ts), "rank threads did not finish"
    return out


def _hot_set(pos, r, world, I, H):
    """local_setup's hot items of rank r: the top H by this rank's positive count, ties by id."""
    mine = pos[pos[:, 0] % world == r]
    cnt = np.bincount(mine[:, 1], minlength=I)
    return [int(x) for x in np.argsort(-cnt, kind="stable")[:H]]


@pytest.mark.parametrize("world,period,dp,overlap", [(2, 2, 3, False), (3, 3, 3, False), (2, 5, 2, False),
                                                     (2, 2, 3, True), (3, 5, 2, True)])
def test_local_dp_serial_replay_matches_oracle(rl, monkeypatch, world, period, dp, overlap):
    monkeypatch.setenv("BPRMF_HOGWILD_SERIAL", "1")
    H = 5
    monkeypatch.setenv("BPRMF_LOCAL_HOT", str(H))
    g = np.random.default_rng(10 * world + period + dp)
    U, I, d, B, steps = 31, 29, 32, 16, 7
    lr, wd = 0.05, 0.01
    # positives with a clear popularity order per rank (hot sets differ across ranks)
    rows = [(u, it) for u in range(U) for it in range(I) if g.random() < 0.25 / (1 + it % 7)]
    pos = np.unique(np.array(rows, np.int64), axis=0)
    P0 = (0.1 * g.standard_normal((U, d))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((I, d))).astype(np.float32)
    trips = []
    for r in range(world):
        users = np.arange(r, U, world)
        u = g.choice(users, steps * B)
        i, j = g.integers(0, I, steps * B), g.integers(0, I, steps * B)
        i[::4] = 0   # popular items often (hot on every rank)
        j[1::6] = 1
        j[:5] = i[:5]  # i == j
        trips.append((u, i, j))
    # global batches: each rank's share of step k is exactly its B triplets
    batches = [tuple(np.concatenate([trips[r][x][k * B:(k + 1) * B] for r in range(world)])
                     for x in range(3)) for k in range(steps)]
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(U, I, d, lr=lr, wd=wd, batch_size=B, device=0, comm=comm,
                            semantics="local", local_steps=period, dp_steps=dp, dp_overlap=overlap)
        m.set_train(pos)
        m.set_weights(sh.shard_rows(P0, r, world), Q0)
        m.attach_runner("loopback", key=7100 + 10 * world + dp + 1000 * overlap)
        st = m.train_replay(batches)
        return m.get_weights(), st

    parts = _threads(rl, world, fn)
    for r in range(1, world):  # one item table on every rank
        assert np.array_equal(parts[r][0][1], parts[0][0][1])
    Pp = [sh.shard_rows(P0, r, world).copy() for r in range(world)]
    hots = [_hot_set(pos, r, world, I, H) for r in range(world)]
    loss, sPs, Qw = O.local_dp_serial(Pp, Q0.copy(), trips, lr, wd, B, hots, period, dp, world,
                                      overlap=overlap)
    a = np.float32(1 - lr * wd)
    for r in range(world):
        Pw = Pp[r] * np.power(np.float64(a), (steps - sPs[r]))[:, None].astype(np.float32)
        np.testing.assert_allclose(parts[r][0][0], Pw, rtol=1e-5, atol=HOG_ATOL)
    np.testing.assert_allclose(parts[0][0][1], Qw, rtol=1e-5, atol=HOG_ATOL)
    got = sum(p[1]["loss"] for p in parts)
    assert got == pytest.approx(loss, rel=1e-5)
    assert all(p[1]["steps"] == steps for p in parts)


@pytest.mark.parametrize("overlap", [False, True])
def test_local_dp_sampled_trains_and_ranks_agree(rl, golden, overlap):
    """The parallel kernels, sampled, 2 ranks on one GPU: loss falls over epochs, tables finite,
    both ranks hold the same item table after every call, each epoch's triplets = the rank's own
    positives x num_ng."""
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    Uu, Ii = int(f["U"]), int(f["I"])
    world, B = 2, 1024
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(Uu, Ii, 32, lr=0.05, wd=0.001, batch_size=B, seed=3, device=0,
                            comm=comm, semantics="local", dp_steps=8, dp_overlap=overlap)
        S = m.set_train(pos)
        m.attach_runner("loopback", key=7300 + overlap)
        hist, qs = [], []
        for e in range(4):
            st = m.train_steps(e, 0, S)
            hist.append(st)
            qs.append(m.get_weights()[1])
        return hist, qs

    parts = _threads(rl, world, fn)
    for e in range(4):
        assert np.array_equal(parts[0][1][e], parts[1][1][e])
        assert np.isfinite(parts[0][1][e]).all()
    for r in range(world):
        mine = int((pos[:, 0] % world == r).sum())
        assert parts[r][0][0]["triplets"] == 4 * mine  # num_ng = 4
    loss = [sum(parts[r][0][e]["loss"] for r in range(world)) for e in range(4)]
    assert loss[-1] < 0.9 * loss[0], loss


def test_local_dp_exports_ipc_handles_and_hogwild_stays_single_gpu(rl):
    """The IPC transport carries this mode too (its all-reduce: tests/test_gpu_ipc.py); the
    hogwild semantics stays single-GPU."""
    sh = rl.sharded
    m = sh.HipShard(10, 10, 8, 0.01, 0.001, 64, 4, 0.01, 0, 0, 0, 2, "local", 0, 0)
    assert len(m.ipc_export()) == rl._lib.IPC_BLOB_BYTES
    with pytest.raises(Exception):
        rl.BPRMF(10, 10, 8, rank=0, world=2, semantics="hogwild")


@pytest.mark.parametrize("overlap", [False, True])
def test_local_dp_rccl_transport_one_rank_matches_oracle(rl, monkeypatch, overlap):
    """The RCCL all-reduce path (in place; overlapped: out of place on the transport's own stream,
    ordered by events) on a one-rank communicator (BPRMF_DP_ONE_RANK=1 runs the item merges at
    world 1): the SERIAL build against local_dp_serial at world 1."""
    import ctypes
    monkeypatch.setenv("BPRMF_DP_ONE_RANK", "1")
    monkeypatch.setenv("BPRMF_HOGWILD_SERIAL", "1")
    H = 4
    monkeypatch.setenv("BPRMF_LOCAL_HOT", str(H))
    g = np.random.default_rng(41 + overlap)
    U, I, d, B, steps, period, dp = 19, 23, 32, 16, 7, 2, 3
    lr, wd = 0.05, 0.01
    rows = [(u, it) for u in range(U) for it in range(I) if g.random() < 0.3 / (1 + it % 5)]
    pos = np.unique(np.array(rows, np.int64), axis=0)
    P0 = (0.1 * g.standard_normal((U, d))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((I, d))).astype(np.float32)
    u, i, j = g.integers(0, U, steps * B), g.integers(0, I, steps * B), g.integers(0, I, steps * B)
    i[::3] = 0
    j[:4] = i[:4]
    m = rl.sharded.HipShard(U, I, d, lr, wd, B, 4, 0.01, 0, 0, 0, 1, "local", period, dp, overlap)
    m.set_train(pos)
    m.set_weights(P0, Q0)
    L = rl._lib.load()
    uid = (ctypes.c_uint8 * 128)()
    rl._lib.check(L.bprmf_dist_unique_id(ctypes.addressof(uid)))
    m.runner_rccl(bytes(uid))
    st = m.runner_train_replay(u, i, j, steps)
    Pg, Qg = m.get_weights()
    Pp = [P0.copy()]
    loss, sPs, Qw = O.local_dp_serial(Pp, Q0.copy(), [(u, i, j)], lr, wd, B, [_hot_set(pos, 0, 1, I, H)],
                                      period, dp, 1, overlap=overlap)
    a = np.float32(1 - lr * wd)
    Pw = Pp[0] * np.power(np.float64(a), (steps - sPs[0]))[:, None].astype(np.float32)
    np.testing.assert_allclose(Pg, Pw, rtol=1e-5, atol=HOG_ATOL)
    np.testing.assert_allclose(Qg, Qw, rtol=1e-5, atol=HOG_ATOL)
    assert st["loss"] == pytest.approx(loss, rel=1e-5)


def test_local_dp_trains_ml100k_protocol(rl, golden):
    """F5 protocol (ml-100k fo/tfo, d=32, B=4096 per rank, 20 epochs) with 4 ranks, overlapped
    merges: HR@10 / NDCG@10 of the merged model inside the reference's spread over seeds (mean
    +- 4 std, as the single-GPU tests), loss falling."""
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "hr_ndcg_ml100k.json")) as fh:
        ref = json.load(fh)
    f = np.load(os.path.join(GOLDEN, "hr_ndcg_ml100k.npz"))
    p = ref["protocol"]
    gt = {int(u): set(f["gt_items"][f["gt_ptr"][k]:f["gt_ptr"][k + 1]].tolist())
          for k, u in enumerate(f["gt_users"])}
    Uu, Ii, world = int(f["U"]), int(f["I"]), 4
    pos = f["positives"].astype(np.int64)
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(Uu, Ii, p["factor_num"], lr=p["lr"], wd=p["wd"], batch_size=p["batch_size"],
                            num_ng=p["num_ng"], seed=11, device=0, comm=comm, semantics="local",
                            dp_steps=64, dp_overlap=True)
        S = m.set_train(pos)
        m.attach_runner("loopback", key=7500)
        losses = [m.train_steps(e, 0, S)["loss"] for e in range(p["epochs"])]
        return m.get_weights(), losses

    parts = _threads(rl, world, fn)
    P = sh.unshard_rows([x[0][0] for x in parts], Uu)
    Q = parts[0][0][1]
    losses = [sum(x[1][e] for x in parts) for e in range(p["epochs"])]
    assert losses[-1] < 0.8 * losses[0]
    m = rl.BPRMF(Uu, Ii, p["factor_num"], lr=p["lr"], wd=p["wd"], batch_size=p["batch_size"])
    m.set_weights(P, Q)
    kpi = rl.metrics.evaluate_topk(m, f["test_data"], gt, p["topk"])
    print("local x4 F5:", kpi, "reference:", ref["summary"])
    for k in ("hr", "ndcg"):
        mu, sd = ref["summary"][k]["mean"], ref["summary"][k]["std"]
        assert abs(kpi[k] - mu) <= 4 * sd + 1e-9, (k, kpi[k], mu, sd)


def test_local_dp_replay_merges_follow_dp_steps_across_chunks(rl, monkeypatch):
    """A replay longer than the runner's chunk (BPRMF_DIST_CHUNK=2 here; 2^20 / B steps by
    default) merges every dp_steps steps and at the call's end, like a sampled call, not at every
    chunk boundary: the SERIAL build against local_dp_serial with dp_steps 5."""
    monkeypatch.setenv("BPRMF_HOGWILD_SERIAL", "1")
    monkeypatch.setenv("BPRMF_DIST_CHUNK", "2")
    H, world, period, dp = 4, 2, 3, 5
    monkeypatch.setenv("BPRMF_LOCAL_HOT", str(H))
    g = np.random.default_rng(77)
    U, I, d, B, steps = 23, 19, 32, 8, 7
    lr, wd = 0.05, 0.01
    rows = [(u, it) for u in range(U) for it in range(I) if g.random() < 0.3 / (1 + it % 5)]
    pos = np.unique(np.array(rows, np.int64), axis=0)
    P0 = (0.1 * g.standard_normal((U, d))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((I, d))).astype(np.float32)
    trips = []
    for r in range(world):
        u = g.choice(np.arange(r, U, world), steps * B)
        i, j = g.integers(0, I, steps * B), g.integers(0, I, steps * B)
        i[::3] = 0
        trips.append((u, i, j))
    batches = [tuple(np.concatenate([trips[r][x][k * B:(k + 1) * B] for r in range(world)])
                     for x in range(3)) for k in range(steps)]
    sh = rl.sharded

    def fn(comm, r):
        m = sh.ShardedBPRMF(U, I, d, lr=lr, wd=wd, batch_size=B, device=0, comm=comm,
                            semantics="local", local_steps=period, dp_steps=dp)
        m.set_train(pos)
        m.set_weights(sh.shard_rows(P0, r, world), Q0)
        m.attach_runner("loopback", key=7700)
        return m.train_replay(batches), m.get_weights()

    parts = _threads(rl, world, fn)
    Pp = [sh.shard_rows(P0, r, world).copy() for r in range(world)]
    hots = [_hot_set(pos, r, world, I, H) for r in range(world)]
    loss, _, Qw = O.local_dp_serial(Pp, Q0.copy(), trips, lr, wd, B, hots, period, dp, world)
    np.testing.assert_allclose(parts[0][1][1], Qw, rtol=1e-5, atol=HOG_ATOL)
    assert np.array_equal(parts[1][1][1], parts[0][1][1])
    assert sum(p[0]["loss"] for p in parts) == pytest.approx(loss, rel=1e-5)


def test_local_dp_refuses_per_step_calls(rl):
    """The per-step sharded API addresses items by owner (i % world); with the item table
    replicated (semantics "local", world > 1) it is refused instead of updating wrong rows."""
    sh = rl.sharded
    pos = np.array([[u, (u * 7 + k) % 13] for u in range(10) for k in range(3)], np.int64)

    def fn(comm, r):
        m = sh.ShardedBPRMF(10, 13, 32, batch_size=8, device=0, comm=comm, semantics="local")
        m.set_train(pos)
        with pytest.raises(ValueError, match="runner"):
            m.step(0, 0)
        with pytest.raises(ValueError, match="runner"):
            m.plan_replay([(np.array([0, 1]), np.array([1, 2]), np.array([3, 4]))])
        # and the C ABI itself refuses (a caller that bypasses the Python check)
        with pytest.raises(Exception, match="replicates the item table"):
            m.b.plan(0, 0, 1)
        return True

    assert all(_threads(rl, 2, fn))
