"""GPU: the split batch builder's cross-workgroup protocol against stale memory (DESIGN.md §3.2,
§6 "the round-3 wrong result").

The split builder's workgroups of one batch exchange their counts (and, when they sample in the
launch, their "staged" marks) through words in the batch buffer tagged with the launch's tag.  In
round 3 the tags were a plain process-wide counter (1, 2, 3, ...) and the buffer came from plain
hipMalloc: a recycled block still held an earlier handle's records (small ints), so in a fresh
process a word could already carry the current launch's tag before its writer published it.  A
part then read garbage counts, or a workgroup read triplets not yet staged, and the step applied
a wrong batch: silently wrong weights.

Fix: the buffer is zeroed when allocated, tags carry a marker bit (bit 31) no record int has, the
sampling board compares a full 64-bit {magic, tag} word.  These tests plant the condition on
purpose: before every build the whole batch buffer is filled with the value the old scheme would
have used as that build's tag (the new tag without its marker bit), and the result must equal a
run on clean memory bit for bit (and the dense oracle for the sharded form, after every step).
"""
import importlib
import threading

import numpy as np
import pytest

from oracle import bpr_oracle as O

pytestmark = pytest.mark.gpu


def _old_style(tag):
    return tag & 0x7FFFFFFF  # what the round-3 counter would have carried for this launch


@pytest.mark.parametrize("smp", ["1", "0"])
def test_single_gpu_split_build_ignores_planted_tags(rl, monkeypatch, smp):
    """Single GPU, sampled chunks (the split builder with in-launch sampling, SMP=1, or after a
    k_sample launch, SMP=0): planted words never change the batches."""
    monkeypatch.setenv("BPRMF_SPLIT_SAMPLE", smp)
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, d, B, seed = 2000, 1500, 32, 1024, 77
    pos = syn.make_positives(U, I, 60_000, seed)
    outs = []
    for plant in (False, True):
        m = rl.BPRMF(U, I, d, batch_size=B, seed=seed)
        m.set_train(pos)  # allocates the batch buffer (zeroed)
        losses = []
        for call in range(4):
            if plant:
                m.debug_fill_batches(_old_style(rl._lib.next_build_tag()))
            losses.append(m.train_steps(0, 5 * call, 5)["loss"])
        outs.append((m.get_weights(), losses))
        m.close()
    (Pa, Qa), la = outs[0]
    (Pb, Qb), lb = outs[1]
    assert np.array_equal(Pa, Pb) and np.array_equal(Qa, Qb)
    assert la == lb


def test_single_gpu_replay_build_ignores_planted_tags(rl):
    """Replayed triplets (the split builder without sampling) with planted words: bitwise equal
    to the clean run."""
    g = np.random.default_rng(5)
    U, I, d, B = 301, 157, 64, 512
    P0 = (0.05 * g.standard_normal((U, d))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, d))).astype(np.float32)
    n = 7 * B
    u, i, j = g.integers(0, U, n), g.integers(0, I, n), g.integers(0, I, n)
    i[:60] = 3  # a hot item
    res = []
    for plant in (False, True):
        m = rl.BPRMF(U, I, d, lr=0.05, wd=0.01, batch_size=B)
        m.set_weights(P0, Q0)
        m.train_triplets(u[:B], i[:B], j[:B])  # allocates the batch buffer
        if plant:
            m.debug_fill_batches(_old_style(rl._lib.next_build_tag()))
        m.train_triplets(u[B:], i[B:], j[B:])
        res.append(m.get_weights())
        m.close()
    for x, y in zip(res[0], res[1]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_plan_build_ignores_planted_tags(rl, world):
    """The round-3 failure's path: in-process shards stepped by the per-step Python orchestration
    (ThreadComm), batches built by the sharded split builder (owner-major slots).  Every shard's
    build runs over a buffer filled with its own launch's old-style tag; the union step must equal
    the dense oracle after EVERY step (failures name the step)."""
    sh = rl.sharded
    U, I, D = 301, 157, 128
    g = np.random.default_rng(40 + world)
    P0 = (0.05 * g.standard_normal((U, D))).astype(np.float32)
    Q0 = (0.05 * g.standard_normal((I, D))).astype(np.float32)
    GB, steps = 512, 6
    batches = []
    for _ in range(steps):
        u, i, j = g.integers(0, U, GB), g.integers(0, I, GB), g.integers(0, I, GB)
        i[:40] = 7
        batches.append((u, i, j))
    lock = threading.Lock()  # one build at a time: each shard knows its launch's tag
    grp = sh.ThreadGroup(world)
    snaps, errs = [[None] * steps for _ in range(world)], []

    def run(r):
        try:
            comm = sh.ThreadComm(grp, r)
            m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=GB, device=0, comm=comm)
            m.set_weights(sh.shard_rows(P0, r, world), sh.shard_rows(Q0, r, world))
            m.plan_replay(batches)  # allocates (and zeroes) the batch buffer
            Ul, Il, Jl, n = m._local_batches(batches)
            with lock:
                m.b.m.debug_fill_batches(_old_style(rl._lib.next_build_tag()))
                send = m.b.plan_replay(Ul, Il, Jl, n)
            recv = comm.exchange_counts(send, m.device)
            m._plan = ("replay", 0, n, send, recv)
            for k in range(steps):
                m.step_replay(k)
                snaps[r][k] = m.get_weights()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    if errs:
        raise errs[0]
    Pr, Qr = P0.copy(), Q0.copy()
    for k, (u, i, j) in enumerate(batches):
        O.bpr_step_dense(Pr, Qr, u, i, j, 0.05, 0.01)
        for r in range(world):
            Pk, Qk = snaps[r][k]
            for name, got, want in (("P", Pk, Pr[r::world]), ("Q", Qk, Qr[r::world])):
                bad = ~np.isclose(got, want, rtol=1e-5, atol=1e-6)
                assert not bad.any(), (f"step {k}, rank {r}: {name} differs from the dense oracle in "
                                       f"{int(bad.sum())} of {bad.size} elements "
                                       f"(max {np.abs(got - want).max():.3g})")


def test_timed_out_build_leaves_tables_untouched(rl):
    """A batch whose split build timed out carries a dead mark (kernels.h kMetaDead) that every
    step workgroup of that batch reads beside meta[0]: the steps skip it and the call fails with
    the builder's error.  The step counter still advances (rows decay lazily as over steps with no
    triplets), so the tables equal the earlier ones times the decay of those steps; the host clears
    the buffer, and the next call trains normally."""
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, d, B, seed = 900, 700, 32, 512, 5
    lr, wd = 0.05, 0.001
    pos = syn.make_positives(U, I, 20_000, seed)
    m = rl.BPRMF(U, I, d, lr=lr, wd=wd, batch_size=B, seed=seed, device=0)
    m.set_train(pos)
    m.train_steps(0, 0, 4)
    P0, Q0 = m.get_weights()
    m.debug_fail_build()
    with pytest.raises(rl.BprmfError, match="batch builder"):
        # a short chunk: the split builder (the one with the timed waits), then fused steps
        m.train_steps(0, 4, 6)
    P1, Q1 = m.get_weights()
    dec = (1 - lr * wd) ** 6  # a real step moves rows by ~1e-2 relative: far outside rtol
    np.testing.assert_allclose(P1, P0 * dec, rtol=2e-6, atol=1e-9)
    np.testing.assert_allclose(Q1, Q0 * dec, rtol=2e-6, atol=1e-9)
    st = m.train_steps(0, 10, 6)
    assert np.isfinite(st["loss"]) and st["loss"] > 0
    P2, _ = m.get_weights()
    assert not np.allclose(P2, P1 * dec, rtol=1e-4)
