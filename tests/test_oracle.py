"""CPU: the oracle is pinned against the reference's own outputs (tests/golden, made by importing
the reference in the build container: tests/golden/make_golden.py) before anything trusts it."""
import json
import os

import numpy as np
import pytest
from scipy import stats

from conftest import GOLDEN
from oracle import bpr_oracle as O
from oracle import c_oracle as C

# Tolerance of the fp32 restatement vs torch (different summation order / fused ops only).
ORACLE_ATOL = 5e-8


def test_dense_step_matches_reference_tiny(golden):
    f = golden("bpr_step_tiny.npz")
    P, Q = f["P0"].copy(), f["Q0"].copy()
    for b in range(f["triplets"].shape[0]):
        t = f["triplets"][b]
        loss = O.bpr_step_dense(P, Q, t[0], t[1], t[2], float(f["lr"]), float(f["wd"]))
        np.testing.assert_allclose(P, f["P"][b], rtol=0, atol=ORACLE_ATOL)
        np.testing.assert_allclose(Q, f["Q"][b], rtol=0, atol=ORACLE_ATOL)
        assert abs(loss - f["loss"][b]) <= 1e-5 * abs(f["loss"][b])


def test_dense_step_matches_reference_ml100k_epoch(golden):
    f = golden("bpr_ml100k_replay.npz")
    tr = f["triplets"].astype(np.int64)
    bd = f["batch_bounds"]
    P, Q = f["P0"].copy(), f["Q0"].copy()
    losses = O.train_replay(P, Q, tr, bd, float(f["lr"]), float(f["wd"]))
    np.testing.assert_allclose(P, f["P_epoch"], rtol=0, atol=ORACLE_ATOL)
    np.testing.assert_allclose(Q, f["Q_epoch"], rtol=0, atol=ORACLE_ATOL)
    np.testing.assert_allclose(losses, f["loss"], rtol=1e-5)


def test_c_dense_step_matches_reference(golden):
    f = golden("bpr_ml100k_replay.npz")
    tr = f["triplets"].astype(np.int32)
    bd = f["batch_bounds"]
    D = C.DenseTrainer(f["P0"], f["Q0"], f["lr"], f["wd"])
    for b in range(10):
        D.step(tr[0, bd[b]:bd[b + 1]], tr[1, bd[b]:bd[b + 1]], tr[2, bd[b]:bd[b + 1]])
    np.testing.assert_allclose(D.P, f["P10"], rtol=0, atol=ORACLE_ATOL)
    np.testing.assert_allclose(D.Q, f["Q10"], rtol=0, atol=ORACLE_ATOL)


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 10 rounds
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = O.philox4x32_10(*ctr, *key)
        assert tuple(int(x) for x in got) == want


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 16, 17, 63, 64, 65, 1000, 4097, 100003])
def test_permutation_is_bijection(n):
    q = O.permute(np.arange(n), n, 987654321, 7)
    assert np.array_equal(np.sort(q), np.arange(n))
    for s in (0, n // 2, n - 1):
        assert C.lib().oracle_permute(s, n, 987654321, 7) == q[s]


@pytest.mark.parametrize("n", [2, 3, 15, 16, 17, 32_557_604, 548_000_000, 10**12 + 7])
def test_feistel_domain_is_tight(n):
    # Z_a x Z_c covers [0, n) with fewer than c extra points: a walk past n is rare (< 1/sqrt(n))
    a, c = O.feistel_dims(n)
    assert a * c >= n and a * c - n < c and (c - 1) ** 2 < n <= c * c
    x = np.arange(min(n, 200_000), dtype=np.int64) * (n // min(n, 200_000))
    q = O.permute(x, n, 11, 3)
    assert (q >= 0).all() and (q < n).all() and len(np.unique(q)) == len(q)
    for k in (0, len(x) // 2, len(x) - 1):  # the C restatement agrees at this size too
        assert C.lib().oracle_permute(int(x[k]), n, 11, 3) == q[k]


def test_kth_nonmember_bruteforce():
    g = np.random.default_rng(3)
    I = 50
    users, items = [], []
    for u in range(20):
        deg = int(g.integers(0, 49))
        for i in g.choice(I, deg, replace=False):
            users.append(u)
            items.append(int(i))
    indptr, indices = O.build_csr(np.array(users), np.array(items), 20)
    for u in range(20):
        pos = set(indices[indptr[u]:indptr[u + 1]].tolist())
        free = [x for x in range(I) if x not in pos]
        ks = np.arange(len(free))
        got = O.kth_nonmember(indptr, indices, np.full(len(ks), u), ks)
        assert got.tolist() == free


def test_sampler_numpy_and_c_restatements_agree(golden):
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    U, I = int(f["U"]), int(f["I"])
    indptr, indices = O.build_csr(pos[:, 0], pos[:, 1], U)
    N = len(pos) * 4
    for epoch, first, cnt in ((0, 0, N), (5, 1234, 5000), (2**31 + 3, N - 777, 777)):
        a = O.sample_triplets(pos[:, 0], pos[:, 1], indptr, indices, I, 4, 0xDEADBEEF12345, epoch, first, cnt)
        b = C.sample(pos[:, 0], pos[:, 1], indptr, indices, I, 4, 0xDEADBEEF12345, epoch, first, cnt)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def _expected_neg_hist(pos, U, I, num_ng):
    indptr, indices = O.build_csr(pos[:, 0], pos[:, 1], U)
    npos_u = np.bincount(pos[:, 0], minlength=U).astype(np.float64)
    deg = np.diff(indptr).astype(np.float64)
    c = np.where(deg < I, num_ng * npos_u / np.maximum(I - deg, 1), 0.0)
    E = np.full(I, c.sum())
    np.subtract.at(E, indices, np.repeat(c, np.diff(indptr)))
    return E


def _chi2_p(obs, E):
    m = E > 0
    chi = ((obs[m] - E[m]) ** 2 / E[m]).sum()
    return stats.chi2.sf(chi, m.sum() - 1)


def test_sampler_distribution_matches_reference_ng_sample(golden):
    """F3: the reference's ng_sample histogram and ours are both consistent with the exact
    'uniform over non-positives' distribution (util/data_loader.py:684-689)."""
    f3 = golden("ng_sample_ml100k.npz")
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    U, I, ng = int(f3["U"]), int(f3["I"]), int(f3["num_ng"])
    E = _expected_neg_hist(pos, U, I, ng)
    assert int(f3["negatives_in_train"]) == 0
    p_ref = _chi2_p(f3["hist_j"].astype(np.float64), E)
    indptr, indices = O.build_csr(pos[:, 0], pos[:, 1], U)
    u, i, j = C.sample(pos[:, 0], pos[:, 1], indptr, indices, I, ng, 42, 0, 0, len(pos) * ng)
    p_ours = _chi2_p(np.bincount(j, minlength=I).astype(np.float64), E)
    assert p_ref > 1e-4, p_ref
    assert p_ours > 1e-4, p_ours
    # per-user negative counts are exactly num_ng x positives, as in the reference
    assert np.array_equal(np.bincount(u, minlength=U), f3["neg_per_user"])
    keys = set(map(tuple, pos.tolist()))
    assert not any((int(a), int(b)) in keys for a, b in zip(u, j))


def test_metrics_known_answers(rl):
    with open(os.path.join(GOLDEN, "metrics_kat.json")) as fh:
        kat = json.load(fh)
    M = rl.metrics
    K = kat["k"]
    for c in kat["cases"]:
        r = c["r"]
        assert M.precision_at_k(r, K) == pytest.approx(c["precision"], abs=1e-12)
        assert M.recall_at_k(r, c["gt_len"], K) == pytest.approx(c["recall"], abs=1e-12)
        assert M.ndcg_at_k(r, K) == pytest.approx(c["ndcg"], abs=1e-12)
        assert M.average_precision(r[:K]) == pytest.approx(c["ap"], abs=1e-12)
    rs = [c["r"][:K] for c in kat["cases"]]
    us = list(range(len(rs)))
    ur = {u: set(range(d)) for u, d in zip(us, kat["aggregate"]["hr_denoms"])}
    assert M.map_at_k(rs) == pytest.approx(kat["aggregate"]["map"], abs=1e-12)
    assert M.mrr_at_k(rs) == pytest.approx(kat["aggregate"]["mrr"], abs=1e-12)
    assert M.hr_at_k(rs, us, ur) == pytest.approx(kat["aggregate"]["hr"], abs=1e-12)


def test_hr_ndcg_fixture_is_consistent():
    with open(os.path.join(GOLDEN, "hr_ndcg_ml100k.json")) as fh:
        j = json.load(fh)
    s = j["summary"]
    assert len(j["runs"]) >= 3
    assert 0 < s["hr"]["mean"] < 1 and s["hr"]["std"] < 0.2 * s["hr"]["mean"]
    f = np.load(os.path.join(GOLDEN, "hr_ndcg_ml100k.npz"))
    assert f["test_data"].shape[1] == 2 and len(f["gt_users"]) == len(f["gt_ptr"]) - 1


def test_metric_eval_ncf_ranks_each_batch(rl):
    """metric_eval(algo='ncf') (util/metrics.py:68-97) with a scoring stub: the ground truth sits
    first in each batch; HR / NDCG follow its rank among the top-k."""
    import torch

    class Stub:  # scores = -item, so smaller ids rank first
        def __call__(self, user, item):
            return -torch.as_tensor(item, dtype=torch.float32)

    batches = [(torch.zeros(5, dtype=torch.long), torch.tensor([3, 9, 1, 7, 5]), torch.zeros(5)),
               (torch.ones(5, dtype=torch.long), torch.tensor([0, 9, 1, 7, 5]), torch.zeros(5))]
    hr, ndcg = rl.metrics.metric_eval(Stub(), batches, 2, algo="ncf")
    # batch 1: top-2 = [1, 3] -> hit at rank 1; batch 2: top-2 = [0, 1] -> hit at rank 0
    assert hr == 1.0
    assert ndcg == pytest.approx((1 / np.log2(3) + 1.0) / 2)
    with pytest.raises(ValueError):
        rl.metrics.metric_eval(Stub(), batches, 2, algo="nfm")


def test_hogwild_spec_equals_reference_step_at_batch_one():
    """The relaxed mode's serial spec (oracle hogwild_serial) is per-triplet SGD with the reference's
    per-step weight decay, so with one triplet per step (B = 1, i != j) it IS the reference step
    (BPRMFRecommender.py:172-176, here oracle bpr_step_dense) applied triplet by triplet, once every
    row is brought to the last step."""
    g = np.random.default_rng(5)
    U, I, d, n, lr, wd = 7, 9, 6, 80, 0.05, 0.02
    P0 = (0.3 * g.standard_normal((U, d))).astype(np.float32)
    Q0 = (0.3 * g.standard_normal((I, d))).astype(np.float32)
    u, i = g.integers(0, U, n), g.integers(0, I, n)
    j = (i + 1 + g.integers(0, I - 1, n)) % I
    P, Q = P0.copy(), Q0.copy()
    loss, sP, sQ = O.hogwild_serial(P, Q, u, i, j, lr, wd, 1)
    a = 1.0 - lr * wd
    P = P * np.power(a, n - sP)[:, None]
    Q = Q * np.power(a, n - sQ)[:, None]
    Pr, Qr = P0.copy(), Q0.copy()
    lr_ = 0.0
    for s in range(n):
        lr_ += O.bpr_step_dense(Pr, Qr, u[s:s + 1], i[s:s + 1], j[s:s + 1], lr, wd)
    np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)
    assert loss == pytest.approx(lr_, rel=1e-5)


def test_local_serial_spec_reduces_to_hogwild_and_merges_deltas():
    """oracle.local_serial (semantics "local"): with no hot items it IS hogwild_serial; with hot
    items and a period longer than the run, a hot row ends as its decayed start plus its change."""
    g = np.random.default_rng(4)
    U, I, d, B, n = 23, 31, 8, 16, 300
    P = (0.1 * g.standard_normal((U, d))).astype(np.float32)
    Q = (0.1 * g.standard_normal((I, d))).astype(np.float32)
    u, i, j = g.integers(0, U, n), g.integers(0, I, n), g.integers(0, I, n)
    P1, Q1, P2, Q2 = P.copy(), Q.copy(), P.copy(), Q.copy()
    a = O.hogwild_serial(P1, Q1, u, i, j, 0.05, 0.01, B)
    b = O.local_serial(P2, Q2, u, i, j, 0.05, 0.01, B, [], 4)
    assert a[0] == b[0] and np.array_equal(P1, P2) and np.array_equal(Q1, Q2)
    # one hot item that no triplet touches: pure decay over the run, in one merge
    i[i == 5] = 6
    j[j == 5] = 6
    P3, Q3 = P.copy(), Q.copy()
    _, _, sQ = O.local_serial(P3, Q3, u, i, j, 0.05, 0.01, B, [5], 10 ** 6)
    T = (n + B - 1) // B
    assert sQ[5] == T
    np.testing.assert_allclose(Q3[5], Q[5] * (1 - 0.05 * 0.01) ** T, rtol=1e-6)


def test_local_dp_spec_one_rank_is_local_serial_and_ranks_add_changes():
    """oracle.local_dp_serial (semantics "local" at world > 1): one rank with one merge period is
    local_serial brought to the end; two ranks whose triplets touch disjoint items each keep their
    own change (the merge adds the other rank's zero change)."""
    g = np.random.default_rng(5)
    U, I, d, B, steps = 20, 24, 8, 8, 6
    P = (0.1 * g.standard_normal((U, d))).astype(np.float32)
    Q = (0.1 * g.standard_normal((I, d))).astype(np.float32)
    n = steps * B
    u, i, j = g.integers(0, U, n), g.integers(0, I, n), g.integers(0, I, n)
    P1, Q1 = P.copy(), Q.copy()
    l1, sP1, sQ1 = O.local_serial(P1, Q1, u, i, j, 0.05, 0.01, B, [3, 4], 2)
    a = np.float32(1 - 0.05 * 0.01)
    Q1T = Q1 * np.power(np.float64(a), steps - sQ1)[:, None].astype(np.float32)
    P2 = [P.copy()]
    l2, sP2, Q2 = O.local_dp_serial(P2, Q.copy(), [(u, i, j)], 0.05, 0.01, B, [[3, 4]], 2, 100, 1)
    assert l2 == pytest.approx(l1, rel=1e-12)
    np.testing.assert_array_equal(sP2[0], sP1)
    np.testing.assert_allclose(P2[0], P1, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(Q2, Q1T, rtol=1e-6, atol=1e-9)
    # two ranks on disjoint items (rank 0: items < 12, rank 1: items >= 12), no hot items, no decay
    tr = []
    for r in range(2):
        uu = g.choice(np.arange(r, U, 2), n)
        ii, jj = g.integers(0, 12, n) + 12 * r, g.integers(0, 12, n) + 12 * r
        tr.append((uu, ii, jj))
    # the overlapped schedule: one rank, or ranks on disjoint items, see no one else's change
    P3 = [P.copy()]
    _, _, Q3 = O.local_dp_serial(P3, Q.copy(), [(u, i, j)], 0.05, 0.01, B, [[3, 4]], 2, 2, 1, overlap=True)
    P4 = [P.copy()]
    _, _, Q4 = O.local_dp_serial(P4, Q.copy(), [(u, i, j)], 0.05, 0.01, B, [[3, 4]], 2, 2, 1)
    np.testing.assert_allclose(Q3, Q4, rtol=1e-5, atol=1e-7)
    Po = [P[r::2].copy() for r in range(2)]
    _, _, Qo = O.local_dp_serial(Po, Q.copy(), tr, 0.05, 0.0, B, [[], []], 3, 2, 2, overlap=True)
    Pp = [P[r::2].copy() for r in range(2)]
    _, _, Qm = O.local_dp_serial(Pp, Q.copy(), tr, 0.05, 0.0, B, [[], []], 3, 2, 2)
    np.testing.assert_allclose(Qo, Qm, rtol=1e-5, atol=1e-7)
    for r in range(2):  # each rank alone on its half of the items
        Pr, Qr = P[r::2].copy(), Q.copy()
        for t0 in range(0, steps, 2):
            sl = slice(t0 * B, (t0 + 2) * B)
            O.local_serial(Pr, Qr, tr[r][0][sl] // 2, tr[r][1][sl], tr[r][2][sl], 0.05, 0.0, B, [], 3, t0=t0)
        half = slice(12 * r, 12 * (r + 1))
        np.testing.assert_allclose(Qm[half], Qr[half], rtol=1e-5, atol=1e-7)


def test_stale1_spec_reduces_to_reference_and_reads_stale_rows():
    """sharded_stale1_serial (semantics "stale1"): with one step per runner chunk every step reads
    the current table, i.e. the reference step exactly; with longer chunks step t's forward reads
    a * Q_{t-2}: checked against a direct construction of step 2 from the stored tables."""
    g = np.random.default_rng(4)
    U_, I_, d = 17, 11, 8
    lr, wd = 0.05, 0.01
    P0 = (0.1 * g.standard_normal((U_, d))).astype(np.float32)
    Q0 = (0.1 * g.standard_normal((I_, d))).astype(np.float32)
    bs = [(g.integers(0, U_, 9), g.integers(0, I_, 9), g.integers(0, I_, 9)) for _ in range(4)]
    P1, Q1 = P0.copy(), Q0.copy()
    l1 = O.sharded_stale1_serial(P1, Q1, bs, lr, wd, 1)
    P2, Q2 = P0.copy(), Q0.copy()
    l2 = [O.bpr_step_dense(P2, Q2, *b, lr, wd) for b in bs]
    assert np.array_equal(P1, P2) and np.array_equal(Q1, Q2) and np.allclose(l1, l2, rtol=0)
    # chunk 4: steps 0 and 1 read Q0 (step 1: a * Q0), step 2 reads a * (Q after step 0)
    P3, Q3 = P0.copy(), Q0.copy()
    O.sharded_stale1_serial(P3, Q3, bs[:3], lr, wd, 4)
    a = np.float32(1) - np.float32(lr) * np.float32(wd)
    Pa, Qa = P0.copy(), Q0.copy()
    O.bpr_step_dense(Pa, Qa, *bs[0], lr, wd)          # step 0: exact
    Q_after0 = Qa.copy()
    O.bpr_step_stale(Pa, Qa, (Q0 * a).astype(np.float32), *bs[1], lr, wd)
    O.bpr_step_stale(Pa, Qa, (Q_after0 * a).astype(np.float32), *bs[2], lr, wd)
    assert np.array_equal(P3, Pa) and np.array_equal(Q3, Qa)
    Pe, Qe = P0.copy(), Q0.copy()
    for b in bs[:3]:
        O.bpr_step_dense(Pe, Qe, *b, lr, wd)
    assert np.abs(Q3 - Qe).max() > 1e-6  # not the reference step
