"""GPU: the NCF path (include/ncf.h) against the reference's own recorded runs (G1,
tests/golden/ncf_steps_tiny.npz: NCF GMF / MLP / NeuMF-end, BCEWithLogitsLoss, Adam) and the
oracle (oracle/ncf_oracle.py).  Tolerances: forward 1e-6 (f32 MFMA vs torch f32); Adam steps
2e-5 absolute on O(0.01-0.3) weights (embedding gradients are f32 atomics: summation order
differs from torch's; Adam's first steps move every element by ~lr regardless of |g|)."""
import numpy as np
import pytest

from oracle import bpr_oracle as BO
from oracle import ncf_oracle as N

pytestmark = pytest.mark.gpu


def _cases(golden):
    f = golden("ncf_steps_tiny.npz")
    for c in range(int(f["n_cases"])):
        pre = f"c{c}_"
        d, L, B, steps, U, I = (int(x) for x in f[pre + "meta"])
        yield f, pre, str(f[pre + "model"]), d, L, B, steps, U, I


def _model(rl, f, pre, model, d, L, B, U, I):
    m = rl.NCF(U, I, d, L, model=model, batch_size=B, seed=1)
    m.load_state_dict({n: f[pre + "init_" + n] for n in m.names})
    return m


def test_forward_matches_reference(rl, golden):
    for f, pre, model, d, L, B, steps, U, I in _cases(golden):
        m = _model(rl, f, pre, model, d, L, B, U, I)
        z = m.predict_logits(f[pre + "u"][0], f[pre + "i"][0])
        np.testing.assert_allclose(z, f[pre + "pred0"], rtol=1e-5, atol=1e-6, err_msg=model)


def test_adam_steps_match_reference(rl, golden):
    for f, pre, model, d, L, B, steps, U, I in _cases(golden):
        m = _model(rl, f, pre, model, d, L, B, U, I)
        for k in range(steps):
            st = m.train_samples(f[pre + "u"][k], f[pre + "i"][k], f[pre + "y"][k])
            assert st["steps"] == 1
            assert abs(st["loss"] - f[pre + "loss"][k]) < 2e-6, (model, k)
            if k + 1 in (1, 3, steps):
                got = m.state_dict()
                for n in m.names:
                    np.testing.assert_allclose(got[n], f[pre + f"after{k + 1}_" + n], rtol=0,
                                               atol=2e-5, err_msg=f"{model} {n} step {k + 1}")


def test_larger_tower_matches_oracle(rl):
    """d=64, 3 layers (the C4 tower: 512 -> 256 -> 128 -> 64), B=256 with duplicates."""
    U, I, d, L, B = 300, 500, 64, 3, 256
    g = np.random.default_rng(5)
    m = rl.NCF(U, I, d, L, batch_size=B, seed=2)
    params = m.state_dict()
    opt = N.Adam(params)
    for k in range(4):
        u = g.integers(0, U, B)
        i = g.integers(0, I, B)
        u[:30] = 7
        y = (g.random(B) < 0.25).astype(np.float32)
        z = m.predict_logits(u, i)
        z_ref, _ = N.forward(params, "NeuMF-end", L, u, i)
        np.testing.assert_allclose(z, z_ref, rtol=1e-4, atol=2e-6)
        grads, loss = N.grads(params, "NeuMF-end", L, u, i, y)
        params = opt.step(params, grads)
        st = m.train_samples(u, i, y)
        assert abs(st["loss"] - loss) < 1e-5
    got = m.state_dict()
    for n in m.names:
        np.testing.assert_allclose(got[n], params[n], rtol=0, atol=5e-5, err_msg=n)


def test_lazy_embedding_adam_matches_dense_over_long_gaps(rl):
    """The embedding rows' zero-gradient Adam steps are applied lazily (k_ncf_catch_up, closed
    form) where torch's Adam moves every row with a nonzero moment every step: cold rows touched at
    steps 3 and 251 (248 zero-gradient steps between, more than the catch-up's 192 terms), a
    predict of cold rows at step 101 (catch-up of the rows read) and state_dict reads (every row)
    in between.  Against the oracle's dense Adam at 1e-6 (measured: 6e-8 lazy, 5e-8 for the dense
    sweep it replaced, tools/dbg/ncf_lazy_check.py)."""
    U, I, d, L, B = 40, 48, 8, 2, 8
    g = np.random.default_rng(17)
    m = rl.NCF(U, I, d, L, batch_size=B, seed=3)
    params = m.state_dict()
    opt = N.Adam(params)
    cold_u, cold_i = np.arange(3 * U // 4, U), np.arange(3 * I // 4, 3 * I // 4 + U // 4)
    seen_u, seen_i = set(), set()
    for k in range(260):
        u = g.integers(0, U // 4, B)
        i = g.integers(0, I // 4, B)
        if k in (2, 250):
            u[: B // 2] = g.integers(3 * U // 4, U, B // 2)
            i[: B // 2] = g.integers(3 * I // 4, I, B // 2)
        y = (g.random(B) < 0.3).astype(np.float32)
        seen_u.update(u.tolist())
        seen_i.update(i.tolist())
        grads, _ = N.grads(params, "NeuMF-end", L, u, i, y)
        params = opt.step(params, grads)
        m.train_samples(u, i, y)
        if k == 100:
            z = m.predict_logits(cold_u, cold_i)
            z_ref, _ = N.forward(params, "NeuMF-end", L, cold_u, cold_i)
            np.testing.assert_allclose(z, z_ref, rtol=0, atol=1e-6)
        if k + 1 in (50, 150, 251, 260):
            got = m.state_dict()
            for n in m.names:
                np.testing.assert_allclose(got[n], params[n], rtol=0, atol=1e-6, err_msg=f"{n} step {k + 1}")
    assert m.active_rows() == (len(seen_u), len(seen_i))
    m.close()


def test_lazy_adam_within_multi_step_calls_matches_dense(rl):
    """The same long-gap stream as above, replayed as two calls of many steps: inside a call the
    next step's rows are caught up beside the middle layers (k_ncf_mid's extra workgroups) and a
    step's row Adam runs in the next step's row launch (k_ncf_rows), both paths a one-step call
    never takes.  Against the oracle's dense Adam at 1e-6."""
    U, I, d, L, B = 40, 48, 8, 2, 8
    g = np.random.default_rng(29)
    m = rl.NCF(U, I, d, L, batch_size=B, seed=5)
    params = m.state_dict()
    opt = N.Adam(params)
    us, is_, ys = [], [], []
    for k in range(260):
        u = g.integers(0, U // 4, B)
        i = g.integers(0, I // 4, B)
        if k in (2, 250):
            u[: B // 2] = g.integers(3 * U // 4, U, B // 2)
            i[: B // 2] = g.integers(3 * I // 4, I, B // 2)
        u[B - 1], i[B - 1] = u[0], i[0]  # a repeated row inside the step
        y = (g.random(B) < 0.3).astype(np.float32)
        grads, _ = N.grads(params, "NeuMF-end", L, u, i, y)
        params = opt.step(params, grads)
        us.append(u), is_.append(i), ys.append(y)
    for lo, hi in ((0, 150), (150, 260)):
        st = m.train_samples(np.concatenate(us[lo:hi]), np.concatenate(is_[lo:hi]), np.concatenate(ys[lo:hi]))
        assert st["steps"] == hi - lo
    got = m.state_dict()
    for n in m.names:
        np.testing.assert_allclose(got[n], params[n], rtol=0, atol=1e-6, err_msg=n)
    m.close()


def test_sampler_matches_oracle_and_ncfdata_semantics(rl, golden):
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    U, I = int(f["U"]), int(f["I"])
    m = rl.NCF(U, I, 8, 1, batch_size=256, num_ng=4, seed=11)
    m.set_train(pos)
    n = m.epoch_size()[0]
    assert n == 5 * len(pos)
    u, i, y = m.sample(3, 0, n)
    indptr, indices = BO.build_csr(pos[:, 0], pos[:, 1], U)
    uo, io, yo = N.sample(pos[:, 0], pos[:, 1], indptr, indices, I, 4, 11, 3, 1000, 5000)
    assert np.array_equal(u[1000:6000], uo) and np.array_equal(i[1000:6000], io)
    assert np.array_equal(y[1000:6000], yo)
    # NCFData.ng_sample: every positive once (label 1) and 4 negatives per positive, none a positive
    assert int(y.sum()) == len(pos)
    posset = set(map(tuple, pos.tolist()))
    neg = y == 0
    assert not any((a, b) in posset for a, b in zip(u[neg].tolist(), i[neg].tolist()))
    cnt = np.bincount(u[neg], minlength=U)
    assert np.array_equal(cnt, 4 * np.bincount(pos[:, 0], minlength=U))


def test_training_reduces_loss_and_ranks(rl, golden):
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    U, I = int(f["U"]), int(f["I"])
    m = rl.NCF(U, I, 16, 2, batch_size=256, num_ng=4, seed=3, lr=0.001)
    m.set_train(pos)
    losses = [m.train_epoch()["loss"] / m.epoch_size()[1] for _ in range(3)]
    assert losses[-1] < losses[0] < 0.7, losses
    # positives now score above random items for most users
    g = np.random.default_rng(0)
    zp = m.predict_logits(pos[:2000, 0], pos[:2000, 1])
    zn = m.predict_logits(pos[:2000, 0], g.integers(0, I, 2000))
    assert (zp > zn).mean() > 0.75
