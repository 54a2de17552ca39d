"""GPU: the rating-SGD path (include/mf.h, mf.hip) through the SVD / RSVD drop-ins, against the
reference's own Cython results (tests/golden/mf_cases.npz) and the C oracle — bit for bit: the
device runs the reference's per-sample loop in dependency levels with the same double operations
in the same order.  predict() goes through numpy like the reference; predict_batch sums the dot
product on the device in factor order (agreement to rounding with numpy's dot: PRED_RTOL)."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

F = np.load(os.path.join(GOLDEN, "mf_cases.npz"))
CASES = [str(c) for c in F["cases"]]
PRED_RTOL = 1e-12


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


def frame(c):
    return pd.DataFrame({"user": c["u"].astype(np.int64), "item": c["i"].astype(np.int64),
                         "rating": c["r"]})


def model_of(rl, c):
    U, I, k, ep = int(c["U"]), int(c["I"]), int(c["k"]), int(c["epochs"])
    if str(c["model"]) == "SVD":
        lr, reg = c["lr"], c["reg"]
        return rl.SVD(U, I, n_factors=k, n_epochs=ep, biased=bool(c["biased"]), lr_bu=lr[0],
                      lr_bi=lr[1], lr_pu=lr[2], lr_qi=lr[3], reg_bu=reg[0], reg_bi=reg[1],
                      reg_pu=reg[2], reg_qi=reg[3], verbose=False)
    return rl.RSVD(U, I, n_factors=k, n_epochs=ep, version=int(c["version"]), lr=float(c["lr"][0]),
                   reg=float(c["reg"][0]), reg2=float(c["reg"][1]), verbose=bool(c["verbose"]))


@pytest.mark.parametrize("name", CASES)
def test_fit_equals_reference_cython_bitwise(rl, name, capsys):
    c = case(name)
    m = model_of(rl, c)
    np.random.seed(int(c["seed"]))  # the reference seeds numpy's global RNG the same way
    m.fit(frame(c))
    if str(c["model"]) == "SVD":
        got = (m.pu, m.qi, m.bu, m.bi)
        assert m.global_mean == float(c["ref_global_mean"])
    else:
        got = (m.ui, m.vj, m.ci, m.dj)
    for g, w in zip(got, (c["P"], c["Q"], c["bu"], c["bi"])):
        assert np.array_equal(g, w)
    u, i = c["u"][:50], c["i"][:50]
    pred = np.array([m.predict(int(a), int(b)) for a, b in zip(u, i)])
    assert np.array_equal(pred, c["pred"])  # the same numpy expression on the same bits
    np.testing.assert_allclose(m.predict_batch(u, i), c["pred"], rtol=PRED_RTOL, atol=1e-15)


def test_larger_random_set_equals_oracle_bitwise(rl):
    g = np.random.default_rng(5)
    U, I, n, k = 3000, 7000, 300_000, 32
    w = 1.0 / np.arange(1, I + 1)
    df = pd.DataFrame({"user": g.integers(0, U, n), "item": g.choice(I, n, p=w / w.sum()),
                       "rating": g.integers(1, 6, n).astype(np.float64)})
    m = rl.SVD(U, I, n_factors=k, n_epochs=3, lr_all=0.01, verbose=False)
    np.random.seed(3)
    m.fit(df)
    np.random.seed(3)
    P0 = np.random.normal(0, .1, (U, k))
    Q0 = np.random.normal(0, .1, (I, k))
    P, Q, bu, bi = C.svd_epochs(df.user.values, df.item.values, df.rating.values, P0, Q0,
                                np.zeros(U), np.zeros(I), df.rating.mean(), 1, [0.01] * 4,
                                [0.02] * 4, 3)
    assert np.array_equal(m.pu, P) and np.array_equal(m.qi, Q)
    assert np.array_equal(m.bu, bu) and np.array_equal(m.bi, bi)
    # levels: at least the longest user or item chain (the Zipf head item), far below the samples
    deg = max(np.bincount(df.user).max(), np.bincount(df.item).max())
    assert deg <= m.last_stats["levels"] < n / 5


def test_predict_rejects_bad_codes(rl):
    m = rl.SVD(10, 20, n_factors=4, n_epochs=1, verbose=False)
    m.fit(pd.DataFrame({"user": [0, 1, 2], "item": [3, 4, 5], "rating": [1.0, 2.0, 3.0]}))
    with pytest.raises(ValueError, match="Invalid user code"):
        m.predict(10, 0)
    with pytest.raises(ValueError, match="Invalid item code"):
        m.predict(0, 20)
    with pytest.raises(ValueError):
        m.predict_batch([0, 10], [0, 0])
    with pytest.raises(ValueError):  # a train row out of range
        m.fit(pd.DataFrame({"user": [0, 11], "item": [0, 0], "rating": [1.0, 1.0]}))


def test_zero_epochs_and_empty_train_set(rl):
    m = rl.SVD(5, 6, n_factors=3, n_epochs=0, verbose=False)
    np.random.seed(1)
    m.fit(pd.DataFrame({"user": [0], "item": [1], "rating": [4.0]}))
    np.random.seed(1)
    assert np.array_equal(m.pu, np.random.normal(0, .1, (5, 3)))
    e = rl.SVD(5, 6, n_factors=3, n_epochs=2, verbose=False)
    e.fit(pd.DataFrame({"user": np.zeros(0, int), "item": np.zeros(0, int), "rating": np.zeros(0)}))
    assert e.last_stats["samples"] == 0
