"""GPU: SVDpp (include/mf.h model MF_SVDPP, mf.hip k_svdpp_epoch) through the SVDpp drop-in,
bit for bit against the reference's own Cython SVDpp.fit (tests/golden/svdpp_cases.npz) and the C
oracle: the device runs the samples in train order with the reference's double operations in the
reference's order (the implicit sum over the user's items in list order, the dot product in
factor order).  predict() is the reference's numpy code on those tables; predict_batch sums on the
device (agreement to rounding: PRED_RTOL)."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

F = np.load(os.path.join(GOLDEN, "svdpp_cases.npz"))
CASES = [str(c) for c in F["cases"]]
PRED_RTOL = 1e-12


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


def model_of(rl, c):
    lr, reg = c["lr"], c["reg"]
    return rl.SVDpp(int(c["U"]), int(c["I"]), n_factors=int(c["k"]), n_epochs=int(c["epochs"]),
                    lr_bu=lr[0], lr_bi=lr[1], lr_pu=lr[2], lr_qi=lr[3], lr_yj=lr[4], reg_bu=reg[0],
                    reg_bi=reg[1], reg_pu=reg[2], reg_qi=reg[3], reg_yj=reg[4], verbose=False)


@pytest.mark.parametrize("name", CASES)
def test_fit_equals_reference_cython_bitwise(rl, name):
    c = case(name)
    m = model_of(rl, c)
    np.random.seed(int(c["seed"]))
    m.fit(pd.DataFrame({"user": c["u"].astype(np.int64), "item": c["i"].astype(np.int64),
                        "rating": c["r"]}))
    assert m.global_mean == float(c["global_mean"])
    for got, want in ((m.pu, c["P"]), (m.qi, c["Q"]), (m.yj, c["Y"]), (m.bu, c["bu"]),
                      (m.bi, c["bi"])):
        np.testing.assert_array_equal(got, want)
    pred = np.array([m.predict(int(a), int(b)) for a, b in c["pairs"]])
    np.testing.assert_array_equal(pred, c["pred"])
    pb = m.predict_batch(c["pairs"][:, 0], c["pairs"][:, 1])
    np.testing.assert_allclose(pb, c["pred"], rtol=PRED_RTOL)


def test_long_lists_and_duplicates_against_oracle(rl):
    """k = 32; a user with 3000 items (16 LDS chunks), a user whose list repeats an item."""
    g = np.random.default_rng(4)
    U, I, k, n = 400, 3200, 32, 12000
    u = g.integers(0, U, n)
    i = g.integers(0, I, n)
    u[:3000], i[:3000] = 7, g.permutation(I)[:3000]
    u[5000:5004], i[5000:5004] = 11, 42  # user 11 rates item 42 four times
    r = g.integers(1, 6, n).astype(np.float64)
    perm = g.permutation(n)
    u, i, r = u[perm], i[perm], r[perm]
    m = rl.SVDpp(U, I, n_factors=k, n_epochs=2, verbose=False)
    np.random.seed(3)
    m.fit(pd.DataFrame({"user": u, "item": i, "rating": r}))
    np.random.seed(3)
    P0 = np.random.normal(0, .1, (U, k))
    Q0 = np.random.normal(0, .1, (I, k))
    Y0 = np.random.normal(0, .1, (I, k))
    P, Q, Y, bu, bi = C.svdpp_epochs(u, i, r, P0, Q0, Y0, np.zeros(U), np.zeros(I), r.mean(),
                                     [0.007] * 5, [0.02] * 5, 2)
    for got, want in ((m.pu, P), (m.qi, Q), (m.yj, Y), (m.bu, bu), (m.bi, bi)):
        np.testing.assert_array_equal(got, want)
    assert m.last_stats["samples"] == 2 * n


def test_bad_codes_and_empty(rl):
    m = rl.SVDpp(5, 6, n_factors=4, n_epochs=1, verbose=False)
    with pytest.raises(ValueError):
        m.fit(pd.DataFrame({"user": [0, 5], "item": [1, 1], "rating": [3.0, 4.0]}))
    np.random.seed(0)
    m.fit(pd.DataFrame({"user": [0, 1], "item": [1, 1], "rating": [3.0, 4.0]}))
    with pytest.raises(ValueError):
        m.predict(5, 0)
    with pytest.raises(ValueError):
        m.predict(0, 6)
    assert np.isfinite(m.predict(4, 5))  # a user with no items: no implicit term
    np.testing.assert_allclose(m.predict_batch(np.array([4, 0]), np.array([5, 1])),
                               [m.predict(4, 5), m.predict(0, 1)], rtol=PRED_RTOL)
    with pytest.raises(ValueError):
        m.predict_batch(np.array([0]), np.array([6]))
