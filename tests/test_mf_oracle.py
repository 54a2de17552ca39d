"""CPU: the C oracle of the rating-SGD path (oracle/mf_cpu.c) against fixtures made by running
the reference's own Cython SVD / RSVD (tests/golden/make_golden_mf.py), bit for bit; and the
dependency-level schedule the device runs (a restatement of mf_capi.cpp's) gives the sequential
loop's bits."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import c_oracle as C

F = np.load(os.path.join(GOLDEN, "mf_cases.npz"))
CASES = [str(c) for c in F["cases"]]


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


def oracle_fit(c, order=None):
    U, I = int(c["U"]), int(c["I"])
    u, i, r = c["u"], c["i"], c["r"]
    if order is not None:
        u, i, r = u[order], i[order], r[order]
    if str(c["model"]) == "SVD":
        return C.svd_epochs(u, i, r, c["P0"], c["Q0"], np.zeros(U), np.zeros(I),
                            float(c["ref_global_mean"]), int(c["biased"]), c["lr"], c["reg"],
                            int(c["epochs"]))
    epochs = int(c["epochs"]) if int(c["verbose"]) else 0  # RSVD trains only when verbose
    return C.rsvd_epochs(u, i, r, c["P0"], c["Q0"], np.zeros(U), np.zeros(I),
                         float(c["global_mean"]), int(c["version"]), float(c["lr"][0]),
                         float(c["reg"][0]), float(c["reg"][1]), epochs)


@pytest.mark.parametrize("name", CASES)
def test_oracle_equals_reference_cython_bitwise(name):
    c = case(name)
    P, Q, b1, b2 = oracle_fit(c)
    for got, want in ((P, c["P"]), (Q, c["Q"]), (b1, c["bu"]), (b2, c["bi"])):
        assert np.array_equal(got, want)


def test_global_mean_is_pandas_mean():
    c = case("svd_biased")
    assert float(c["ref_global_mean"]) == float(c["global_mean"])


@pytest.mark.parametrize("name", ["svd_biased", "rsvd_v2"])
def test_level_schedule_equals_sequential_bitwise(name):
    c = case(name)
    order, off = C.mf_levels(c["u"], c["i"], int(c["U"]), int(c["I"]))
    u, i = c["u"][order], c["i"][order]
    for L in range(len(off) - 1):  # a level touches every user and every item at most once
        lu, li = u[off[L]:off[L + 1]], i[off[L]:off[L + 1]]
        assert len(np.unique(lu)) == len(lu) and len(np.unique(li)) == len(li)
    P, Q, b1, b2 = oracle_fit(c, order)
    assert np.array_equal(P, c["P"]) and np.array_equal(Q, c["Q"])
    assert np.array_equal(b1, c["bu"]) and np.array_equal(b2, c["bi"])
