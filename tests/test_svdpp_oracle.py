"""CPU: the SVDpp oracle (oracle/mf_cpu.c:oracle_svdpp_epochs) is bit-identical to the
reference's Cython SVDpp.fit (tests/golden/svdpp_cases.npz, made by running the reference
module), including a user whose item list holds an item twice."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import c_oracle as C

F = np.load(os.path.join(GOLDEN, "svdpp_cases.npz"))
CASES = [str(c) for c in F["cases"]]


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


@pytest.mark.parametrize("name", CASES)
def test_oracle_equals_reference_bitwise(name):
    c = case(name)
    U, I = int(c["U"]), int(c["I"])
    P, Q, Y, bu, bi = C.svdpp_epochs(c["u"], c["i"], c["r"], c["P0"], c["Q0"], c["Y0"],
                                     np.zeros(U), np.zeros(I), float(c["global_mean"]),
                                     c["lr"], c["reg"], int(c["epochs"]))
    for got, want in ((P, c["P"]), (Q, c["Q"]), (Y, c["Y"]), (bu, c["bu"]), (bi, c["bi"])):
        np.testing.assert_array_equal(got, want)


def test_duplicate_case_has_a_repeated_item():
    c = case("pp_dup")
    pairs = set()
    dup = False
    for a, b in zip(c["u"], c["i"]):
        dup |= (a, b) in pairs
        pairs.add((a, b))
    assert dup
