"""CPU: the BPR-FM oracle (oracle/bprfm_oracle.py, float64) against fixtures made by running the
reference's BPRFM module (tests/golden/make_golden_bprfm.py; float32 torch)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import bprfm_oracle as O

F = np.load(os.path.join(GOLDEN, "bprfm_steps.npz"))
CASES = [str(c) for c in F["cases"]]
GRAD_RTOL = 2e-5  # first-step gradients: float32 reference vs float64 oracle (sum orders)
# Parameters after several steps: Adagrad's early updates are ~lr * g / |g| (the accumulator
# starts at 1e-8), so a gradient that nearly cancels (an item's +/- references, a user's two
# sides) turns float32 rounding noise into updates of up to lr; the reference itself is not
# reproducible below that level.  Measured oracle-vs-reference: <= 1e-4 after 6 steps.
PARAM_ATOL = 5e-4


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


def init_state(c):
    bn = bool(c["bn"])
    return O.State(c["init_embeddings_weight"], c["init_biases_weight"], c["init_bias_"],
                   c["init_FM_layers_0_weight"] if bn else None,
                   c["init_FM_layers_0_bias"] if bn else None)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_steps(name):
    c = case(name)
    st = init_state(c)
    U = int(c["U"])
    for s in range(int(c["steps"])):
        t = c["triplets"][s]
        g = {}
        loss = O.step(st, U, t[0], t[1], t[2], float(c["lr"]), grads_out=g)
        # step 0 from identical parameters; later steps carry the Adagrad noise above
        assert loss == pytest.approx(float(c["loss"][s]), rel=1e-6 if s == 0 else 1e-4)
        if s == 0:
            scale = np.abs(c["grad0_embeddings_weight"]).max()
            np.testing.assert_allclose(g["E"], c["grad0_embeddings_weight"], rtol=0,
                                       atol=GRAD_RTOL * scale)
            np.testing.assert_allclose(g["b"], c["grad0_biases_weight"].reshape(-1), rtol=0,
                                       atol=GRAD_RTOL * np.abs(c["grad0_biases_weight"]).max())
            if st.bn:
                np.testing.assert_allclose(g["gamma"], c["grad0_FM_layers_0_weight"], rtol=GRAD_RTOL,
                                           atol=GRAD_RTOL * scale)
                np.testing.assert_allclose(g["beta"], c["grad0_FM_layers_0_bias"], rtol=GRAD_RTOL,
                                           atol=GRAD_RTOL * scale)
    np.testing.assert_allclose(st.E, c["final_embeddings_weight"], rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(st.b, c["final_biases_weight"].reshape(-1), rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(st.bias_, c["final_bias_"], rtol=0, atol=PARAM_ATOL)
    if st.bn:
        np.testing.assert_allclose(st.gamma, c["final_FM_layers_0_weight"], rtol=0, atol=PARAM_ATOL)
        np.testing.assert_allclose(st.beta, c["final_FM_layers_0_bias"], rtol=0, atol=PARAM_ATOL)
        np.testing.assert_allclose(st.run_mean, c["final_FM_layers_0_running_mean"], rtol=1e-3,
                                   atol=1e-7)
        np.testing.assert_allclose(st.run_var, c["final_FM_layers_0_running_var"], rtol=1e-3)
