"""CPU: the NCF oracle (oracle/ncf_oracle.py) reproduces the reference NCF's predictions, gradients,
losses and Adam steps recorded in tests/golden/ncf_steps_tiny.npz (G1)."""
import numpy as np
import pytest

from oracle import ncf_oracle as N


def _cases(golden):
    f = golden("ncf_steps_tiny.npz")
    for c in range(int(f["n_cases"])):
        pre = f"c{c}_"
        d, L = (int(x) for x in f[pre + "meta"][:2])
        model = str(f[pre + "model"])
        names = [str(x) for x in f[pre + "names"]]
        yield f, pre, model, d, L, names


def test_forward_and_grads_match_reference(golden):
    for f, pre, model, d, L, names in _cases(golden):
        params = {n: f[pre + "init_" + n] for n in names}
        u, i, y = f[pre + "u"][0], f[pre + "i"][0], f[pre + "y"][0]
        z, _ = N.forward(params, model, L, u, i)
        np.testing.assert_allclose(z, f[pre + "pred0"], rtol=1e-5, atol=1e-7)
        g, loss = N.grads(params, model, L, u, i, y)
        assert abs(loss - f[pre + "loss"][0]) < 1e-6
        for n in names:
            key = pre + "grad0_" + n
            if key in f.files:
                np.testing.assert_allclose(g[n], f[key], rtol=1e-4, atol=1e-9, err_msg=n)
            else:
                assert n not in g, n  # no gradient: the branch the model does not use


def test_adam_steps_match_reference(golden):
    for f, pre, model, d, L, names in _cases(golden):
        params = {n: f[pre + "init_" + n].copy() for n in names}
        opt = N.Adam(params)
        steps = int(f[pre + "meta"][3])
        for k in range(steps):
            g, loss = N.grads(params, model, L, f[pre + "u"][k], f[pre + "i"][k], f[pre + "y"][k])
            assert abs(loss - f[pre + "loss"][k]) < 1e-5, (model, k)
            params = opt.step(params, g)
            if k + 1 in (1, 3, steps):
                for n in names:
                    np.testing.assert_allclose(params[n], f[pre + f"after{k + 1}_" + n],
                                               rtol=0, atol=2e-6, err_msg=f"{model} {n} step {k + 1}")
