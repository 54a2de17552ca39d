"""NCF embedding Adam: the library in use (BPRMF_DIAG_LIB may name another build, e.g. the dense
sweep) against the oracle's dense Adam over a run with long gaps between a row's touches
(cold rows touched at step 2 and again at step 250: more zero-gradient steps than the catch-up's
term count), with a predict and a state_dict read inside the run.  Prints the max deviation per
parameter at a few steps.

  python tools/dbg/ncf_lazy_check.py [--steps 260]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def batches(steps, U, I, B, seed):
    g = np.random.default_rng(seed)
    out = []
    for k in range(steps):
        u = g.integers(0, U // 4, B)
        i = g.integers(0, I // 4, B)
        if k in (2, 250):  # the cold rows
            u[: B // 2] = g.integers(3 * U // 4, U, B // 2)
            i[: B // 2] = g.integers(3 * I // 4, I, B // 2)
        out.append((u, i, (g.random(B) < 0.3).astype(np.float32)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=260)
    ap.add_argument("--model", default="NeuMF-end")
    a = ap.parse_args()
    rl = importlib.import_module("recommend-lib_amd")
    from oracle import ncf_oracle as N
    U, I, d, L, B = 40, 48, 8, 2, 8
    m = rl.NCF(U, I, d, L, model=a.model, batch_size=B, seed=3)
    params = m.state_dict()
    opt = N.Adam(params)
    res = {}
    for k, (u, i, y) in enumerate(batches(a.steps, U, I, B, 17)):
        grads, _ = N.grads(params, a.model, L, u, i, y)
        params = opt.step(params, grads)
        m.train_samples(u, i, y)
        if k == 100:
            z = m.predict_logits(np.arange(3 * U // 4, U), np.arange(3 * I // 4, 3 * I // 4 + U // 4))
            zr, _ = N.forward(params, a.model, L, np.arange(3 * U // 4, U),
                              np.arange(3 * I // 4, 3 * I // 4 + U // 4))
            res["predict_100"] = float(np.abs(z - zr).max())
        if k + 1 in (50, 150, 251, a.steps):
            got = m.state_dict()
            res[f"step_{k + 1}"] = {n: float(np.abs(got[n] - params[n]).max()) for n in m.names}
    print(json.dumps({"lib": os.environ.get("BPRMF_DIAG_LIB", "product"), **res}, indent=1))


if __name__ == "__main__":
    main()
