"""Debug: C4 NCF at ml-20m shape vs the oracle, per step and per parameter (GPU box)."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa
from oracle import ncf_oracle as N
rl = importlib.import_module("recommend-lib_amd")
U, I, d, L, B = [int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (138493, 26744, 64, 3, 256))]
g = np.random.default_rng(44)
m = rl.NCF(U, I, d, L, batch_size=B, seed=9)
params = m.state_dict()
opt = N.Adam(params)
for k in range(3):
    u = g.integers(0, U, B); i = g.integers(0, I, B)
    u[:20] = 5; i[10:40] = 11
    y = (g.random(B) < 0.2).astype(np.float32)
    z = m.predict_logits(u, i)
    z_ref, _ = N.forward(params, "NeuMF-end", L, u, i)
    print(f"step {k}: forward max|dz| {np.abs(z - z_ref).max():.3e}  (|z| ~ {np.abs(z_ref).mean():.3e})")
    grads, loss = N.grads(params, "NeuMF-end", L, u, i, y)
    params = opt.step(params, grads)
    st = m.train_samples(u, i, y)
    print(f"   loss gpu {st['loss']:.8f} oracle {loss:.8f}")
    got = m.state_dict()
    for n in m.names:
        dd = np.abs(got[n] - params[n])
        gn = np.abs(grads[n])
        big = dd > 5e-5
        print(f"   {n:28s} max|d| {dd.max():.3e}  n>5e-5 {int(big.sum())}  "
              f"min|g| among them {gn[big].min() if big.any() else 0:.3e}  median|g| {np.median(gn[gn>0]) if (gn>0).any() else 0:.3e}")
