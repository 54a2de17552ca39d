"""Generate the NCF golden fixtures by IMPORTING the reference (read-only)
in the build container.  Test infrastructure only: never run on the GPU box; only its outputs
travel.  It imports `NCFRecommender.NCF` from /root/reference and drives it the way
`NCFRecommender.py:262-288` does (zero_grad, forward, BCEWithLogitsLoss, backward, Adam.step),
with the torch RNG seeded for the initialisation.

Fixture written next to this file:
  G1 ncf_steps_tiny.npz  for each case (model, factor_num, num_layers): the initial parameters,
     6 batches of (user, item, label) (one with a repeated (user, item)), the loss of every step,
     the gradients of the first step, the predictions of the first batch, and every parameter
     after steps 1, 3 and 6 (Adam, lr 0.001, the reference defaults).
Run:  python tests/golden/make_golden_ncf.py
"""
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
CASES = [("NeuMF-end", 8, 3), ("GMF", 8, 3), ("MLP", 8, 3), ("NeuMF-end", 16, 2)]
U, I, B, STEPS = 30, 50, 64, 6


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    import NCFRecommender as N
    out = {}
    g = np.random.default_rng(2024)
    for ci, (name, d, L) in enumerate(CASES):
        torch.manual_seed(100 + ci)
        model = N.NCF(U, I, d, L, 0.0, name)
        opt = torch.optim.Adam(model.parameters(), lr=0.001)
        loss_fn = torch.nn.BCEWithLogitsLoss()
        names = [n for n, _ in model.named_parameters()]
        pre = f"c{ci}_"
        out[pre + "meta"] = np.array([d, L, B, STEPS, U, I])
        out[pre + "model"] = np.array(name)
        out[pre + "names"] = np.array(names)
        for n, p in model.named_parameters():
            out[pre + "init_" + n] = p.detach().numpy().copy()
        batches = []
        for k in range(STEPS):
            u = g.integers(0, U, B)
            i = g.integers(0, I, B)
            y = (g.random(B) < 0.2).astype(np.float32)
            if k == 2:
                u[:10], i[:10] = 3, 7  # the same (user, item) ten times in one batch
            batches.append((u, i, y))
        out[pre + "u"] = np.stack([b[0] for b in batches]).astype(np.int32)
        out[pre + "i"] = np.stack([b[1] for b in batches]).astype(np.int32)
        out[pre + "y"] = np.stack([b[2] for b in batches])
        losses = []
        for k, (u, i, y) in enumerate(batches):
            ut, it, yt = torch.as_tensor(u), torch.as_tensor(i), torch.as_tensor(y)
            model.zero_grad()
            pred = model(ut, it)
            loss = loss_fn(pred, yt)
            loss.backward()
            if k == 0:
                out[pre + "pred0"] = pred.detach().numpy().copy()
                for n, p in model.named_parameters():
                    if p.grad is not None:
                        out[pre + "grad0_" + n] = p.grad.detach().numpy().copy()
            opt.step()
            losses.append(float(loss.item()))
            if k + 1 in (1, 3, STEPS):
                for n, p in model.named_parameters():
                    out[pre + f"after{k + 1}_" + n] = p.detach().numpy().copy()
        out[pre + "loss"] = np.array(losses)
    out["n_cases"] = np.array(len(CASES))
    np.savez_compressed(os.path.join(OUT, "ncf_steps_tiny.npz"), **out)
    print("wrote", os.path.join(OUT, "ncf_steps_tiny.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
