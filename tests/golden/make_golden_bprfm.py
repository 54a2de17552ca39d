"""Generate the BPR-FM fixtures by IMPORTING the reference's model class (BPRFMRecommender.BPRFM,
BPRFMRecommender.py:28-79) in the build container and driving it exactly as its training loop
does (:203-227): model.train(), zero_grad, forward on (features_i, values_i, features_j,
values_j), loss = -(pred_i - pred_j).sigmoid().log().sum(), backward, Adagrad(lr,
initial_accumulator_value=1e-8).step().  The reference is not copied; only its outputs are
written.  Dropout is 0 here (the reference's dropout draws from torch's RNG and cannot be matched
bit for bit; the GPU path's dropout is tested statistically), BatchNorm on and off.

Features follow BPRFMData (util/data_loader.py:574-627): two fields [user feature, item feature],
values 1; user features in [0, U), item features in [U, U + I).
bprfm_steps.npz, per case c: U, I, k, bn, lr, B, steps, triplets [steps, 3, B] (u, i, j), the
initial parameters, the first step's gradients, per-step losses and the parameters after the
last step.
Run:  python tests/golden/make_golden_bprfm.py
"""
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    torch.set_num_threads(1)
    from BPRFMRecommender import BPRFM  # the reference model (:28-79)

    out = {}
    cases = [("bn", 40, 60, 8, True, 64, 6, 0.05, 1), ("nobn", 40, 60, 8, False, 64, 6, 0.05, 2),
             ("bn16", 100, 150, 16, True, 256, 4, 0.05, 3)]
    for name, U, I, k, bn, B, steps, lr, seed in cases:
        torch.manual_seed(seed)
        model = BPRFM(U + I, k, bn, [0.0, 0.0])
        opt = torch.optim.Adagrad(model.parameters(), lr=lr, initial_accumulator_value=1e-8)
        g = np.random.default_rng(seed)
        trip = np.stack([g.integers(0, U, (steps, B)), g.integers(0, I, (steps, B)),
                         g.integers(0, I, (steps, B))], 1)
        trip[0, 0, :8] = trip[0, 0, 0]  # a user repeated within a batch
        trip[0, 1, :12] = 3             # a hot item
        trip[1, 2, :5] = trip[1, 1, :5]  # i == j
        sd = {n: p.detach().numpy().copy() for n, p in model.state_dict().items()}
        losses = []
        for s in range(steps):
            u, i, j = (torch.from_numpy(trip[s, x].astype(np.int64)) for x in range(3))
            fi = torch.stack([u, i + U], 1)
            fj = torch.stack([u, j + U], 1)
            ones = torch.ones(B, 2)
            model.train()
            model.zero_grad()
            pi, pj = model(fi, ones, fj, ones)
            loss = -(pi - pj).sigmoid().log().sum()
            loss.backward()
            if s == 0:  # the first step's gradients (well-conditioned, unlike Adagrad's output)
                grads0 = {n: p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
            opt.step()
            losses.append(float(loss.detach()))
        fin = {n: p.detach().numpy().copy() for n, p in model.state_dict().items()}
        c = dict(U=U, I=I, k=k, bn=int(bn), lr=lr, B=B, steps=steps, triplets=trip.astype(np.int32),
                 loss=np.array(losses))
        for n, v in sd.items():
            c["init_" + n.replace(".", "_")] = v
        for n, v in fin.items():
            c["final_" + n.replace(".", "_")] = v
        for n, v in grads0.items():
            c["grad0_" + n.replace(".", "_")] = v
        for key, v in c.items():
            out[f"{name}_{key}"] = np.asarray(v)
        print(name, sorted(sd), file=sys.stderr)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(OUT, "bprfm_steps.npz"), **out)


if __name__ == "__main__":
    main()
