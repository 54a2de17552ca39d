"""Measurement of the NCF row (BASELINE config C4): NeuMF-end training on
the ml-20m shape (138,493 users x 26,744 items, ~1e7 synthetic positives), factor_num 64,
3 tower layers (512 -> 256 -> 128 -> 64), batch 256, num_ng 4, Adam lr 0.001 (NCFRecommender.py
defaults, factor 64 per the config).

  python tools/bench_ncf.py [--steps K] [--warmup W] [--batch-size B]

A step is the reference's: forward + BCE + backward over B samples, then Adam over EVERY
parameter (torch's dense Adam: every embedding row with a nonzero moment moves every step; here
the rows' zero-gradient steps are applied lazily, in closed form, before anything reads them).
The warm-up first replays a stream that touches every user and item once (the steady state of an
epoch), then W sampler steps; the K timed steps come from the device sampler.  One JSON line:
samples/s, the per-launch split from HIP events, the tower's MFMA rate against the f32 MFMA peak
(the step is latency-bound: 16 sample groups of 16 carry the per-sample layers), and a CPU
baseline: the same step in torch on this host (a module written here with the reference's math,
not the reference), a bounded number of steps.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
F32_MFMA_PEAK_TFS = 157.3  # MI355X f32-input MFMA (MI355X_MICROARCH.md)


def cpu_baseline(U, I, d, L, B, steps=20):
    import torch
    import torch.nn as nn
    E = d * 2 ** (L - 1)

    class Tower(nn.Module):  # NeuMF-end: GMF product + ReLU tower, one logit
        def __init__(self):
            super().__init__()
            self.pg, self.qg = nn.Embedding(U, d), nn.Embedding(I, d)
            self.pm, self.qm = nn.Embedding(U, E), nn.Embedding(I, E)
            layers, n = [], 2 * E
            for _ in range(L):
                layers += [nn.Linear(n, n // 2), nn.ReLU()]
                n //= 2
            self.mlp = nn.Sequential(*layers)
            self.out = nn.Linear(2 * d, 1)

        def forward(self, u, i):
            g = self.pg(u) * self.qg(i)
            h = self.mlp(torch.cat([self.pm(u), self.qm(i)], -1))
            return self.out(torch.cat([g, h], -1)).view(-1)

    torch.manual_seed(0)
    m = Tower()
    opt = torch.optim.Adam(m.parameters(), lr=0.001)
    lf = nn.BCEWithLogitsLoss()
    g = torch.Generator().manual_seed(1)
    batches = [(torch.randint(0, U, (B,), generator=g), torch.randint(0, I, (B,), generator=g),
                (torch.rand(B, generator=g) < 0.2).float()) for _ in range(steps + 2)]
    for u, i, y in batches[:2]:  # warm-up (allocates Adam state)
        opt.zero_grad()
        lf(m(u, i), y).backward()
        opt.step()
    t0 = time.perf_counter()
    for u, i, y in batches[2:]:
        opt.zero_grad()
        lf(m(u, i), y).backward()
        opt.step()
    el = time.perf_counter() - t0
    return dict(value=round(steps * B / el, 1), unit="samples/s", cores=torch.get_num_threads(),
                kind="port", sample=f"{steps} torch-CPU steps of B={B} (same model, dense Adam "
                                    f"over the full {U}x{I} tables)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--factor", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--users", type=int, default=138493)
    ap.add_argument("--items", type=int, default=26744)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, d, L, B = a.users, a.items, a.factor, a.layers, a.batch_size
    pos = syn.make_positives(U, I, 10_000_000, 20261015)
    m = rl.NCF(U, I, d, L, batch_size=B, num_ng=4, seed=7)
    m.set_train(pos)
    # steady state: every user and item row has been touched once (as after the first epoch)
    n = max(U, I)
    cover_u = np.arange(n) % U
    cover_i = np.random.default_rng(0).permutation(n) % I
    m.train_samples(cover_u, cover_i, np.zeros(n, np.float32))
    m.train_steps(0, 0, a.warmup)
    au, ai = m.active_rows()
    m.profile(True)
    st = m.train_steps(0, a.warmup, a.steps)
    kp = m.profile_read()
    m.profile(False)
    step_s = st["seconds"] / a.steps
    E = d * 2 ** (L - 1)
    per_kind = {k: v["ms"] / max(1, v["count"]) * 1e3 for k, v in kp.items()}  # us per launch
    # tower MACs per sample: forward, dX and dW each sum nin * nout over the layers (+ predict)
    macs = sum((2 * E >> l) * (E >> l) for l in range(L)) + 2 * d
    flops = 3 * 2 * macs * B
    tf = flops / step_s / 1e12
    out = {"metric": "NCF NeuMF-end training samples/s, ml-20m shape, factor 64 (config C4)",
           "value": round(a.steps * B / st["seconds"], 1), "unit": "samples/s", "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(step_s * 1e3, 4),
           "dtype": "f32 (tower on v_mfma_f32_16x16x4_f32)", "data": "synthetic ml-20m-shaped positives",
           "config": {"users": U, "items": I, "factor_num": d, "num_layers": L, "batch_size": B,
                      "num_ng": 4, "optimizer": "Adam(lr=0.001), torch's dense semantics (lazy rows)",
                      "active_rows": [au, ai]},
           "launch_us": {"rows (prev row Adam + catch-up)": round(per_kind["catch_up"], 2),
                         "front + mid + back": round(per_kind["fwd_bwd"], 2)},
           "roofline": {"bound": "latency", "kernel": "the step's tower math (forward, dX, dW)",
                        "achieved": round(tf, 3), "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(tf / F32_MFMA_PEAK_TFS, 4), "flops_per_step": flops},
           "loss_per_step": round(st["loss"] / a.steps, 5),
           "cpu_baseline": None if a.no_cpu_baseline else cpu_baseline(U, I, d, L, B)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
