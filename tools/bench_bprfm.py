"""Measurement of the BPR-FM row: the reference's BPRFM training loop
(BPRFMRecommender.py:196-227) on the GPU with the reference defaults (hidden_factor 64,
batch_norm on, dropout 0.5, Adagrad lr 0.05, batch_size 4096, num_ng 4).

  python tools/bench_bprfm.py [--epochs E] [--factors K] [--batch B] [--no-bn] [--dropout P]

Workload: ml-100k's shape (943 users + 1,682 items = 2,625 features, 99,057 train rows after the
leave-one-out split, x 4 negatives = 396,228 triplets per epoch), synthetic (the GPU box has no
data): users by lognormal activity, items by Zipf 0.5, negatives uniform.  One JSON line:
triplets/s over the timed epochs (device time of bprfm_train, triplets already host-side like the
reference's DataLoader output), us/step, and the roofline of the step: algorithmic bytes per
triplet = 3 rows x (embedding read + write, accumulator read + write) x 4 B x k (Adagrad's
minimum traffic; gradients and BatchNorm scratch are not counted), per step x B, over the step's
device time.  CPU baseline: the oracle's numpy step (float64, oracle/bprfm_oracle.py) on a bounded
sample of the same batches.
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (/opt/skills/guides/MI355X_MICROARCH.md)


def triplets(U, I, rows, num_ng, seed=7):
    g = np.random.default_rng(seed)
    act = g.lognormal(0.0, 1.0, U)
    u = g.choice(U, rows, p=act / act.sum())
    w = 1.0 / np.arange(1, I + 1) ** 0.5
    i = g.permutation(I)[g.choice(I, rows, p=w / w.sum())]
    u, i = np.repeat(u, num_ng), np.repeat(i, num_ng)
    j = g.integers(0, I, len(u))
    perm = g.permutation(len(u))  # the DataLoader's shuffle
    return (u[perm].astype(np.int32), (U + i[perm]).astype(np.int32),
            (U + j[perm]).astype(np.int32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--factors", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--no-bn", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=20)
    a = ap.parse_args()
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    rl = importlib.import_module("recommend-lib_amd")
    from oracle import bprfm_oracle as O
    U, I, rows, ng = 943, 1682, 99_057, 4
    u, i, j = triplets(U, I, rows, ng)
    n, k, B, bn = len(u), a.factors, a.batch, not a.no_bn
    m = rl.BPRFM(U + I, k, bn, [a.dropout, 0.2], lr=0.05, max_batch=B, seed=1)
    m.train_triplets(u[: 4 * B], i[: 4 * B], j[: 4 * B], B)  # warm-up
    secs, steps, loss = 0.0, 0, 0.0
    t0 = time.perf_counter()
    for _ in range(a.epochs):
        loss = m.train_triplets(u, i, j, B)
        secs += m.last_stats["seconds"]
        steps += m.last_stats["steps"]
    wall = time.perf_counter() - t0
    gpu = n * a.epochs / secs
    us_step = secs / steps * 1e6
    alg = 3 * 4 * 4 * k * B  # bytes per full step
    achieved = alg / (us_step * 1e-6) / 1e9
    # CPU: the oracle step on the first cpu_steps batches
    sd = m.state_dict()
    st = O.State(sd["embeddings.weight"], sd["biases.weight"], sd["bias_"],
                 sd.get("FM_layers.0.weight"), sd.get("FM_layers.0.bias"))
    cs = min(a.cpu_steps, (n + B - 1) // B)
    t0 = time.perf_counter()
    for s in range(cs):
        sl = slice(s * B, (s + 1) * B)
        masks = None
        if a.dropout > 0:
            masks = (np.random.default_rng(s).random((2, len(u[sl]), k)) >= a.dropout) / (1 - a.dropout)
        O.step(st, 0, u[sl], i[sl], j[sl], 0.05, masks=masks)
    cpu_s = time.perf_counter() - t0
    cpu = min(n, cs * B) / cpu_s
    out = {"metric": "BPR-FM training triplets/s (BPRFMRecommender.py train loop)",
           "value": round(gpu, 1), "unit": "triplets/s", "n_gpus": 1, "epochs": a.epochs,
           "ms_per_step": round(us_step / 1e3, 5), "dtype": "f32", "data": "synthetic ml-100k shape",
           "config": {"workload": "BPR-FM epoch, ml-100k shape", "features": U + I,
                      "triplets_per_epoch": n, "hidden_factor": k, "batch_size": B,
                      "batch_norm": bn, "dropout": a.dropout, "lr": 0.05, "opt": "Adagrad"},
           "last_epoch_loss": loss, "device_seconds": round(secs, 4), "wall_seconds": round(wall, 4),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "per_step_bytes": alg},
           "cpu_baseline": {"value": round(cpu, 1), "unit": "triplets/s", "cores": 1, "kind": "port",
                            "sample": f"{cs} steps of B={B} through the numpy oracle (float64)"}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
