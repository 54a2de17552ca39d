"""Measurement of the rating-SGD row: the reference's Cython SVD.fit
(util/matrix_factorization.pyx:104-155) on the GPU, exact per-sample SGD in dependency levels.

  python tools/bench_mf.py [--shape ml-1m|ml-100k] [--factors K] [--epochs E]

Workloads: ml-100k is the reference's own data/ml-100k ratings when present (it is not on the
GPU box: then a synthetic set of its shape); ml-1m is synthetic at ml-1m's shape (6,040 users x
3,706 items, 1,000,209 ratings) with a popularity skew matched to ml-1m's (the most rated movie
holds ~0.3 % of the ratings: Zipf alpha 0.4 over the items; lognormal user activity).  SVD with
the reference defaults (n_factors 100, lr 0.005, reg 0.02, biased).  One JSON line: samples/s
(train rows x epochs / device time), dependency levels per epoch, and the CPU baseline: the
oracle's C restatement of the same loop on one host core (the loop is a strict sequence; the
reference's own Cython, measured in the build container at ~40.5 k samples/s for d=32, is
slower still: SURVEY.md §6).  Results are bit-identical to the reference's (tests/test_gpu_mf.py).
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


def ratings(shape, seed=7):
    g = np.random.default_rng(seed)
    if shape == "ml-100k":
        path = "/root/reference/data/ml-100k/u.data"
        if os.path.exists(path):
            a = np.loadtxt(path, dtype=np.int64)
            _, u = np.unique(a[:, 0], return_inverse=True)
            _, i = np.unique(a[:, 1], return_inverse=True)
            return u, i, a[:, 2].astype(np.float64), "reference data/ml-100k/u.data"
        U, I, n, alpha = 943, 1682, 100_000, 0.5
    else:
        U, I, n, alpha = 6040, 3706, 1_000_209, 0.4
    act = g.lognormal(0.0, 1.0, U)
    u = g.choice(U, n, p=act / act.sum())
    w = 1.0 / np.arange(1, I + 1) ** alpha
    i = g.permutation(I)[g.choice(I, n, p=w / w.sum())]
    r = g.integers(1, 6, n).astype(np.float64)
    return u, i, r, f"synthetic {shape} shape ({U} users x {I} items, {n} ratings, Zipf {alpha})"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ml-1m", choices=["ml-1m", "ml-100k"])
    ap.add_argument("--factors", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--cpu-epochs", type=int, default=1)
    ap.add_argument("--model", default="svd", choices=["svd", "svdpp"])
    a = ap.parse_args()
    import pandas as pd
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    rl = importlib.import_module("recommend-lib_amd")
    from oracle import c_oracle as C
    u, i, r, what = ratings(a.shape)
    if a.model == "svdpp":  # one rating per (user, item), as in real rating data
        _, keep = np.unique(u.astype(np.int64) * (int(i.max()) + 1) + i, return_index=True)
        keep.sort()
        u, i, r = u[keep], i[keep], r[keep]
        what += f", duplicate (user, item) pairs dropped: {len(u)} ratings"
    U, I = int(u.max()) + 1, int(i.max()) + 1
    df = pd.DataFrame({"user": u, "item": i, "rating": r})
    if a.model == "svdpp":
        m = rl.SVDpp(U, I, n_factors=a.factors, n_epochs=1, verbose=False)
    else:
        m = rl.SVD(U, I, n_factors=a.factors, n_epochs=1, verbose=False)
    np.random.seed(0)
    m.fit(df)  # warm-up (kernel load, schedule build)
    m.n_epochs = a.epochs
    np.random.seed(0)
    t0 = time.perf_counter()
    m.fit(df)
    wall = time.perf_counter() - t0
    st = m.last_stats
    gpu = st["samples"] / st["seconds"]
    # CPU: the same loop in C (one core), from the same initial tables
    np.random.seed(0)
    P0 = np.random.normal(0, .1, (U, a.factors))
    Q0 = np.random.normal(0, .1, (I, a.factors))
    t0 = time.perf_counter()
    if a.model == "svdpp":
        Y0 = np.random.normal(0, .1, (I, a.factors))
        C.svdpp_epochs(u, i, r, P0, Q0, Y0, np.zeros(U), np.zeros(I), df.rating.mean(),
                       [0.007] * 5, [0.02] * 5, a.cpu_epochs)
    else:
        C.svd_epochs(u, i, r, P0, Q0, np.zeros(U), np.zeros(I), df.rating.mean(), 1,
                     [0.005] * 4, [0.02] * 4, a.cpu_epochs)
    cpu_s = time.perf_counter() - t0
    cpu = len(u) * a.cpu_epochs / cpu_s
    name = "SVDpp" if a.model == "svdpp" else "SVD"
    lr, reg = (0.007, 0.02) if a.model == "svdpp" else (0.005, 0.02)
    out = {"metric": f"{name}.fit per-sample SGD samples/s (util/matrix_factorization.pyx)",
           "value": round(gpu, 1), "unit": "samples/s", "n_gpus": 1, "epochs": a.epochs,
           "dtype": "f64", "data": what,
           "config": {"workload": f"{name} fit, {a.shape} shape", "users": U, "items": I,
                      "ratings": int(len(u)), "n_factors": a.factors, "lr": lr, "reg": reg},
           "levels_per_epoch": st["levels"], "us_per_level": round(st["seconds"] / a.epochs / st["levels"] * 1e6, 3),
           "device_seconds": round(st["seconds"], 4), "wall_seconds_fit": round(wall, 4),
           "semantics": "bit-identical to the reference's sequential Cython loop",
           "cpu_baseline": {"value": round(cpu, 1), "unit": "samples/s", "cores": 1, "kind": "port",
                            "sample": f"{a.cpu_epochs} epoch(s) of the C restatement (oracle/mf_cpu.c)"}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
