"""Measurement of the ranking row: full-catalogue top-k for every user of
the ml-20m shape (138,493 users x 26,744 items, d=128, k=10, training positives skipped), the
serving form of BPRMFRecommender.py:196-207's ranking.

  python tools/bench_topk.py [--users N] [--k K] [--repeat R]

Prints one JSON line: users/s, the kernel's time from HIP events (bprmf_profile, kind topk_all),
its MFMA roofline (2*U*I*d flops over the f32 MFMA peak, 157.3 TF; MI355X_MICROARCH.md), and a
CPU baseline: numpy f32 GEMM + argpartition over a bounded sample of users on this host's cores.
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
MFMA_F32_PEAK_TF = 157.3


def blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max(int(x.get("num_threads", 1)) for x in threadpool_info()) or 1
    except Exception:  # noqa: BLE001
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=138493)
    ap.add_argument("--items", type=int, default=26744)
    ap.add_argument("--factor", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--cpu-users", type=int, default=4096)
    a = ap.parse_args()
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, d, k = a.users, a.items, a.factor, a.k
    pos = syn.make_positives(U, I, 10_000_000, 20261015)
    m = rl.BPRMF(U, I, d, seed=1)
    m.set_train(pos)
    m.train_steps(0, 0, 50)  # some rows carry pending decay, as in serving after training
    users = np.arange(U, dtype=np.int32)
    m.topk_all(users[:4096], k)  # warm-up
    m.profile(True)
    t0 = time.perf_counter()
    for _ in range(a.repeat):
        items, scores = m.topk_all(users, k)
    wall = (time.perf_counter() - t0) / a.repeat
    kp = m.profile_read()["topk_all"]
    m.profile(False)
    kern_s = kp["ms"] / kp["count"] * 1e-3
    flops = 2.0 * U * I * d
    ach = flops / kern_s / 1e12
    # CPU baseline: the same ranking with numpy on the host (f32 GEMM, argpartition), sample
    P, Q = m.get_weights()
    n = min(a.cpu_users, U)
    t0 = time.perf_counter()
    S = P[:n] @ Q.T
    order = np.argsort(pos[:, 0], kind="stable")
    pu, pi = pos[order, 0], pos[order, 1]
    starts = np.searchsorted(pu, np.arange(n + 1))
    for u in range(n):
        S[u, pi[starts[u]:starts[u + 1]]] = -np.inf
    top = np.argpartition(-S, k, axis=1)[:, :k]
    top = np.take_along_axis(top, np.argsort(-np.take_along_axis(S, top, 1), 1), 1)
    cpu_s = time.perf_counter() - t0
    agree = float(np.mean([len(set(top[u]) & set(items[u])) / k for u in range(n)]))
    out = {"metric": "full-catalogue top-k users/s, ml-20m shape", "value": round(U / kern_s, 1),
           "unit": "users/s", "k": k, "factor_num": d, "users": U, "items": I,
           "kernel_ms": round(kern_s * 1e3, 3), "call_ms_incl_copies": round(wall * 1e3, 3),
           "dtype": "f32 (MFMA 16x16x4 f32, exact f32)",
           "roofline": {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F32_PEAK_TF,
                        "unit": "TFLOP/s", "frac": round(ach / MFMA_F32_PEAK_TF, 4),
                        "flops_per_launch": flops},
           "cpu_baseline": {"value": round(n / cpu_s, 1), "unit": "users/s",
                            "cores": blas_threads(), "kind": "numpy",
                            "sample": f"{n} users: f32 GEMM vs all {I} items + argpartition"},
           "topk_agreement_vs_cpu": round(agree, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
