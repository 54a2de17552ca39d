"""Measurement of the Item2Vec row: the reference's SGNS training loop
(Item2VecRecommender.py:272-287) on the GPU with its defaults (e_dim 300, n_negs 20, window 5,
mb 4096, uniform negatives, Adam lr 1e-3).

  python tools/bench_sgns.py [--epochs E] [--dim E] [--negs N] [--mb B] [--items I]

Workload: ml-100k's shape, synthetic (943 users, 1,682 items, 100,000 ratings, Zipf 0.5 item
popularity), the corpus built by BuildCorpus from all ratings and converted from the 80 % train
split (data_split 'fo'): ~80 k examples per epoch, vocabulary ~1,684.  One JSON line: examples/s
over the timed epochs (device time of sgns_train, examples host-side like the DataLoader's),
ms/step, and the step's roofline against HBM: algorithmic bytes per example = (1 + C + C n) table
rows x E x 4 B read by the forward (the rows the reference's three embedding lookups gather);
the tables (2 x 2 MB) sit in L2 / MALL, so this is a lower bound on the traffic the step moves.
CPU baseline: the numpy oracle step (float64, oracle/sgns_oracle.py) on a bounded sample.
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

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--negs", type=int, default=20)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--mb", type=int, default=4096)
    ap.add_argument("--items", type=int, default=1682)
    ap.add_argument("--cpu-steps", type=int, default=2)
    a = ap.parse_args()
    import pandas as pd
    import torch
    rl = importlib.import_module("recommend-lib_amd")
    from oracle import sgns_oracle as O
    g = np.random.default_rng(7)
    U, I, n = 943, a.items, 100_000
    act = g.lognormal(0.0, 1.0, U)
    w = 1.0 / np.arange(1, I + 1) ** 0.5
    df = pd.DataFrame({"user": g.choice(U, n, p=act / act.sum()),
                       "item": g.permutation(I)[g.choice(I, n, p=w / w.sum())]})
    pre = rl.BuildCorpus(df, window=a.window, max_vocab=20000).build()
    train = df.sample(frac=0.8, random_state=1)
    iw, ow = pre.convert(train, 0)
    V = len(pre.idx2word)
    C = 2 * a.window
    torch.manual_seed(0)
    m = rl.Item2Vec(V, a.dim)
    s = rl.SGNS(m, V, n_negs=a.negs, context=C, max_batch=a.mb, seed=1)
    s.train_examples(iw[: 2 * a.mb], ow[: 2 * a.mb], batch_size=a.mb)  # warm-up (rocBLAS init)
    secs, steps = 0.0, 0
    data = rl.PermutedSubsampledCorpus((iw, ow))
    np.random.seed(0)
    t0 = time.perf_counter()
    for _ in range(a.epochs):
        s.train_epoch(data, a.mb)
        secs += s.last_stats["seconds"]
        steps += s.last_stats["steps"]
    wall = time.perf_counter() - t0
    ex = len(iw) * a.epochs
    gpu = ex / secs
    ms_step = secs / steps * 1e3
    R = 1 + C + C * a.negs
    per_step = a.mb * R * a.dim * 4
    achieved = per_step / (ms_step * 1e-3) / 1e9
    # CPU: the oracle step on the first cpu_steps batches (its own negatives)
    sd = s.state_dict()
    st = O.State(sd["embedding.ivectors.weight"], sd["embedding.ovectors.weight"])
    cs = a.cpu_steps
    t0 = time.perf_counter()
    for k in range(cs):
        sl = slice(k * a.mb, (k + 1) * a.mb)
        nw = g.integers(0, V - 1, (len(iw[sl]), C * a.negs))
        O.step(st, iw[sl], ow[sl], nw)
    cpu_s = time.perf_counter() - t0
    cpu = cs * a.mb / cpu_s
    out = {"metric": "Item2Vec SGNS training examples/s (Item2VecRecommender.py train loop)",
           "value": round(gpu, 1), "unit": "examples/s", "n_gpus": 1, "epochs": a.epochs,
           "ms_per_step": round(ms_step, 5), "dtype": "f32", "data": "synthetic ml-100k shape",
           "config": {"workload": "Item2Vec epoch, ml-100k shape", "vocab": V,
                      "examples_per_epoch": int(len(iw)), "e_dim": a.dim, "n_negs": a.negs,
                      "window": a.window, "mb": a.mb, "opt": "Adam", "negatives": "uniform"},
           "device_seconds": round(secs, 4), "wall_seconds": round(wall, 4),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "per_step_bytes": per_step},
           "cpu_baseline": {"value": round(cpu, 1), "unit": "examples/s", "cores": 1,
                            "kind": "port",
                            "sample": f"{cs} steps of mb={a.mb} through the numpy oracle (float64)"}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
