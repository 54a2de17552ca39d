"""HR@10 / NDCG@10 of the exact step and the relaxed ones (hogwild, local) on the same data, one
JSON line per (workload, mode).  GPU box:  python tools/hr_modes.py [--epochs E] [--users-eval N]

Workloads:
  f5     the reference protocol of tests/golden/hr_ndcg_ml100k.* (ml-100k fo/tfo, d=32, B=4096,
         20 epochs, the reference's own split and candidates), scored as BPRMFRecommender.py:196-229
         with metrics.evaluate_topk; the reference's mean / std over 5 seeds beside it.
  ml20m  the bench workload (synthetic ml-20m shape, d=128, B=4096): each user's last positive held
         out (leave-one-out), 99 non-positive candidates drawn per user plus the held-out item,
         HR@10 / NDCG@10 over `--users-eval` users after `--epochs` epochs.  Synthetic data has no
         taste structure beyond item popularity, so this compares the two modes with each other,
         not with any published number.
Throughput of each run (stats.seconds: host wall clock per epoch call) is printed beside it."""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def f5(rl, mode, seed):
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "hr_ndcg_ml100k.json")) as fh:
        ref = json.load(fh)
    f = np.load(os.path.join(g, "hr_ndcg_ml100k.npz"))
    p = ref["protocol"]
    gt = {int(u): set(f["gt_items"][f["gt_ptr"][k]:f["gt_ptr"][k + 1]].tolist())
          for k, u in enumerate(f["gt_users"])}
    m = rl.BPRMF(int(f["U"]), int(f["I"]), p["factor_num"], lr=p["lr"], wd=p["wd"],
                 batch_size=p["batch_size"], num_ng=p["num_ng"], seed=seed, semantics=mode)
    t0 = time.perf_counter()
    m.fit(f["positives"].astype(np.int64), epochs=p["epochs"])
    el = time.perf_counter() - t0
    kpi = rl.metrics.evaluate_topk(m, f["test_data"], gt, p["topk"])
    return dict(workload="f5 ml-100k fo/tfo d=32", mode=mode, seed=seed, epochs=p["epochs"],
                hr10=round(kpi["hr"], 5), ndcg10=round(kpi["ndcg"], 5),
                final_loss=round(m.history[-1]["loss"], 2), train_s=round(el, 3),
                reference=dict(hr10=ref["summary"]["hr"], ndcg10=ref["summary"]["ndcg"]))


def ml20m(rl, mode, seed, epochs, n_eval):
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I = 138493, 26744
    pos = syn.make_positives(U, I, 10_000_000, 20261015)
    last = np.r_[np.flatnonzero(np.diff(pos[:, 0])), len(pos) - 1]  # each user's last row
    test = pos[last]
    train = np.delete(pos, last, axis=0)
    g = np.random.default_rng(7)
    users = np.sort(g.choice(U, size=min(n_eval, U), replace=False))
    starts = np.searchsorted(pos[:, 0], users)
    ends = np.searchsorted(pos[:, 0], users, side="right")
    lists = []
    for u, b, e in zip(users, starts, ends):
        seen = set(pos[b:e, 1].tolist())
        cand = []
        while len(cand) < 99:
            x = int(g.integers(0, I))
            if x not in seen:
                seen.add(x)
                cand.append(x)
        lists.append([int(test[u, 1])] + cand)  # the held-out item first
    m = rl.BPRMF(U, I, 128, batch_size=4096, seed=seed, semantics=mode)
    m.set_train(train)
    secs, trip = 0.0, 0
    for _ in range(epochs):
        st = m.train_epoch()
        secs += st["seconds"]
        trip += st["triplets"]
    p, _ = m.topk_lists(users, lists, 10)
    hit = (p == 0).any(1)
    rank = np.where(p == 0, np.arange(10)[None, :], 99).min(1)
    ndcg = np.where(hit, 1.0 / np.log2(rank + 2.0), 0.0)
    return dict(workload="ml-20m shape synthetic, loo + 99 negatives, d=128, B=4096", mode=mode,
                seed=seed, epochs=epochs, users_eval=int(len(users)), hr10=round(float(hit.mean()), 5),
                ndcg10=round(float(ndcg.mean()), 5), final_loss=round(m.history[-1]["loss"], 2),
                triplets_per_s=round(trip / secs, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--users-eval", type=int, default=20000)
    ap.add_argument("--seeds", default="11,12,13")
    ap.add_argument("--which", default="f5,ml20m")
    ap.add_argument("--modes", default="exact,hogwild,local")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    rl = importlib.import_module("recommend-lib_amd")
    for w in a.which.split(","):
        for mode in a.modes.split(","):
            for seed in (int(x) for x in a.seeds.split(",")):
                r = f5(rl, mode, seed) if w == "f5" else ml20m(rl, mode, seed, a.epochs, a.users_eval)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
