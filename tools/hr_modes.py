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
  planted  the ml-20m shape (138,493 x 26,744, ~10M positives, d=128, B=4096) drawn from a
         ground-truth low-rank model (synthetic.make_planted: P* Q* of rank 8 plus Zipf
         popularity), one random positive per user held out, 99 non-positive candidates: here a
         model that learns the user-item structure beats the popularity ranking, so the modes
         can be told apart.
Throughput of each run (stats.seconds: host wall clock per epoch call) is printed beside it.
Mode "popularity": no training; candidates ranked by their positive count in the training set
(the baseline a model has to beat).  Every trained mode also reports eval_loss: the BPR loss
of its FINAL tables, sum over a fixed sample of (u, i, j) (train positive, uniform non-positive)
per 1e6 triplets, next to final_loss (the loss summed while the last epoch trained).

Mode "local_dpW" (e.g. local_dp8): semantics "local" at world W: W ranks, users
sharded, each with the whole item table, merged every --dp-steps steps; rehearsed as W in-process
ranks sharing this one GPU (threads + the loopback transport), so its quality is what W GPUs
would train (its throughput here is not: the ranks share one GPU)."""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def train_local_dp(rl, W, U, I, d, pos, epochs, seed, dp_steps, dp_overlap=False, local_steps=0, **kw):
    """W ranks of semantics "local" (threads + loopback on this GPU); returns a single-GPU model
    holding the trained (P, Q) for scoring, the per-epoch loss, seconds and triplets."""
    import threading
    sh = rl.sharded
    grp = sh.ThreadGroup(W)
    out, errs = [None] * W, []

    def run(r):
        try:
            m = sh.ShardedBPRMF(U, I, d, seed=seed, device=0, comm=sh.ThreadComm(grp, r),
                                semantics="local", dp_steps=dp_steps, dp_overlap=dp_overlap,
                                local_steps=local_steps, **kw)
            S = m.set_train(pos)
            m.attach_runner("loopback", key=9100 + W)
            hist = [m.train_steps(e, 0, S) for e in range(epochs)]
            out[r] = (m.get_weights(), hist)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    t0 = time.perf_counter()
    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    el = time.perf_counter() - t0
    if errs:
        raise errs[0]
    P = sh.unshard_rows([o[0][0] for o in out], U)
    Q = out[0][0][1]
    m = rl.BPRMF(U, I, d, **{k: v for k, v in kw.items() if k in ("lr", "wd", "batch_size", "num_ng")})
    m.set_weights(P, Q)
    m.history = [{"loss": sum(o[1][e]["loss"] for o in out)} for e in range(epochs)]
    trip = sum(o[1][e]["triplets"] for o in out for e in range(epochs))
    return m, el, trip


def dp_world(mode):
    return int(mode[len("local_dp"):]) if mode.startswith("local_dp") else 0


def big_batch(mode):
    """"exact_bN": the exact step with per-step batch N (the union batch of N / 4096 ranks of the
    exact sharded runner; B > 8192 takes the f32-atomic sums)."""
    return int(mode[len("exact_b"):]) if mode.startswith("exact_b") else 0


def eval_loss(m, pos, I, n=1_000_000, seed=8):
    """BPR loss of the model's final tables on a fixed triplet sample: (u, i) uniform over the
    training positives, j uniform over u's non-positives; -log sigmoid(s_ui - s_uj) summed, per
    1e6 triplets (the same sample for every mode of one workload)."""
    g = np.random.default_rng(seed)
    k = g.integers(0, len(pos), n)
    u, i = pos[k, 0], pos[k, 1]
    keys = np.sort(pos[:, 0] * I + pos[:, 1])
    j = g.integers(0, I, n)
    for _ in range(20):
        q = u * I + j
        hit = keys[np.minimum(np.searchsorted(keys, q), len(keys) - 1)] == q
        if not hit.any():
            break
        j[hit] = g.integers(0, I, int(hit.sum()))
    x = m.score(u, i).astype(np.float64) - m.score(u, j).astype(np.float64)
    return float(np.logaddexp(0.0, -x).sum() * (1e6 / n))


class PopModel:
    """The popularity baseline: a candidate's score is its positive count in the training set."""

    def __init__(self, pos, I):
        self.cnt = np.bincount(pos[:, 1], minlength=I).astype(np.float64)

    def topk_lists(self, users, lists, k):
        out = []
        for lst in lists:
            sc = self.cnt[np.asarray(lst)]
            # ties: the later position first, as topk_lists / np.argsort(pred)[::-1] rank them
            o = np.lexsort((-np.arange(len(lst)), -sc))[:k]
            out.append(np.r_[o, np.full(k - len(o), -1)])
        return np.array(out, dtype=np.int64), None


_PLANTED = {}


def planted_data(U=138493, I=26744, npos=10_000_000, seed=20261101):
    key = (U, I, npos, seed)
    if key not in _PLANTED:
        import torch
        syn = importlib.import_module("recommend-lib_amd.synthetic")
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        pos, _, _ = syn.make_planted(U, I, npos, seed, device=dev)
        g = np.random.default_rng(7)
        start = np.searchsorted(pos[:, 0], np.arange(U))
        deg = np.diff(np.r_[start, len(pos)])
        held = start + (g.random(U) * deg).astype(np.int64)  # one random positive per user
        test = pos[held]
        train = np.delete(pos, held, axis=0)
        _PLANTED[key] = (pos, train, test)
    return _PLANTED[key]


def candidates(pos, test, U, I, n_eval, seed=7):
    g = np.random.default_rng(seed)
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
    return users, lists


def planted(rl, mode, seed, epochs, n_eval, dp_steps=64, dp_overlap=False, local_steps=0):
    U, I = 138493, 26744
    pos, train, test = planted_data(U, I)
    users, lists = candidates(pos, test, U, I, n_eval)
    secs, trip, fl, el = 0.0, 0, None, None
    if mode == "popularity":
        m = PopModel(train, I)
    elif dp_world(mode):
        m, secs, trip = train_local_dp(rl, dp_world(mode), U, I, 128, train, epochs, seed, dp_steps,
                                       dp_overlap, local_steps, batch_size=4096)
        fl = m.history[-1]["loss"]
    else:
        m = rl.BPRMF(U, I, 128, batch_size=4096, seed=seed, semantics=mode, local_steps=local_steps)
        m.set_train(train)
        for _ in range(epochs):
            st = m.train_epoch()
            secs += st["seconds"]
            trip += st["triplets"]
        fl = m.history[-1]["loss"]
    if mode != "popularity":
        el = eval_loss(m, train, I)
    p, _ = m.topk_lists(users, lists, 10)
    hit = (p == 0).any(1)
    rank = np.where(p == 0, np.arange(10)[None, :], 99).min(1)
    ndcg = np.where(hit, 1.0 / np.log2(rank + 2.0), 0.0)
    return dict(workload="planted ml-20m shape (rank-8 P*Q* + Zipf popularity), 1 held-out positive "
                         "+ 99 negatives, d=128, B=4096", mode=mode, seed=seed, epochs=epochs,
                users_eval=int(len(users)), hr10=round(float(hit.mean()), 5),
                ndcg10=round(float(ndcg.mean()), 5),
                final_loss=None if fl is None else round(fl, 2),
                eval_loss_per_1e6=None if el is None else round(el, 1),
                triplets_per_s=round(trip / secs, 1) if secs else None)


def f5(rl, mode, seed, dp_steps=64, dp_overlap=False, local_steps=0):
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "hr_ndcg_ml100k.json")) as fh:
        ref = json.load(fh)
    f = np.load(os.path.join(g, "hr_ndcg_ml100k.npz"))
    p = ref["protocol"]
    gt = {int(u): set(f["gt_items"][f["gt_ptr"][k]:f["gt_ptr"][k + 1]].tolist())
          for k, u in enumerate(f["gt_users"])}
    if mode == "popularity":
        m, el = PopModel(f["positives"].astype(np.int64), int(f["I"])), 0.0
        m.history = [{"loss": None}]
    elif dp_world(mode):
        m, el, _ = train_local_dp(rl, dp_world(mode), int(f["U"]), int(f["I"]), p["factor_num"],
                                  f["positives"].astype(np.int64), p["epochs"], seed, dp_steps,
                                  dp_overlap, local_steps, lr=p["lr"], wd=p["wd"], batch_size=p["batch_size"], num_ng=p["num_ng"])
    else:
        m = rl.BPRMF(int(f["U"]), int(f["I"]), p["factor_num"], lr=p["lr"], wd=p["wd"],
                     batch_size=p["batch_size"], num_ng=p["num_ng"], seed=seed, semantics=mode,
                     local_steps=local_steps)
        t0 = time.perf_counter()
        m.fit(f["positives"].astype(np.int64), epochs=p["epochs"])
        el = time.perf_counter() - t0
    if mode == "popularity":
        kpi = rl.metrics.evaluate_topk(m, f["test_data"], gt, p["topk"])
        ev = None
    else:
        kpi = rl.metrics.evaluate_topk(m, f["test_data"], gt, p["topk"])
        ev = eval_loss(m, f["positives"].astype(np.int64), int(f["I"]), n=200_000)
    fl = m.history[-1]["loss"]
    return dict(workload="f5 ml-100k fo/tfo d=32", mode=mode, seed=seed, epochs=p["epochs"],
                hr10=round(kpi["hr"], 5), ndcg10=round(kpi["ndcg"], 5),
                final_loss=None if fl is None else round(fl, 2),
                eval_loss_per_1e6=None if ev is None else round(ev, 1), train_s=round(el, 3),
                reference=dict(hr10=ref["summary"]["hr"], ndcg10=ref["summary"]["ndcg"]))


def ml20m(rl, mode, seed, epochs, n_eval, dp_steps=64, dp_overlap=False, local_steps=0):
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
    if dp_world(mode):
        m, secs, trip = train_local_dp(rl, dp_world(mode), U, I, 128, train, epochs, seed, dp_steps,
                                       dp_overlap, local_steps, batch_size=4096)
    else:
        if big_batch(mode):
            m = rl.BPRMF(U, I, 128, batch_size=big_batch(mode), seed=seed)
        else:
            m = rl.BPRMF(U, I, 128, batch_size=4096, seed=seed, semantics=mode, local_steps=local_steps)
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
    ap.add_argument("--dp-steps", type=int, default=64, help="local_dpW: steps between item merges")
    ap.add_argument("--dp-overlap", action="store_true", help="local_dpW: all-reduce beside the next period")
    ap.add_argument("--local-steps", type=int, default=0, help="local: steps between XCD merges (0: 128)")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    rl = importlib.import_module("recommend-lib_amd")
    for w in a.which.split(","):
        if w == "planted":
            r = planted(rl, "popularity", 0, 0, a.users_eval)
            print(json.dumps(r), flush=True)
        for mode in a.modes.split(","):
            for seed in (int(x) for x in a.seeds.split(",")):
                if w == "f5":
                    r = f5(rl, mode, seed, a.dp_steps, a.dp_overlap, a.local_steps)
                elif w == "planted":
                    r = planted(rl, mode, seed, a.epochs, a.users_eval, a.dp_steps, a.dp_overlap,
                                a.local_steps)
                else:
                    r = ml20m(rl, mode, seed, a.epochs, a.users_eval, a.dp_steps, a.dp_overlap,
                              a.local_steps)
                if mode == "local" or dp_world(mode):
                    r["local_steps"] = a.local_steps or 128
                if dp_world(mode):
                    r["dp_steps"] = a.dp_steps
                    r["dp_overlap"] = a.dp_overlap
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
