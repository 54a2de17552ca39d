"""Generate the golden fixtures F1-F5 by IMPORTING the reference (read-only) in the
build container.  Test infrastructure only: this script is never run on the GPU box
(/root/reference does not exist there); only its outputs travel.

It does not copy reference source.  It imports `BPRMFRecommender.BPR`,
`util.data_loader.{load_mat,BPRData}` and `util.metrics` from /root/reference and
drives them the way `BPRMFRecommender.py:135-229` does, with every RNG seeded.

Environment shims (the reference is left untouched):
  * `np.asfarray` was removed in NumPy 2; `util/metrics.py:178` needs it.
  * The working split protocol is data_split='fo', val_method='tfo' (SURVEY.md §8c).

Fixtures written next to this file:
  F1 bpr_step_tiny.npz      U=50 I=80 d=8, 6 batches (one all-duplicates), P,Q after each step
  F2 bpr_ml100k_replay.npz  ml-100k fo/tfo split, d=32, ONE full epoch of reference triplets
                            (BPRData.ng_sample + shuffled DataLoader, B=4096), P,Q after batch 10
                            and after the epoch, per-batch loss
  F3 ng_sample_ml100k.npz   histogram of sampled negatives j and per-user negative counts of the
                            same ng_sample call (distributional sampler parity)
  F4 metrics_kat.json       precision/recall/map/ndcg/hr/mrr@K and _bpr_topk on fixed inputs
  F5 hr_ndcg_ml100k.npz/.json  test candidates + ground truth of the split and the final
                            HR@10/NDCG@10/... of 20-epoch reference runs over 5 training seeds
Run:  python tests/golden/make_golden.py [--quick]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    if not hasattr(np, "asfarray"):
        np.asfarray = lambda a, dtype=float: np.asarray(a, dtype=dtype)
    import torch
    import BPRMFRecommender as R
    from util import data_loader as D
    from util import metrics as M
    return torch, R, D, M


def _seed_all(torch, s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def _ref_step(torch, model, opt, u, i, j):
    """One training step exactly as BPRMFRecommender.py:172-176."""
    model.zero_grad()
    pi, pj = model(u, i, j)
    loss = -(pi - pj).sigmoid().log().sum()
    loss.backward()
    opt.step()
    return float(loss.item())


def make_f1(torch, R):
    _seed_all(torch, 1234)
    U, I, d, B, lr, wd = 50, 80, 8, 64, 0.01, 0.001
    model = R.BPR(U, I, d)
    opt = torch.optim.SGD(model.parameters(), lr=lr, weight_decay=wd)
    P0 = model.embed_user.weight.detach().numpy().copy()
    Q0 = model.embed_item.weight.detach().numpy().copy()
    g = np.random.default_rng(7)
    trip, Ps, Qs, losses = [], [], [], []
    nb = 6
    for b in range(nb):
        u = g.integers(0, U, B)
        i = g.integers(0, I, B)
        j = g.integers(0, I, B)
        if b == 3:  # all-duplicate batch: one user, one positive, 8 negatives
            u[:] = 5
            i[:] = 11
            j = g.integers(0, 8, B) + 20
        if b == 4:  # i == j for half the rows (x = 0, item grads cancel)
            j[: B // 2] = i[: B // 2]
        trip.append(np.stack([u, i, j]).astype(np.int32))
        tu, ti, tj = (torch.tensor(a, dtype=torch.long) for a in (u, i, j))
        losses.append(_ref_step(torch, model, opt, tu, ti, tj))
        Ps.append(model.embed_user.weight.detach().numpy().copy())
        Qs.append(model.embed_item.weight.detach().numpy().copy())
    np.savez_compressed(
        os.path.join(OUT, "bpr_step_tiny.npz"),
        U=U, I=I, d=d, B=B, lr=lr, wd=wd, P0=P0, Q0=Q0,
        triplets=np.stack(trip), P=np.stack(Ps), Q=np.stack(Qs),
        loss=np.array(losses, dtype=np.float64))


def _load_split(torch, D, seed):
    """load_mat(ml-100k, fo, by_time=1, tfo) with the data seed fixed (util/data_loader.py:444-548)."""
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        _seed_all(torch, seed)
        out = D.load_mat("ml-100k", data_split="fo", by_time=1, val_method="tfo")
    finally:
        os.chdir(cwd)
    train_list, test_data, user_num, item_num, train_mat_list, ur, val_list = out
    return train_list[0], test_data, int(user_num), int(item_num), train_mat_list[0], ur, val_list[0]


def make_f2_f3(torch, R, D, split):
    train, test_data, U, I, train_mat, ur, val = split
    d, B, lr, wd, num_ng = 32, 4096, 0.01, 0.001, 4
    _seed_all(torch, 2024)
    ds = D.BPRData(train, I, train_mat, num_ng, True)
    t0 = time.time()
    ds.ng_sample()
    t_ng = time.time() - t0
    gen = torch.Generator().manual_seed(2024)
    loader = torch.utils.data.DataLoader(ds, batch_size=B, shuffle=True, num_workers=0, generator=gen)
    torch.manual_seed(99)
    model = R.BPR(U, I, d)
    opt = torch.optim.SGD(model.parameters(), lr=lr, weight_decay=wd)
    P0 = model.embed_user.weight.detach().numpy().copy()
    Q0 = model.embed_item.weight.detach().numpy().copy()
    batches, losses = [], []
    P10 = Q10 = None
    t0 = time.time()
    for bi, (u, i, j) in enumerate(loader):
        batches.append(np.stack([u.numpy(), i.numpy(), j.numpy()]).astype(np.int16))
        losses.append(_ref_step(torch, model, opt, u, i, j))
        if bi == 9:
            P10 = model.embed_user.weight.detach().numpy().copy()
            Q10 = model.embed_item.weight.detach().numpy().copy()
    t_train = time.time() - t0
    trip = np.concatenate(batches, axis=1)
    bounds = np.cumsum([0] + [b.shape[1] for b in batches]).astype(np.int64)
    pos = np.asarray(train, dtype=np.int16)
    np.savez_compressed(
        os.path.join(OUT, "bpr_ml100k_replay.npz"),
        U=U, I=I, d=d, B=B, lr=lr, wd=wd, num_ng=num_ng, positives=pos,
        P0=P0, Q0=Q0, triplets=trip, batch_bounds=bounds,
        P10=P10, Q10=Q10,
        P_epoch=model.embed_user.weight.detach().numpy(),
        Q_epoch=model.embed_item.weight.detach().numpy(),
        loss=np.array(losses, dtype=np.float64),
        ref_seconds=np.array([t_ng, t_train]))
    # F3: negatives of the same ng_sample call (features_fill order, before the shuffle)
    fill = np.asarray(ds.features_fill, dtype=np.int64)
    hist_j = np.bincount(fill[:, 2], minlength=I).astype(np.int64)
    neg_per_user = np.bincount(fill[:, 0], minlength=U).astype(np.int64)
    in_train = sum(1 for (uu, _, jj) in ds.features_fill if (uu, jj) in train_mat)
    np.savez_compressed(
        os.path.join(OUT, "ng_sample_ml100k.npz"),
        U=U, I=I, num_ng=num_ng, hist_j=hist_j, neg_per_user=neg_per_user,
        n_triplets=len(fill), negatives_in_train=in_train,
        first_rows=fill[:64].astype(np.int32))
    print(f"F2/F3: {len(fill)} triplets, ng_sample {t_ng:.2f}s, epoch train {t_train:.2f}s")


def make_f4(torch, R, M):
    g = np.random.default_rng(11)
    K = 10
    cases = []
    for n in range(40):
        L = int(g.integers(K, 3 * K))
        r = (g.random(L) < 0.25).astype(int).tolist()
        if n == 0:
            r = [0] * L
        if n == 1:
            r = [1] * L
        gt_len = int(sum(r) + g.integers(0, 4))
        cases.append(dict(r=r, gt_len=gt_len,
                          precision=float(M.precision_at_k(r, K)),
                          recall=float(M.recall_at_k(r, gt_len, K)),
                          ndcg=float(M.ndcg_at_k(r, K)),
                          ap=float(M.average_precision(r[:K]))))
    rs = [c["r"][:K] for c in cases]
    us = list(range(len(rs)))
    ur = {u: set(range(max(1, c["gt_len"]))) for u, c in zip(us, cases)}
    agg = dict(map=float(M.map_at_k(rs)), mrr=float(M.mrr_at_k(rs)), hr=float(M.hr_at_k(rs, us, ur)),
               hr_denoms=[len(ur[u]) for u in us])
    # _bpr_topk on a tiny model: 6 users x 100 candidates, candidate 0 is the ground truth
    _seed_all(torch, 5)
    model = R.BPR(6, 300, 16)
    cand = []
    for u in range(6):
        items = g.choice(300, 100, replace=False)
        cand += [[u, int(x)] for x in items]
    ds = [(torch.tensor(u), torch.tensor(i), torch.tensor(i)) for u, i in cand]
    loader = torch.utils.data.DataLoader(ds, batch_size=100, shuffle=False)
    hr, ndcg = M.metric_eval(model, loader, K)
    topk = dict(P=model.embed_user.weight.detach().numpy().tolist(),
                Q=model.embed_item.weight.detach().numpy().tolist(),
                candidates=cand, k=K, hr=float(hr), ndcg=float(ndcg))
    with open(os.path.join(OUT, "metrics_kat.json"), "w") as f:
        json.dump(dict(k=K, cases=cases, aggregate=agg, bpr_topk=topk), f)


def _kpi(torch, M, model, test_data, ur, topk=10):
    """Final KPI of BPRMFRecommender.py:195-229 (scores computed per user in one batched forward
    of the same module instead of one forward per candidate; same embedding+mul+sum ops)."""
    from collections import defaultdict
    test_u_is = defaultdict(set)
    for ele in test_data:
        test_u_is[int(ele[0])].add(int(ele[1]))
    preds = {}
    with torch.no_grad():
        for u in test_u_is.keys():
            items = list(test_u_is[u])
            it = torch.tensor(items, dtype=torch.long)
            s = model(torch.full_like(it, u), it, it)[0].numpy()
            rec_idx = np.argsort(s)[::-1][:topk]
            preds[u] = list(np.array(items)[rec_idx])
    rel = {u: [1 if e in ur[u] else 0 for e in p] for u, p in preds.items()}
    return dict(
        precision=float(np.mean([M.precision_at_k(r, topk) for r in rel.values()])),
        recall=float(np.mean([M.recall_at_k(r, len(ur[u]), topk) for u, r in rel.items()])),
        map=float(M.map_at_k(list(rel.values()))),
        ndcg=float(np.mean([M.ndcg_at_k(r, topk) for r in rel.values()])),
        hr=float(M.hr_at_k(list(rel.values()), list(rel.keys()), ur)),
        mrr=float(M.mrr_at_k(list(rel.values()))))


def make_f5(torch, R, D, M, split, seeds, epochs):
    train, test_data, U, I, train_mat, ur, val = split
    d, B, lr, wd, num_ng = 32, 4096, 0.01, 0.001, 4
    runs = []
    for s in seeds:
        t0 = time.time()
        _seed_all(torch, 1000 + s)
        ds = D.BPRData(train, I, train_mat, num_ng, True)
        gen = torch.Generator().manual_seed(1000 + s)
        loader = torch.utils.data.DataLoader(ds, batch_size=B, shuffle=True, num_workers=0, generator=gen)
        model = R.BPR(U, I, d)
        opt = torch.optim.SGD(model.parameters(), lr=lr, weight_decay=wd)
        for _ in range(epochs):
            model.train()
            loader.dataset.ng_sample()
            for u, i, j in loader:
                _ref_step(torch, model, opt, u, i, j)
        model.eval()
        kpi = _kpi(torch, M, model, test_data, ur)
        kpi["seed"] = 1000 + s
        kpi["seconds"] = time.time() - t0
        runs.append(kpi)
        print("F5 run", kpi)
    keys = ["precision", "recall", "map", "ndcg", "hr", "mrr"]
    summary = {k: dict(mean=float(np.mean([r[k] for r in runs])), std=float(np.std([r[k] for r in runs], ddof=1)))
               for k in keys}
    test_arr = np.asarray(test_data, dtype=np.int16)
    gt_u = np.array(sorted(ur.keys()), dtype=np.int16)
    gt_ptr = np.cumsum([0] + [len(ur[u]) for u in sorted(ur.keys())]).astype(np.int32)
    gt_items = np.array([x for u in sorted(ur.keys()) for x in sorted(ur[u])], dtype=np.int16)
    np.savez_compressed(os.path.join(OUT, "hr_ndcg_ml100k.npz"), test_data=test_arr,
                        gt_users=gt_u, gt_ptr=gt_ptr, gt_items=gt_items, U=U, I=I,
                        positives=np.asarray(train, dtype=np.int16))
    with open(os.path.join(OUT, "hr_ndcg_ml100k.json"), "w") as f:
        json.dump(dict(protocol=dict(dataset="ml-100k", data_split="fo", by_time=1, val_method="tfo",
                                     factor_num=d, batch_size=B, lr=lr, wd=wd, num_ng=num_ng,
                                     epochs=epochs, topk=10, split_seed=2024),
                       runs=runs, summary=summary), f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip F5 (the 20-epoch runs)")
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch, R, D, M = _import_reference()
    torch.set_num_threads(8)
    only = set(a.only.split(",")) if a.only else {"f1", "f2", "f4", "f5"}
    if "f1" in only:
        make_f1(torch, R)
    if "f4" in only:
        make_f4(torch, R, M)
    if only & {"f2", "f5"}:
        split = _load_split(torch, D, 2024)
        if "f2" in only:
            make_f2_f3(torch, R, D, split)
        if "f5" in only and not a.quick:
            make_f5(torch, R, D, M, split, range(a.seeds), a.epochs)


if __name__ == "__main__":
    main()
