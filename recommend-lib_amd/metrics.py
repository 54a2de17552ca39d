"""Top-K evaluation of the BPR-MF path (drop-in for util/metrics.py, BPR parts).

`metric_eval` / `_bpr_topk` keep the reference batch protocol (util/metrics.py:46-66,88-94):
each loader batch is one user's [ground truth, negatives...]; the ground truth is item_i[0].
`evaluate_topk` is the final KPI of BPRMFRecommender.py:196-229 with every candidate scored AND
ranked on the GPU in one launch (bprmf_topk_lists) instead of one scalar forward per candidate
(the reference's 43 s loop); `metric_eval` ranks all loader batches in one launch the same way.
The scalar metric functions restate util/metrics.py:99-195 (NumPy-2 safe: no np.asfarray).
"""
from collections import defaultdict

import numpy as np


def _hit(gt_item, pred_items):
    return 1 if gt_item in pred_items else 0


def _ndcg(gt_item, pred_items):
    if gt_item in pred_items:
        return float(np.reciprocal(np.log2(pred_items.index(gt_item) + 2)))
    return 0


def _bpr_topk(model, test_loader, top_k):
    import torch
    if hasattr(model, "topk_lists"):  # every batch ranked on the device in one launch
        users, lists = [], []
        for user, item_i, _ in test_loader:
            users.append(int(torch.as_tensor(user).reshape(-1)[0]))
            lists.append(torch.as_tensor(item_i).reshape(-1).cpu().numpy())
        if not users:
            return np.mean([]), np.mean([])
        pos, _ = model.topk_lists(users, lists, top_k)
        HR, NDCG = [], []
        for l, p in zip(lists, pos):
            recommends = l[p[p >= 0]].tolist()
            HR.append(_hit(int(l[0]), recommends))
            NDCG.append(_ndcg(int(l[0]), recommends))
        return np.mean(HR), np.mean(NDCG)
    HR, NDCG = [], []
    for user, item_i, item_j in test_loader:
        prediction_i, _ = model(user, item_i, item_j)
        _, indices = torch.topk(prediction_i.cpu(), top_k)
        recommends = torch.take(torch.as_tensor(item_i).cpu(), indices).numpy().tolist()
        gt_item = int(torch.as_tensor(item_i)[0])
        HR.append(_hit(gt_item, recommends))
        NDCG.append(_ndcg(gt_item, recommends))
    return np.mean(HR), np.mean(NDCG)


def _ncf_topk(model, test_loader, top_k):
    """util/metrics.py:68-86: each batch is one user's [ground truth, negatives] with labels;
    model(user, item) scores them (NCF.forward, on the device)."""
    import torch
    HR, NDCG = [], []
    for user, item, _ in test_loader:  # _ is the label
        predictions = torch.as_tensor(model(user, item)).reshape(-1).cpu()
        _, indices = torch.topk(predictions, top_k)
        recommends = torch.take(torch.as_tensor(item).cpu(), indices).numpy().tolist()
        gt_item = int(torch.as_tensor(item).reshape(-1)[0])
        HR.append(_hit(gt_item, recommends))
        NDCG.append(_ndcg(gt_item, recommends))
    return np.mean(HR), np.mean(NDCG)


def metric_eval(model, test_loader, top_k, algo="bpr"):
    """util/metrics.py:88-97 (algo 'bpr' or 'ncf')."""
    if algo == "bpr":
        return _bpr_topk(model, test_loader, top_k)
    if algo == "ncf":
        return _ncf_topk(model, test_loader, top_k)
    raise ValueError(f"unknown algo {algo!r}")


def precision_at_k(r, k):
    assert k >= 1
    r = np.asarray(r)[:k] != 0
    if r.size != k:
        raise ValueError("Relevance score length < k")
    return sum(r) / len(r)


def recall_at_k(r, groud_truth_len, k):
    if groud_truth_len == 0:
        return 0
    assert k >= 1
    r = np.asarray(r)[:k] != 0
    if r.size != k:
        raise ValueError("Relevance score length < k")
    return sum(r) / groud_truth_len


def mrr_at_k(rs):
    res = 0
    for r in rs:
        for index, item in enumerate(r):
            if item == 1:
                res += 1 / (index + 1)
    return res / len(rs)


def average_precision(r):
    r = np.asarray(r) != 0
    out = [precision_at_k(r, k + 1) for k in range(r.size) if r[k]]
    if not out:
        return 0.
    return np.sum(out) / len(r)


def map_at_k(rs):
    return np.mean([average_precision(r) for r in rs])


def hr_at_k(rs, us, ur):
    assert len(rs) == len(us)
    nom, denom = 0, 0
    for idx in range(len(rs)):
        nom += np.sum(rs[idx])
        denom += len(ur[us[idx]])
    return nom / denom


def dcg_at_k(r, k):
    r = np.asarray(r, dtype=float)[:k] != 0
    if r.size:
        return np.sum(np.subtract(np.power(2, r), 1) / np.log2(np.arange(2, r.size + 2)))
    return 0.


def ndcg_at_k(r, k):
    idcg = dcg_at_k(sorted(r, reverse=True), k)
    if not idcg:
        return 0.
    return dcg_at_k(r, k) / idcg


def evaluate_topk(model, test_data, test_ur, topk=10):
    """Final KPI of BPRMFRecommender.py:196-229.

    test_data: [[u, i], ...] candidates (load_mat test_data); test_ur: {u: set(gt items)}.
    Candidates are grouped per user exactly as the reference does (a set per user, listed in set
    order), then scored and ranked on the device in one launch with np.argsort(...)[::-1][:k]'s
    order (score descending, ties by the later position).
    Returns dict(precision, recall, map, ndcg, hr, mrr).
    """
    test_u_is = defaultdict(set)
    for ele in test_data:
        test_u_is[int(ele[0])].add(int(ele[1]))
    users = list(test_u_is.keys())
    lists = [list(test_u_is[u]) for u in users]
    preds = {}
    if users:
        pos, _ = model.topk_lists(users, lists, topk)  # scoring + ranking on the device
        for u, l, p in zip(users, lists, pos):
            preds[u] = [1 if e in test_ur[u] else 0 for e in np.array(l)[p[p >= 0]]]
    rel = list(preds.values())
    return dict(
        precision=float(np.mean([precision_at_k(r, topk) for r in rel])),
        recall=float(np.mean([recall_at_k(r, len(test_ur[u]), topk) for u, r in preds.items()])),
        map=float(map_at_k(rel)),
        ndcg=float(np.mean([ndcg_at_k(r, topk) for r in rel])),
        hr=float(hr_at_k(rel, list(preds.keys()), test_ur)),
        mrr=float(mrr_at_k(rel)))
