"""Ingestion oracle (TEST INFRASTRUCTURE ONLY; nothing in the product imports this).

A numpy restatement of the reference's ratings ingestion, pinned by
tests/golden/ingest_ml100k_slice.npz (made by importing the reference, make_golden_ingest.py):
  load_rate      util/data_loader.py:27-146   rating >= 4 for ml-1m/10m/20m (:35,:39,:43);
                 sort_values(['user', 'item', 'timestamp']) (:118); prepro '5core'/'10core'
                 (:122-144): ONE pass, counts over the unfiltered rows, inner merges keep order
  codes          :447-451                      pd.Categorical(ids).codes = rank among the sorted
                                               unique ids; user_num / item_num = max code + 1
  _split_loo     :410-414 (by_time=1)          rank(method='first', ascending=False) == 1 per user
  _split_fo      :422-427 (by_time=1)          first ceil(0.8 n) rows in time order (the reference
                                               orders equal timestamps randomly; here row order)
  KFold          :496-503 (val 'cv')           contiguous folds, the first n % k one row longer
  tfo            :525-535                      first ceil(0.9 n) train rows in time order
Rows are numpy arrays (user, item, rating, timestamp) of raw ids in file order.
"""
import math

import numpy as np


def load_rate_rows(raw, min_rating=0.0, core=0):
    """Indices into `raw` of load_rate's output rows, in its order."""
    raw = np.asarray(raw)
    keep = np.flatnonzero(raw[:, 2] >= min_rating)
    if core:
        u, i = raw[keep, 0], raw[keep, 1]
        _, ui, cu = np.unique(u, return_inverse=True, return_counts=True)
        _, ii, ci = np.unique(i, return_inverse=True, return_counts=True)
        keep = keep[(cu[ui] >= core) & (ci[ii] >= core)]
    # lexsort is stable: equal (user, item, timestamp) keep file order
    o = np.lexsort((raw[keep, 3], raw[keep, 1], raw[keep, 0]))
    return keep[o]


def codes(ids):
    """pd.Categorical(ids).codes for integer ids and the categories (raw id per code)."""
    cats, inv = np.unique(ids, return_inverse=True)
    return inv.astype(np.int64), cats


def split_loo(users, ts):
    """is_test per row (rows ordered by (user, item, timestamp)): the first row per user holding
    its latest timestamp."""
    n = len(users)
    o = np.lexsort((np.arange(n), -np.asarray(ts), users))
    head = np.ones(n, bool)
    head[1:] = users[o[1:]] != users[o[:-1]]
    t = np.zeros(n, bool)
    t[o[head]] = True
    return t


def split_fo(ts, test_frac=0.2):
    """(is_test per row, the time order): rows past ceil(n (1 - test_frac)) in stable time order."""
    o = np.argsort(ts, kind="stable")
    k = int(math.ceil(len(ts) * (1 - test_frac)))
    t = np.zeros(len(ts), bool)
    t[o[k:]] = True
    return t, o


def kfold_bounds(n, k):
    sizes = np.full(k, n // k, np.int64)
    sizes[: n % k] += 1
    return np.concatenate([[0], np.cumsum(sizes)])


def load_mat(raw, data_split="loo", val_method="cv", fold_num=5, min_rating=0.0, core=0):
    """The deterministic outputs of load_mat(by_time=1): dict(user_num, item_num, train (rows
    [u, i] of the test split's train part, in load_mat's order), folds_tr, folds_va, is_test,
    users, items, ts (coded rows in load_rate order))."""
    rows = load_rate_rows(raw, min_rating, core)
    r = np.asarray(raw)[rows]
    u, _ = codes(r[:, 0])
    i, _ = codes(r[:, 1])
    ts = r[:, 3]
    U, I = int(u.max()) + 1, int(i.max()) + 1
    if data_split == "loo":
        is_test = split_loo(u, ts)
        tr_rows = np.flatnonzero(~is_test)
    else:
        is_test, o = split_fo(ts)
        tr_rows = o[~is_test[o]]
    train = np.stack([u[tr_rows], i[tr_rows]], 1)
    folds_tr, folds_va = [], []
    if val_method == "cv":
        b = kfold_bounds(len(train), fold_num)
        for f in range(fold_num):
            folds_va.append(train[b[f]:b[f + 1]])
            folds_tr.append(np.concatenate([train[: b[f]], train[b[f + 1]:]]))
    elif val_method == "tfo":
        o2 = np.argsort(ts[tr_rows], kind="stable")
        k = int(math.ceil(len(train) * 0.9))
        folds_tr.append(train[o2][:k])
        folds_va.append(train[o2][k:])
    return dict(user_num=U, item_num=I, train=train, folds_tr=folds_tr, folds_va=folds_va,
                is_test=is_test, users=u, items=i, ts=ts)
