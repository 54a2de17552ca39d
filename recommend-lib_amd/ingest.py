"""Ratings ingestion — drop-in for util/data_loader.py:load_rate (:27-146) and load_mat (:444-548)
on the MovieLens sources.

Parsing, the rating filter, the k-core filter, the (user, item, timestamp) ordering, the dense id
codes, the loo / fo test splits and the test candidate lists run in libbprmf_amd.so
(include/bprmf.h `bprmf_dataset_*`, host C++ on all cores); this module only slices the arrays it
returns into the reference's output shapes.

Differences from the reference, all where it draws from an unseeded RNG or fails:
  * fo (by_time=1) and tfo / tloo: the reference shuffles before an unstable time sort, so rows
    with equal timestamps land in random order; here they keep (user, item) row order;
  * test candidates (loo's 999 negatives, fo's fill-up to test_num) are drawn from a seeded
    per-user stream and listed ascending (loo: ground truth first);
  * load_mat's loo `ur` holds each user's test item (the reference stores `int(str[1])`, the first
    character of the user id, data_loader.py:467);
  * val_method 'tloo' / 'loo' return [user, item] lists like 'tfo' (the reference builds the
    train_mat from a DataFrame there and raises IndexError, :538-543);
  * by_time=0 splits are not provided (they are unseeded random splits in the reference).
"""
import ctypes
import math
import os
from collections import defaultdict

import numpy as np

from . import _lib

# load_rate's file and rating filter per source (data_loader.py:28-43)
SOURCES = {
    "ml-100k": ("u.data", 0.0),
    "ml-1m": ("ratings.dat", 4.0),
    "ml-10m": ("ratings.dat", 4.0),
    "ml-20m": ("ratings.csv", 4.0),
}
PREPRO = {"origin": 0, "5core": 5, "10core": 10}
LOO, FO = 0, 1  # BPRMF_SPLIT_LOO_TIME / BPRMF_SPLIT_FO_TIME


class Ratings:
    """One parsed ratings file (a bprmf_dataset): rows ordered by (user, item, timestamp), ids
    coded densely; `user_ids[code]` / `item_ids[code]` are the raw ids."""

    def __init__(self, path, min_rating=0.0, core=0, threads=0):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self._L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._L.bprmf_dataset_load(os.fsencode(path), float(min_rating), int(core),
                                              int(threads), ctypes.byref(h)))
        self._h = h
        n, U, I = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.bprmf_dataset_info(h, ctypes.byref(n), ctypes.byref(U), ctypes.byref(I)))
        self.n, self.user_num, self.item_num = n.value, U.value, I.value
        self.users = np.empty(self.n, np.int32)
        self.items = np.empty(self.n, np.int32)
        self.ratings = np.empty(self.n, np.float32)
        self.timestamps = np.empty(self.n, np.int64)
        self.user_ids = np.empty(self.user_num, np.int64)
        self.item_ids = np.empty(self.item_num, np.int64)
        _lib.check(self._L.bprmf_dataset_copy(h, _lib.ptr(self.users), _lib.ptr(self.items),
                                              _lib.ptr(self.ratings), _lib.ptr(self.timestamps),
                                              _lib.ptr(self.user_ids), _lib.ptr(self.item_ids)))

    def close(self):
        if getattr(self, "_h", None):
            self._L.bprmf_dataset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.n

    def split(self, method, test_frac=0.2):
        """Boolean is_test per row (LOO: each user's latest row; FO: the last test_frac in time)."""
        m = np.zeros(self.n, np.uint8)
        _lib.check(self._L.bprmf_dataset_split(self._h, int(method), float(test_frac), _lib.ptr(m)))
        return m.view(bool)

    def candidates(self, is_test, method, count, seed=0):
        """Test lists as (users, items) rows (bprmf_dataset_candidates)."""
        t = np.ascontiguousarray(np.asarray(is_test, dtype=bool)).view(np.uint8)
        if len(t) != self.n:
            raise ValueError("is_test must have one entry per row")
        n = ctypes.c_int64(0)
        _lib.check(self._L.bprmf_dataset_candidates(self._h, _lib.ptr(t), int(method), int(count),
                                                    int(seed) & (2**64 - 1), ctypes.byref(n), None,
                                                    None))
        u, i = np.empty(n.value, np.int32), np.empty(n.value, np.int32)
        _lib.check(self._L.bprmf_dataset_candidates(self._h, _lib.ptr(t), int(method), int(count),
                                                    int(seed) & (2**64 - 1), ctypes.byref(n),
                                                    _lib.ptr(u), _lib.ptr(i)))
        return u, i

    def frame(self, raw_ids=True):
        """The rows as a DataFrame(user, item, rating, timestamp) (load_rate's return value)."""
        import pandas as pd
        u = self.user_ids[self.users] if raw_ids else self.users
        i = self.item_ids[self.items] if raw_ids else self.items
        return pd.DataFrame({"user": u, "item": i, "rating": self.ratings, "timestamp": self.timestamps})


def read_ratings(path, min_rating=0.0, prepro="origin", threads=0):
    return Ratings(path, min_rating, PREPRO[prepro] if isinstance(prepro, str) else int(prepro), threads)


def _source_path(src, data_dir):
    if src not in SOURCES:
        raise ValueError("Invalid Dataset Error")
    return os.path.join(data_dir, src, SOURCES[src][0]), SOURCES[src][1]


def load_rate(src="ml-100k", prepro="origin", data_dir="./data", threads=0):
    """DataFrame(user, item, rating, timestamp) with raw ids, ordered by (user, item, timestamp)."""
    if prepro not in PREPRO:
        raise ValueError("Invalid dataset preprocess type, origin/5core/10core expected")
    path, min_rating = _source_path(src, data_dir)
    r = read_ratings(path, min_rating, prepro, threads)
    try:
        return r.frame()
    finally:
        r.close()


def kfold(n, fold_num):
    """sklearn KFold(n_splits=fold_num, shuffle=False) fold bounds: contiguous, the first
    n % fold_num folds one longer."""
    sizes = np.full(fold_num, n // fold_num, np.int64)
    sizes[: n % fold_num] += 1
    return np.concatenate([[0], np.cumsum(sizes)])


def _latest_first(users, ts, order):
    """Rows (indices into users/ts, in `order`) ranked 1 by rank(method='first',
    ascending=False) of the timestamp within each user: the first latest row in that order."""
    u = users[order]
    t = ts[order]
    # within each user, the first position holding the maximum timestamp
    o2 = np.lexsort((np.arange(len(order)), -t, u))
    head = np.ones(len(o2), bool)
    head[1:] = u[o2[1:]] != u[o2[:-1]]
    pick = np.zeros(len(order), bool)
    pick[o2[head]] = True
    return pick


class TrainMat:
    """The train positives as CSR (what BPRData / BPRMF.set_train read); `todok()` gives the
    reference's scipy dok_matrix((user_num, item_num), float32)."""

    def __init__(self, users, items, shape):
        import scipy.sparse as sp
        self.shape = tuple(int(x) for x in shape)
        m = sp.csr_matrix((np.ones(len(users), np.float32), (np.asarray(users), np.asarray(items))),
                          shape=self.shape)
        m.sum_duplicates()
        m.data[:] = 1.0
        self._csr = m
        self.nnz = m.nnz

    def tocsr(self):
        return self._csr

    def tocoo(self):
        return self._csr.tocoo()

    def todok(self):
        return self._csr.todok()

    def keys(self):
        c = self._csr.tocoo()
        return list(zip(c.row.tolist(), c.col.tolist()))

    def __contains__(self, key):
        u, i = key
        return self._csr[u, i] != 0

    def __getitem__(self, key):
        return self._csr[key]


def load_mat(src="ml-100k", test_num=1000, data_split="loo", by_time=1, val_method="cv",
             fold_num=5, prepro="origin", data_dir="./data", seed=0, threads=0, as_lists=True,
             train_mat="dok", path=None, min_rating=None):
    """-> (train_data_list, test_data, user_num, item_num, train_mat_list, ur, val_data_list)
    (data_loader.py:444-548).  `path` / `min_rating` read any file in the supported format
    instead of data_dir/src.  as_lists=False gives [n, 2] arrays (int64 train / val, int32 test)
    instead of Python lists;
    train_mat='csr' gives TrainMat objects instead of dok matrices."""
    if not by_time:
        raise ValueError("by_time=0 (unseeded random splits) is not provided; use by_time=1")
    if data_split not in ("loo", "fo"):
        raise ValueError("Invalid data_split value, expect: loo, fo")
    if val_method not in ("cv", "tloo", "loo", "tfo"):
        raise ValueError("Invalid val_method value, expect: cv, loo, tloo, tfo")
    if path is None:
        path, mr = _source_path(src, data_dir)
    else:
        mr = 0.0
    r = read_ratings(path, mr if min_rating is None else min_rating, prepro, threads)
    try:
        U, I = r.user_num, r.item_num
        users, items, ts = r.users, r.items, r.timestamps
        if data_split == "loo":
            is_test = r.split(LOO)
            train_rows = np.flatnonzero(~is_test)  # row order (user, item, timestamp)
            tu, ti = r.candidates(is_test, LOO, 999, seed)
            ur = defaultdict(set)
            for u, i in zip(users[is_test].tolist(), items[is_test].tolist()):
                ur[u].add(i)
        else:
            is_test = r.split(FO, 0.2)
            order = np.argsort(ts, kind="stable")  # time order, ties in row order
            train_rows = order[~is_test[order]]
            tu, ti = r.candidates(is_test, FO, test_num, seed)
            ur = defaultdict(set)
            for u, i in zip(users[is_test].tolist(), items[is_test].tolist()):
                ur[u].add(i)
    finally:
        r.close()
    train = np.stack([users[train_rows], items[train_rows]], 1).astype(np.int64)
    train_ts = ts[train_rows]
    folds_tr, folds_va = [], []
    if val_method == "cv":
        b = kfold(len(train), fold_num)
        for f in range(fold_num):
            folds_va.append(train[b[f]:b[f + 1]])
            folds_tr.append(np.concatenate([train[: b[f]], train[b[f + 1]:]]))
    elif val_method in ("tfo", "tloo"):
        o = np.argsort(train_ts, kind="stable")
        t = train[o]
        if val_method == "tfo":
            k = int(math.ceil(len(t) * 0.9))
            folds_tr.append(t[:k])
            folds_va.append(t[k:])
        else:
            pick = _latest_first(t[:, 0], train_ts[o], np.arange(len(t)))
            folds_tr.append(t[~pick])
            folds_va.append(t[pick])
    else:  # 'loo': one seeded random train row per user for validation
        g = np.random.default_rng(seed)
        key = g.random(len(train))
        pick = _latest_first(train[:, 0], key, np.arange(len(train)))
        folds_tr.append(train[~pick])
        folds_va.append(train[pick][np.argsort(train[pick][:, 0], kind="stable")])
    mats = []
    for f in folds_tr:
        m = TrainMat(f[:, 0], f[:, 1], (U, I))
        mats.append(m.todok() if train_mat == "dok" else m)
    test = np.stack([tu, ti], 1)
    if as_lists:
        folds_tr = [f.tolist() for f in folds_tr]
        folds_va = [f.tolist() for f in folds_va]
        test = test.tolist()
    return folds_tr, test, U, I, mats, ur, folds_va


def write_ncf_files(out_dir, name, src_path, min_rating=0.0, seed=0, threads=0):
    """The `.train.rating` / `.test.rating` / `.test.negative` files of data_loader.py:1191-1220:
    the loo split by time of a ratings file (coded ids), and per user "(user,gt)" followed by its
    999 negatives, tab-separated."""
    r = read_ratings(src_path, min_rating, "origin", threads)
    try:
        is_test = r.split(LOO)
        tu, ti = r.candidates(is_test, LOO, 999, seed)
        rows = np.arange(r.n)
        os.makedirs(out_dir, exist_ok=True)

        def fmt(v):  # integral ratings print as integers, like the reference's int64 rows
            return str(int(v)) if float(v).is_integer() else repr(float(v))

        for suffix, sel in ((".train.rating", ~is_test), (".test.rating", is_test)):
            with open(os.path.join(out_dir, name + suffix), "w") as f:
                for k in rows[sel]:
                    f.write("\t".join((str(r.users[k]), str(r.items[k]), fmt(r.ratings[k]),
                                       str(r.timestamps[k]))) + "\n")
        with open(os.path.join(out_dir, name + ".test.negative"), "w") as f:
            for s in range(0, len(tu), 1000):
                negs = "\t".join(str(x) for x in ti[s + 1: s + 1000])
                f.write(f"({tu[s]},{ti[s]})\t{negs}\n")
    finally:
        r.close()
