"""Generate the ingestion golden fixture by IMPORTING the reference
(read-only) in the build container.  Test infrastructure only: never run on the GPU box; only its
output travels.

Input: a slice of the reference's data/ml-100k/u.data (raw user id <= 300, users with more than
I - 999 ratings dropped so that `_negative_sampling`'s random.sample(.., 999) can succeed), written
into a scratch ./data tree three ways -- ml-100k u.data ('\\t'), ml-1m ratings.dat ('::', the
rating >= 4 filter) and ml-20m ratings.csv (header, half-star ratings) -- and then read by the
reference's own `util.data_loader.load_rate` / `load_mat` with cwd at the scratch tree and
`random` / `np.random` seeded (and KFold given the old-sklearn reading of its arguments, below).

Fixture written next to this file, ingest_ml100k_slice.npz:
  raw                      the slice (user, item, rating, timestamp) in file order
  rate_<src>_<prepro>_rows load_rate's output rows as indices into `raw` (its rating and timestamp
                           columns are checked here against those rows)
  loo_cv_*                 load_mat('ml-100k', data_split='loo', by_time=1, val_method='cv'):
                           user_num, item_num, the 5 val folds (concatenated + lengths; fold f's
                           train list is checked here to be the other folds in order), the
                           train list lengths, each fold's train_mat nnz, the test_data length and
                           its ground-truth rows (the random negatives are checked by property)
  (val_method 'tloo' / 'loo' are absent: load_mat raises IndexError there, :538-543 iterate the
  DataFrame those branches return, so the reference has no output to pin them with)
  fo_tfo_*, fo_cv_*        data_split='fo' (time order with shuffled ties: compared by property)
Run:  python tests/golden/make_golden_ingest.py
"""
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.dont_write_bytecode = True
    raw = np.loadtxt(os.path.join(REF, "data/ml-100k/u.data"), dtype=np.int64)
    raw = raw[raw[:, 0] <= 300]
    items = len(np.unique(raw[:, 1]))
    users, cnt = np.unique(raw[:, 0], return_counts=True)
    raw = raw[~np.isin(raw[:, 0], users[cnt > items - 1000])]
    out = {"raw": raw.astype(np.int64)}
    half = (raw[:, 3] % 2 == 1) & (raw[:, 2] < 5)  # half-star ratings for the csv form
    with tempfile.TemporaryDirectory() as tmp:
        for d in ("ml-100k", "ml-1m", "ml-20m"):
            os.makedirs(os.path.join(tmp, "data", d))
        with open(os.path.join(tmp, "data/ml-100k/u.data"), "w") as f:
            for u, i, r, t in raw:
                f.write(f"{u}\t{i}\t{r}\t{t}\n")
        with open(os.path.join(tmp, "data/ml-1m/ratings.dat"), "w") as f:
            for u, i, r, t in raw:
                f.write(f"{u}::{i}::{r}::{t}\n")
        with open(os.path.join(tmp, "data/ml-20m/ratings.csv"), "w") as f:
            f.write("userId,movieId,rating,timestamp\n")
            for (u, i, r, t), h in zip(raw, half):
                f.write(f"{u},{i},{r + 0.5 if h else float(r)},{t}\n")
        cwd = os.getcwd()
        os.chdir(tmp)
        sys.path.insert(0, REF)
        try:
            import util.data_loader as D
            from sklearn.model_selection import KFold

            # sklearn < 0.24 (the reference's era) ignored random_state when shuffle=False; the
            # installed one raises on load_mat's KFold(.., shuffle=False, random_state=2019) call
            D.KFold = lambda n_splits, shuffle=False, random_state=None: KFold(n_splits=n_splits, shuffle=shuffle)
            pos = {(u, i): r for r, (u, i) in enumerate(raw[:, :2].tolist())}  # (user, item) unique
            for src, pre in (("ml-100k", "origin"), ("ml-100k", "5core"), ("ml-100k", "10core"),
                             ("ml-1m", "origin"), ("ml-20m", "origin")):
                df = D.load_rate(src, pre)
                rows = np.array([pos[(u, i)] for u, i in zip(df["user"], df["item"])], np.int32)
                assert np.array_equal(df["timestamp"].to_numpy(), raw[rows, 3])
                want = raw[rows, 2] + np.where(half[rows], 0.5, 0.0) if src == "ml-20m" else raw[rows, 2]
                assert np.array_equal(df["rating"].to_numpy(np.float64), want)
                out[f"rate_{src}_{pre}_rows"] = rows  # load_rate's rows as indices into `raw`
            for split, val in (("loo", "cv"), ("fo", "tfo"), ("fo", "cv")):
                random.seed(7)
                np.random.seed(7)
                tr, test, U, I, mats, ur, va = D.load_mat("ml-100k", data_split=split, by_time=1,
                                                          val_method=val, fold_num=5)
                k = f"{split}_{val}_"
                out[k + "shape"] = np.array([U, I])
                tr = [np.asarray(f.values if hasattr(f, "values") else f, np.int64).reshape(-1, 2) for f in tr]
                va = [np.asarray(f.values if hasattr(f, "values") else f, np.int64).reshape(-1, 2) for f in va]
                if val == "cv":  # fold f's train list is the other folds' val lists, in order
                    for f in range(len(tr)):
                        assert np.array_equal(tr[f], np.concatenate(va[:f] + va[f + 1:]))
                else:
                    out[k + "train"] = np.concatenate(tr).astype(np.int32)
                out[k + "train_len"] = np.array([len(f) for f in tr])
                out[k + "val"] = np.concatenate(va).astype(np.int32)
                out[k + "val_len"] = np.array([len(f) for f in va])
                out[k + "mat_nnz"] = np.array([m.nnz for m in mats])
                test = np.asarray(test, np.int64).reshape(-1, 2)
                out[k + "test_len"] = np.array(len(test))
                if split == "loo":  # [gt, 999 random negatives] per user: keep the gt rows
                    out[k + "test_gt"] = test[::1000].astype(np.int32)
                elif val == "tfo":  # random candidates: keep the ground truth sets
                    gu = sorted(ur)
                    out[k + "ur_user"] = np.array(gu, np.int64)
                    out[k + "ur_len"] = np.array([len(ur[u]) for u in gu])
                    out[k + "ur_item"] = np.array([i for u in gu for i in sorted(ur[u])], np.int32)
                    out[k + "test_users"] = np.array(list(dict.fromkeys(test[:, 0].tolist())), np.int32)
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(OUT, "ingest_ml100k_slice.npz"), **out)
    print({k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
