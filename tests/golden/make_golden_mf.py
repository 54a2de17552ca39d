"""Generate the golden fixtures of the rating-SGD path (util/matrix_factorization.pyx SVD / RSVD)
by RUNNING the reference's own Cython module, built from /root/reference by
oracle/build_ref_mf.py into oracle/_ref/ (build container only; /root/reference never reaches
the GPU box, only the .npz written here does).

Data: data/ml-100k/u.data of the reference (user, item, rating, timestamp; tab separated), ids
mapped to dense codes the way util/data_loader.py:447-448 does (pd.Categorical(...).codes).
Every fit is preceded by np.random.seed(seed); the initial tables are recovered by re-seeding and
drawing exactly as fit() does (SVD: pu then qi, :125-126; RSVD: ui then vj, :37-38).

mf_cases.npz, per case c (prefix c_): u, i, r (the train rows in iterrows order), U, I, k, epochs,
global_mean (train_set.rating.mean()), the hyper-parameters, the initial and final tables.
Run:  python oracle/build_ref_mf.py && python tests/golden/make_golden_mf.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DATA = "/root/reference/data/ml-100k/u.data"


def _ref():
    sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))
    import matrix_factorization as mf  # noqa: E402  (the reference's compiled Cython module)
    return mf


def _ratings(n=None):
    df = pd.read_csv(DATA, sep="\t", header=None, names=["user", "item", "rating", "timestamp"])
    df["user"] = pd.Categorical(df.user).codes
    df["item"] = pd.Categorical(df.item).codes
    df = df[["user", "item", "rating"]]
    if n:
        df = df.iloc[:n].reset_index(drop=True)
    return df.astype({"user": np.int64, "item": np.int64, "rating": np.float64})


def main():
    mf = _ref()
    out = {}
    cases = [
        # name, model, rows, kwargs, seed
        ("svd_biased", "SVD", None, dict(n_factors=16, n_epochs=3), 11),
        ("svd_plain", "SVD", 20000, dict(n_factors=8, n_epochs=2, biased=False, lr_all=0.01), 12),
        ("svd_rates", "SVD", 20000, dict(n_factors=5, n_epochs=2, lr_bu=0.01, lr_bi=0.002,
                                         lr_pu=0.007, lr_qi=0.003, reg_bu=0.1, reg_bi=0.05,
                                         reg_pu=0.03, reg_qi=0.01), 13),
        ("rsvd_v2", "RSVD", 20000, dict(n_factors=12, n_epochs=2, version=2, lr=0.003), 14),
        ("rsvd_v1", "RSVD", 20000, dict(n_factors=6, n_epochs=2, version=1, lr=0.003), 15),
        ("rsvd_quiet", "RSVD", 5000, dict(n_factors=4, n_epochs=2, verbose=False), 16),
    ]
    for name, model, rows, kw, seed in cases:
        df = _ratings(rows)
        U, I = int(df.user.max()) + 1, int(df.item.max()) + 1
        cls = getattr(mf, model)
        m = cls(U, I, **kw)
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            m.fit(df)
        np.random.seed(seed)
        k = m.n_factors
        P0 = np.random.normal(m.init_mean, m.init_std_dev, size=(U, k))
        Q0 = np.random.normal(m.init_mean, m.init_std_dev, size=(I, k))
        c = {"u": df.user.values.astype(np.int32), "i": df.item.values.astype(np.int32),
             "r": df.rating.values.astype(np.float64), "U": U, "I": I, "k": k,
             "epochs": m.n_epochs, "global_mean": float(df.rating.mean()), "P0": P0, "Q0": Q0,
             "model": model, "seed": seed}
        if model == "SVD":
            c.update(biased=int(m.biased), lr=np.array([m.lr_bu, m.lr_bi, m.lr_pu, m.lr_qi]),
                     reg=np.array([m.reg_bu, m.reg_bi, m.reg_pu, m.reg_qi]),
                     P=m.pu, Q=m.qi, bu=m.bu, bi=m.bi, ref_global_mean=m.global_mean)
            c["pred"] = np.array([m.predict(int(a), int(b)) for a, b in zip(df.user[:50], df.item[:50])])
        else:
            c.update(version=m.version, lr=np.array([m.lr]), reg=np.array([m.reg, m.reg2]),
                     verbose=int(m.verbose))
            if hasattr(m, "ui"):
                c.update(P=m.ui, Q=m.vj, bu=m.ci, bi=m.dj)
                c["pred"] = np.array([m.predict(int(a), int(b)) for a, b in zip(df.user[:50], df.item[:50])])
        for key, v in c.items():
            out[f"{name}_{key}"] = np.asarray(v)
        print(name, U, I, k, len(df), file=sys.stderr)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "mf_cases.npz"), **out)


if __name__ == "__main__":
    main()
