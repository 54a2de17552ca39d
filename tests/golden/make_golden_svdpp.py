"""Generate the SVDpp fixtures by RUNNING the reference's own Cython module
(util/matrix_factorization.pyx SVDpp, :169-287), built from /root/reference by
oracle/build_ref_mf.py into oracle/_ref/ (build container only).

Data: slices of the reference's data/ml-100k/u.data with dense codes (util/data_loader.py:447-448),
plus one case with a repeated (user, item) row, so a user's item list holds an item twice.
fit() is preceded by np.random.seed(seed); the initial tables are recovered by re-seeding and
drawing as fit() does (pu, qi, yj: :218-221).

svdpp_cases.npz, per case c (prefix c_): u, i, r, U, I, k, epochs, global_mean, lr [5], reg [5]
(bu, bi, pu, qi, yj), P0, Q0, Y0, and after fit: P, Q, Y, bu, bi, pairs [m, 2] and pred (the
reference's predict on them).
Run:  python oracle/build_ref_mf.py && python tests/golden/make_golden_svdpp.py
"""
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_mf import _ratings, _ref  # noqa: E402


def main():
    mf = _ref()
    out = {}
    cases = [
        # name, rows, kwargs, seed, duplicate row
        ("pp_small", 3000, dict(n_factors=8, n_epochs=2), 21, False),
        ("pp_rates", 4000, dict(n_factors=20, n_epochs=2, lr_bu=0.01, lr_bi=0.002, lr_pu=0.007,
                                lr_qi=0.003, lr_yj=0.005, reg_bu=0.1, reg_bi=0.05, reg_pu=0.03,
                                reg_qi=0.01, reg_yj=0.04), 22, False),
        ("pp_dup", 1500, dict(n_factors=6, n_epochs=3, lr_all=0.01), 23, True),
    ]
    for name, rows, kw, seed, dup in cases:
        df = _ratings(rows)
        if dup:  # the user of row 10 rates its item again
            df = df._append(df.iloc[10], ignore_index=True).astype(df.dtypes.to_dict())
        U, I = int(df.user.max()) + 1, int(df.item.max()) + 1
        m = mf.SVDpp(U, I, verbose=False, **kw)
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            m.fit(df)
        np.random.seed(seed)
        k = kw["n_factors"]
        P0 = np.random.normal(0, .1, size=(U, k))
        Q0 = np.random.normal(0, .1, size=(I, k))
        Y0 = np.random.normal(0, .1, size=(I, k))
        g = np.random.default_rng(seed)
        pairs = np.stack([g.integers(0, U, 50), g.integers(0, I, 50)], 1)
        pred = np.array([m.predict(int(a), int(b)) for a, b in pairs])
        c = dict(u=df.user.values.astype(np.int32), i=df.item.values.astype(np.int32),
                 r=df.rating.values.astype(np.float64), U=U, I=I, k=k, epochs=kw["n_epochs"],
                 global_mean=m.global_mean,
                 lr=np.array([m.lr_bu, m.lr_bi, m.lr_pu, m.lr_qi, m.lr_yj]),
                 reg=np.array([m.reg_bu, m.reg_bi, m.reg_pu, m.reg_qi, m.reg_yj]),
                 P0=P0, Q0=Q0, Y0=Y0, P=m.pu, Q=m.qi, Y=m.yj, bu=m.bu, bi=m.bi, pairs=pairs,
                 pred=pred, seed=seed)
        for key, v in c.items():
            out[f"{name}_{key}"] = np.asarray(v)
        print(name, U, I, len(df), file=sys.stderr)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "svdpp_cases.npz"), **out)


if __name__ == "__main__":
    main()
