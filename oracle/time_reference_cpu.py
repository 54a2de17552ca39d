"""Times the reference's own CPU training paths in the BUILD CONTAINER (8 CPUs, no GPU), by
importing its modules from /root/reference (test infrastructure: /root/reference does not exist on
the GPU box, so these numbers are recorded in profiles/r01_reference_cpu.json and cited in
DESIGN.md next to the device numbers; nothing here runs in a product path).

  python oracle/time_reference_cpu.py > profiles/r01_reference_cpu.json

* BPR-FM: BPRFMRecommender.BPRFM (hidden 64, BatchNorm, dropout 0.5) + Adagrad(0.05), the loop
  body of :223-227 on batches of 4096 triplets over 2,625 features (ml-100k shape).
* Item2Vec: Item2VecRecommender.Item2Vec + SGNS (E 300, 20 negatives, window 5) + Adam, the loop
  body of :283-286 on batches of 4096 examples, vocabulary 1,684 (ml-100k shape).
* SVDpp: the reference's compiled Cython SVDpp.fit (oracle/_ref, built by build_ref_mf.py) on the
  first 3,000 ratings of its data/ml-100k/u.data, and on tools/bench_mf.py's SVDpp workload
  (synthetic ml-100k shape), k = 20, one epoch.
"""
import json
import os
import sys
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def bprfm(steps=10):
    import torch
    from BPRFMRecommender import BPRFM
    torch.manual_seed(0)
    U, I, B = 943, 1682, 4096
    model = BPRFM(U + I, 64, True, [0.5, 0.2])
    opt = torch.optim.Adagrad(model.parameters(), lr=0.05, initial_accumulator_value=1e-8)
    g = np.random.default_rng(0)
    ones = torch.ones(B, 2)
    batches = []
    for _ in range(steps + 2):
        u = torch.from_numpy(g.integers(0, U, B))
        batches.append((torch.stack([u, U + torch.from_numpy(g.integers(0, I, B))], 1),
                        torch.stack([u, U + torch.from_numpy(g.integers(0, I, B))], 1)))
    model.train()

    def one(fi, fj):
        model.zero_grad()
        pi, pj = model(fi, ones, fj, ones)
        loss = -(pi - pj).sigmoid().log().sum()
        loss.backward()
        opt.step()

    for fi, fj in batches[:2]:
        one(fi, fj)
    t0 = time.perf_counter()
    for fi, fj in batches[2:]:
        one(fi, fj)
    dt = time.perf_counter() - t0
    return {"triplets_per_s": round(steps * B / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
            "steps": steps, "batch": B, "threads": torch.get_num_threads()}


def sgns(steps=5):
    import torch
    from Item2VecRecommender import Item2Vec, SGNS
    torch.manual_seed(0)
    V, E, C, n, B = 1684, 300, 10, 20, 4096
    model = Item2Vec(vocab_size=V, embedding_size=E)
    s = SGNS(embedding=model, vocab_size=V, n_negs=n)
    opt = torch.optim.Adam(s.parameters())
    g = np.random.default_rng(0)
    batches = [(torch.from_numpy(g.integers(1, V, B)), torch.from_numpy(g.integers(0, V, (B, C))))
               for _ in range(steps + 1)]

    def one(iw, ow):
        loss = s(iw, ow)
        opt.zero_grad()
        loss.backward()
        opt.step()

    one(*batches[0])
    t0 = time.perf_counter()
    for iw, ow in batches[1:]:
        one(iw, ow)
    dt = time.perf_counter() - t0
    return {"examples_per_s": round(steps * B / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
            "steps": steps, "batch": B, "threads": torch.get_num_threads()}


def svdpp():
    import contextlib
    import io
    sys.path.insert(0, os.path.join(HERE, "_ref"))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests", "golden"))
    import matrix_factorization as mf
    from make_golden_mf import _ratings
    df = _ratings(3000)
    U, I = int(df.user.max()) + 1, int(df.item.max()) + 1
    m = mf.SVDpp(U, I, n_factors=20, n_epochs=1, verbose=False)
    np.random.seed(0)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        m.fit(df)
    dt = time.perf_counter() - t0
    return {"samples_per_s": round(len(df) / dt, 1), "us_per_sample": round(dt / len(df) * 1e6, 1),
            "ratings": len(df), "mean_items_per_user": round(len(df) / df.user.nunique(), 1)}


def svdpp_bench_shape():
    """The reference's Cython SVDpp.fit on tools/bench_mf.py's SVDpp workload (synthetic ml-100k
    shape, one rating per pair), one epoch: the device's number in DESIGN §9 is on this data."""
    import contextlib
    import io
    import pandas as pd
    sys.path.insert(0, os.path.join(HERE, "_ref"))
    import matrix_factorization as mf
    g = np.random.default_rng(7)  # tools/bench_mf.py:ratings('ml-100k') without the data file
    U, I, n = 943, 1682, 100_000
    act = g.lognormal(0.0, 1.0, U)
    u = g.choice(U, n, p=act / act.sum())
    w = 1.0 / np.arange(1, I + 1) ** 0.5
    i = g.permutation(I)[g.choice(I, n, p=w / w.sum())]
    r = g.integers(1, 6, n).astype(np.float64)
    _, keep = np.unique(u.astype(np.int64) * (int(i.max()) + 1) + i, return_index=True)
    keep.sort()
    df = pd.DataFrame({"user": u[keep], "item": i[keep], "rating": r[keep]})
    m = mf.SVDpp(int(df.user.max()) + 1, int(df.item.max()) + 1, n_factors=20, n_epochs=1,
                 verbose=False)
    np.random.seed(0)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        m.fit(df)
    dt = time.perf_counter() - t0
    return {"samples_per_s": round(len(df) / dt, 1), "us_per_sample": round(dt / len(df) * 1e6, 1),
            "ratings": len(df)}


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    out = {"host": f"build container, {os.cpu_count()} CPUs", "bprfm": bprfm(), "sgns": sgns(),
           "svdpp_cython": svdpp(), "svdpp_cython_bench_shape": svdpp_bench_shape()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
