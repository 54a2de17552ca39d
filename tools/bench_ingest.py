"""Ingestion throughput: a synthetic ml-20m-shaped ratings.csv (138,493
users, 26,744 items, 20,000,263 rows, half-star ratings, lognormal user degree / Zipf items) read
by the native path (libbprmf_amd.so bprmf_dataset_*, host C++) and, when /root/reference is
present (the build container only), by the reference's own util.data_loader.load_rate plus the
coding step of load_mat (pandas), on the same file.

    python tools/bench_ingest.py [--rows N] [--threads T] [--no-reference]
Prints one JSON line.  Host-only: no GPU is used.
"""
import argparse
import importlib
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference"


def make_csv(path, rows, users=138493, items=26744, seed=0):
    g = np.random.default_rng(seed)
    deg = g.lognormal(0.0, 1.0, users)
    deg = np.maximum(1, np.round(deg / deg.sum() * rows)).astype(np.int64)
    deg[np.argmax(deg)] += rows - deg.sum()
    u = np.repeat(np.arange(1, users + 1), deg)
    zipf = 1.0 / np.arange(1, items + 1) ** 0.8
    it = g.choice(items, size=rows, p=zipf / zipf.sum()) + 1
    r = g.integers(1, 11, rows) / 2.0
    t = g.integers(789652009, 1427784002, rows)
    with open(path, "w") as f:
        f.write("userId,movieId,rating,timestamp\n")
        step = 1 << 20
        for s in range(0, rows, step):
            e = min(rows, s + step)
            f.write("".join(f"{a},{b},{c},{d}\n" for a, b, c, d in
                            zip(u[s:e].tolist(), it[s:e].tolist(), r[s:e].tolist(), t[s:e].tolist())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_263)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    rl = importlib.import_module("recommend-lib_amd")
    tmp = tempfile.mkdtemp(dir="/tmp")
    d = os.path.join(tmp, "data", "ml-20m")
    os.makedirs(d)
    path = os.path.join(d, "ratings.csv")
    t0 = time.perf_counter()
    make_csv(path, a.rows)
    gen_s = time.perf_counter() - t0
    size = os.path.getsize(path)
    out = {"metric": "ratings ingested/s (ml-20m-shaped ratings.csv, rating >= 4)", "rows": a.rows,
           "bytes": size, "gen_s": round(gen_s, 1)}
    # native: parse + filter + sort + code, then the fo split and the test lists
    t0 = time.perf_counter()
    r = rl.ingest.read_ratings(path, 4.0, "origin", a.threads)
    t_cold = time.perf_counter() - t0  # the process's first large allocations fault their pages in
    r.close()
    t0 = time.perf_counter()
    r = rl.ingest.read_ratings(path, 4.0, "origin", a.threads)
    t_load = time.perf_counter() - t0
    t0 = time.perf_counter()
    is_test = r.split(rl.ingest.FO, 0.2)
    t_split = time.perf_counter() - t0
    t0 = time.perf_counter()
    tu, _ = r.candidates(is_test, rl.ingest.FO, 1000, 0)
    t_cand = time.perf_counter() - t0
    out["native"] = {"load_s": round(t_load, 3), "load_first_call_s": round(t_cold, 3), "rows_kept": r.n, "users": r.user_num,
                     "items": r.item_num, "rows_per_s": round(a.rows / t_load),
                     "GB_per_s": round(size / t_load / 1e9, 3), "fo_split_s": round(t_split, 3),
                     "test_lists_s": round(t_cand, 3), "test_rows": int(len(tu)),
                     "threads": a.threads or os.cpu_count()}
    r.close()
    # the whole load_mat (fo split, tfo validation) into arrays + CSR train_mat, and into the
    # reference's types (Python lists, dok_matrix)
    for kind, kw in (("arrays_csr", dict(as_lists=False, train_mat="csr")), ("lists_dok", {})):
        t0 = time.perf_counter()
        rl.load_mat(data_split="fo", val_method="tfo", path=path, min_rating=4.0,
                    threads=a.threads, **kw)
        out["native"][f"load_mat_fo_tfo_{kind}_s"] = round(time.perf_counter() - t0, 3)
    if not a.no_reference and os.path.isdir(REF):
        import pandas as pd
        cwd = os.getcwd()
        os.chdir(tmp)
        sys.path.insert(0, REF)
        try:
            import util.data_loader as D
            t0 = time.perf_counter()
            df = D.load_rate("ml-20m")
            t_ref = time.perf_counter() - t0
            t0 = time.perf_counter()
            df["user"] = pd.Categorical(df.user).codes
            df["item"] = pd.Categorical(df.item).codes
            t_codes = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
        out["reference"] = {"load_rate_s": round(t_ref, 3), "codes_s": round(t_codes, 3),
                            "rows_kept": len(df), "rows_per_s": round(a.rows / (t_ref + t_codes)),
                            "cores": 1, "note": "util/data_loader.py:41-43,118 + :447-448 (pandas)"}
        out["speedup_load"] = round((t_ref + t_codes) / t_load, 1)
    os.remove(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
