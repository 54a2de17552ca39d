"""Timing of bprmf_topk_lists (candidate-list ranking, metrics protocol) at the ml-20m shape:
20,000 users x 100 / 1,000 candidates, k = 10; one call includes the host copies.
  python tools/ubench_topk_lists.py   (GPU box)"""
import importlib, sys, time, os
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
rl = importlib.import_module("recommend-lib_amd")
U, I, d = 138493, 26744, 128
m = rl.BPRMF(U, I, d, seed=1)
g = np.random.default_rng(0)
for n_c in (100, 1000):
    users = g.integers(0, U, 20000)
    flat = g.integers(0, I, 20000 * n_c).astype(np.int32)
    offs = np.arange(0, 20000 * n_c + 1, n_c, dtype=np.int64)
    m.topk_lists(users, (offs, flat), 10)
    t = time.perf_counter()
    for _ in range(5):
        m.topk_lists(users, (offs, flat), 10)
    print(f"topk_lists 20000 users x {n_c} candidates, k=10: {(time.perf_counter() - t) / 5 * 1e3:.2f} ms per call (host copies included)")
