"""Upper bound of VERDICT r5 item 2's lever (pre-summing in LDS the contribution rows of items
referenced more than once inside one K1 workgroup), computed from the exact batch structure the
step sees: the oracle sampler's triplets at the ml-20m shape (the bench's synthetic positives),
each batch sorted by (user, slot) as the builder does, K1 workgroups of T consecutive positions.

Counted per step (row = d floats = 512 B at d = 128):
  today    K1 writes one contribution row c*P_u per triplet holding a multi-reference item (both
           sides share it); K2 reads one row per reference to a multi-reference item.
  presum   K1 writes one partial row per (workgroup, multi-reference item) group instead; K2 reads
           one row per such group.
The bound assumes a free in-LDS sum; it only counts the contribution bytes the lever moves.

  python tools/presum_bound.py [--batches 8] [--T 8,16,32]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--T", default="8,16,32")
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--d", type=int, default=128)
    a = ap.parse_args()
    from oracle import bpr_oracle as O
    from oracle import c_oracle as C
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, NPOS, seed = 138493, 26744, 10_000_000, 20261015  # bench.py's workload
    pos = syn.make_positives(U, I, NPOS, seed)
    indptr, indices = O.build_csr(pos[:, 0], pos[:, 1], U)
    B, row = a.B, 4 * a.d
    u, i, j = C.sample(pos[:, 0], pos[:, 1], indptr, indices, I, 4, seed, 0, 0, a.batches * B)
    res = {}
    for T in [int(x) for x in a.T.split(",")]:
        acc = dict(triplets=0, multi_refs=0, contrib_writes=0, presum_groups=0, hot_refs=0,
                   presum_hot_groups=0)
        for b in range(a.batches):
            s = slice(b * B, (b + 1) * B)
            bu, bi, bj = u[s], i[s], j[s]
            order = np.lexsort((np.arange(B), bu))  # user order, stable by slot
            bu, bi, bj = bu[order], bi[order], bj[order]
            items = np.concatenate([bi, bj])
            cnt = np.bincount(items, minlength=I)
            multi_i, multi_j = cnt[bi] > 1, cnt[bj] > 1
            hot = cnt > 16
            acc["triplets"] += B
            acc["multi_refs"] += int(multi_i.sum() + multi_j.sum())
            acc["hot_refs"] += int(hot[bi].sum() + hot[bj].sum())
            acc["contrib_writes"] += int((multi_i | multi_j).sum())
            wg = np.arange(B) // T
            refs_wg = np.concatenate([wg[multi_i], wg[multi_j]])
            refs_it = np.concatenate([bi[multi_i], bj[multi_j]])
            key = refs_wg.astype(np.int64) * I + refs_it
            groups = np.unique(key)
            acc["presum_groups"] += int(groups.size)
            acc["presum_hot_groups"] += int(hot[groups % I].sum())
        n = a.batches
        per = {k: v / n for k, v in acc.items()}
        today = (per["contrib_writes"] + per["multi_refs"]) * row
        presum = 2 * per["presum_groups"] * row
        res[f"T={T}"] = dict(
            per_step={k: round(v, 1) for k, v in per.items()},
            contrib_bytes_today=round(today), contrib_bytes_presum=round(presum),
            k2_reads_saved_bytes=round((per["multi_refs"] - per["presum_groups"]) * row),
            k1_writes_added_bytes=round((per["presum_groups"] - per["contrib_writes"]) * row))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
