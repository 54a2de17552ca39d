"""Exchange volume of the sharded step at the ml-20m shape (DESIGN.md §6 "What 8 GPUs can reach"):
per world size, each rank's distinct items per step, how many are remote, the largest per-owner
request count (the exchange capacity), the union of all ranks' items per step, and the share of a
rank's rows at step k+1 that some rank updated at step k.  CPU only (the oracle's C sampler, each
rank's shard seed, 8 steps of B = 4096).

  python tools/xch_stats.py            # ml-20m shape (C3), then the one-hop schedule
  python tools/xch_stats.py c5         # the C5 shape (100M items, d = 256): drawn directly

C5 (BASELINE configs[4]: 10M users x 100M items, d = 256, 8 GPUs): building the 1.4e8-positive
set and its sampler is not needed for the exchange volume -- a step's positive items follow the
items' popularity (Zipf alpha = 1 over a random order, synthetic.make_positives) and its negatives
are uniform over the catalogue, so each rank's 8 steps are drawn that way (the user side never
crosses a link)."""
import sys, importlib, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import bpr_oracle as O
from oracle import c_oracle as C
syn = importlib.import_module("recommend-lib_amd.synthetic")
U, I, B = 138493, 26744, 4096

if len(sys.argv) > 1 and sys.argv[1] == "c5":
    I5, d5, steps = 100_000_000, 256, 8
    g = np.random.default_rng(5)
    # inverse CDF of Zipf(1) over ranks 1..I5: H(r) ~ ln r + gamma
    gamma = 0.5772156649
    HN = np.log(I5) + gamma
    order_seed = np.random.default_rng(6)
    perm_a, perm_b = int(order_seed.integers(1, I5)) | 1, int(order_seed.integers(0, I5))

    def item_of_rank(r):  # a fixed random order of the catalogue (affine bijection mod I5)
        return (perm_a * r + perm_b) % I5

    for W in (1, 2, 4, 8):
        caps, distinct, remote, union, upd = [], [], [], [], []
        sets = [[None] * steps for _ in range(W)]
        for r in range(W):
            for k in range(steps):
                # B positives (each triplet one; a positive recurs num_ng times per epoch) + B negatives
                rk = np.minimum(np.exp(g.random(B) * HN - gamma), I5 - 1).astype(np.int64)
                i = item_of_rank(rk)
                j = g.integers(0, I5, B)
                it = np.unique(np.concatenate([i, j]))
                sets[r][k] = it
                distinct.append(len(it))
                own = np.bincount(it % W, minlength=W)
                caps.append(own.max())
                remote.append(len(it) - own[r])
        for k in range(steps):
            union.append(len(np.unique(np.concatenate([sets[r][k] for r in range(W)]))))
        for r in range(W):
            for k in range(steps - 1):
                prev = np.unique(np.concatenate([sets[q][k] for q in range(W)]))
                upd.append(np.isin(sets[r][k + 1], prev).mean())
        rb = 4 * d5
        print(f"C5 W={W}: distinct/rank/step {np.mean(distinct):.0f} of {2 * B} refs, remote "
              f"{np.mean(remote):.0f}, max per-owner cap {np.max(caps)}, union/step {np.mean(union):.0f}, "
              f"frac of next-step rows updated last step {np.mean(upd):.3f}, per-link bytes/hop "
              f"(padded cap x {rb} B) {np.max(caps) * rb / 1e3:.0f} KB, all links/rank/hop "
              f"{np.max(caps) * rb * max(W - 1, 0) / 1e6:.2f} MB")
    sys.exit(0)
pos = syn.make_positives(U, I, 10_000_000, 20261015)
for W in (1, 2, 4, 8):
    caps, distinct, remote, union = [], [], [], []
    per_step_sets = []
    for r in range(W):
        mine = pos[pos[:, 0] % W == r]
        indptr, indices = O.build_csr(mine[:, 0], mine[:, 1], U)
        u, i, j = C.sample(mine[:, 0], mine[:, 1], indptr, indices, I, 4,
                           (20261015 + r * 0x9E3779B97F4A7C15) & (2**64 - 1), 0, 0, 8 * B)
        sets = []
        for k in range(8):
            it = np.unique(np.concatenate([i[k*B:(k+1)*B], j[k*B:(k+1)*B]]))
            sets.append(it)
            distinct.append(len(it))
            own = np.bincount(it % W, minlength=W)
            caps.append(own.max())
            remote.append(len(it) - own[r])
        per_step_sets.append(sets)
    for k in range(8):
        union.append(len(np.unique(np.concatenate([per_step_sets[r][k] for r in range(W)]))))
    # rows a rank needs at step k+1 that the union updated at step k
    upd = []
    for r in range(W):
        for k in range(7):
            prev = np.unique(np.concatenate([per_step_sets[q][k] for q in range(W)]))
            upd.append(np.isin(per_step_sets[r][k+1], prev).mean())
    print(f"W={W}: distinct/rank/step {np.mean(distinct):.0f}, remote {np.mean(remote):.0f}, "
          f"max per-owner cap {np.max(caps)}, mean cap {np.mean(caps):.0f}, union/step {np.mean(union):.0f}, "
          f"frac of next-step rows updated last step {np.mean(upd):.3f}, "
          f"per-link bytes/hop (mean remote/(W-1)*512) {np.mean(remote)/max(W-1,1)*512/1e3:.0f} KB, padded cap {np.max(caps)*512/1e3:.0f} KB")


# The one-hop schedule: gradients of step k go straight from each producer rank to
# every rank that reads the item at step k+1 (and its owner); rows are prefetched from the owner
# one step early.  Rows crossing links per step for W = 8, all items direct or the top-H hot items
# replicated (their gradients all-gathered: every producer to every other rank).
W = 8
sets = []
for r in range(W):
    mine = pos[pos[:, 0] % W == r]
    indptr, indices = O.build_csr(mine[:, 0], mine[:, 1], U)
    u, i, j = C.sample(mine[:, 0], mine[:, 1], indptr, indices, I, 4,
                       (20261015 + r * 0x9E3779B97F4A7C15) & (2**64 - 1), 0, 0, 8 * B)
    sets.append([np.unique(np.concatenate([i[k*B:(k+1)*B], j[k*B:(k+1)*B]])) for k in range(8)])
cnt = np.bincount(pos[:, 1], minlength=I)
hot_order = np.argsort(-cnt, kind="stable")
for H in (0, 256, 1024, 4096):
    hot = np.zeros(I, bool)
    hot[hot_order[:H]] = True
    tot_direct, tot_hot = [], []
    for k in range(7):
        m = np.zeros((W, I), bool)
        n = np.zeros((W, I), bool)
        for r in range(W):
            m[r, sets[r][k]] = True
            n[r, sets[r][k + 1]] = True
        own = np.arange(I) % W
        rows = 0
        for p in range(W):
            its = np.nonzero(m[p] & ~hot)[0]
            dest = n[:, its].copy()
            dest[own[its], np.arange(len(its))] = True  # the owner keeps its base current
            dest[p] = False
            rows += int(dest.sum())
        hot_rows = int((m[:, hot].sum(0) * (W - 1)).sum())
        tot_direct.append(rows)
        tot_hot.append(hot_rows)
    per_link = (np.mean(tot_direct) + np.mean(tot_hot)) / (W * (W - 1)) * 512 / 1e3
    print(f"one-hop W=8, H={H}: cold gradient rows/step {np.mean(tot_direct):.0f}, hot all-gather rows "
          f"{np.mean(tot_hot):.0f}, per link {per_link:.0f} KB (owner scheme: 2 hops x ~402 KB)")
