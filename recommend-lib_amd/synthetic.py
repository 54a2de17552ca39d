"""Synthetic interaction data of a given shape (no dataset download is possible on the box).

make_positives(U, I, npos, seed): the ml-20m-shaped (or C5-shaped) positive set of SURVEY.md §8d:
user degree lognormal, clipped at >= 10; item popularity Zipf(alpha=1.0) over a random item order;
positives de-duplicated per user.  Returns int64 [n, 2] (user, item) rows, n close to npos,
ordered by user (the `features` list of util/data_loader.py:BPRData).
"""
import numpy as np


def make_positives(U, I, npos, seed=20261015, alpha=1.0, min_deg=10, sigma=1.0):
    g = np.random.default_rng(seed)
    U, I, npos = int(U), int(I), int(npos)
    deg = g.lognormal(0.0, sigma, U)
    deg = np.maximum(np.round(deg * (npos / deg.sum())), min_deg)
    deg = np.minimum(deg, I // 2).astype(np.int64)
    # oversample ~8% to make up for per-user duplicates removed below
    draw = np.ceil(deg * 1.08).astype(np.int64)
    total = int(draw.sum())
    w = 1.0 / np.power(np.arange(1, I + 1, dtype=np.float64), alpha)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    ranks = np.searchsorted(cdf, g.random(total), side="right")
    ranks = np.minimum(ranks, I - 1)
    order = g.permutation(I)
    items = order[ranks]
    users = np.repeat(np.arange(U, dtype=np.int64), draw)
    key = np.unique(users * I + items)
    users, items = key // I, key % I
    # trim each user back to its target degree (keeps the lognormal shape)
    start = np.searchsorted(users, np.arange(U))
    rank_in_user = np.arange(len(users)) - start[users]
    keep = rank_in_user < deg[users]
    return np.stack([users[keep], items[keep]], axis=1)
