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


def make_planted(U, I, npos, seed=20261101, k=8, beta=1.0, alpha=1.0, min_deg=10, sigma=1.0,
                 device="cpu", chunk=2048):
    """Positives with latent taste structure: a ground-truth low-rank model
    P* [U, k], Q* [I, k] (N(0, 1) entries) and a Zipf(alpha) popularity over a random item order;
    user u draws deg(u) distinct items (lognormal degree as make_positives) without replacement
    with probability proportional to exp(beta <P*_u, Q*_i> + log pop_i) (Gumbel top-k, chunks of
    users on `device`).  A model that learns the user-item structure beats the popularity ranking
    on held-out positives; on make_positives' data nothing but popularity can be learnt.
    Returns (positives int64 [n, 2] sorted by (user, item), P*, Q*) as numpy arrays.  The draw
    depends on the device's RNG (CPU and GPU give different, equally distributed sets)."""
    import torch
    g = np.random.default_rng(seed)
    U, I, npos = int(U), int(I), int(npos)
    deg = g.lognormal(0.0, sigma, U)
    deg = np.maximum(np.round(deg * (npos / deg.sum())), min_deg)
    deg = np.minimum(deg, I // 2).astype(np.int64)
    w = 1.0 / np.power(np.arange(1, I + 1, dtype=np.float64), alpha)
    logpop = np.empty(I)
    logpop[g.permutation(I)] = np.log(w / w.sum())
    tg = torch.Generator(device=device).manual_seed(int(seed))
    Ps = torch.randn(U, k, generator=tg, device=device)
    Qs = torch.randn(I, k, generator=tg, device=device)
    lp = torch.as_tensor(logpop, dtype=torch.float32, device=device)
    users, items = [], []
    for a in range(0, U, chunk):
        b = min(U, a + chunk)
        logits = beta * (Ps[a:b] @ Qs.T) + lp
        u01 = torch.rand(logits.shape, generator=tg, device=device).clamp_(1e-12, 1.0 - 1e-7)
        keys = logits - torch.log(-torch.log(u01))  # + Gumbel(0, 1)
        kmax = int(deg[a:b].max())
        top = torch.topk(keys, kmax, dim=1).indices.cpu().numpy()
        d = deg[a:b]
        mask = np.arange(kmax)[None, :] < d[:, None]
        users.append(np.repeat(np.arange(a, b, dtype=np.int64), d))
        items.append(top[mask].astype(np.int64))
    users, items = np.concatenate(users), np.concatenate(items)
    o = np.lexsort((items, users))
    return (np.stack([users[o], items[o]], axis=1), Ps.cpu().numpy(), Qs.cpu().numpy())
