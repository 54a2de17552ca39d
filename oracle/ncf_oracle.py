"""NCF oracle (TEST INFRASTRUCTURE ONLY; nothing in the product imports this).

A numpy restatement of the reference NCF training step, pinned by tests/golden/ncf_steps_tiny.npz
(G1, made by importing the reference):
  model      NCFRecommender.py:27-124   GMF (embed_user_GMF * embed_item_GMF), MLP tower over
             concat(embed_user_MLP, embed_item_MLP) with num_layers x [Linear(n, n/2), ReLU],
             predict_layer Linear(d or 2d, 1); models 'GMF', 'MLP', 'NeuMF-end' (dropout 0)
  loss       NCFRecommender.py:255,282   BCEWithLogitsLoss (mean over the batch)
  optimiser  NCFRecommender.py:259-260   torch Adam(lr, betas=(0.9, 0.999), eps=1e-8), dense
             gradients: every embedding row with a nonzero moment moves every step; a parameter
             with no gradient (the unused branch of 'GMF' / 'MLP') is not stepped at all
Arithmetic in float64 on float32 parameters (the reference is fp32; parity is by tolerance).
Parameter names follow the reference's state_dict.
"""
import numpy as np


def param_names(model, num_layers):
    names = ["embed_user_GMF.weight", "embed_item_GMF.weight", "embed_user_MLP.weight",
             "embed_item_MLP.weight"]
    for l in range(num_layers):
        names += [f"MLP_layers.{3 * l + 1}.weight", f"MLP_layers.{3 * l + 1}.bias"]
    return names + ["predict_layer.weight", "predict_layer.bias"]


def used(model, name):
    """Parameters that receive a gradient (NCFRecommender.py:103-118)."""
    if model == "GMF":
        return "MLP" not in name
    if model == "MLP":
        return "GMF" not in name
    return True


def forward(params, model, num_layers, u, i):
    """NCF.forward (NCFRecommender.py:103-124); returns prediction and the activations."""
    p = {k: np.asarray(v, np.float64) for k, v in params.items()}
    act = {}
    parts = []
    if model != "MLP":
        act["eu"] = p["embed_user_GMF.weight"][u]
        act["ei"] = p["embed_item_GMF.weight"][i]
        parts.append(act["eu"] * act["ei"])
    if model != "GMF":
        h = np.concatenate([p["embed_user_MLP.weight"][u], p["embed_item_MLP.weight"][i]], 1)
        act["h0"] = h
        for l in range(num_layers):
            n = 3 * l + 1
            h = np.maximum(h @ p[f"MLP_layers.{n}.weight"].T + p[f"MLP_layers.{n}.bias"], 0.0)
            act[f"h{l + 1}"] = h
        parts.append(h)
    x = np.concatenate(parts, 1)
    act["x"] = x
    z = x @ p["predict_layer.weight"][0] + p["predict_layer.bias"][0]
    return z, act


def bce_with_logits(z, y):
    """mean(max(z,0) - z*y + log(1 + exp(-|z|)))  (torch's stable BCEWithLogitsLoss)."""
    return float(np.mean(np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z)))))


def grads(params, model, num_layers, u, i, y):
    """Dense gradients of the mean BCE loss (what loss.backward() leaves in .grad)."""
    p = {k: np.asarray(v, np.float64) for k, v in params.items()}
    z, act = forward(params, model, num_layers, u, i)
    B = len(u)
    dz = (1.0 / (1.0 + np.exp(-z)) - y) / B
    g = {k: np.zeros_like(v) for k, v in p.items()}
    x = act["x"]
    g["predict_layer.weight"][0] = dz @ x
    g["predict_layer.bias"][0] = dz.sum()
    dx = np.outer(dz, p["predict_layer.weight"][0])
    d = p["embed_user_GMF.weight"].shape[1]
    off = 0
    if model != "MLP":
        dg = dx[:, :d]
        np.add.at(g["embed_user_GMF.weight"], u, dg * act["ei"])
        np.add.at(g["embed_item_GMF.weight"], i, dg * act["eu"])
        off = d
    if model != "GMF":
        dh = dx[:, off:]
        for l in reversed(range(num_layers)):
            n = 3 * l + 1
            h_out, h_in = act[f"h{l + 1}"], act[f"h{l}"]
            dpre = dh * (h_out > 0)
            g[f"MLP_layers.{n}.weight"] = dpre.T @ h_in
            g[f"MLP_layers.{n}.bias"] = dpre.sum(0)
            dh = dpre @ p[f"MLP_layers.{n}.weight"]
        E = p["embed_user_MLP.weight"].shape[1]
        np.add.at(g["embed_user_MLP.weight"], u, dh[:, :E])
        np.add.at(g["embed_item_MLP.weight"], i, dh[:, E:])
    return {k: v for k, v in g.items() if used(model, k)}, bce_with_logits(z, y)


class Adam:
    """torch.optim.Adam, single-tensor form: m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
    p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)."""

    def __init__(self, params, lr=0.001, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps
        self.m = {k: np.zeros(np.shape(v)) for k, v in params.items()}
        self.v = {k: np.zeros(np.shape(v)) for k, v in params.items()}
        self.t = {k: 0 for k in params}

    def step(self, params, grads):
        for k, g in grads.items():
            self.t[k] += 1
            t = self.t[k]
            m = self.m[k] = self.m[k] + (1 - self.b1) * (g - self.m[k])
            v = self.v[k] = self.b2 * self.v[k] + (1 - self.b2) * g * g
            denom = np.sqrt(v) / np.sqrt(1 - self.b2 ** t) + self.eps
            params[k] = (np.asarray(params[k], np.float64)
                         - (self.lr / (1 - self.b1 ** t)) * m / denom).astype(np.float32)
        return params


def sample(pos_u, pos_i, indptr, indices, item_num, num_ng, seed, epoch, first, count):
    """Samples [first, first+count) of an epoch -> (u, i, label): the device sampler's spec.

    NCFData.ng_sample (util/data_loader.py:941-956) lists every positive (label 1), then num_ng
    negatives per positive (label 0); the DataLoader shuffles.  Here slot s -> q = permute(s) over
    (1 + num_ng) * npos (the BPR sampler's Feistel permutation); q < npos is positive q, else
    positive p = (q - npos) // num_ng with the negative = the k-th non-positive item of its user,
    k = the Lemire-bounded Philox draw of q (bpr_oracle._bounded)."""
    from oracle import bpr_oracle as O
    npos = len(pos_u)
    n = npos * (1 + num_ng)
    s = np.arange(first, first + count, dtype=np.int64)
    q = O.permute(s, n, seed, epoch)
    is_pos = q < npos
    p = np.where(is_pos, q, (q - npos) // max(num_ng, 1))
    u = np.asarray(pos_u, dtype=np.int64)[p]
    i = np.asarray(pos_i, dtype=np.int64)[p].copy()
    neg = ~is_pos
    if neg.any():
        un = u[neg]
        free = item_num - (indptr[un + 1] - indptr[un])
        k0, k1 = O._seed_key(seed)
        k = O._bounded(q[neg], epoch, free, k0, k1)
        i[neg] = O.kth_nonmember(indptr, indices, un, k)
    return u.astype(np.int32), i.astype(np.int32), is_pos.astype(np.float32)
