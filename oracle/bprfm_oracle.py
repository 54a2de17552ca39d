"""ORACLE (test infrastructure only) — numpy restatement of the reference's BPR-FM training step.

Model BPRFMRecommender.py:28-79, loop :203-227: two fields per side (user feature u, item feature
U + x), values 1 (util/data_loader.py:574-627); per side
    fm   = 0.5 * ((e_u + e_x)^2 - (e_u^2 + e_x^2))                       (Bi-Interaction, :68-73)
    y    = BatchNorm1d(fm) in training mode (batch mean, biased variance, eps 1e-5) if batch_norm;
           running mean / variance (unbiased) updated with momentum 0.1, side i then side j
    y    = Dropout(p)(y)                                                   (:51-52)
    pred = sum_k y + b_u + b_x + bias_                                     (:74-79)
loss = -sum log sigmoid(pred_i - pred_j) (:220), dense gradients, Adagrad over every parameter
(lr, initial_accumulator_value 1e-8, eps 1e-10: torch.optim.Adagrad): rows with a zero gradient
keep their value and accumulator exactly.  float64 here; the reference is float32 (tolerances in
tests/test_bprfm_oracle.py).  `masks`: optional dropout keep-masks [2, B, k] (already scaled by
1 / (1 - p)), so the GPU's dropout draws can be replayed.
"""
import numpy as np

BN_EPS = 1e-5
ADAGRAD_EPS = 1e-10


class State:
    def __init__(self, E, b, bias_, gamma=None, beta=None, init_acc=1e-8):
        self.E = np.array(E, np.float64)
        self.b = np.array(b, np.float64).reshape(-1)
        self.bias_ = np.array(bias_, np.float64).reshape(1)
        self.bn = gamma is not None
        self.gamma = None if gamma is None else np.array(gamma, np.float64)
        self.beta = None if beta is None else np.array(beta, np.float64)
        k = self.E.shape[1]
        self.run_mean, self.run_var = np.zeros(k), np.ones(k)
        self.acc = {n: np.full_like(getattr(self, n), init_acc)
                    for n in ("E", "b", "bias_", "gamma", "beta") if getattr(self, n) is not None}


def _side(st, u, xf, mask):
    a, c = st.E[u], st.E[xf]
    s = a + c
    fm = 0.5 * (s * s - (a * a + c * c))
    cache = dict(a=a, c=c, s=s)
    if st.bn:
        mean = fm.mean(0)
        var = fm.var(0)
        inv = 1.0 / np.sqrt(var + BN_EPS)
        xhat = (fm - mean) * inv
        y = st.gamma * xhat + st.beta
        cache.update(xhat=xhat, inv=inv)
        B = fm.shape[0]
        st.run_mean = 0.9 * st.run_mean + 0.1 * mean
        st.run_var = 0.9 * st.run_var + 0.1 * (var * B / (B - 1) if B > 1 else var)
    else:
        y = fm
    if mask is not None:
        y = y * mask
    pred = y.sum(1) + st.b[u] + st.b[xf] + st.bias_[0]
    return pred, cache


def _back(st, g, u, xf, cache, mask, grads):
    gy = np.repeat(g[:, None], st.E.shape[1], 1)
    if mask is not None:
        gy = gy * mask
    if st.bn:
        xhat, inv = cache["xhat"], cache["inv"]
        grads["gamma"] += (gy * xhat).sum(0)
        grads["beta"] += gy.sum(0)
        gx = gy * st.gamma
        gfm = inv * (gx - gx.mean(0) - xhat * (gx * xhat).mean(0))
    else:
        gfm = gy
    s = cache["s"]
    np.add.at(grads["E"], u, gfm * (s - cache["a"]))
    np.add.at(grads["E"], xf, gfm * (s - cache["c"]))
    np.add.at(grads["b"], u, g)
    np.add.at(grads["b"], xf, g)
    grads["bias_"][0] += g.sum()


def step(st, U, u, i, j, lr, masks=None, grads_out=None):
    """One reference step on triplets (u, i, j); returns the loss.  Updates `st` in place;
    `grads_out` (a dict) receives the step's gradients."""
    u, i, j = (np.asarray(x, np.int64) for x in (u, i, j))
    pi, ci = _side(st, u, U + i, None if masks is None else masks[0])
    pj, cj = _side(st, u, U + j, None if masks is None else masks[1])
    d = pi - pj
    loss = float(np.sum(np.logaddexp(0.0, -d)))  # -log sigmoid(d)
    c = 1.0 / (1.0 + np.exp(d))                  # sigmoid(-d)
    grads = {n: np.zeros_like(v) for n, v in st.acc.items()}
    _back(st, -c, u, U + i, ci, None if masks is None else masks[0], grads)
    _back(st, c, u, U + j, cj, None if masks is None else masks[1], grads)
    if grads_out is not None:
        grads_out.update({n: g.copy() for n, g in grads.items()})
    for n, gr in grads.items():
        st.acc[n] += gr * gr
        p = getattr(st, n)
        p -= lr * gr / (np.sqrt(st.acc[n]) + ADAGRAD_EPS)
    return loss


def predict(st, u, x):
    """model.eval() forward of one side (:61-79): BatchNorm on the running statistics."""
    u, x = np.asarray(u, np.int64), np.asarray(x, np.int64)
    a, c = st.E[u], st.E[x]
    s = a + c
    fm = 0.5 * (s * s - (a * a + c * c))
    if st.bn:
        fm = (fm - st.run_mean) / np.sqrt(st.run_var + BN_EPS) * st.gamma + st.beta
    return fm.sum(1) + st.b[u] + st.b[x] + st.bias_[0]
