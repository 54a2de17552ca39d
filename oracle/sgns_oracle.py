"""ORACLE (test infrastructure only) — numpy restatement of the reference's Item2Vec path.

* build_corpus: util/data_loader.py BuildCorpus (:1118-1171).  Sentences are each user's items in
  frame order (groupby('user'), users ascending).  wc counts the items and starts with
  {UNK: 1}; idx2word = [UNK] + the max_vocab - 1 most frequent keys of wc (a stable sort by
  count, descending, ties in first-seen order; UNK itself is a key of wc, so it may appear a
  second time); word2idx keeps the LAST index of a word, so UNK's index is that second one when
  it exists.  skipgram(i) pads both sides of the window with UNK.
* step: SGNS.forward (Item2VecRecommender.py:82-97) + dense backward + torch.optim.Adam (:272,
  defaults lr 1e-3, betas (0.9, 0.999), eps 1e-8).  Both tables are nn.Embedding with
  padding_idx 0: row 0 gets no gradient.  Negatives are supplied (the reference draws them from
  torch's RNG; tests/golden/make_golden_sgns.py records them).  float64.
"""
import numpy as np

UNK = -1  # the UNK token among item ids


def build_corpus(users, items, max_vocab):
    """(idx2word, word2idx): UNK as -1."""
    wc = {UNK: 1}
    for u in np.unique(users):
        for w in items[users == u]:
            w = int(w)
            wc[w] = wc.get(w, 0) + 1
    idx2word = [UNK] + sorted(wc, key=wc.get, reverse=True)[: max_vocab - 1]
    word2idx = {w: x for x, w in enumerate(idx2word)}
    return idx2word, word2idx, wc


def convert(users, items, word2idx, window):
    """BuildCorpus.convert: (iwords [n], owords [n, 2 window]) in user order."""
    unk = word2idx[UNK]
    iws, ows = [], []
    for u in np.unique(users):
        sent = [word2idx.get(int(w), unk) if int(w) in word2idx else unk for w in items[users == u]]
        for x in range(len(sent)):
            left = sent[max(x - window, 0): x]
            right = sent[x + 1: x + 1 + window]
            iws.append(sent[x])
            ows.append([unk] * (window - len(left)) + left + right + [unk] * (window - len(right)))
    return np.array(iws, np.int64), np.array(ows, np.int64).reshape(-1, 2 * window)


def _logsig(x):
    return -np.logaddexp(0.0, -x)


class State:
    def __init__(self, I, O, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
        self.I = np.array(I, np.float64)
        self.O = np.array(O, np.float64)
        self.m = {n: np.zeros_like(getattr(self, n)) for n in ("I", "O")}
        self.v = {n: np.zeros_like(getattr(self, n)) for n in ("I", "O")}
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps


def step(st, iwords, owords, nwords, grads_out=None):
    """One reference step; returns the loss.  iwords [B], owords [B, C], nwords [B, C * n]."""
    iw = np.asarray(iwords, np.int64)
    ow = np.asarray(owords, np.int64)
    nw = np.asarray(nwords, np.int64)
    B, C = ow.shape
    n = nw.shape[1] // C
    iv = st.I[iw]                                    # [B, E]
    so = np.einsum("bce,be->bc", st.O[ow], iv)       # o . i
    sn = np.einsum("bke,be->bk", st.O[nw], iv)       # n . i (the reference negates n)
    oloss = _logsig(so).mean(1)
    nloss = _logsig(-sn).reshape(B, C, n).sum(2).mean(1)
    loss = float(-(oloss + nloss).mean())
    go = -(1.0 - 1.0 / (1.0 + np.exp(-so))) / (B * C)   # d loss / d (o . i)
    gn = (1.0 / (1.0 + np.exp(-sn))) / (B * C)          # d loss / d (n . i)
    gI = np.zeros_like(st.I)
    gO = np.zeros_like(st.O)
    np.add.at(gI, iw, np.einsum("bc,bce->be", go, st.O[ow]) + np.einsum("bk,bke->be", gn, st.O[nw]))
    np.add.at(gO, ow.reshape(-1), (go[:, :, None] * iv[:, None, :]).reshape(-1, iv.shape[1]))
    np.add.at(gO, nw.reshape(-1), (gn[:, :, None] * iv[:, None, :]).reshape(-1, iv.shape[1]))
    gI[0] = 0.0  # padding_idx
    gO[0] = 0.0
    if grads_out is not None:
        grads_out.update(I=gI.copy(), O=gO.copy())
    st.t += 1
    bc1 = 1.0 - st.b1 ** st.t
    bc2 = 1.0 - st.b2 ** st.t
    for name, g in (("I", gI), ("O", gO)):
        m, v, p = st.m[name], st.v[name], getattr(st, name)
        m += (1.0 - st.b1) * (g - m)
        v *= st.b2
        v += (1.0 - st.b2) * g * g
        p -= (st.lr / bc1) * (m / (np.sqrt(v) / np.sqrt(bc2) + st.eps))
    return loss
