"""Item2Vec / SGNS — drop-in for the reference's Item2Vec path.

`Item2VecRecommender.py` Item2Vec (:39-68), SGNS (:70-97) with Adam and its training loop
(:272-291), and `util/data_loader.py` BuildCorpus / PermutedSubsampledCorpus (:1118-1189).  The
tables and Adam's moments live on the GPU (include/sgns.h, sgns.hip); state_dict() uses the
reference module's parameter names and optimizer_state_dict() torch's Adam layout, so the
--conti resume (:266-275) round-trips.  The corpus is built on the host exactly as the reference
builds it, quirks included (UNK is a key of the word counts, so idx2word may list it twice and
word2idx keeps the second index), but in memory instead of pickles under ./data.
"""
import ctypes
import random

import numpy as np

from . import _lib

UNK_DEFAULT = "<UNK>"


class SgnsConfig(ctypes.Structure):  # sgns_config, include/sgns.h
    _fields_ = [("vocab_size", ctypes.c_int64), ("embedding_size", ctypes.c_int32),
                ("n_negs", ctypes.c_int32), ("context", ctypes.c_int32),
                ("max_batch", ctypes.c_int32), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("seed", ctypes.c_uint64),
                ("device", ctypes.c_int32), ("reserved", ctypes.c_int32 * 3)]


class SgnsStats(ctypes.Structure):  # sgns_stats
    _fields_ = [("examples", ctypes.c_int64), ("steps", ctypes.c_int64), ("loss", ctypes.c_double),
                ("seconds", ctypes.c_double)]


def _i32(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a), np.int32)
    return a if shape is None else a.reshape(shape)


# ------------------------------------------------------------------------------------------------
# corpus (util/data_loader.py:1118-1189)
# ------------------------------------------------------------------------------------------------
class BuildCorpus:
    """BuildCorpus(corpus_df, window, max_vocab, unk, dataset): build() makes the vocabulary
    (wc, idx2word, word2idx, vocab), convert(train_df, idx) the skip-gram rows, returned as
    (iwords [n], owords [n, 2 window]) int32 arrays and kept in self.data[idx]."""

    def __init__(self, corpus_df, window=5, max_vocab=20000, unk=UNK_DEFAULT, dataset="ml-100k"):
        self.window, self.max_vocab, self.unk = window, max_vocab, unk
        self.dataset = dataset
        self.corpus = self._sentences(corpus_df)
        self.data = {}

    @staticmethod
    def _sentences(df):
        # groupby('user')['item'].apply(list): users ascending, items in frame order
        u = np.asarray(df["user"].values)
        it = np.asarray(df["item"].values)
        order = np.argsort(u, kind="stable")
        us, starts = np.unique(u[order], return_index=True)
        bounds = list(starts) + [len(order)]
        return [it[order[bounds[k]:bounds[k + 1]]].tolist() for k in range(len(us))]

    def skipgram(self, sentence, i):
        iword = sentence[i]
        left = sentence[max(i - self.window, 0): i]
        right = sentence[i + 1: i + 1 + self.window]
        return iword, ([self.unk] * (self.window - len(left)) + left + right
                       + [self.unk] * (self.window - len(right)))

    def build(self):
        self.wc = {self.unk: 1}
        for sent in self.corpus:
            for w in sent:
                self.wc[w] = self.wc.get(w, 0) + 1
        self.idx2word = [self.unk] + sorted(self.wc, key=self.wc.get, reverse=True)[: self.max_vocab - 1]
        self.word2idx = {self.idx2word[x]: x for x in range(len(self.idx2word))}
        self.vocab = set(self.word2idx)
        return self

    def convert(self, corpus_train_df, idx=0):
        w2i, unk = self.word2idx, self.unk
        iws, ows = [], []
        for sent in self._sentences(corpus_train_df):
            sent = [w if w in self.vocab else unk for w in sent]
            for x in range(len(sent)):
                iword, owords = self.skipgram(sent, x)
                iws.append(w2i[iword])
                ows.append([w2i[o] for o in owords])
        out = (np.array(iws, np.int32), np.array(ows, np.int32).reshape(-1, 2 * self.window))
        self.data[idx] = out
        return out

    def word_counts(self):
        """wf of the script (:255): counts in idx2word order (for SGNS weights)."""
        return np.array([self.wc[w] for w in self.idx2word], np.float64)


class PermutedSubsampledCorpus:
    """PermutedSubsampledCorpus(data, ws=None): keeps (iword, owords) with random.random() >
    ws[iword] (Python's random, in the reference's order); data = (iwords, owords) arrays."""

    def __init__(self, data, ws=None):
        iw, ow = data
        if ws is not None:
            keep = np.array([random.random() > ws[w] for w in iw], bool)
            iw, ow = iw[keep], ow[keep]
        self.iwords, self.owords = np.asarray(iw, np.int32), np.asarray(ow, np.int32)

    def __len__(self):
        return len(self.iwords)

    def __getitem__(self, idx):
        return int(self.iwords[idx]), np.array(self.owords[idx])


# ------------------------------------------------------------------------------------------------
# model (Item2VecRecommender.py:39-97)
# ------------------------------------------------------------------------------------------------
class Item2Vec:
    """The embedding pair.  Initial tables as the reference draws them (torch's global RNG:
    row 0 zeros, the rest uniform(-0.5/E, 0.5/E)), uploaded when SGNS wraps it; without torch,
    the device draws its own (same distribution)."""

    def __init__(self, vocab_size=20000, embedding_size=100, padding_idx=0, torch_init=True):
        if padding_idx != 0:
            raise ValueError("padding_idx must be 0 (the reference's)")
        self.vocab_size, self.embedding_size = int(vocab_size), int(embedding_size)
        self._init = None
        if torch_init:
            try:
                import torch
            except ImportError:
                torch = None
            if torch is not None:
                V, E = self.vocab_size, self.embedding_size
                for _ in range(2):  # the two nn.Embedding(...) constructions draw normal_ first
                    torch.empty(V, E).normal_()
                tabs = []
                for _ in range(2):  # ivectors, then ovectors (:46-53)
                    t = torch.cat([torch.zeros(1, E),
                                   torch.FloatTensor(V - 1, E).uniform_(-0.5 / E, 0.5 / E)])
                    tabs.append(t.numpy().copy())
                self._init = tabs
        self._sgns = None

    def _bound(self):
        if self._sgns is None:
            raise RuntimeError("wrap the model in SGNS(embedding=model, ...) first")
        return self._sgns

    def forward(self, data):
        return self.forward_i(data)

    __call__ = forward

    def forward_i(self, data):
        return self._bound()._lookup(0, data)

    def forward_o(self, data):
        return self._bound()._lookup(1, data)

    @property
    def ivectors_weight(self):
        return self._bound().state_dict()["embedding.ivectors.weight"]

    @property
    def ovectors_weight(self):
        return self._bound().state_dict()["embedding.ovectors.weight"]


class SGNS:
    """SGNS(embedding, vocab_size, n_negs, weights) + optim.Adam(lr, betas, eps).

    train_step(iword, owords) = the loop body (loss, zero_grad, backward, step) and returns the
    loss; train_epoch(dataset, mb) = one shuffled DataLoader pass.  `context` is the owords
    width, 2 x window."""

    def __init__(self, embedding, vocab_size=20000, n_negs=20, weights=None, context=10, lr=1e-3,
                 betas=(0.9, 0.999), eps=1e-8, max_batch=4096, seed=0, device=0):
        if int(vocab_size) != embedding.vocab_size:
            raise ValueError("vocab_size differs from the embedding's")
        self.embedding, self.vocab_size, self.n_negs = embedding, int(vocab_size), int(n_negs)
        self.context, self.max_batch = int(context), int(max_batch)
        self._L = _lib.load()
        cfg = SgnsConfig(vocab_size=self.vocab_size, embedding_size=embedding.embedding_size,
                         n_negs=self.n_negs, context=self.context, max_batch=self.max_batch,
                         lr=float(lr), beta1=float(betas[0]), beta2=float(betas[1]), eps=float(eps),
                         seed=int(seed) & (2**64 - 1), device=int(device))
        h = ctypes.c_void_p()
        _lib.check(self._L.sgns_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.weights = None
        if weights is not None:
            w = np.ascontiguousarray(np.asarray(weights, np.float64).reshape(-1))
            if len(w) != self.vocab_size:
                raise ValueError("weights must have vocab_size entries")
            _lib.check(self._L.sgns_set_noise(self._h, _lib.ptr(w)))
            wf = np.power(w, 0.75)
            self.weights = wf / wf.sum()
        if embedding._init is not None:
            I, O = embedding._init
            _lib.check(self._L.sgns_set_weights(self._h, _lib.ptr(I), _lib.ptr(O)))
        embedding._sgns = self
        self.last_stats = None

    def close(self):
        if getattr(self, "_h", None):
            self._L.sgns_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    # --- training (:276-287) ---
    def train_examples(self, iwords, owords, nwords=None, batch_size=None):
        """The loop body over the examples in the given order, batch_size (default max_batch)
        per step; nwords [n, context * n_negs] replays given negatives.  Returns the summed loss
        of the batches."""
        batch_size = self.max_batch if batch_size is None else int(batch_size)
        iw = _i32(iwords).reshape(-1)
        ow = _i32(owords, (-1, self.context))
        if len(ow) != len(iw):
            raise ValueError("owords must be [n, context]")
        nw = None
        if nwords is not None:
            nw = _i32(nwords, (-1, self.context * self.n_negs))
            if len(nw) != len(iw):
                raise ValueError("nwords must be [n, context * n_negs]")
        st = SgnsStats()
        _lib.check(self._L.sgns_train(self._h, _lib.ptr(iw), _lib.ptr(ow), _lib.ptr(nw), len(iw),
                                      batch_size, ctypes.byref(st)))
        self.last_stats = dict(examples=st.examples, steps=st.steps, loss=st.loss,
                               seconds=st.seconds)
        return st.loss

    def train_step(self, iword, owords, nwords=None):
        return self.train_examples(iword, owords, nwords, batch_size=len(np.asarray(iword).reshape(-1)))

    def train_epoch(self, dataset, mb=None, shuffle=True):
        """One pass of DataLoader(dataset, batch_size=mb, shuffle=True) (the permutation from
        numpy's RNG instead of torch's)."""
        iw, ow = dataset.iwords, dataset.owords
        if shuffle:
            p = np.random.permutation(len(iw))
            iw, ow = iw[p], ow[p]
        return self.train_examples(iw, ow, batch_size=mb)

    def negatives(self, B):
        """The negatives [B, context * n_negs] the next step draws for a batch of B."""
        out = np.empty((int(B), self.context * self.n_negs), np.int32)
        _lib.check(self._L.sgns_negatives(self._h, int(B), _lib.ptr(out)))
        return out

    def _lookup(self, which, data):
        idx = _i32(data)
        out = np.empty(idx.shape + (self.embedding.embedding_size,), np.float32)
        _lib.check(self._L.sgns_lookup(self._h, which, _lib.ptr(idx.reshape(-1)), idx.size,
                                       _lib.ptr(out)))
        return out

    # --- state (torch.save(sgns.state_dict()) / optimizer.state_dict(), :288-291) ---
    def state_dict(self):
        V, E = self.vocab_size, self.embedding.embedding_size
        I, O = np.empty((V, E), np.float32), np.empty((V, E), np.float32)
        _lib.check(self._L.sgns_get_weights(self._h, _lib.ptr(I), _lib.ptr(O)))
        return {"embedding.ivectors.weight": I, "embedding.ovectors.weight": O}

    def load_state_dict(self, sd):
        V, E = self.vocab_size, self.embedding.embedding_size
        arrs = []
        for n in ("embedding.ivectors.weight", "embedding.ovectors.weight"):
            v = sd.get(n)
            if v is not None:
                v = np.ascontiguousarray(np.asarray(v, np.float32))
                if v.shape != (V, E):
                    raise ValueError(f"{n}: expected {(V, E)}, got {v.shape}")
            arrs.append(v)
        _lib.check(self._L.sgns_set_weights(self._h, _lib.ptr(arrs[0]), _lib.ptr(arrs[1])))

    @property
    def steps(self):
        step = ctypes.c_int64()
        _lib.check(self._L.sgns_get_adam(self._h, ctypes.byref(step), None, None, None, None))
        return step.value

    def optimizer_state_dict(self):
        V, E = self.vocab_size, self.embedding.embedding_size
        m = [np.empty((V, E), np.float32) for _ in range(4)]
        step = ctypes.c_int64()
        _lib.check(self._L.sgns_get_adam(self._h, ctypes.byref(step), *[_lib.ptr(x) for x in m]))
        st = {q: {"step": float(step.value), "exp_avg": m[2 * q], "exp_avg_sq": m[2 * q + 1]}
              for q in range(2)}
        return {"state": st if step.value else {}, "param_groups": [{"params": [0, 1]}]}

    def load_optimizer_state_dict(self, sd):
        st = sd.get("state", {})
        if not st:
            return
        step = int(float(np.asarray(st[0]["step"])))
        arrs = [np.ascontiguousarray(np.asarray(st[q][k], np.float32))
                for q in range(2) for k in ("exp_avg", "exp_avg_sq")]
        _lib.check(self._L.sgns_set_adam(self._h, step, *[_lib.ptr(a) for a in arrs]))
