"""BPRData — drop-in for util/data_loader.py:667-700, with ng_sample() on the GPU.

Reference semantics kept: `features` = [[u, i], ...] train positives; `ng_sample()` (training only,
AssertionError otherwise, :681) draws `num_ng` negatives per positive, each uniform over the items
the user has NOT interacted with in `train_mat` (:684-689); `__len__` = num_ng * len(features) when
training (:692-693); `__getitem__` -> (user, item_i, item_j) with item_j = item_i when not
training (:695-700).
Difference: the RNG is Philox4x32-10 keyed by `seed` (reproducible, parallel) instead of the
unseeded global MT19937, and `features_fill` comes back already in shuffled epoch order (a
DataLoader(shuffle=True) on top only reshuffles a uniform order).
"""
import numpy as np


def _pairs(features):
    a = np.asarray(features)
    if a.size == 0:
        return np.zeros((0, 2), dtype=np.int64)
    return a[:, :2].astype(np.int64)


def train_mat_pairs(train_mat):
    """(users, items) of the positives of a dok/csr/coo matrix or a set of (u, i) tuples."""
    if train_mat is None:
        return None
    if hasattr(train_mat, "tocoo"):
        c = train_mat.tocoo()
        keep = c.data != 0
        return c.row[keep].astype(np.int32), c.col[keep].astype(np.int32)
    keys = np.array(list(train_mat.keys() if hasattr(train_mat, "keys") else train_mat), dtype=np.int64)
    if keys.size == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    return keys[:, 0].astype(np.int32), keys[:, 1].astype(np.int32)


class BPRData:
    def __init__(self, features, num_item, train_mat=None, num_ng=0, is_training=None, seed=0,
                 device=0, num_user=None):
        self.features = features
        self.num_item = int(num_item)
        self.train_mat = train_mat
        self.num_ng = int(num_ng)
        self.is_training = is_training
        self.seed = int(seed)
        self.device = int(device)
        self.num_user = num_user
        self.epoch = 0
        self._sampler = None
        self.features_fill = None

    def _make_sampler(self):
        from .model import BPRMF
        pairs = _pairs(self.features)
        ex = train_mat_pairs(self.train_mat)
        nu = self.num_user
        if nu is None:
            nu = int(pairs[:, 0].max()) + 1 if len(pairs) else 1
            if ex is not None and len(ex[0]):
                nu = max(nu, int(ex[0].max()) + 1)
        s = BPRMF(nu, self.num_item, factor_num=1, batch_size=4096, num_ng=max(self.num_ng, 1),
                  seed=self.seed, device=self.device, init_std=0.0)
        s.set_train(pairs, exclude=ex)
        return s

    def ng_sample(self):
        assert self.is_training, "no need to sampling when testing"
        if self._sampler is None:
            self._sampler = self._make_sampler()
        u, i, j = self._sampler.sample(self.epoch)
        self.epoch += 1
        self.features_fill = np.stack([u, i, j], axis=1).astype(np.int64)

    def __len__(self):
        return self.num_ng * len(self.features) if self.is_training else len(self.features)

    def __getitem__(self, idx):
        features = self.features_fill if self.is_training else self.features
        user = int(features[idx][0])
        item_i = int(features[idx][1])
        item_j = int(features[idx][2]) if self.is_training else int(features[idx][1])
        return user, item_i, item_j

    def triplets(self):
        """(u, i, j) int32 arrays of the current epoch (for BPRMF.train_triplets)."""
        f = np.asarray(self.features_fill if self.is_training else self.features)
        if not self.is_training:
            return f[:, 0].astype(np.int32), f[:, 1].astype(np.int32), f[:, 1].astype(np.int32)
        return f[:, 0].astype(np.int32), f[:, 1].astype(np.int32), f[:, 2].astype(np.int32)
