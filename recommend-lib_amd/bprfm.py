"""BPR-FM — drop-in for the reference's factorization-machine BPR.

`BPRFMRecommender.py` BPRFM (:28-79) with its Adagrad training loop (:196-227) and
`util/data_loader.py` BPRFMData (:574-627).  The model state lives on the GPU (include/bprfm.h,
bprfm.hip); state_dict() / load_state_dict() use the reference module's parameter names, so a
reference checkpoint loads as is.  Triplets are feature indices: BPRFMData builds them exactly as
the reference does (numpy's global RNG, rejection sampling against the train pairs).
"""
import ctypes

import numpy as np

from . import _lib


class BPRFMConfig(ctypes.Structure):  # bprfm_config, include/bprfm.h
    _fields_ = [("num_features", ctypes.c_int64), ("num_factors", ctypes.c_int32),
                ("batch_norm", ctypes.c_int32), ("drop_prob", ctypes.c_float),
                ("lr", ctypes.c_float), ("init_std", ctypes.c_float),
                ("max_batch", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("device", ctypes.c_int32), ("reserved", ctypes.c_int32 * 3)]


class BPRFMStats(ctypes.Structure):  # bprfm_stats
    _fields_ = [("triplets", ctypes.c_int64), ("steps", ctypes.c_int64), ("loss", ctypes.c_double),
                ("seconds", ctypes.c_double)]


def _i32(a):
    return np.ascontiguousarray(np.asarray(a).reshape(-1), np.int32)


class BPRFM:
    """BPRFM(num_features, num_factors, batch_norm, drop_prob) + Adagrad(lr, 1e-8).

    drop_prob is the reference's list (drop_prob[0] is the FM dropout; a float is accepted too).
    """

    def __init__(self, num_features, num_factors, batch_norm, drop_prob, lr=0.05, max_batch=4096,
                 seed=0, device=0, init_std=0.01):
        p = drop_prob[0] if hasattr(drop_prob, "__len__") else drop_prob
        self.num_features, self.num_factors = int(num_features), int(num_factors)
        self.batch_norm, self.drop_prob = bool(batch_norm), drop_prob
        self.lr, self.max_batch = float(lr), int(max_batch)
        self._L = _lib.load()
        cfg = BPRFMConfig(num_features=self.num_features, num_factors=self.num_factors,
                          batch_norm=int(self.batch_norm), drop_prob=float(p), lr=self.lr,
                          init_std=float(init_std), max_batch=self.max_batch,
                          seed=int(seed) & (2**64 - 1), device=int(device))
        h = ctypes.c_void_p()
        _lib.check(self._L.bprfm_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.last_stats = None

    def close(self):
        if getattr(self, "_h", None):
            self._L.bprfm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    # --- state ---
    def state_dict(self):
        F, k = self.num_features, self.num_factors
        E, b, b0 = np.empty((F, k), np.float32), np.empty((F, 1), np.float32), np.empty(1, np.float32)
        g, be, rm, rv = (np.empty(k, np.float32) for _ in range(4))
        _lib.check(self._L.bprfm_get_weights(self._h, _lib.ptr(E), _lib.ptr(b), _lib.ptr(b0),
                                             _lib.ptr(g), _lib.ptr(be), _lib.ptr(rm), _lib.ptr(rv)))
        sd = {"bias_": b0, "embeddings.weight": E, "biases.weight": b}
        if self.batch_norm:
            sd.update({"FM_layers.0.weight": g, "FM_layers.0.bias": be,
                       "FM_layers.0.running_mean": rm, "FM_layers.0.running_var": rv,
                       "FM_layers.0.num_batches_tracked": np.array(2 * self.steps, np.int64)})
        return sd

    def load_state_dict(self, sd):
        def get(name, shape):
            v = sd.get(name)
            if v is None:
                return None
            v = np.ascontiguousarray(np.asarray(v, np.float32))
            if v.size != int(np.prod(shape)):
                raise ValueError(f"{name}: expected {shape}, got {v.shape}")
            return v
        F, k = self.num_features, self.num_factors
        arrs = [get("embeddings.weight", (F, k)), get("biases.weight", (F,)), get("bias_", (1,)),
                get("FM_layers.0.weight", (k,)), get("FM_layers.0.bias", (k,)),
                get("FM_layers.0.running_mean", (k,)), get("FM_layers.0.running_var", (k,))]
        _lib.check(self._L.bprfm_set_weights(self._h, *[_lib.ptr(a) for a in arrs]))

    @property
    def steps(self):
        return int(self._L.bprfm_steps(self._h))

    # --- training (:211-227) ---
    def train_triplets(self, u, i, j, batch_size=None):
        """One pass of the inner training loop over the triplets in the given order, batch_size
        (default max_batch) per optimizer step; returns the summed loss of the batches."""
        batch_size = self.max_batch if batch_size is None else batch_size
        u, i, j = _i32(u), _i32(i), _i32(j)
        if not (len(u) == len(i) == len(j)):
            raise ValueError("u, i, j must have one length")
        st = BPRFMStats()
        _lib.check(self._L.bprfm_train(self._h, _lib.ptr(u), _lib.ptr(i), _lib.ptr(j), len(u),
                                       int(batch_size), ctypes.byref(st)))
        self.last_stats = dict(triplets=st.triplets, steps=st.steps, loss=st.loss, seconds=st.seconds)
        return st.loss

    def fit_epoch(self, dataset, batch_size=None, shuffle=True):
        """model.train(); dataset.ng_sample(); one shuffled pass (DataLoader(shuffle=True) draws
        its permutation from torch's RNG, this one from numpy's)."""
        dataset.ng_sample()
        u, i, j = dataset.triplets()
        if shuffle:
            perm = np.random.permutation(len(u))
            u, i, j = u[perm], i[perm], j[perm]
        return self.train_triplets(u, i, j, batch_size)

    def dropout_mask(self, B):
        """The keep-scales [2, B, k] the next optimizer step draws for a batch of B."""
        out = np.empty((2, int(B), self.num_factors), np.float32)
        _lib.check(self._L.bprfm_dropout_mask(self._h, int(B), _lib.ptr(out)))
        return out

    # --- model.eval() forward (:55-79) ---
    def _out(self, features, values=None):
        f = np.asarray(features).reshape(-1, 2)
        if values is not None and not np.all(np.asarray(values) == 1):
            raise ValueError("feature values must be 1 (BPRFMData's only shape)")
        u, x = _i32(f[:, 0]), _i32(f[:, 1])
        out = np.empty(len(u), np.float32)
        _lib.check(self._L.bprfm_predict(self._h, _lib.ptr(u), _lib.ptr(x), len(u), _lib.ptr(out)))
        return out

    def forward(self, features_i, feature_values_i, features_j, feature_values_j):
        return self._out(features_i, feature_values_i), self._out(features_j, feature_values_j)

    __call__ = forward

    def predict(self, features, feature_values=None):
        return self._out(features, feature_values)


class BPRFMData:
    """util/data_loader.py BPRFMData (:574-627) over a DataFrame[user, item, ...]: features are
    feature_map[col value + feat_idx_dict[col]] per row; ng_sample draws num_ng negatives per row
    with np.random.randint(num_item), rejecting (u, j) train pairs, in the reference's order."""

    def __init__(self, df, feat_idx_dict, feature_map, num_item, num_ng=0, is_training=None):
        self.feat_idx_dict, self.feature_map = feat_idx_dict, feature_map
        self.num_ng, self.num_item, self.is_training = num_ng, num_item, is_training
        users = np.asarray(df["user"].values, np.int64)
        items = np.asarray(df["item"].values, np.int64)
        self.train_mat = set(zip(users.tolist(), items.tolist()))
        cols = [c for c in df.columns if c not in ("rating", "timestamp")]
        if cols != ["user", "item"]:
            raise ValueError(f"BPR-FM rows are [user, item] features, got columns {cols}")
        self.cols = cols
        fmap = np.vectorize(feature_map.__getitem__, otypes=[np.int64])
        self.fu = fmap(users + feat_idx_dict["user"]) if len(users) else users
        self.fi = fmap(items + feat_idx_dict["item"]) if len(items) else items
        self._fill = None

    def ng_sample(self):
        assert self.is_training, "no need to sampling when testing"
        n = len(self.fu)
        u = np.repeat(self.fu, self.num_ng)
        i = np.repeat(self.fi, self.num_ng)
        j = np.empty(n * self.num_ng, np.int64)
        off = self.feat_idx_dict["item"]
        q = 0
        for x in range(n):
            ux = int(self.fu[x])
            for _ in range(self.num_ng):
                jj = np.random.randint(self.num_item)
                while (ux, jj) in self.train_mat:
                    jj = np.random.randint(self.num_item)
                j[q] = self.feature_map[jj + off]
                q += 1
        self._fill = (u, i, j)

    def triplets(self):
        """(u, i, j) feature indices of the sampled training rows (ng_sample first)."""
        if self._fill is None:
            raise RuntimeError("call ng_sample() first")
        return self._fill

    def __len__(self):
        return self.num_ng * len(self.fu) if self.is_training else len(self.fu)

    def __getitem__(self, idx):
        one = np.ones(2, np.float32)
        if self.is_training:
            u, i, j = (a[idx] for a in self.triplets())
            return np.array([u, i]), one, np.array([u, j]), one
        f = np.array([self.fu[idx], self.fi[idx]])
        return f, one, f, one
