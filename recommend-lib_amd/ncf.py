"""NCF — the drop-in model object of the MI355X NCF path.

Mirrors the reference contract:
  * `NCF(user_num, item_num, factor_num, num_layers, dropout, model)` with
    `forward(user, item) -> prediction` (NCFRecommender.py:27-124), so util/metrics.py's
    `_ncf_topk` and the KPI loop of NCFRecommender.py run unchanged;
  * the training loop of NCFRecommender.py:262-288 (BCEWithLogitsLoss, Adam(lr) over every
    parameter, `NCFData.ng_sample()` + shuffled DataLoader every epoch) as `fit()` / `train_epoch()`;
  * `NCFData(features, num_item, train_mat, num_ng, is_training)` (util/data_loader.py:931-972),
    its negatives drawn by the device sampler.
Models 'GMF', 'MLP', 'NeuMF-end' with dropout 0 (the reference default).  All compute runs in
libbprmf_amd.so (include/ncf.h); parameters live in HBM and are reached through `state_dict()`.
"""
import ctypes

import numpy as np

from . import _lib

MODELS = {"NeuMF-end": 0, "GMF": 1, "MLP": 2}


class NCF:
    def __init__(self, user_num, item_num, factor_num=32, num_layers=3, dropout=0.0,
                 model="NeuMF-end", GMF_model=None, MLP_model=None, lr=0.001, batch_size=256,
                 num_ng=4, epochs=20, seed=0, device=0, betas=(0.9, 0.999), eps=1e-8):
        if model not in MODELS:
            raise ValueError(f"model must be one of {sorted(MODELS)} (NeuMF-pre: build NeuMF-end "
                             "and load_state_dict the pre-trained tensors)")
        if dropout:
            raise ValueError("dropout > 0 is not supported (the reference default is 0.0)")
        self.user_num, self.item_num = int(user_num), int(item_num)
        self.factor_num, self.num_layers, self.model = int(factor_num), int(num_layers), model
        self.batch_size, self.num_ng, self.epochs = int(batch_size), int(num_ng), int(epochs)
        self.device = int(device)
        self.epoch = 0
        self.history = []
        L = _lib.load()
        cfg = _lib.NcfConfig(user_num=self.user_num, item_num=self.item_num,
                             factor_num=self.factor_num, num_layers=self.num_layers,
                             model=MODELS[model], batch_size=self.batch_size, num_ng=self.num_ng,
                             lr=float(lr), beta1=float(betas[0]), beta2=float(betas[1]),
                             eps=float(eps), init_std=0.01, seed=int(seed) & (2**64 - 1),
                             device=self.device)
        h = ctypes.c_void_p()
        _lib.check(L.ncf_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h, self._L = h, L
        self._has_train = False
        n = ctypes.c_int32()
        _lib.check(L.ncf_param_count(h, ctypes.byref(n)))
        self.names = ["embed_user_GMF.weight", "embed_item_GMF.weight", "embed_user_MLP.weight",
                      "embed_item_MLP.weight"]
        for l in range(self.num_layers):
            self.names += [f"MLP_layers.{3 * l + 1}.weight", f"MLP_layers.{3 * l + 1}.bias"]
        self.names += ["predict_layer.weight", "predict_layer.bias"]
        assert len(self.names) == n.value
        self._shapes = []
        for k in range(n.value):
            r, c = ctypes.c_int64(), ctypes.c_int64()
            _lib.check(L.ncf_param_shape(h, k, ctypes.byref(r), ctypes.byref(c)))
            bias = self.names[k].endswith(".bias")
            self._shapes.append((r.value,) if bias else (r.value, c.value))

    def close(self):
        if getattr(self, "_h", None):
            self._L.ncf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- nn.Module surface used by the reference driver ------------------------------------------
    def train(self, mode=True):
        return self

    def eval(self):
        return self

    def cuda(self, *a, **k):
        return self

    def cpu(self):
        return self

    def zero_grad(self):
        pass

    def state_dict(self):
        out = {}
        for k, (name, shape) in enumerate(zip(self.names, self._shapes)):
            a = np.empty(shape, dtype=np.float32)
            _lib.check(self._L.ncf_get_param(self._h, k, _lib.ptr(a)))
            out[name] = a
        return out

    def load_state_dict(self, state):
        for k, (name, shape) in enumerate(zip(self.names, self._shapes)):
            if name not in state:
                continue
            a = np.ascontiguousarray(np.asarray(state[name], dtype=np.float32).reshape(shape))
            _lib.check(self._L.ncf_set_param(self._h, k, _lib.ptr(a)))

    # -- data ------------------------------------------------------------------------------------
    def set_train(self, train_set):
        """Positives [[u, i], ...] (NCFData features / load_mat train list)."""
        if hasattr(train_set, "features_ps"):
            train_set = train_set.features_ps
        a = np.asarray(train_set)
        u = np.ascontiguousarray(a[:, 0], dtype=np.int32)
        i = np.ascontiguousarray(a[:, 1], dtype=np.int32)
        _lib.check(self._L.ncf_set_train(self._h, _lib.ptr(u), _lib.ptr(i), len(u)))
        self._has_train = True
        return self

    def epoch_size(self):
        n, s = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.ncf_epoch_size(self._h, ctypes.byref(n), ctypes.byref(s)))
        return n.value, s.value

    def sample(self, epoch, first=0, n=None):
        if n is None:
            n = self.epoch_size()[0] - first
        u, i = np.empty(n, np.int32), np.empty(n, np.int32)
        y = np.empty(n, np.float32)
        _lib.check(self._L.ncf_sample(self._h, int(epoch), int(first), int(n), _lib.ptr(u),
                                      _lib.ptr(i), _lib.ptr(y)))
        return u, i, y

    # -- training --------------------------------------------------------------------------------
    def fit(self, train_set=None, epochs=None):
        if train_set is not None:
            self.set_train(train_set)
        if not self._has_train:
            raise ValueError("fit() needs a train_set")
        for _ in range(self.epochs if epochs is None else int(epochs)):
            self.train_epoch()
        return self

    def train_epoch(self, epoch=None):
        e = self.epoch if epoch is None else int(epoch)
        st = _lib.Stats()
        _lib.check(self._L.ncf_train_epoch(self._h, e, ctypes.byref(st)))
        self.epoch = e + 1
        d = st.as_dict()
        self.history.append(d)
        return d

    def train_steps(self, epoch, first_step, n_steps):
        st = _lib.Stats()
        _lib.check(self._L.ncf_train_steps(self._h, int(epoch), int(first_step), int(n_steps),
                                           ctypes.byref(st)))
        return st.as_dict()

    def train_samples(self, user, item, label):
        """Replay reference-format samples in order, batch_size per Adam step; returns stats with
        loss = the sum of the steps' mean BCE losses."""
        u = np.ascontiguousarray(np.asarray(user).reshape(-1), dtype=np.int32)
        i = np.ascontiguousarray(np.asarray(item).reshape(-1), dtype=np.int32)
        y = np.ascontiguousarray(np.asarray(label).reshape(-1), dtype=np.float32)
        st = _lib.Stats()
        _lib.check(self._L.ncf_train_samples(self._h, _lib.ptr(u), _lib.ptr(i), _lib.ptr(y),
                                             len(u), ctypes.byref(st)))
        return st.as_dict()

    # -- scoring ---------------------------------------------------------------------------------
    def predict_logits(self, users, items):
        u = np.ascontiguousarray(np.asarray(users).reshape(-1), dtype=np.int32)
        i = np.ascontiguousarray(np.asarray(items).reshape(-1), dtype=np.int32)
        if len(u) != len(i):
            raise ValueError("users and items must have the same length")
        out = np.empty(len(u), np.float32)
        _lib.check(self._L.ncf_predict(self._h, _lib.ptr(u), _lib.ptr(i), len(u), _lib.ptr(out)))
        return out

    def forward(self, user, item):
        """NCF.forward (NCFRecommender.py:103-124): prediction logits, shape [B] (view(-1))."""
        import torch
        u = torch.as_tensor(user)
        dev = u.device
        z = self.predict_logits(u.reshape(-1).cpu().numpy(), torch.as_tensor(item).reshape(-1).cpu().numpy())
        return torch.from_numpy(z).to(dev)

    __call__ = forward

    def active_rows(self):
        """(users, items) whose embedding rows Adam moves every step (ever touched)."""
        u, i = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.ncf_active_rows(self._h, ctypes.byref(u), ctypes.byref(i)))
        return u.value, i.value

    def profile(self, enable=True):
        _lib.check(self._L.ncf_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        kp = _lib.KProf()
        _lib.check(self._L.ncf_profile_read(self._h, ctypes.byref(kp)))
        return {k: dict(count=int(kp.count[n]), ms=float(kp.ms[n]))
                for n, k in enumerate(("sample", "fwd_bwd", "adam", "catch_up"))}


class NCFData:
    """util/data_loader.py:931-972 drop-in: (user, item, label) samples; ng_sample() draws the
    negatives with the device sampler of an NCF handle (a new epoch order per call)."""

    def __init__(self, features, num_item, train_mat=None, num_ng=0, is_training=None, seed=0,
                 device=0):
        self.features_ps = [list(map(int, x[:2])) for x in features]
        self.num_item = int(num_item)
        self.train_mat = train_mat
        self.num_ng = int(num_ng)
        self.is_training = is_training
        self.labels = [0 for _ in range(len(self.features_ps))]
        self._epoch = 0
        self._seed, self._device = seed, device
        self.features_fill, self.labels_fill = None, None

    def ng_sample(self):
        assert self.is_training, "no need to sampling when testing"
        pos = np.asarray(self.features_ps, dtype=np.int64).reshape(-1, 2)
        users = int(pos[:, 0].max()) + 1 if len(pos) else 1
        if self.train_mat is not None:
            keys = list(self.train_mat.keys())
            if keys:
                users = max(users, max(int(k[0]) for k in keys) + 1)
        m = NCF(users, self.num_item, 4, 1, model="GMF", num_ng=self.num_ng,
                batch_size=256, seed=self._seed, device=self._device)
        m.set_train(pos)
        n = len(pos) * (1 + self.num_ng)
        u, i, y = m.sample(self._epoch, 0, n)
        m.close()
        self._epoch += 1
        # the reference lists positives first, then negatives; the shuffle is the DataLoader's
        neg = y == 0
        self.features_fill = self.features_ps + [[int(a), int(b)] for a, b in zip(u[neg], i[neg])]
        self.labels_fill = [1] * len(self.features_ps) + [0] * int(neg.sum())

    def __len__(self):
        return (self.num_ng + 1) * len(self.labels)

    def __getitem__(self, idx):
        features = self.features_fill if self.is_training else self.features_ps
        labels = self.labels_fill if self.is_training else self.labels
        return features[idx][0], features[idx][1], labels[idx]
