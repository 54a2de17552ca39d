"""SVD / RSVD / SVDpp — drop-ins for the reference's Cython rating-SGD models.

`util/matrix_factorization.pyx` SVD (:81-167), RSVD (:5-78) and SVDpp (:169-287): the same
constructor arguments,
`fit(train_set)` with a DataFrame[user, item, rating] and `predict(u, i)` raising
ValueError('Invalid user code' / 'Invalid item code').  fit() draws the initial tables from
numpy's global RNG exactly as the reference does (np.random.normal, users then items) and
computes global_mean as train_set.rating.mean(); the epochs then run on the GPU
(include/mf.h, mf.hip) with results bit-identical to the Cython loop's.
"""
import ctypes

import numpy as np

from . import _lib


class MfConfig(ctypes.Structure):  # mf_config, include/mf.h
    _fields_ = [("user_num", ctypes.c_int64), ("item_num", ctypes.c_int64),
                ("n_factors", ctypes.c_int32), ("model", ctypes.c_int32),
                ("variant", ctypes.c_int32), ("device", ctypes.c_int32),
                ("lr", ctypes.c_double * 4), ("reg", ctypes.c_double * 4),
                ("lr_yj", ctypes.c_double), ("reg_yj", ctypes.c_double)]


class MfStats(ctypes.Structure):  # mf_stats
    _fields_ = [("samples", ctypes.c_int64), ("levels", ctypes.c_int64), ("seconds", ctypes.c_double)]


MF_SVD, MF_RSVD, MF_SVDPP = 0, 1, 2


def _rows(train_set):
    """(users, items, ratings, global_mean) in iterrows order; the mean as the reference takes it."""
    if hasattr(train_set, "columns"):
        u = np.asarray(train_set["user"].values)
        i = np.asarray(train_set["item"].values)
        r = np.asarray(train_set["rating"].values, dtype=np.float64)
        gm = float(train_set["rating"].mean())
    else:
        a = np.asarray(train_set)
        u, i, r = a[:, 0], a[:, 1], np.asarray(a[:, 2], dtype=np.float64)
        gm = float(r.mean()) if len(r) else float("nan")
    return (np.ascontiguousarray(u, np.int32), np.ascontiguousarray(i, np.int32),
            np.ascontiguousarray(r, np.float64), gm)


class _MF:
    _model = MF_SVD

    def _open(self, user_num, item_num, n_factors, variant, lr, reg, device, lr_yj=0.0, reg_yj=0.0):
        self._L = _lib.load()
        cfg = MfConfig(user_num=int(user_num), item_num=int(item_num), n_factors=int(n_factors),
                       model=self._model, variant=int(variant), device=int(device),
                       lr_yj=float(lr_yj), reg_yj=float(reg_yj))
        for x in range(4):
            cfg.lr[x] = float(lr[x])
            cfg.reg[x] = float(reg[x])
        h = ctypes.c_void_p()
        _lib.check(self._L.mf_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.last_stats = None

    def close(self):
        if getattr(self, "_h", None):
            self._L.mf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    def _run(self, train_set, P0, Q0, epochs, gm=None):
        u, i, r, mean = _rows(train_set)
        gm = mean if gm is None else gm
        _lib.check(self._L.mf_set_train(self._h, _lib.ptr(u), _lib.ptr(i), _lib.ptr(r), len(u),
                                        ctypes.c_double(gm)))
        P0 = np.ascontiguousarray(P0, np.float64)
        Q0 = np.ascontiguousarray(Q0, np.float64)
        _lib.check(self._L.mf_set_weights(self._h, _lib.ptr(P0), _lib.ptr(Q0), None, None))
        st = MfStats()
        _lib.check(self._L.mf_fit(self._h, int(epochs), ctypes.byref(st)))
        self.last_stats = dict(samples=st.samples, levels=st.levels, seconds=st.seconds)
        U, I, k = self.user_num, self.item_num, self.n_factors
        P, Q = np.empty((U, k)), np.empty((I, k))
        b1, b2 = np.empty(U), np.empty(I)
        _lib.check(self._L.mf_get_weights(self._h, _lib.ptr(P), _lib.ptr(Q), _lib.ptr(b1), _lib.ptr(b2)))
        return gm, P, Q, b1, b2

    def _check_ids(self, a, b):
        if a >= self.user_num:
            raise ValueError('Invalid user code')
        if b >= self.item_num:
            raise ValueError('Invalid item code')

    def predict_batch(self, users, items):
        """predict() for arrays of pairs, on the device (the dot product summed in factor order)."""
        u = np.ascontiguousarray(users, np.int32)
        i = np.ascontiguousarray(items, np.int32)
        out = np.empty(len(u), np.float64)
        _lib.check(self._L.mf_predict(self._h, _lib.ptr(u), _lib.ptr(i), len(u), _lib.ptr(out)))
        return out


class SVD(_MF):
    """util/matrix_factorization.pyx:81-167 (biased MF trained by per-sample SGD)."""
    _model = MF_SVD

    def __init__(self, user_num, item_num, n_factors=100, n_epochs=20, biased=True, init_mean=0,
                 init_std_dev=.1, lr_all=.005, reg_all=.02, lr_bu=None, lr_bi=None, lr_pu=None,
                 lr_qi=None, reg_bu=None, reg_bi=None, reg_pu=None, reg_qi=None, random_state=None,
                 verbose=True, device=0):
        self.user_num, self.item_num = user_num, item_num
        self.n_factors, self.n_epochs, self.biased = n_factors, n_epochs, biased
        self.init_mean, self.init_std_dev = init_mean, init_std_dev
        self.lr_bu = lr_bu if lr_bu is not None else lr_all
        self.lr_bi = lr_bi if lr_bi is not None else lr_all
        self.lr_pu = lr_pu if lr_pu is not None else lr_all
        self.lr_qi = lr_qi if lr_qi is not None else lr_all
        self.reg_bu = reg_bu if reg_bu is not None else reg_all
        self.reg_bi = reg_bi if reg_bi is not None else reg_all
        self.reg_pu = reg_pu if reg_pu is not None else reg_all
        self.reg_qi = reg_qi if reg_qi is not None else reg_all
        self.random_state, self.verbose = random_state, verbose
        self._open(user_num, item_num, n_factors, 1 if biased else 0,
                   (self.lr_bu, self.lr_bi, self.lr_pu, self.lr_qi),
                   (self.reg_bu, self.reg_bi, self.reg_pu, self.reg_qi), device)

    def fit(self, train_set):
        # :123-126: zero biases, N(init_mean, init_std_dev) tables from numpy's global RNG
        pu = np.random.normal(self.init_mean, self.init_std_dev, size=(self.user_num, self.n_factors))
        qi = np.random.normal(self.init_mean, self.init_std_dev, size=(self.item_num, self.n_factors))
        gm, self.pu, self.qi, self.bu, self.bi = self._run(train_set, pu, qi, self.n_epochs)
        self.global_mean = gm if self.biased else 0  # :128-131
        return self

    def predict(self, u, i):
        self._check_ids(u, i)
        if self.biased:
            return self.global_mean + self.bu[u] + self.bi[i] + np.dot(self.qi[i], self.pu[u])
        return np.dot(self.qi[i], self.pu[u])


class RSVD(_MF):
    """util/matrix_factorization.pyx:5-78 (regularised SVD, version 1 or 2 with biases).

    Mirrors the reference including its quirk that training runs only when verbose=True (the
    epoch loop sits inside `if self.verbose`, :41-44); pass train_when_quiet=True to train anyway.
    """
    _model = MF_RSVD

    def __init__(self, user_num, item_num, n_factors=96, n_epochs=20, version=2, init_mean=0,
                 init_std_dev=.1, lr=.001, reg=.02, reg2=.05, random_state=None, verbose=True,
                 device=0, train_when_quiet=False):
        self.user_num, self.item_num = user_num, item_num
        self.n_factors, self.n_epochs, self.version = n_factors, n_epochs, version
        self.init_mean, self.init_std_dev = init_mean, init_std_dev
        self.lr, self.reg, self.reg2 = lr, reg, reg2
        self.random_state, self.verbose = random_state, verbose
        self.train_when_quiet = train_when_quiet
        self._open(user_num, item_num, n_factors, version, (lr, 0, 0, 0), (reg, reg2, 0, 0), device)

    def fit(self, train_set):
        ui = np.random.normal(self.init_mean, self.init_std_dev, size=(self.user_num, self.n_factors))
        vj = np.random.normal(self.init_mean, self.init_std_dev, size=(self.item_num, self.n_factors))
        epochs = self.n_epochs if (self.verbose or self.train_when_quiet) else 0
        if self.verbose:
            for epoch in range(self.n_epochs):
                print(f'Processing epoch {epoch + 1}')
        _, self.ui, self.vj, self.ci, self.dj = self._run(train_set, ui, vj, epochs)
        return self

    def predict(self, i, j):
        self._check_ids(i, j)
        if self.version == 2:
            return self.ci[i] + self.dj[j] + np.dot(self.ui[i], self.vj[j])
        return np.dot(self.ui[i], self.vj[j])


class SVDpp(_MF):
    """util/matrix_factorization.pyx:169-287 (SVD++: implicit feedback y_j of the user's items).

    fit() draws pu, qi, yj from numpy's global RNG as the reference does (:218-221); the epochs
    run on the device sample by sample (include/mf.h), bit-identical to the Cython loop.
    """
    _model = MF_SVDPP

    def __init__(self, user_num, item_num, n_factors=20, n_epochs=20, init_mean=0, init_std_dev=.1,
                 lr_all=.007, reg_all=.02, lr_bu=None, lr_bi=None, lr_pu=None, lr_qi=None,
                 lr_yj=None, reg_bu=None, reg_bi=None, reg_pu=None, reg_qi=None, reg_yj=None,
                 random_state=None, verbose=True, device=0):
        self.user_num, self.item_num = user_num, item_num
        self.n_factors, self.n_epochs = n_factors, n_epochs
        self.init_mean, self.init_std_dev = init_mean, init_std_dev
        pick = lambda v: v if v is not None else lr_all  # noqa: E731
        self.lr_bu, self.lr_bi, self.lr_pu, self.lr_qi, self.lr_yj = (
            pick(lr_bu), pick(lr_bi), pick(lr_pu), pick(lr_qi), pick(lr_yj))
        pick = lambda v: v if v is not None else reg_all  # noqa: E731
        self.reg_bu, self.reg_bi, self.reg_pu, self.reg_qi, self.reg_yj = (
            pick(reg_bu), pick(reg_bi), pick(reg_pu), pick(reg_qi), pick(reg_yj))
        self.random_state, self.verbose = random_state, verbose
        self._open(user_num, item_num, n_factors, 1,
                   (self.lr_bu, self.lr_bi, self.lr_pu, self.lr_qi),
                   (self.reg_bu, self.reg_bi, self.reg_pu, self.reg_qi), device,
                   self.lr_yj, self.reg_yj)

    def fit(self, train_set):
        U, I, k = self.user_num, self.item_num, self.n_factors
        pu = np.random.normal(self.init_mean, self.init_std_dev, size=(U, k))
        qi = np.random.normal(self.init_mean, self.init_std_dev, size=(I, k))
        yj = np.random.normal(self.init_mean, self.init_std_dev, size=(I, k))
        u, i, r, _ = _rows(train_set)
        Y = np.ascontiguousarray(yj, np.float64)
        # ur (:222-224): each user's (item, rating) in train order
        self.ur = {}
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            self.ur.setdefault(a, []).append((b, c))
        if self.verbose:
            for epoch in range(self.n_epochs):
                print(f'processing epoch {epoch + 1}')
        # the tables and the train set go up first, then yj, then the epochs
        self._train_with_implicit(train_set, pu, qi, Y)
        return self

    def _train_with_implicit(self, train_set, pu, qi, Y):
        u, i, r, gm = _rows(train_set)
        _lib.check(self._L.mf_set_train(self._h, _lib.ptr(u), _lib.ptr(i), _lib.ptr(r), len(u),
                                        ctypes.c_double(gm)))
        P0 = np.ascontiguousarray(pu, np.float64)
        Q0 = np.ascontiguousarray(qi, np.float64)
        _lib.check(self._L.mf_set_weights(self._h, _lib.ptr(P0), _lib.ptr(Q0), None, None))
        _lib.check(self._L.mf_set_implicit(self._h, _lib.ptr(Y)))
        st = MfStats()
        _lib.check(self._L.mf_fit(self._h, int(self.n_epochs), ctypes.byref(st)))
        self.last_stats = dict(samples=st.samples, levels=st.levels, seconds=st.seconds)
        U, I, k = self.user_num, self.item_num, self.n_factors
        self.pu, self.qi, self.yj = np.empty((U, k)), np.empty((I, k)), np.empty((I, k))
        self.bu, self.bi = np.empty(U), np.empty(I)
        _lib.check(self._L.mf_get_weights(self._h, _lib.ptr(self.pu), _lib.ptr(self.qi),
                                          _lib.ptr(self.bu), _lib.ptr(self.bi)))
        _lib.check(self._L.mf_get_implicit(self._h, _lib.ptr(self.yj)))
        self.global_mean = gm

    def predict(self, u, i):
        est = self.global_mean
        self._check_ids(u, i)
        est += self.bu[u] + self.bi[i]
        Iu = len(self.ur.get(u, []))
        if Iu == 0:
            u_impl_feedback = 0
        else:
            u_impl_feedback = (sum(self.yj[j] for (j, _) in self.ur[u]) / np.sqrt(Iu))
        est += np.dot(self.qi[i], self.pu[u] + u_impl_feedback)
        return est
