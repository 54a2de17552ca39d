"""ORACLE (test infrastructure only) — ctypes binding of oracle/bpr_cpu.c (liboracle_bpr.so).

Used by tests/ as a checker and by bench.py's cpu_baseline leg as the timed CPU port.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BPRMF_ORACLE_LIB_DIR: prebuilt variants of the same sources (tests/sanitize: ASan + UBSan)
LIB_DIR = os.environ.get("BPRMF_ORACLE_LIB_DIR") or HERE
LIB = os.path.join(LIB_DIR, "liboracle_bpr.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


def build():
    src = os.path.join(HERE, "bpr_cpu.c")
    if LIB_DIR == HERE and (not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src)):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        L.oracle_sample.argtypes = [_i32p, _i32p, ctypes.c_int64, _i64p, _i32p, ctypes.c_int64,
                                    ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                                    ctypes.c_int64, _i32p, _i32p, _i32p]
        L.oracle_sample.restype = ctypes.c_int
        L.oracle_step_dense.argtypes = [_f32p, _f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                        _i32p, _i32p, _i32p, ctypes.c_int64, ctypes.c_float,
                                        ctypes.c_float, _f32p, _f32p]
        L.oracle_step_dense.restype = ctypes.c_double
        L.oracle_permute.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.oracle_permute.restype = ctypes.c_uint64
        L.oracle_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def sample(pos_u, pos_i, indptr, indices, item_num, num_ng, seed, epoch, first, count):
    L = lib()
    pos_u = np.ascontiguousarray(pos_u, dtype=np.int32)
    pos_i = np.ascontiguousarray(pos_i, dtype=np.int32)
    out = [np.empty(count, dtype=np.int32) for _ in range(3)]
    rc = L.oracle_sample(pos_u, pos_i, len(pos_u), np.ascontiguousarray(indptr, dtype=np.int64),
                         np.ascontiguousarray(indices, dtype=np.int32), int(item_num), int(num_ng),
                         int(seed) & (2**64 - 1), int(epoch), int(first), int(count), *out)
    if rc != 0:
        raise ValueError("user with no negative item")
    return tuple(out)


class DenseTrainer:
    """The reference step on CPU (dense grads + dense weight decay), tables in float32."""

    def __init__(self, P, Q, lr, wd):
        self.P = np.ascontiguousarray(P, dtype=np.float32)
        self.Q = np.ascontiguousarray(Q, dtype=np.float32)
        self.gP = np.empty_like(self.P)
        self.gQ = np.empty_like(self.Q)
        self.lr, self.wd = float(lr), float(wd)

    def step(self, u, i, j):
        u = np.ascontiguousarray(u, dtype=np.int32)
        i = np.ascontiguousarray(i, dtype=np.int32)
        j = np.ascontiguousarray(j, dtype=np.int32)
        U, d = self.P.shape
        return lib().oracle_step_dense(self.P, self.Q, U, self.Q.shape[0], d, u, i, j, len(u),
                                       self.lr, self.wd, self.gP, self.gQ)


def threads():
    return int(lib().oracle_threads())


# ---- rating SGD (oracle/mf_cpu.c: util/matrix_factorization.pyx SVD / RSVD) ----------------------
_mf = None
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def mf_lib():
    global _mf
    if _mf is None:
        src = os.path.join(HERE, "mf_cpu.c")
        so = os.path.join(LIB_DIR, "liboracle_mf.so")
        if LIB_DIR == HERE and (not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src)):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(so)
        L.oracle_svd_epochs.argtypes = [ctypes.c_int64, _i32p, _i32p, _f64p, ctypes.c_int,
                                        ctypes.c_double, ctypes.c_int, _f64p, _f64p, _f64p, _f64p,
                                        _f64p, _f64p, ctypes.c_int]
        L.oracle_rsvd_epochs.argtypes = [ctypes.c_int64, _i32p, _i32p, _f64p, ctypes.c_int,
                                         ctypes.c_double, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, _f64p, _f64p, _f64p,
                                         _f64p, ctypes.c_int]
        L.oracle_svdpp_epochs.argtypes = [ctypes.c_int64, _i32p, _i32p, _f64p, ctypes.c_int,
                                          ctypes.c_double, _f64p, _f64p, _f64p, _f64p, _f64p,
                                          _f64p, _f64p, _i64p, _i32p, _f64p, ctypes.c_int]
        _mf = L
    return _mf


def svd_epochs(u, i, r, P, Q, bu, bi, gm, biased, lr, reg, epochs):
    """SVD.fit epochs on copies of the tables; returns (P, Q, bu, bi)."""
    P, Q = np.array(P, np.float64, order="C"), np.array(Q, np.float64, order="C")
    bu, bi = np.array(bu, np.float64), np.array(bi, np.float64)
    mf_lib().oracle_svd_epochs(len(u), np.ascontiguousarray(u, np.int32),
                               np.ascontiguousarray(i, np.int32), np.ascontiguousarray(r, np.float64),
                               P.shape[1], float(gm), int(biased), np.asarray(lr, np.float64),
                               np.asarray(reg, np.float64), P, Q, bu, bi, int(epochs))
    return P, Q, bu, bi


def rsvd_epochs(u, i, r, P, Q, bu, bi, gm, version, lr, reg, reg2, epochs):
    """RSVD.fit epochs (as when verbose) on copies; returns (ui, vj, ci, dj)."""
    P, Q = np.array(P, np.float64, order="C"), np.array(Q, np.float64, order="C")
    bu, bi = np.array(bu, np.float64), np.array(bi, np.float64)
    mf_lib().oracle_rsvd_epochs(len(u), np.ascontiguousarray(u, np.int32),
                                np.ascontiguousarray(i, np.int32),
                                np.ascontiguousarray(r, np.float64), P.shape[1], float(gm),
                                int(version), float(lr), float(reg), float(reg2), P, Q, bu, bi,
                                int(epochs))
    return P, Q, bu, bi


def user_items(u, i, U):
    """ur of SVDpp.fit (:222-224): each user's items in train-set order, as CSR (uoff, uitems)."""
    u = np.asarray(u, np.int64)
    order = np.argsort(u, kind="stable")
    uoff = np.zeros(U + 1, np.int64)
    np.add.at(uoff, u + 1, 1)
    return np.cumsum(uoff), np.ascontiguousarray(np.asarray(i, np.int32)[order])


def svdpp_epochs(u, i, r, P, Q, Y, bu, bi, gm, lr, reg, epochs):
    """SVDpp.fit epochs on copies of the tables; returns (P, Q, Y, bu, bi)."""
    P, Q, Y = (np.array(x, np.float64, order="C") for x in (P, Q, Y))
    bu, bi = np.array(bu, np.float64), np.array(bi, np.float64)
    uoff, uitems = user_items(u, i, P.shape[0])
    impl = np.zeros(P.shape[1])
    mf_lib().oracle_svdpp_epochs(len(u), np.ascontiguousarray(u, np.int32),
                                 np.ascontiguousarray(i, np.int32),
                                 np.ascontiguousarray(r, np.float64), P.shape[1], float(gm),
                                 np.asarray(lr, np.float64), np.asarray(reg, np.float64), P, Q, Y,
                                 bu, bi, uoff, uitems, impl, int(epochs))
    return P, Q, Y, bu, bi


def mf_levels(u, i, U, I):
    """The device's schedule (mf_capi.cpp:mf_set_train), restated: level(s) = 1 + the last level
    of s's user or item among earlier samples; returns (order, offsets) of the stable sort by
    level.  Running the samples in `order` must equal the sequential loop bit for bit."""
    lu = np.full(U, -1, np.int64)
    li = np.full(I, -1, np.int64)
    lvl = np.empty(len(u), np.int64)
    for s in range(len(u)):
        a, b = int(u[s]), int(i[s])
        lvl[s] = lu[a] = li[b] = max(lu[a], li[b]) + 1
    order = np.argsort(lvl, kind="stable")
    L = int(lvl.max()) + 1 if len(lvl) else 0
    off = np.searchsorted(lvl[order], np.arange(L + 1))
    return order, off
