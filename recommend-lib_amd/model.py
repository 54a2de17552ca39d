"""BPRMF — the drop-in model object of the MI355X BPR-MF path.

Mirrors, in one object, the three parts of the reference contract:
  * `BPR(user_num, item_num, factor_num)` + `forward(user, item_i, item_j) -> (pred_i, pred_j)`
    (BPRMFRecommender.py:28-50), so util/metrics.py:46-66 `_bpr_topk` and the KPI loop of
    BPRMFRecommender.py:196-207 run unchanged;
  * the training loop of BPRMFRecommender.py:154-178 (SGD(lr, weight_decay), sum-of-log-sigmoid
    loss, `ng_sample()` + shuffled DataLoader every epoch) as `fit()` / `train_epoch()`;
  * the `fit(train_set)` / `predict(u, i)` convention of util/matrix_factorization.pyx:81-167
    (`predict` raises ValueError('Invalid user code' / 'Invalid item code')).
All compute runs in libbprmf_amd.so (HIP, gfx950).  Tables live in HBM; the host only sees them
through get_weights() / embed_user.weight / embed_item.weight.
"""
import ctypes
from types import SimpleNamespace

import numpy as np

from . import _lib


def _as_pairs(train_set):
    """Accept list of [u,i], ndarray [n,>=2], DataFrame(user,item,...) or a BPRData."""
    if hasattr(train_set, "features") and hasattr(train_set, "num_item"):
        train_set = train_set.features
    if hasattr(train_set, "columns"):  # pandas DataFrame, matrix_factorization.pyx:104 style
        u = np.asarray(train_set["user"].values)
        i = np.asarray(train_set["item"].values)
        return u.astype(np.int32), i.astype(np.int32)
    a = np.asarray(train_set)
    if a.ndim != 2 or a.shape[1] < 2:
        if a.size == 0:
            return np.zeros(0, np.int32), np.zeros(0, np.int32)
        raise ValueError("train_set must be pairs [[user, item], ...]")
    return np.ascontiguousarray(a[:, 0], dtype=np.int32), np.ascontiguousarray(a[:, 1], dtype=np.int32)


# step semantics (include/bprmf.h BPRMF_SEM_*): "exact" is the reference's batch-synchronous SGD
# (the default); "hogwild" is the opt-in relaxed mode (lock-free per-triplet updates, weight decay
# still once per row per step; single GPU); "local" is hogwild with the hot items
# in per-XCD replicas merged every local_steps steps
SEMANTICS = {"exact": 0, "hogwild": 1, "local": 2, "stale1": 3}
# how an exact step sums duplicate rows (include/bprmf.h BPRMF_STEP_*): "segmented" = sorted,
# one writer per row, bitwise reproducible (batch_size <= 8192); "atomic" = f32 atomics, any batch
# size, the same step up to the order of the fp32 sums
STEP_MODES = {"segmented": 0, "atomic": 1}


class BPRMF:
    """BPR matrix factorisation trained on one MI355X (or one shard of a multi-GPU run).

    Parameters follow the reference CLI (BPRMFRecommender.py:53-116): lr=0.01, wd=0.001,
    batch_size=4096, epochs=20, factor_num=32, num_ng=4; init N(0, 0.01^2) (:39-40).
    `seed` makes init, negative sampling and the epoch shuffle reproducible (the reference is
    unseeded).  `semantics="hogwild"` opts into relaxed synchronisation (not the reference's
    step; faster, nondeterministic; see DESIGN.md §5b for its HR@10 / NDCG@10 against exact).
    `semantics="local"`: hogwild for users and cold items, the hot items trained in one replica
    per XCD and merged every `local_steps` steps (default 128; bounded staleness).
    With world > 1 and `semantics="local"` the handle keeps its users' rows but the WHOLE item
    table, merged with the other ranks every `dp_steps` steps (default 256) and at every call's end
    (sharded.ShardedBPRMF drives it); `dp_overlap=True` runs each merge's
    all-reduce beside the next period and adds its sum one period later.
    `step="atomic"` sums duplicate rows with f32 atomics instead of the sorted one-writer sums
    (any batch size; the reference step up to fp32 summation order, not bitwise reproducible).
    """

    def __init__(self, user_num, item_num, factor_num=32, lr=0.01, wd=0.001, batch_size=4096,
                 num_ng=4, epochs=20, init_std=0.01, seed=0, device=0, rank=0, world=1,
                 verbose=False, semantics="exact", step="segmented", local_steps=0,
                 dp_steps=0, dp_overlap=False):
        self.user_num, self.item_num = int(user_num), int(item_num)
        self.factor_num = int(factor_num)
        self.lr, self.wd = float(lr), float(wd)
        self.batch_size, self.num_ng, self.epochs = int(batch_size), int(num_ng), int(epochs)
        self.seed, self.device = int(seed), int(device)
        self.rank, self.world = int(rank), int(world)
        self.verbose = verbose
        if semantics not in SEMANTICS:
            raise ValueError(f"semantics must be one of {sorted(SEMANTICS)}")
        self.semantics = semantics
        if step not in STEP_MODES:
            raise ValueError(f"step must be one of {sorted(STEP_MODES)}")
        self.step_mode = step
        self.epoch = 0
        self.history = []
        L = _lib.load()
        cfg = _lib.Config(user_num=self.user_num, item_num=self.item_num,
                          factor_num=self.factor_num, lr=self.lr, weight_decay=self.wd,
                          batch_size=self.batch_size, num_ng=self.num_ng, init_std=float(init_std),
                          seed=self.seed & (2**64 - 1), device=self.device, rank=self.rank,
                          world=self.world, semantics=SEMANTICS[semantics],
                          step_mode=STEP_MODES[step], local_steps=int(local_steps),
                          dp_steps=int(dp_steps), dp_overlap=int(bool(dp_overlap)))
        h = ctypes.c_void_p()
        _lib.check(L.bprmf_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._L = L
        self._has_train = False

    # -- lifecycle -----------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.bprmf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream):
        """Run on a hipStream_t (int) or a torch.cuda.Stream; None = own stream."""
        s = getattr(stream, "cuda_stream", stream)
        _lib.check(self._L.bprmf_set_stream(self._h, ctypes.c_void_p(s) if s else None))

    def synchronize(self):
        _lib.check(self._L.bprmf_synchronize(self._h))

    # -- drop-in no-ops of nn.Module used by the reference driver --------------------------------
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

    # -- data ----------------------------------------------------------------------------------
    def set_train(self, train_set, exclude=None):
        """Positives in features order; `exclude` = extra (users, items) never drawn as negatives
        (the keys of a train_mat larger than the features list)."""
        if hasattr(train_set, "features") and hasattr(train_set, "num_item") and exclude is None:
            from .data import train_mat_pairs
            exclude = train_mat_pairs(getattr(train_set, "train_mat", None))
        u, i = _as_pairs(train_set)
        if exclude is None:
            eu = ei = np.zeros(0, dtype=np.int32)
        else:
            eu = np.ascontiguousarray(exclude[0], dtype=np.int32)
            ei = np.ascontiguousarray(exclude[1], dtype=np.int32)
        _lib.check(self._L.bprmf_set_train_ex(self._h, _lib.ptr(u), _lib.ptr(i), len(u),
                                              _lib.ptr(eu), _lib.ptr(ei), len(eu)))
        self._has_train = True
        return self

    def epoch_size(self):
        n, s = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.bprmf_epoch_size(self._h, ctypes.byref(n), ctypes.byref(s)))
        return n.value, s.value

    @property
    def steps_taken(self):
        t = ctypes.c_int64()
        _lib.check(self._L.bprmf_step_count(self._h, ctypes.byref(t)))
        return t.value

    # -- training ------------------------------------------------------------------------------
    def fit(self, train_set=None, epochs=None):
        """ng_sample + shuffled batches + SGD(weight_decay) for `epochs` epochs
        (BPRMFRecommender.py:157-178).  Returns self (matrix_factorization.pyx:104 convention)."""
        if train_set is not None:
            self.set_train(train_set)
        if not self._has_train:
            raise ValueError("fit() needs a train_set")
        for _ in range(self.epochs if epochs is None else int(epochs)):
            st = self.train_epoch()
            if self.verbose:
                print(f"epoch {self.epoch:03d}: loss {st['loss']:.4f} "
                      f"{st['triplets'] / max(st['seconds'], 1e-12):.3e} triplets/s")
        return self

    def train_epoch(self, epoch=None):
        e = self.epoch if epoch is None else int(epoch)
        st = _lib.Stats()
        _lib.check(self._L.bprmf_train_epoch(self._h, e, ctypes.byref(st)))
        self.epoch = e + 1
        d = st.as_dict()
        self.history.append(d)
        return d

    def train_steps(self, epoch, first_step, n_steps):
        st = _lib.Stats()
        _lib.check(self._L.bprmf_train_steps(self._h, int(epoch), int(first_step), int(n_steps),
                                             ctypes.byref(st)))
        return st.as_dict()

    def train_triplets(self, user, item_i, item_j):
        """Replay reference-format triplets (BPRData __getitem__ order), batch_size per step."""
        if hasattr(user, "is_cuda") and user.is_cuda:
            import torch
            u, i, j = (x.to(torch.int32).contiguous() for x in (user, item_i, item_j))
            st = _lib.Stats()
            _lib.check(self._L.bprmf_train_triplets_dev(self._h, u.data_ptr(), i.data_ptr(),
                                                        j.data_ptr(), u.numel(), ctypes.byref(st)))
            return st.as_dict()
        u, i, j = (np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.int32)
                   for x in (user, item_i, item_j))
        if not (len(u) == len(i) == len(j)):
            raise ValueError("user, item_i, item_j must have the same length")
        st = _lib.Stats()
        _lib.check(self._L.bprmf_train_triplets(self._h, _lib.ptr(u), _lib.ptr(i), _lib.ptr(j),
                                                len(u), ctypes.byref(st)))
        return st.as_dict()

    def sample(self, epoch, first=0, n=None):
        """The device sampler's triplets for slots [first, first+n) of `epoch` (host arrays)."""
        N, _ = self.epoch_size()
        n = N - first if n is None else int(n)
        out = [np.empty(n, dtype=np.int32) for _ in range(3)]
        _lib.check(self._L.bprmf_sample(self._h, int(epoch), int(first), n, *map(_lib.ptr, out)))
        return tuple(out)

    # -- measurement ---------------------------------------------------------------------------
    def profile(self, enable=True):
        """Start (and reset) / stop live HIP-event timing of every kernel launch."""
        _lib.check(self._L.bprmf_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        k = _lib.KProf()
        _lib.check(self._L.bprmf_profile_read(self._h, ctypes.byref(k)))
        return k.as_dict()

    # -- test hooks ----------------------------------------------------------------------------
    def debug_fill_batches(self, value):
        """Fill the batch buffer with int32 `value` (deliberately stale memory; tests only)."""
        v = int(value) & 0xFFFFFFFF
        _lib.check(self._L.bprmf_debug_fill_batches(self._h, v - (1 << 32) if v >> 31 else v))

    def debug_fail_build(self):
        """Leave the batches as a timed-out build would (tests only): the next call fails."""
        _lib.check(self._L.bprmf_debug_fail_build(self._h))

    # -- weights -------------------------------------------------------------------------------
    def local_rows(self):
        u, i = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.bprmf_local_rows(self._h, ctypes.byref(u), ctypes.byref(i)))
        return u.value, i.value

    def get_weights(self):
        """(P [users, d], Q [items, d]) fp32 with all pending weight decay applied."""
        U, I = self.local_rows()
        P = np.empty((U, self.factor_num), dtype=np.float32)
        Q = np.empty((I, self.factor_num), dtype=np.float32)
        _lib.check(self._L.bprmf_get_weights(self._h, _lib.ptr(P), _lib.ptr(Q)))
        return P, Q

    def get_rows(self, table, rows):
        """Rows of embed_user (table 'user' / 0) or embed_item ('item' / 1) as of the current step,
        [len(rows), factor_num] fp32; rows are local row ids.  Reads only those rows (no flush)."""
        t = {"user": 0, "item": 1}.get(table, table)
        r = np.ascontiguousarray(np.asarray(rows).reshape(-1), dtype=np.int32)
        out = np.empty((len(r), self.factor_num), dtype=np.float32)
        _lib.check(self._L.bprmf_get_rows(self._h, int(t), _lib.ptr(r), len(r), _lib.ptr(out)))
        return out

    def set_weights(self, P, Q):
        U, I = self.local_rows()
        P = np.ascontiguousarray(P, dtype=np.float32)
        Q = np.ascontiguousarray(Q, dtype=np.float32)
        if P.shape != (U, self.factor_num) or Q.shape != (I, self.factor_num):
            raise ValueError(f"expected P {(U, self.factor_num)} and Q {(I, self.factor_num)}")
        _lib.check(self._L.bprmf_set_weights(self._h, _lib.ptr(P), _lib.ptr(Q)))

    @property
    def embed_user(self):
        import torch
        return SimpleNamespace(weight=torch.from_numpy(self.get_weights()[0]))

    @property
    def embed_item(self):
        import torch
        return SimpleNamespace(weight=torch.from_numpy(self.get_weights()[1]))

    def save(self, path):
        P, Q = self.get_weights()
        np.savez(path, embed_user=P, embed_item=Q, steps=self.steps_taken, epoch=self.epoch)

    # -- scoring -------------------------------------------------------------------------------
    def predict(self, u, i):
        """Scalar <P_u, Q_i>; ValueError on out-of-range codes (matrix_factorization.pyx:157-161)."""
        if int(u) >= self.user_num or int(u) < 0:
            raise ValueError("Invalid user code")
        if int(i) >= self.item_num or int(i) < 0:
            raise ValueError("Invalid item code")
        return float(self.score(np.array([u]), np.array([i]))[0])

    def score(self, users, items):
        u = np.ascontiguousarray(np.asarray(users).reshape(-1), dtype=np.int32)
        i = np.ascontiguousarray(np.asarray(items).reshape(-1), dtype=np.int32)
        if len(u) != len(i):
            raise ValueError("users and items must have the same length")
        out = np.empty(len(u), dtype=np.float32)
        _lib.check(self._L.bprmf_score(self._h, _lib.ptr(u), _lib.ptr(i), len(u), _lib.ptr(out)))
        return out

    def topk_lists(self, users, lists, k):
        """Per user, the k best of its candidate list (one device launch for all users): positions
        into the list and scores, score descending, ties by the later position first (what
        np.argsort(pred)[::-1][:k] ranks, BPRMFRecommender.py:196-207); -1 / -inf past the end.
        users: [n]; lists: n sequences of item ids (or (offsets[n+1], flat items))."""
        u = np.ascontiguousarray(np.asarray(users).reshape(-1), dtype=np.int32)
        if isinstance(lists, tuple) and len(lists) == 2:
            offs = np.ascontiguousarray(lists[0], dtype=np.int64)
            flat = np.ascontiguousarray(lists[1], dtype=np.int32)
        else:
            lens = np.fromiter((len(x) for x in lists), dtype=np.int64, count=len(lists))
            offs = np.zeros(len(lists) + 1, dtype=np.int64)
            np.cumsum(lens, out=offs[1:])
            flat = (np.concatenate([np.asarray(x, dtype=np.int32).reshape(-1) for x in lists])
                    if len(lists) else np.zeros(0, np.int32))
            flat = np.ascontiguousarray(flat, dtype=np.int32)
        if len(offs) != len(u) + 1:
            raise ValueError("one candidate list per user")
        pos = np.empty((len(u), int(k)), dtype=np.int32)
        sc = np.empty((len(u), int(k)), dtype=np.float32)
        _lib.check(self._L.bprmf_topk_lists(self._h, _lib.ptr(u), _lib.ptr(offs), _lib.ptr(flat),
                                            len(u), int(k), _lib.ptr(pos), _lib.ptr(sc)))
        return pos, sc

    def topk_all(self, users, k, exclude_train=True):
        """The k best items of the whole catalogue per user (scores on f32 MFMA), skipping the
        user's training positives unless exclude_train=False: (items [n, k], scores [n, k]),
        score descending, ties by the smaller item; -1 / -inf when fewer items remain."""
        u = np.ascontiguousarray(np.asarray(users).reshape(-1), dtype=np.int32)
        items = np.empty((len(u), int(k)), dtype=np.int32)
        sc = np.empty((len(u), int(k)), dtype=np.float32)
        _lib.check(self._L.bprmf_topk_all(self._h, _lib.ptr(u), len(u), int(k),
                                          1 if exclude_train else 0, _lib.ptr(items), _lib.ptr(sc)))
        return items, sc

    def forward(self, user, item_i, item_j=None):
        """BPR.forward (BPRMFRecommender.py:42-50): int64 tensors (0-d or [B]) -> fp32 (pred_i, pred_j).
        CUDA inputs stay on the GPU; CPU inputs are scored on the GPU and returned on CPU."""
        import torch
        if item_j is None:
            item_j = item_i
        user, item_i, item_j = (torch.as_tensor(x) for x in (user, item_i, item_j))
        shape = user.shape
        back_to_cpu = not user.is_cuda
        dev = torch.device("cuda", self.device)
        u, i, j = (x.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
                   for x in (user, item_i, item_j))
        if not (u.numel() == i.numel() == j.numel()):
            raise ValueError("user, item_i, item_j must have the same number of elements")
        oi = torch.empty(u.numel(), dtype=torch.float32, device=dev)
        oj = torch.empty_like(oi)
        # the library runs on a dedicated non-default stream ordered after the caller's (torch's
        # default stream is handle 0, which bprmf_set_stream reads as "own stream", unordered)
        caller = torch.cuda.current_stream(dev)
        if getattr(self, "_fwd_stream", None) is None:
            self._fwd_stream = torch.cuda.Stream(dev)
        s = self._fwd_stream
        s.wait_stream(caller)
        self.set_stream(s)
        try:
            _lib.check(self._L.bprmf_forward_dev(self._h, u.data_ptr(), i.data_ptr(), j.data_ptr(),
                                                 u.numel(), oi.data_ptr(), oj.data_ptr()))
        finally:
            self.set_stream(None)
        caller.wait_stream(s)
        for t in (u, i, j, oi, oj):
            t.record_stream(s)
        oi, oj = oi.reshape(shape), oj.reshape(shape)
        if back_to_cpu:
            oi, oj = oi.cpu(), oj.cpu()
        return oi, oj

    __call__ = forward
