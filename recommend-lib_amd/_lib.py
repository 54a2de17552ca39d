"""ctypes binding of libbprmf_amd.so (include/bprmf.h, ncf.h, mf.h, bprfm.h, sgns.h).

The HIP library is the only compute path: if it is missing or no GPU is visible, handle creation
raises — there is no CPU fallback in the product.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbprmf_amd.so")
# diagnostic variants only (tools/ubench_build.py loads a stamped build); never set by the product
if os.environ.get("BPRMF_DIAG_LIB"):
    LIB_PATH = os.environ["BPRMF_DIAG_LIB"]

E_INVALID, E_RANGE, E_HIP, E_STATE, E_NO_NEGATIVE, E_UNSUPPORTED = -1, -2, -3, -4, -5, -6


class BprmfError(RuntimeError):
    """A HIP / state failure inside libbprmf_amd."""


class Config(ctypes.Structure):
    _fields_ = [("user_num", ctypes.c_int64), ("item_num", ctypes.c_int64),
                ("factor_num", ctypes.c_int32), ("lr", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("batch_size", ctypes.c_int32),
                ("num_ng", ctypes.c_int32), ("init_std", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("device", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("world", ctypes.c_int32), ("semantics", ctypes.c_int32),
                ("step_mode", ctypes.c_int32), ("local_steps", ctypes.c_int32),
                ("dp_steps", ctypes.c_int32), ("dp_overlap", ctypes.c_int32)]


class NcfConfig(ctypes.Structure):  # ncf_config, include/ncf.h
    _fields_ = [("user_num", ctypes.c_int64), ("item_num", ctypes.c_int64),
                ("factor_num", ctypes.c_int32), ("num_layers", ctypes.c_int32),
                ("model", ctypes.c_int32), ("batch_size", ctypes.c_int32),
                ("num_ng", ctypes.c_int32), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("init_std", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("device", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 4)]


class Stats(ctypes.Structure):
    _fields_ = [("triplets", ctypes.c_int64), ("steps", ctypes.c_int64),
                ("loss", ctypes.c_double), ("seconds", ctypes.c_double)]

    def as_dict(self):
        return dict(triplets=self.triplets, steps=self.steps, loss=self.loss, seconds=self.seconds)


class KProf(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64 * 8), ("ms", ctypes.c_double * 8)]

    KINDS = ("sample", "user_step", "item_step", "owner_apply", "step_graph", "topk_all")

    def as_dict(self):
        return {k: dict(count=int(self.count[n]), ms=float(self.ms[n])) for n, k in enumerate(self.KINDS)}


IPC_BLOB_BYTES = 512  # BPRMF_IPC_BLOB_BYTES
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
# name -> argtypes (restype int unless noted); mirrors include/bprmf.h
SIGNATURES = {
    "bprmf_create": [ctypes.POINTER(Config), ctypes.POINTER(ctypes.c_void_p)],
    "bprmf_destroy": [_P],
    "bprmf_last_error": [],
    "bprmf_version": [],
    "bprmf_set_stream": [_P, _P],
    "bprmf_synchronize": [_P],
    "bprmf_set_train": [_P, _P, _P, _I64],
    "bprmf_set_train_ex": [_P, _P, _P, _I64, _P, _P, _I64],
    "bprmf_epoch_size": [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "bprmf_set_weights": [_P, _P, _P],
    "bprmf_get_weights": [_P, _P, _P],
    "bprmf_get_rows": [_P, ctypes.c_int32, _P, _I64, _P],
    "bprmf_local_rows": [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "bprmf_step_count": [_P, ctypes.POINTER(_I64)],
    "bprmf_train_epoch": [_P, ctypes.c_uint32, ctypes.POINTER(Stats)],
    "bprmf_train_steps": [_P, ctypes.c_uint32, _I64, _I64, ctypes.POINTER(Stats)],
    "bprmf_train_triplets": [_P, _P, _P, _P, _I64, ctypes.POINTER(Stats)],
    "bprmf_train_triplets_dev": [_P, _P, _P, _P, _I64, ctypes.POINTER(Stats)],
    "bprmf_sample": [_P, ctypes.c_uint32, _I64, _I64, _P, _P, _P],
    "bprmf_score": [_P, _P, _P, _I64, _P],
    "bprmf_forward_dev": [_P, _P, _P, _P, _I64, _P, _P],
    "bprmf_dist_plan": [_P, ctypes.c_uint32, _I64, _I64, _P],
    "bprmf_dist_plan_replay": [_P, _P, _P, _P, _I64, _P],
    "bprmf_dist_request_ids": [_P, _I64, _P, _I64],
    "bprmf_dist_gather_items": [_P, _P, _I64, _P],
    "bprmf_dist_user_step": [_P, _I64, _P],
    "bprmf_dist_item_grads": [_P, _I64, _P],
    "bprmf_dist_apply_items": [_P, _P, _P, _I64],
    "bprmf_dist_end_step": [_P, ctypes.POINTER(ctypes.c_double)],
    "bprmf_dist_sample_dev": [_P, ctypes.c_uint32, _I64, _I64, _P, _P, _P],
    "bprmf_topk_lists": [_P, _P, _P, _P, _I64, ctypes.c_int32, _P, _P],
    "bprmf_topk_all": [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32, _P, _P],
    "bprmf_dist_unique_id": [_P],
    "bprmf_dist_init_rccl": [_P, _P],
    "bprmf_dist_init_loopback": [_P, _I64],
    "bprmf_dist_ipc_export": [_P, _P],
    "bprmf_dist_init_ipc": [_P, _P],
    "bprmf_dist_train_steps": [_P, ctypes.c_uint32, _I64, _I64, _P],
    "bprmf_dist_train_replay": [_P, _P, _P, _P, _I64, _P],
    "bprmf_dist_exchange_stats": [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                                  ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "bprmf_row_stride": [_P, ctypes.POINTER(ctypes.c_int32)],
    "bprmf_dataset_load": [ctypes.c_char_p, ctypes.c_float, ctypes.c_int32, ctypes.c_int32,
                           ctypes.POINTER(ctypes.c_void_p)],
    "bprmf_dataset_info": [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "bprmf_dataset_copy": [_P, _P, _P, _P, _P, _P, _P],
    "bprmf_dataset_split": [_P, ctypes.c_int32, ctypes.c_double, _P],
    "bprmf_dataset_candidates": [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                 ctypes.POINTER(_I64), _P, _P],
    "bprmf_dataset_free": [_P],
    "bprmf_node_barrier_open": [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_void_p)],
    "bprmf_node_barrier_wait": [_P, ctypes.c_double],
    "bprmf_node_barrier_close": [_P],
    "bprmf_debug_next_build_tag": [ctypes.POINTER(ctypes.c_uint32)],
    "bprmf_debug_fill_batches": [_P, ctypes.c_int32],
    "bprmf_debug_fail_build": [_P],
    "bprmf_profile": [_P, ctypes.c_int32],
    "bprmf_profile_read": [_P, ctypes.POINTER(KProf)],
    # include/ncf.h
    "ncf_create": [ctypes.POINTER(NcfConfig), ctypes.POINTER(ctypes.c_void_p)],
    "ncf_destroy": [_P],
    "ncf_param_count": [_P, ctypes.POINTER(ctypes.c_int32)],
    "ncf_param_shape": [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
    "ncf_set_param": [_P, ctypes.c_int32, _P],
    "ncf_get_param": [_P, ctypes.c_int32, _P],
    "ncf_set_train": [_P, _P, _P, _I64],
    "ncf_epoch_size": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
    "ncf_train_samples": [_P, _P, _P, _P, _I64, _P],
    "ncf_train_steps": [_P, ctypes.c_uint32, _I64, _I64, _P],
    "ncf_train_epoch": [_P, ctypes.c_uint32, _P],
    "ncf_sample": [_P, ctypes.c_uint32, _I64, _I64, _P, _P, _P],
    "ncf_predict": [_P, _P, _P, _I64, _P],
    "ncf_active_rows": [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
    "ncf_profile": [_P, ctypes.c_int32],
    "ncf_profile_read": [_P, ctypes.POINTER(KProf)],
    # include/mf.h (mf_config / mf_stats: recommend-lib_amd/mf.py)
    "mf_create": [_P, ctypes.POINTER(ctypes.c_void_p)],
    "mf_destroy": [_P],
    "mf_set_train": [_P, _P, _P, _P, _I64, ctypes.c_double],
    "mf_set_weights": [_P, _P, _P, _P, _P],
    "mf_get_weights": [_P, _P, _P, _P, _P],
    "mf_fit": [_P, ctypes.c_int32, _P],
    "mf_predict": [_P, _P, _P, _I64, _P],
    "mf_set_implicit": [_P, _P],
    "mf_get_implicit": [_P, _P],
    # include/bprfm.h (bprfm_config / bprfm_stats: recommend-lib_amd/bprfm.py)
    "bprfm_create": [_P, ctypes.POINTER(ctypes.c_void_p)],
    "bprfm_destroy": [_P],
    "bprfm_set_weights": [_P, _P, _P, _P, _P, _P, _P, _P],
    "bprfm_get_weights": [_P, _P, _P, _P, _P, _P, _P, _P],
    "bprfm_train": [_P, _P, _P, _P, _I64, ctypes.c_int32, _P],
    "bprfm_dropout_mask": [_P, ctypes.c_int32, _P],
    "bprfm_predict": [_P, _P, _P, _I64, _P],
    "bprfm_steps": [_P],
    # include/sgns.h (sgns_config / sgns_stats: recommend-lib_amd/item2vec.py)
    "sgns_create": [_P, ctypes.POINTER(ctypes.c_void_p)],
    "sgns_destroy": [_P],
    "sgns_set_noise": [_P, _P],
    "sgns_set_weights": [_P, _P, _P],
    "sgns_get_weights": [_P, _P, _P],
    "sgns_set_adam": [_P, _I64, _P, _P, _P, _P],
    "sgns_get_adam": [_P, _P, _P, _P, _P, _P],
    "sgns_train": [_P, _P, _P, _P, _I64, ctypes.c_int32, _P],
    "sgns_negatives": [_P, ctypes.c_int32, _P],
    "sgns_lookup": [_P, ctypes.c_int32, _P, _I64, _P],
}
RESTYPES = {"bprmf_last_error": ctypes.c_char_p, "bprfm_steps": ctypes.c_int64}

_lib = None


def load():
    """Load (never build) the in-tree library; raise ImportError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    # torch links its bundled HIP runtime as "libamdhip64.so" (SONAME libamdhip64.so.7); loading
    # torch first lets our NEEDED libamdhip64.so.7 resolve to that same copy.  Loading ours first
    # would bring in a second HIP runtime and torch would then see no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    diag = bool(os.environ.get("BPRMF_DIAG_LIB"))
    for name, args in SIGNATURES.items():
        f = getattr(L, name, None)
        if f is None:
            # a diagnostic variant may hold a subset (tests/sanitize: the host-only ingestion)
            if diag:
                continue
            raise ImportError(f"{LIB_PATH} does not export {name}")
        f.argtypes = args
        f.restype = RESTYPES.get(name, ctypes.c_int)
    _lib = L
    return L


def next_build_tag():
    """The launch tag the process's next split batch build will carry (test hook)."""
    t = ctypes.c_uint32()
    check(load().bprmf_debug_next_build_tag(ctypes.byref(t)))
    return t.value


def check(rc):
    if rc == 0:
        return
    msg = (load().bprmf_last_error() or b"").decode(errors="replace")
    if rc in (E_INVALID, E_RANGE):
        raise ValueError(msg)
    if rc == E_NO_NEGATIVE:
        raise ValueError(msg)
    raise BprmfError(f"libbprmf_amd error {rc}: {msg}")


def ptr(a):
    """Raw address of a numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data
