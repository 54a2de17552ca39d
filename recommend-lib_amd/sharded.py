"""Multi-GPU BPR-MF: one process per GPU, users and items row-sharded, RCCL all-to-all.

North-star layout: user u lives on rank u % world and each rank samples triplets
only for its own users, so user-row updates stay local; item i lives on rank i % world (strided,
spreading Zipf-hot items).  Per step, on every rank:

  1. request_ids   distinct items of the local batch, owner-major (from the batch builder)
  2. all-to-all    ids -> owners
  3. gather_items  owners send their rows, brought to the current step (lazy decay applied)
  4. all-to-all    rows -> requesters
  5. user_step     local users vs received rows: c, user gradient, user rows updated in place
  6. item_grads    one gradient row per requested item (fixed-order sum of -/+ c*P_u)
  7. all-to-all    grads -> owners
  8. apply_items   owners sum the grads of every requester and apply SGD + weight decay

A step over the union of the ranks' batches is the reference step on that union (sums of
per-row gradients are order-independent up to fp rounding): G ranks x batch B == one GPU x G*B.
Exchange sizes are planned once per chunk of steps (one host sync per chunk, not per step).
The reference has no distributed code at all: this is the build's addition.
"""
import ctypes
import threading

import numpy as np

from . import _lib


# ------------------------------------------------------------------------------------------------
# communicators
# ------------------------------------------------------------------------------------------------

IPC_BUS_ID_OFF = 5 * 64  # csrc/dist.cpp: kIpcHandles hipIpcMemHandle_t (64 B), then the bus id

class TorchComm:
    """torch.distributed (backend "nccl" = RCCL on ROCm, or "gloo" for CPU tests)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)

    def _dev(self, like):
        import torch
        return like.device if self.backend != "gloo" else torch.device("cpu")

    def all_to_all(self, out, inp, out_splits, in_splits):
        self.dist.all_to_all_single(out, inp, [int(x) for x in out_splits],
                                    [int(x) for x in in_splits], group=self.group)

    def exchange_counts(self, counts, device):
        """counts[k][r] = rows this rank requests from r at step k -> recv[k][r] = rows r requests
        from this rank."""
        import torch
        n, w = counts.shape
        dev = torch.device("cpu") if self.backend == "gloo" else device
        send = torch.from_numpy(np.ascontiguousarray(counts.T)).to(dev)  # [w, n]
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send, group=self.group)
        return recv.cpu().numpy().T.copy()

    def allreduce_max(self, x, device):
        import torch
        dev = torch.device("cpu") if self.backend == "gloo" else device
        t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def all_gather_bytes(self, data, device):
        """every rank's bytes (equal lengths), in rank order."""
        import torch
        dev = torch.device("cpu") if self.backend == "gloo" else device
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [bytes(x.cpu().numpy().tobytes()) for x in out]

    def broadcast_bytes(self, data, device):
        """rank 0's bytes to every rank (the RCCL unique id of the library's communicator)."""
        import torch
        dev = torch.device("cpu") if self.backend == "gloo" else device
        t = torch.zeros(len(data), dtype=torch.uint8, device=dev)
        if self.rank == 0:
            t.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        src = self.dist.get_global_rank(self.group, 0) if self.group is not None else 0
        self.dist.broadcast(t, src=src, group=self.group)
        return bytes(t.cpu().numpy().tobytes())


class ThreadGroup:
    """Shared state of an in-process group: `world` shards stepped by `world` threads (used to run
    several shards on one GPU, e.g. to test the sharded kernels without a multi-GPU node)."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [[None] * world for _ in range(world)]
        self.vals = [None] * world


class ThreadComm:
    def __init__(self, group, rank):
        self.g = group
        self.rank = rank
        self.world = group.world

    def _sync(self):
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.g.barrier.wait()

    def all_to_all(self, out, inp, out_splits, in_splits):
        import torch
        offs = np.concatenate([[0], np.cumsum(in_splits)]).astype(int)
        for r in range(self.world):
            self.g.slots[self.rank][r] = inp[offs[r]:offs[r + 1]]
        self._sync()
        parts = [self.g.slots[r][self.rank] for r in range(self.world)]
        if out.numel():
            torch.cat(parts, dim=0, out=out)
        self._sync()

    def exchange_counts(self, counts, device):
        self.g.vals[self.rank] = counts
        self._sync()
        recv = np.stack([self.g.vals[r][:, self.rank] for r in range(self.world)], axis=1)
        self._sync()
        return recv.astype(np.int32)

    def allreduce_max(self, x, device):
        self.g.vals[self.rank] = int(x)
        self._sync()
        m = max(self.g.vals)
        self._sync()
        return m


# ------------------------------------------------------------------------------------------------
# the HIP shard backend (libbprmf_amd.so through the C ABI)
# ------------------------------------------------------------------------------------------------
class HipShard:
    """One shard's state in HBM and its step phases (include/bprmf.h, bprmf_dist_*)."""

    def __init__(self, user_num, item_num, factor_num, lr, wd, batch_size, num_ng, init_std, seed,
                 device, rank, world, semantics="exact", local_steps=0, dp_steps=0,
                 dp_overlap=False):
        from .model import BPRMF
        self.m = BPRMF(user_num, item_num, factor_num, lr=lr, wd=wd, batch_size=batch_size,
                       num_ng=num_ng, init_std=init_std, seed=seed, device=device, rank=rank,
                       world=world, semantics=semantics, local_steps=local_steps,
                       dp_steps=dp_steps, dp_overlap=dp_overlap)
        self.L, self.h = _lib.load(), self.m.handle
        ld = ctypes.c_int32()
        _lib.check(self.L.bprmf_row_stride(self.h, ctypes.byref(ld)))
        self.ld = ld.value
        self.batch_size = batch_size
        self.world = world
        import torch
        self.device = torch.device("cuda", device)

    def stream(self):
        """The dedicated (non-default) torch stream every per-step phase runs on.  The library
        and torch's collectives are ordered on it; binding torch's default stream instead would
        hand the library handle 0, which bprmf_set_stream reads as "the handle's own stream"."""
        import torch
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream(self.device)
        return self._stream

    def bind_stream(self):
        self.m.set_stream(self.stream())

    def set_train(self, pos):
        self.m.set_train(pos)
        return self.m.epoch_size()[1]

    def plan(self, epoch, first_step, n_steps):
        counts = np.empty((n_steps, self.world), dtype=np.int32)
        _lib.check(self.L.bprmf_dist_plan(self.h, int(epoch), int(first_step), int(n_steps),
                                          counts.ctypes.data))
        return counts

    def plan_replay(self, u, i, j, n_steps):
        counts = np.empty((n_steps, self.world), dtype=np.int32)
        u, i, j = (np.ascontiguousarray(x, dtype=np.int32) for x in (u, i, j))
        _lib.check(self.L.bprmf_dist_plan_replay(self.h, u.ctypes.data, i.ctypes.data,
                                                 j.ctypes.data, int(n_steps), counts.ctypes.data))
        return counts

    def request_ids(self, k, ids, n):
        _lib.check(self.L.bprmf_dist_request_ids(self.h, int(k), ids.data_ptr(), int(n)))

    def gather_items(self, rows, n, out):
        _lib.check(self.L.bprmf_dist_gather_items(self.h, rows.data_ptr(), int(n), out.data_ptr()))

    def user_step(self, k, item_rows):
        _lib.check(self.L.bprmf_dist_user_step(self.h, int(k), item_rows.data_ptr()))

    def item_grads(self, k, grads):
        _lib.check(self.L.bprmf_dist_item_grads(self.h, int(k), grads.data_ptr()))

    def apply_items(self, rows, grads, n):
        _lib.check(self.L.bprmf_dist_apply_items(self.h, rows.data_ptr(), grads.data_ptr(), int(n)))

    def end_step(self, want_loss=False):
        if not want_loss:
            _lib.check(self.L.bprmf_dist_end_step(self.h, None))
            return None
        loss = ctypes.c_double()
        _lib.check(self.L.bprmf_dist_end_step(self.h, ctypes.byref(loss)))
        return loss.value

    # -- the library-driven runner (bprmf_dist_init_* / bprmf_dist_train_*) --------------------
    def runner_rccl(self, uid):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        _lib.check(self.L.bprmf_dist_init_rccl(self.h, ctypes.addressof(buf)))

    def ipc_export(self):
        """This rank's IPC handles (raises on failure)."""
        blob = (ctypes.c_uint8 * _lib.IPC_BLOB_BYTES)()
        _lib.check(self.L.bprmf_dist_ipc_export(self.h, ctypes.addressof(blob)))
        return bytes(blob)

    def ipc_init(self, blobs):
        allb = (ctypes.c_uint8 * len(blobs)).from_buffer_copy(blobs)
        _lib.check(self.L.bprmf_dist_init_ipc(self.h, ctypes.addressof(allb)))

    def runner_ipc(self, all_gather_bytes):
        blob = self.ipc_export()
        self.ipc_init(b"".join(all_gather_bytes(blob)))

    def runner_loopback(self, key):
        _lib.check(self.L.bprmf_dist_init_loopback(self.h, int(key)))

    def runner_train_steps(self, epoch, first_step, n_steps):
        st = _lib.Stats()
        _lib.check(self.L.bprmf_dist_train_steps(self.h, int(epoch), int(first_step), int(n_steps),
                                                 ctypes.byref(st)))
        return st.as_dict()

    def runner_train_replay(self, u, i, j, n_steps):
        st = _lib.Stats()
        u, i, j = (np.ascontiguousarray(x, dtype=np.int32) for x in (u, i, j))
        _lib.check(self.L.bprmf_dist_train_replay(self.h, u.ctypes.data, i.ctypes.data,
                                                  j.ctypes.data, int(n_steps), ctypes.byref(st)))
        return st.as_dict()

    def exchange_stats(self):
        v = [ctypes.c_int64() for _ in range(4)]
        _lib.check(self.L.bprmf_dist_exchange_stats(self.h, *map(ctypes.byref, v)))
        return dict(zip(("steps", "row_bytes", "grad_bytes", "id_bytes"), (x.value for x in v)))

    def get_weights(self):
        return self.m.get_weights()

    def set_weights(self, P, Q):
        self.m.set_weights(P, Q)

    def profile(self, on=True):
        self.m.profile(on)

    def profile_read(self):
        return self.m.profile_read()


# ------------------------------------------------------------------------------------------------
# the orchestrator
# ------------------------------------------------------------------------------------------------
class ShardedBPRMF:
    """One rank of a sharded BPR-MF run.  `comm`: TorchComm (default, one process per GPU) or a
    ThreadComm; `backend`: the shard's compute (HipShard by default).

    semantics="local" (opt-in, not the reference step): users stay sharded but
    every rank holds and trains the WHOLE item table with the single-GPU local step, and the ranks'
    tables are merged (decayed base + the sum of the ranks' changes; one all-reduce) every
    `dp_steps` steps and at the end of every call (`dp_overlap`: each merge's all-reduce runs
    beside the next period, its sum added one period later).  Runner only (attach_runner "rccl" or
    "loopback"); get_weights / set_weights then take (P_local, Q_full).

    semantics="stale1" (opt-in, not the reference step): the exact sharded step with
    the item rows one step stale (oracle/bpr_oracle.py sharded_stale1_serial): each step's
    gradient exchange and the owners' apply run beside the next step's compute.  Runner only:
    attach_runner "rccl" or "loopback" (a second stream), or "ipc" with one rank per GPU (the
    device-flag form, inside the next step's launch)."""

    def __init__(self, user_num, item_num, factor_num=32, lr=0.01, wd=0.001, batch_size=4096,
                 num_ng=4, init_std=0.01, seed=0, device=0, group=None, comm=None, backend=None,
                 chunk_steps=256, semantics="exact", local_steps=0, dp_steps=0, dp_overlap=False):
        self.comm = comm if comm is not None else TorchComm(group)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.user_num, self.item_num, self.factor_num = int(user_num), int(item_num), int(factor_num)
        self.batch_size = int(batch_size)
        self.semantics = semantics
        self.b = backend if backend is not None else HipShard(
            user_num, item_num, factor_num, lr, wd, batch_size, num_ng, init_std, seed, device,
            self.rank, self.world, semantics, local_steps, dp_steps, dp_overlap)
        self.ld = self.b.ld
        self.device = self.b.device
        self.chunk_steps = int(chunk_steps)
        self.steps_per_epoch = None
        self._plan = None  # (epoch, first_step, n, send_counts, recv_counts)
        self.runner = None  # attach_runner(): "ipc" | "rccl" | "loopback"
        self.transport_error = None

    # -- data -----------------------------------------------------------------------------------
    def set_train(self, positives):
        """Global positives [[u, i], ...]; every rank passes the same list and keeps its users."""
        local_steps = self.b.set_train(positives)
        self.steps_per_epoch = self.comm.allreduce_max(local_steps, self.device)
        self._plan = None
        return self.steps_per_epoch

    def _per_step_ok(self):
        # semantics "local" keeps the whole item table on every rank; the per-step calls address
        # items by owner (i % world), so only the runner (train_steps / train_replay) runs it
        if self.semantics in ("local", "stale1"):
            raise ValueError(f'semantics="{self.semantics}" runs through the library runner only '
                             '(attach_runner + train_steps / train_replay), not per-step orchestration')

    def _ensure_plan(self, epoch, step):
        self._per_step_ok()
        p = self._plan
        if p is not None and p[0] == epoch and p[1] <= step < p[1] + p[2]:
            return
        first = (step // self.chunk_steps) * self.chunk_steps
        n = min(self.chunk_steps, self.steps_per_epoch - first)
        send = self.b.plan(epoch, first, n)
        recv = self.comm.exchange_counts(send, self.device)
        self._plan = (epoch, first, n, send, recv)

    def _local_batches(self, batches):
        """This rank's share of GLOBAL batches (list of (u, i, j), one per step), batch_size slots
        per step, u = -1 in empty slots (a batch of G*B global triplets splits unevenly across
        ranks, so the local capacity batch_size must hold every rank's share)."""
        B = self.batch_size
        n = len(batches)
        U = np.full(n * B, -1, np.int32)
        I = np.zeros(n * B, np.int32)
        J = np.zeros(n * B, np.int32)
        for k, (u, i, j) in enumerate(batches):
            u, i, j = (np.asarray(x).astype(np.int64) for x in (u, i, j))
            mine = (u % self.world) == self.rank
            c = int(mine.sum())
            if c > B:
                raise ValueError(f"rank {self.rank} gets {c} triplets at step {k} > batch_size {B}")
            U[k * B:k * B + c], I[k * B:k * B + c], J[k * B:k * B + c] = u[mine], i[mine], j[mine]
        return U, I, J, n

    def plan_replay(self, batches):
        """Replay plan (per-step Python orchestration) from GLOBAL batches, see _local_batches."""
        self._per_step_ok()
        U, I, J, n = self._local_batches(batches)
        send = self.b.plan_replay(U, I, J, n)
        recv = self.comm.exchange_counts(send, self.device)
        self._plan = ("replay", 0, n, send, recv)

    # -- the library-driven runner: whole chunks of steps, exchanges issued from C++ -------------
    def attach_runner(self, transport="rccl", key=0):
        """transport "ipc": kernels write each peer's block straight into its buffers (hipIpc
        mappings exchanged over the process group; one process per GPU, one node); "rccl": the
        library's own RCCL communicator (rank 0 makes the unique id, the process group broadcasts
        it); "loopback": in-process shards sharing group `key` (tests)."""
        if transport == "rccl":
            uid = bytes(128)
            if self.rank == 0:
                buf = (ctypes.c_uint8 * 128)()
                _lib.check(_lib.load().bprmf_dist_unique_id(ctypes.addressof(buf)))
                uid = bytes(buf)
            uid = self.comm.broadcast_bytes(uid, self.device)
            self.b.runner_rccl(uid)
        elif transport == "ipc":
            self.b.runner_ipc(lambda blob: self.comm.all_gather_bytes(blob, self.device))
        elif transport == "auto" and self.semantics == "local":
            return self.attach_runner("rccl")  # the item merge is an all-reduce
        elif transport == "auto":  # ipc where every rank can map its peers, else rccl
            # Every rank joins every collective whatever failed locally: a status byte travels
            # with the handles, so a rank whose export failed cannot leave its peers waiting in
            # the all-gather, and the fallback is agreed on by all ranks together.
            ok, blob = 1, bytes(_lib.IPC_BLOB_BYTES)
            try:
                blob = self.b.ipc_export()
            except Exception as e:  # noqa: BLE001 (reported, then the fallback is agreed on)
                self.transport_error = str(e)
                ok = 0
            got = self.comm.all_gather_bytes(bytes([ok]) + blob, self.device)
            # stale1 over IPC is the device-flag form: one rank per GPU (every blob carries its
            # device's PCI bus id after the five handles); ranks sharing a GPU take rccl
            if self.semantics == "stale1" and all(g[0] == 1 for g in got):
                bus = [bytes(g[1 + IPC_BUS_ID_OFF:1 + IPC_BUS_ID_OFF + 64]) for g in got]
                if len(set(bus)) < len(bus):
                    return self.attach_runner("rccl")
            if all(g[0] == 1 for g in got):
                try:
                    self.b.ipc_init(b"".join(g[1:] for g in got))
                except Exception as e:  # noqa: BLE001
                    self.transport_error = str(e)
                    ok = 0
            else:
                ok = 0
            if -self.comm.allreduce_max(-ok, self.device) == 1:
                transport = "ipc"
            else:
                return self.attach_runner("rccl")
        elif transport == "loopback":
            self.b.runner_loopback(key)
        else:
            raise ValueError(f"unknown transport {transport!r}")
        self.runner = transport

    def train_steps(self, epoch, first_step, n_steps):
        """Global steps [first_step, first_step + n_steps) of `epoch` on every rank (same args)."""
        return self.b.runner_train_steps(epoch, first_step, n_steps)

    def exchange_stats(self):
        """Bytes this rank sent to peers since attach_runner (rows, gradients, request lists) and
        the steps they cover (the runner's padded exchange volume)."""
        return self.b.exchange_stats()

    def train_epoch(self, epoch):
        return self.train_steps(epoch, 0, self.steps_per_epoch)

    def train_replay(self, batches):
        """GLOBAL batches (list of (u, i, j), one per step) through the runner."""
        U, I, J, n = self._local_batches(batches)
        return self.b.runner_train_replay(U, I, J, n)

    # -- one step (per-step Python orchestration over `comm`) -----------------------------------
    def step(self, epoch, step, want_loss=False):
        """Global step `step` of `epoch` (every rank calls it with the same arguments)."""
        self._ensure_plan(epoch, step)
        return self._run(step - self._plan[1], want_loss)

    def step_replay(self, k, want_loss=False):
        self._per_step_ok()
        return self._run(k, want_loss)

    def _run(self, k, want_loss):
        import contextlib
        import torch
        if hasattr(self.b, "stream"):
            # one non-default stream for the library's kernels, torch's allocations and the
            # collectives, then the caller's stream waits for it
            s = self.b.stream()
            self.b.bind_stream()
            caller = torch.cuda.current_stream(self.device)
            s.wait_stream(caller)
            with torch.cuda.stream(s):
                out = self._run_on_stream(k, want_loss)
            caller.wait_stream(s)
            return out
        with contextlib.nullcontext():
            return self._run_on_stream(k, want_loss)

    def _run_on_stream(self, k, want_loss):
        import torch
        _, _, _, send, recv = self._plan
        sc, rc = send[k], recv[k]
        ns, nr = int(sc.sum()), int(rc.sum())
        dev, ld = self.device, self.ld
        ids = torch.empty(max(ns, 1), dtype=torch.int32, device=dev)
        self.b.request_ids(k, ids, ns)
        rids = torch.empty(max(nr, 1), dtype=torch.int32, device=dev)
        self.comm.all_to_all(rids[:nr], ids[:ns], rc, sc)
        rows_out = torch.empty((max(nr, 1), ld), dtype=torch.float32, device=dev)
        self.b.gather_items(rids, nr, rows_out)
        rows_in = torch.empty((max(ns, 1), ld), dtype=torch.float32, device=dev)
        self.comm.all_to_all(rows_in[:ns], rows_out[:nr], sc, rc)
        self.b.user_step(k, rows_in)
        grads = torch.empty((max(ns, 1), ld), dtype=torch.float32, device=dev)
        self.b.item_grads(k, grads)
        rgrads = torch.empty((max(nr, 1), ld), dtype=torch.float32, device=dev)
        self.comm.all_to_all(rgrads[:nr], grads[:ns], rc, sc)
        self.b.apply_items(rids, rgrads, nr)
        return self.b.end_step(want_loss)

    # -- weights / measurement --------------------------------------------------------------------
    def get_weights(self):
        """This shard's (P_local, Q_local): global user = local*world + rank, same for items
        (semantics "local": Q is the whole item table, the same on every rank)."""
        return self.b.get_weights()

    def set_weights(self, P_local, Q_local):
        self.b.set_weights(P_local, Q_local)

    def profile(self, on=True):
        self.b.profile(on)

    def profile_read(self):
        return self.b.profile_read()


class NodeBarrier:
    """The ranks of one node meeting on two shared words of a /dev/shm file (include/bprmf.h
    bprmf_node_barrier_*; ~1 us instead of a process group's ~0.1 ms).  One rank constructs it
    with create=True before the others open the same path."""

    def __init__(self, path, world, rank, create):
        self.L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self.L.bprmf_node_barrier_open(str(path).encode(), int(world), int(rank),
                                                  int(bool(create)), ctypes.byref(h)))
        self.h = h

    def wait(self, timeout=120.0):
        _lib.check(self.L.bprmf_node_barrier_wait(self.h, float(timeout)))

    def close(self):
        if self.h:
            self.L.bprmf_node_barrier_close(self.h)
            self.h = None


def shard_rows(global_table, rank, world):
    """Rows of a global table owned by `rank` (strided sharding)."""
    return np.ascontiguousarray(global_table[rank::world])


def unshard_rows(parts, n_rows):
    """Inverse of shard_rows over all ranks' parts."""
    world = len(parts)
    out = np.empty((n_rows,) + parts[0].shape[1:], dtype=parts[0].dtype)
    for r, p in enumerate(parts):
        out[r::world] = p
    return out
