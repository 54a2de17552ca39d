// dist.cpp — the sharded multi-GPU runner behind bprmf_dist_train_* (include/bprmf.h).
//
// One handle per GPU (one process per GPU under torch.distributed.run).  The runner drives whole
// chunks of steps from C++: no Python per step.  Transports:
//   ipc       kernels write each peer's block straight into the peer's buffer (mapped with
//             hipIpc; xGMI peer writes) and raise a per-source flag.  Per step, the owners'
//             gather writes the rows into the requesters' landing buffers itself and K1 waits on
//             its row flags; the owners' apply waits on its gradient flags, no host in the loop:
//             two launches per step, the owner phase beside K1 (step.hip k_dist_front) and K2
//             writing its gradients straight into the owners' landing buffers
//             (k_item_step_push).  Ranks sharing one device: push kernels + receive copies.
//   rccl      an RCCL communicator owned by the handle (ncclCommInitRank from a unique id the
//             caller broadcasts); per-peer blocks move with grouped ncclSend/ncclRecv over xGMI.
//   loopback  handles of one process exchanging through a shared table + device copies (the
//             in-process test transport: several shards on one GPU, one host thread each).
// A chunk of n steps (dist.hip has the buffer layouts):
//   build_batches(slots padded by S per owner) -> cap = max requests per (step, owner), max over
//   ranks -> pack + exchange the chunk's requests once -> owner apply plan;
//   per step k: owner_gather -> exchange rows -> user_step (SH) -> item_step (SH: per-slot grads)
//   -> exchange grads -> owner_apply.  A rank's requests to itself never enter the exchange: the
//   gather writes them into its slots and the apply reads their gradients in place.
// Exchange sizes are cap rows per peer per step (uniform), so every rank posts matching sizes
// without a per-step count exchange.  Semantics: SURVEY.md §8e — a world-W run with per-rank
// batch B equals one step over the union batch (BPRMFRecommender.py:172-176).
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <vector>

#include "handle.h"
#include "host_plan.h"

namespace bprmf {

enum XKind { X_ROWS = 0, X_GRADS = 1, X_IDS = 2, X_MAX = 3, X_KINDS = 4 };

struct Xchg {  // one all-to-all of per-peer blocks
  int kind;
  const void* const* send;  // send[p]: the block for rank p (nullptr at this rank: already placed)
  void* const* recv;        // recv[p]: where the block from rank p lands (this rank's memory)
  size_t bytes;
  const int32_t* tbase;  // per-step exchange: sequence number *tbase + k + 1 (graph-safe)
  int k;
  int32_t seq;  // per-chunk exchange (tbase == nullptr)
};

struct Transport {
  virtual ~Transport() = default;
  // another rank's kernels run on this rank's GPU (one-GPU rehearsals, in-process shards): no
  // launch may wait on workgroups of its own grid that come after it (the split builder's
  // in-launch sampling board does), since a peer's spinning workgroups can hold the CUs they need
  virtual bool shares_device() const { return false; }
  virtual int exchange(bprmf_handle* h, const Xchg& x) = 0;
  // in-place max over ranks of one device int32; vals: [world] scratch peers may write into
  virtual int max_i32(bprmf_handle* h, int32_t* dev, int32_t* vals, int32_t seq) {
    const int W = h->cfg.world;
    if (W == 1 && !self_exchange) return 0;  // the max over one rank
    std::vector<const void*> sp(W, dev);
    std::vector<void*> rp(W);
    for (int p = 0; p < W; ++p) rp[p] = vals + p;
    if (int r = exchange(h, Xchg{X_MAX, sp.data(), rp.data(), 4, nullptr, 0, seq})) return r;
    HIPCHK(max_vals(vals, W, dev, h->stream));
    return 0;
  }
  // semantics LOCAL at world > 1: the sum over ranks of every rank's buf (n floats), the same
  // bits on every rank; *out = where it landed (buf itself, or the transport's scratch)
  virtual int allreduce_sum(bprmf_handle* h, float* buf, int64_t n, const float** out) {
    (void)h;
    (void)buf;
    (void)n;
    (void)out;
    return fail(BPRMF_E_UNSUPPORTED, "this transport has no all-reduce: use rccl (or loopback)");
  }
  // the same sum, started beside the caller's stream (dp_overlap): into `dst` (or the transport's
  // scratch, *out says which); allreduce_wait orders the caller's stream after it.  Default: the
  // blocking form (its result is ready when the call returns).
  virtual int allreduce_start(bprmf_handle* h, float* buf, float* dst, int64_t n, const float** out) {
    (void)dst;
    return allreduce_sum(h, buf, n, out);
  }
  virtual int allreduce_wait(bprmf_handle* h) {
    (void)h;
    return 0;
  }
  // exchange() only enqueues stream work (no host synchronisation): hipGraph-capturable
  virtual bool capturable() const { return false; }
  virtual bool ready() const { return true; }
  // device memory that peers write into (the IPC transport exports it)
  virtual int alloc_shared(bprmf_handle* h, int kind, size_t bytes, void** p) {
    (void)h;
    (void)kind;
    *p = nullptr;
    HIPCHK(hipMalloc(p, bytes));
    return 0;
  }
  virtual void free_shared(void* p) {
    if (p) (void)!hipFree(p);
  }
  bool self_exchange = false;  // test hook: this rank's own blocks also go through the transport
};

#define NCCLCHK(x)                                                                      \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) return fail(BPRMF_E_HIP, "%s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

struct RcclTransport final : Transport {
  ncclComm_t comm = nullptr;
  hipStream_t side = nullptr;  // dp_overlap: the all-reduce beside the training stream
  hipEvent_t ev_in = nullptr, ev_done = nullptr;
  ~RcclTransport() override {
    if (side) (void)!hipStreamSynchronize(side);
    if (comm) ncclCommDestroy(comm);
    if (ev_in) (void)!hipEventDestroy(ev_in);
    if (ev_done) (void)!hipEventDestroy(ev_done);
    if (side) (void)!hipStreamDestroy(side);
  }
  bool capturable() const override { return true; }
  int exchange(bprmf_handle* h, const Xchg& x) override {
    if (!x.bytes) return 0;
    const int W = h->cfg.world, R = h->cfg.rank;
    if (x.send[R] && !self_exchange)
      HIPCHK(hipMemcpyAsync(x.recv[R], x.send[R], x.bytes, hipMemcpyDeviceToDevice, h->stream));
    if (W == 1 && !self_exchange) return 0;
    NCCLCHK(ncclGroupStart());
    for (int p = 0; p < W; ++p) {
      if (p == R && (!self_exchange || !x.send[R])) continue;
      NCCLCHK(ncclSend(x.send[p], x.bytes, ncclUint8, p, comm, h->stream));
      NCCLCHK(ncclRecv(x.recv[p], x.bytes, ncclUint8, p, comm, h->stream));
    }
    NCCLCHK(ncclGroupEnd());
    return 0;
  }
  int max_i32(bprmf_handle* h, int32_t* dev, int32_t* vals, int32_t seq) override {
    (void)vals;
    (void)seq;
    if (h->cfg.world == 1) return 0;
    NCCLCHK(ncclAllReduce(dev, dev, 1, ncclInt32, ncclMax, comm, h->stream));
    return 0;
  }
  // in place; ring and tree all-reduces reduce each element once and broadcast the result, so
  // every rank holds the same bits
  int allreduce_sum(bprmf_handle* h, float* buf, int64_t n, const float** out) override {
    *out = buf;
    NCCLCHK(ncclAllReduce(buf, buf, (size_t)n, ncclFloat, ncclSum, comm, h->stream));
    return 0;
  }
  int allreduce_start(bprmf_handle* h, float* buf, float* dst, int64_t n, const float** out) override {
    if (!side) {
      HIPCHK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(ev_in, h->stream));  // the delta pass has written buf
    HIPCHK(hipStreamWaitEvent(side, ev_in, 0));
    NCCLCHK(ncclAllReduce(buf, dst, (size_t)n, ncclFloat, ncclSum, comm, side));
    HIPCHK(hipEventRecord(ev_done, side));
    *out = dst;
    return 0;
  }
  int allreduce_wait(bprmf_handle* h) override {
    if (side) HIPCHK(hipStreamWaitEvent(h->stream, ev_done, 0));
    return 0;
  }
};

// ---- IPC: blocks pushed by a kernel straight into the peers' buffers (xGMI peer writes) -----
// Peers write into "landing" buffers, allocated uncached (their writes bypass this GPU's L2, so
// no reader sees a stale line) and exported with hipIpcGetMemHandle; each rank maps the peers'
// handles.  Layouts are symmetric: the block rank R sends to p lands in p's buffer at the offset
// where R's own buffer keeps the block from R.  Completion: per-(kind, source) flags carrying the
// exchange's sequence number (the step number for per-step exchanges).  Rows and request lists
// are then copied by a receive kernel (which waits per peer) into ordinary cached buffers, since
// the step kernels read them many times; gradients and capacities are read once, in place.
constexpr int kIpcHandles = X_KINDS + 1;  // the four landing buffers + the flag array
constexpr int kBusIdBytes = 64;          // a PCI bus id string, after the handles in the blob
struct IpcTransport final : Transport {
  int world = 0, rank = 0;
  void* recv_base[X_KINDS] = {};          // the buffers the runner reads (alloc_shared)
  void* local[kIpcHandles] = {};          // this rank's landing buffers (X_KINDS: flags)
  std::vector<void*> remote[kIpcHandles];  // [world] peers' mappings (self: local)
  // completion boards (device_common.h board_mark / board_finish), kBoardMax words each: the
  // push kernels' by exchange kind, then the owner phase's, then the fused step's K2
  int32_t* boards = nullptr;
  static constexpr int kBoardOwner = X_KINDS, kBoardK2 = X_KINDS + 1, kBoards = X_KINDS + 2;
  int32_t* board(int b) const { return boards + (size_t)b * kBoardMax; }
  bool opened = false;
  bool shared_device = false;  // some peer runs on this rank's GPU (rehearsals on one device)
  bool shares_device() const override { return shared_device; }
  // owner workgroups per launch: they spin on the peers' gradient flags before applying, so with
  // ranks sharing one GPU a full grid of them could hold every CU a peer needs to produce those
  // gradients (measured: 2 ranks, ~1,500 owner workgroups, timed out); one rank per GPU: no cap
  int owner_blocks() const { return shared_device ? 160 : kBoardMax; }
  static bool copied(int kind) { return kind == X_ROWS || kind == X_IDS; }
  ~IpcTransport() override {
    for (int b = 0; b < kIpcHandles; ++b)
      for (int p = 0; p < (int)remote[b].size(); ++p)
        if (p != rank && remote[b][p]) (void)!hipIpcCloseMemHandle(remote[b][p]);
    for (int b = 0; b < kIpcHandles; ++b) {
      if (b < X_KINDS && copied(b) && recv_base[b]) (void)!hipFree(recv_base[b]);
      if (local[b]) (void)!hipFree(local[b]);
    }
    if (boards) (void)!hipFree(boards);
  }
  bool capturable() const override { return true; }
  bool ready() const override { return opened; }
  int alloc_shared(bprmf_handle* h, int kind, size_t bytes, void** p) override {
    (void)h;
    *p = nullptr;
    // landing memory uncached: a reader never sees a stale L2 line after a peer's xGMI write
    // (fine-grained and plain allocations measured the same)
    HIPCHK(hipExtMallocWithFlags(&local[kind], std::max<size_t>(bytes, 256), hipDeviceMallocUncached));
    if (copied(kind)) {
      HIPCHK(hipMalloc(&recv_base[kind], std::max<size_t>(bytes, 256)));
    } else {
      recv_base[kind] = local[kind];
    }
    *p = recv_base[kind];
    return 0;
  }
  void free_shared(void* p) override { (void)p; }  // owned (and freed) by the transport
  int32_t* flags() const { return static_cast<int32_t*>(local[X_KINDS]); }
  // per-step fusion (enqueue_steps): the owners' gather writes rows straight into the peers' row
  // landing buffers, K1 reads them there after waiting on its flags, and the apply waits on the
  // gradient flags itself; only the gradient push remains a separate kernel
  // The fused forms need one rank per GPU: their consumers wait inside kernels (K1 workgroups on
  // the row flags, owner workgroups on the gradient flags), and ranks sharing a device fill it
  // with spinning workgroups until a peer cannot run the kernel that would release them (8
  // ranks on one GPU timed out).  Shared device: every exchange is a push kernel plus a receive
  // copy (or one waiting block), and no step kernel spins.  BPRMF_DIST_FUSE=0/1 forces either
  // (1: also at world 1 or on a shared device, to measure and test the fused form there).
  // The fused form is two launches per step (step.hip k_dist_front + k_item_step_push): the
  // owner phase beside K1, K2's gradients straight into the owners' landing buffers.  (A
  // three-launch form, owner step / K1 / K2 + a push kernel, measured slower and was removed in
  // round 6; a chunk whose plan has no rows to exchange, cap 0, still runs its launch sequence.)
  bool fused() const {
    if (!opened || self_exchange) return false;
    const char* e = getenv("BPRMF_DIST_FUSE");
    if (e && *e) return e[0] != '0';
    return world > 1 && !shared_device;
  }
  // stale-1's device-flag form: as fused(), at world 1 too (no single-GPU step to dispatch to)
  bool device_flags() const {
    if (!opened || self_exchange) return false;
    const char* e = getenv("BPRMF_DIST_FUSE");
    if (e && *e) return e[0] != '0';
    return !shared_device;
  }
  float* landing(int kind) const { return static_cast<float*>(local[kind]); }
  void* peer_landing(int kind, int p) const { return remote[kind][p]; }
  int32_t* peer_flag(int kind, int p) const {
    return static_cast<int32_t*>(remote[X_KINDS][p]) + kind * kMaxWorld + rank;
  }
  const int32_t* my_flags(int kind) const { return flags() + kind * kMaxWorld; }
  // the push half of an exchange: every peer's block into its landing buffer + its flag
  int push(bprmf_handle* h, const Xchg& x) {
    PushArgs a{};
    const char* base = static_cast<const char*>(recv_base[x.kind]);
    const ptrdiff_t off = static_cast<const char*>(x.recv[rank]) - base;  // this rank's block
    for (int p = 0; p < world; ++p) {
      a.src[p] = x.send[p];
      if (p == rank) {
        a.dst[p] = x.recv[p];
      } else {
        a.dst[p] = static_cast<char*>(remote[x.kind][p]) + off;
        a.flag[p] = peer_flag(x.kind, p);
      }
    }
    HIPCHK(ipc_push(a, world, (int64_t)x.bytes, x.tbase, x.k, x.seq, board(x.kind), h->d_err, h->stream));
    return 0;
  }
  // semantics LOCAL at world > 1 (dist.cpp dp_merge): the item tables' all-reduce as a
  // reduce-scatter and an all-gather of pushes over the full mesh (each rank owns a slice of
  // ceil(I / W) rows): every rank pushes its slice p of buf into rank p's landing buffer (kind
  // X_ROWS, block = the sender), waits for the W blocks of its own slice, sums them in rank order
  // into its sum buffer (kind X_GRADS), pushes that slice into every peer's sum buffer and waits
  // for theirs.  The sums are the loopback transport's, bit for bit.  A slice's landing blocks
  // are reused by the next all-reduce only after every peer has pushed (so read) this one's.
  int64_t dp_seq = 0;
  int allreduce_sum(bprmf_handle* h, float* buf, int64_t n, const float** out) override {
    const int W = world, R = rank;
    const int64_t ld = h->geom.ld, slice = (h->I + W - 1) / W * ld;  // floats per slice
    if (n != h->I * ld || !local[X_ROWS] || !local[X_GRADS])
      return fail(BPRMF_E_STATE, "ipc all-reduce: the item-table buffers are not attached");
    const int32_t seq = (int32_t)++dp_seq;
    float* land = static_cast<float*>(local[X_ROWS]);
    float* sum = static_cast<float*>(local[X_GRADS]);
    PushArgs a{};
    for (int p = 0; p < W; ++p) {
      a.src[p] = buf + (int64_t)p * slice;
      a.dst[p] = (p == R ? land : static_cast<float*>(remote[X_ROWS][p])) + (int64_t)R * slice;
      if (p != R) a.flag[p] = static_cast<int32_t*>(remote[X_KINDS][p]) + X_ROWS * kMaxWorld + R;
    }
    HIPCHK(ipc_push(a, W, slice * (int64_t)sizeof(float), nullptr, 0, seq, board(X_ROWS), h->d_err, h->stream));
    HIPCHK(ipc_wait(flags() + X_ROWS * kMaxWorld, W, R, nullptr, 0, seq, h->d_err, h->stream));
    DpSrcs src{};
    for (int p = 0; p < W; ++p) src.p[p] = land + (int64_t)p * slice;
    HIPCHK(dp_sum(src, W, sum + (int64_t)R * slice, slice, h->stream));
    PushArgs c{};
    for (int p = 0; p < W; ++p) {
      if (p == R) continue;
      c.src[p] = sum + (int64_t)R * slice;
      c.dst[p] = static_cast<float*>(remote[X_GRADS][p]) + (int64_t)R * slice;
      c.flag[p] = static_cast<int32_t*>(remote[X_KINDS][p]) + X_GRADS * kMaxWorld + R;
    }
    HIPCHK(ipc_push(c, W, slice * (int64_t)sizeof(float), nullptr, 0, seq, board(X_GRADS), h->d_err, h->stream));
    HIPCHK(ipc_wait(flags() + X_GRADS * kMaxWorld, W, R, nullptr, 0, seq, h->d_err, h->stream));
    *out = sum;
    return 0;
  }
  int exchange(bprmf_handle* h, const Xchg& x) override {
    if (!x.bytes) return 0;
    if (world == 1) {  // no peers: only a self block, if the caller did not place it
      if (x.send[0]) HIPCHK(hipMemcpyAsync(x.recv[0], x.send[0], x.bytes, hipMemcpyDeviceToDevice, h->stream));
      return 0;
    }
    PushArgs a{};
    const char* base = static_cast<const char*>(recv_base[x.kind]);
    const ptrdiff_t off = static_cast<const char*>(x.recv[rank]) - base;  // this rank's block
    for (int p = 0; p < world; ++p) {
      a.src[p] = x.send[p];
      if (p == rank) {
        a.dst[p] = x.recv[p];
      } else {
        a.dst[p] = static_cast<char*>(remote[x.kind][p]) + off;
        a.flag[p] = static_cast<int32_t*>(remote[X_KINDS][p]) + x.kind * kMaxWorld + rank;
      }
    }
    HIPCHK(ipc_push(a, world, (int64_t)x.bytes, x.tbase, x.k, x.seq, board(x.kind), h->d_err, h->stream));
    const int32_t* fl = flags() + x.kind * kMaxWorld;
    if (!copied(x.kind)) {
      HIPCHK(ipc_wait(fl, world, rank, x.tbase, x.k, x.seq, h->d_err, h->stream));
      return 0;
    }
    PushArgs c{};  // landing -> working buffer, per peer
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      const ptrdiff_t o = static_cast<const char*>(x.recv[p]) - base;
      c.src[p] = static_cast<const char*>(local[x.kind]) + o;
      c.dst[p] = x.recv[p];
    }
    HIPCHK(ipc_recv(c, world, rank, (int64_t)x.bytes, fl, x.tbase, x.k, x.seq, h->d_err, h->stream));
    return 0;
  }
};

// ---- loopback: shards of one process (tests) ----------------------------------------------
struct LoopGroup {
  std::mutex m;
  std::condition_variable cv;
  int world = 0, arrived = 0, refs = 0;
  int64_t gen = 0;
  std::vector<const void* const*> send;
  std::vector<int32_t> val;
  std::vector<const float*> fbuf;  // allreduce_sum: every rank's buffer
  void barrier() {
    std::unique_lock<std::mutex> l(m);
    const int64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(l, [&] { return gen != g; });
    }
  }
};
static std::mutex g_loops_m;
static std::map<int64_t, LoopGroup*> g_loops;

struct LoopTransport final : Transport {
  bool shares_device() const override { return true; }  // in-process shards on one GPU
  int64_t key = 0;
  LoopGroup* g = nullptr;
  float* scratch = nullptr;  // allreduce_sum's result (peers still read this rank's buffer)
  int64_t scratch_n = 0;
  ~LoopTransport() override {
    if (scratch) (void)!hipFree(scratch);
    std::lock_guard<std::mutex> l(g_loops_m);
    if (g && --g->refs == 0) {
      g_loops.erase(key);
      delete g;
    }
  }
  int exchange(bprmf_handle* h, const Xchg& x) override {
    const int W = h->cfg.world, R = h->cfg.rank;
    HIPCHK(hipStreamSynchronize(h->stream));  // this shard's blocks are complete
    g->send[R] = x.send;
    g->barrier();
    int rc = 0;
    for (int p = 0; p < W && !rc && x.bytes; ++p) {
      if (!g->send[p][R]) continue;
      const hipError_t e = hipMemcpyAsync(x.recv[p], g->send[p][R], x.bytes, hipMemcpyDeviceToDevice, h->stream);
      if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback copy: %s", hipGetErrorString(e));
    }
    const hipError_t e = hipStreamSynchronize(h->stream);
    if (!rc && e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback sync: %s", hipGetErrorString(e));
    g->barrier();  // every peer has read this shard's send blocks
    return rc;
  }
  // every rank sums all ranks' buffers in rank order into its scratch (the same bits everywhere)
  int allreduce_sum(bprmf_handle* h, float* buf, int64_t n, const float** out) override {
    const int W = h->cfg.world, R = h->cfg.rank;
    int rc = 0;
    if (n > scratch_n) {
      if (scratch) (void)!hipFree(scratch);
      scratch = nullptr;
      scratch_n = 0;
      if (hipMalloc((void**)&scratch, sizeof(float) * n) == hipSuccess) scratch_n = n;
      else rc = fail(BPRMF_E_HIP, "loopback all-reduce scratch");
    }
    hipError_t e = hipStreamSynchronize(h->stream);  // this rank's buffer is complete
    if (!rc && e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback sync: %s", hipGetErrorString(e));
    g->fbuf[R] = buf;
    g->barrier();
    bool all = true;
    DpSrcs src{};
    for (int p = 0; p < W; ++p) {
      src.p[p] = g->fbuf[p];
      all = all && src.p[p];
    }
    if (!rc && all) {
      e = dp_sum(src, W, scratch, n, h->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
      if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback all-reduce: %s", hipGetErrorString(e));
    } else if (!rc) {
      rc = fail(BPRMF_E_STATE, "loopback all-reduce: a peer failed");
    }
    g->barrier();  // every peer has read this rank's buffer
    g->fbuf[R] = nullptr;
    *out = scratch;
    return rc;
  }
  int max_i32(bprmf_handle* h, int32_t* dev, int32_t* vals, int32_t seq) override {
    (void)vals;
    (void)seq;
    int32_t v = 0;
    HIPCHK(hipMemcpyAsync(&v, dev, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    g->val[h->cfg.rank] = v;
    g->barrier();
    const int32_t m = *std::max_element(g->val.begin(), g->val.end());
    g->barrier();
    HIPCHK(hipMemcpyAsync(dev, &m, 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
  }
};

struct DistGraph {  // a captured chunk of sharded steps (fixed n, cap and buffers)
  int64_t n = 0;
  int cap = 0;
  const void* bufs[4] = {};
  hipGraphExec_t exec = nullptr;  // null: seen once, not captured yet
};

// Buffers of the runner.  Sizes are fixed at attach (peers of the IPC transport hold mappings of
// the shared ones): S = slot stride per owner, nmax = steps per chunk.  The request lists and
// their apply plans alternate between two parities, so a rank may publish chunk c+1's requests
// while a slower peer still applies chunk c.
struct DistState {
  Transport* tr = nullptr;
  std::vector<DistGraph> graphs;
  int S = 0;             // requester-side slot stride per owner (rows)
  int cap = 0;           // rows per peer per step of the current chunk
  int64_t nmax = 0;      // steps per chunk
  int64_t chunks = 0;    // chunks run (parity, per-chunk sequence numbers)
  // bytes this rank sent over peer links since attach (padded to the exchange capacity, what the
  // transport moves): item rows (owner -> requesters), gradients (requester -> owners), request
  // lists (once per chunk); steps they cover (bprmf_dist_exchange_stats)
  int64_t x_steps = 0, x_rows = 0, x_grads = 0, x_ids = 0;
  int64_t aplan_n[2] = {0, 0};
  int32_t* ids_send = nullptr;     // [W][n][cap]
  int32_t* ids_recv = nullptr;     // shared, 2 parities x [W][nmax][S]
  int32_t* aplan[2] = {nullptr, nullptr};  // per parity: aplan [n][W][cap][W], then gdep
                                           // [n][W][cap][W], then gfree [n][W][cap]
  int32_t* vals = nullptr;         // shared, 2 parities x [W] (capacity max)
  int32_t* d_cap = nullptr;
  float* rows_send = nullptr;   // owner:     [W][cap][ld]
  float* rows_recv = nullptr;   // shared, requester: [W][S][ld] (slot order)
  float* grads_send = nullptr;  // requester: [W][S][ld]
  float* grads_recv = nullptr;  // shared, owner: [W][cap][ld] (cap <= S)
  // semantics STALE1 (enqueue_stale1): the second parity of rows_recv and grads_send, the owner
  // stream (gradient exchange, apply, gather, row exchange) and the events that order it against
  // the compute stream (h->stream)
  float* rows_recv1 = nullptr;
  float* grads_send1 = nullptr;
  hipStream_t xs = nullptr;
  hipEvent_t ev_rows[4] = {}, ev_k2[4] = {}, ev_fork = nullptr, ev_join = nullptr;
};

static void drop_dist_graphs(DistState* d) {
  for (auto& g : d->graphs)
    if (g.exec) (void)!hipGraphExecDestroy(g.exec);
  d->graphs.clear();
}

void dist_free(DistState* d) {
  if (!d) return;
  drop_dist_graphs(d);
  if (d->xs) (void)!hipStreamSynchronize(d->xs);
  for (hipEvent_t e : {d->ev_rows[0], d->ev_rows[1], d->ev_rows[2], d->ev_rows[3], d->ev_k2[0],
                       d->ev_k2[1], d->ev_k2[2], d->ev_k2[3], d->ev_fork, d->ev_join})
    if (e) (void)!hipEventDestroy(e);
  if (d->xs) (void)!hipStreamDestroy(d->xs);
  for (void* p : {(void*)d->rows_recv1, (void*)d->grads_send1})
    if (p) (void)!hipFree(p);
  void* shared[] = {d->ids_recv, d->vals, d->rows_recv, d->grads_recv};
  for (void* p : shared) d->tr->free_shared(p);
  void* ptrs[] = {d->ids_send, d->aplan[0], d->aplan[1], d->d_cap, d->rows_send, d->grads_send};
  for (void* p : ptrs)
    if (p) (void)!hipFree(p);
  delete d->tr;
  delete d;
}

int64_t dist_chunk_steps(const bprmf_handle* h) {
  // BPRMF_DIST_CHUNK: a shorter chunk, so tests reach chunk boundaries with small replays
  // (read per call: a test sets it for one handle)
  if (const char* e = getenv("BPRMF_DIST_CHUNK"))
    if (*e) return std::max<int64_t>(1, atoll(e));
  return std::max<int64_t>(1, (int64_t(1) << 20) / h->cfg.batch_size);
}

static int ensure_aplan(bprmf_handle* h, int par, int64_t n, int cap);

static int dist_attach(bprmf_handle* h, Transport* tr) {
  if (h->dp_mode) {  // LOCAL at world > 1: the item merge needs only the transport
    if (h->dist) {
      HIPCHK(hipStreamSynchronize(h->stream));
      dist_free(h->dist);
    }
    h->dist = new DistState();
    h->dist->tr = tr;
    if (dynamic_cast<IpcTransport*>(tr)) {  // its all-reduce's landing and sum buffers (exported)
      const int64_t W = h->cfg.world;
      const size_t bytes = sizeof(float) * (size_t)(W * ((h->I + W - 1) / W) * h->geom.ld);
      void* p = nullptr;
      if (int r = tr->alloc_shared(h, X_ROWS, bytes, &p)) return r;
      if (int r = tr->alloc_shared(h, X_GRADS, bytes, &p)) return r;
      // (the other kinds are unused here, but every exported handle needs a buffer)
      if (int r = tr->alloc_shared(h, X_IDS, 256, &p)) return r;
      if (int r = tr->alloc_shared(h, X_MAX, 256, &p)) return r;
    }
    return 0;
  }
  if (!seg_mode(h)) {
    delete tr;
    return fail(BPRMF_E_UNSUPPORTED, "sharded steps need batch_size <= %d", kMaxSegBatch);
  }
  if (h->dist) {
    HIPCHK(hipStreamSynchronize(h->stream));
    dist_free(h->dist);
    h->dist = nullptr;
  }
  auto* d = new DistState();
  d->tr = tr;
  tr->self_exchange = getenv("BPRMF_DIST_SELF_EXCHANGE") != nullptr;
  h->dist = d;
  const int64_t W = h->cfg.world;
  RunnerGeom rg;  // host_plan.cpp (sanitizer-tested host code)
  if (int r = runner_geom(h->cfg.batch_size, h->cfg.item_num, (int)W, h->geom.ld, dist_chunk_steps(h), &rg))
    return r;
  d->S = rg.S;
  d->nmax = rg.nmax;
  const int64_t rows = rg.row_elems;
  const int64_t ids = rg.id_elems;
  auto* ipc = dynamic_cast<IpcTransport*>(tr);
  const bool stale1 = h->semantics == BPRMF_SEM_STALE1;
  // stale-1 over IPC (enqueue_stale1_ipc): the row and gradient landing buffers in two parities
  const int64_t land = stale1 && ipc ? 2 * rows : rows;
  void* p = nullptr;
  if (int r = tr->alloc_shared(h, X_ROWS, sizeof(float) * land, &p)) return r;
  d->rows_recv = static_cast<float*>(p);
  if (int r = tr->alloc_shared(h, X_GRADS, sizeof(float) * land, &p)) return r;
  d->grads_recv = static_cast<float*>(p);
  if (int r = tr->alloc_shared(h, X_IDS, sizeof(int32_t) * 2 * ids, &p)) return r;
  d->ids_recv = static_cast<int32_t*>(p);
  if (int r = tr->alloc_shared(h, X_MAX, sizeof(int32_t) * 2 * W, &p)) return r;
  d->vals = static_cast<int32_t*>(p);
  if (int r = dalloc(&d->d_cap, 1)) return r;
  HIPCHK(hipMemsetAsync(d->d_cap, 0, sizeof(int32_t), h->stream));  // the split builder's max starts at 0
  if (int r = dalloc(&d->ids_send, ids)) return r;
  if (int r = dalloc(&d->rows_send, rows)) return r;
  if (int r = dalloc(&d->grads_send, rows)) return r;
  // both parities' apply plans at their largest (a full chunk at the largest capacity), so no
  // chunk ever reallocates one inside a call (a free synchronises the device)
  for (int par = 0; par < 2; ++par)
    if (int r = ensure_aplan(h, par, d->nmax, d->S)) return r;
  if (stale1) {  // the second parities; enqueue_stale1's stream and events
    if (int r = dalloc(&d->grads_send1, rows)) return r;
    HIPCHK(hipMemsetAsync(d->grads_send1, 0, sizeof(float) * rows, h->stream));
  }
  if (stale1 && !ipc) {
    if (int r = dalloc(&d->rows_recv1, rows)) return r;
    HIPCHK(hipMemsetAsync(d->rows_recv1, 0, sizeof(float) * rows, h->stream));
    HIPCHK(hipStreamCreateWithFlags(&d->xs, hipStreamNonBlocking));
    for (hipEvent_t* e : {&d->ev_rows[0], &d->ev_rows[1], &d->ev_rows[2], &d->ev_rows[3], &d->ev_k2[0],
                          &d->ev_k2[1], &d->ev_k2[2], &d->ev_k2[3], &d->ev_fork, &d->ev_join})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  // rows past a peer's request count are sent but never read; keep them finite
  HIPCHK(hipMemsetAsync(d->rows_send, 0, sizeof(float) * rows, h->stream));
  HIPCHK(hipMemsetAsync(d->grads_send, 0, sizeof(float) * rows, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

static int ensure_aplan(bprmf_handle* h, int par, int64_t n, int cap) {
  DistState* d = h->dist;
  const int64_t ap = aplan_words(n, h->cfg.world, cap);  // rec, gdep, gfree
  if (ap <= d->aplan_n[par]) return 0;
  if (d->aplan[par]) HIPCHK(hipFree(d->aplan[par]));
  d->aplan[par] = nullptr;
  d->aplan_n[par] = 0;
  if (int r = dalloc(&d->aplan[par], ap)) return r;
  d->aplan_n[par] = ap;
  return 0;
}

// Semantics STALE1 (include/bprmf.h, spec oracle/bpr_oracle.py sharded_stale1_serial): the
// owner side of step k (its gradient exchange, the owners' apply, then the gather and row
// exchange of step k+2) runs on the owner stream d->xs while step k+1 computes on h->stream.
//   owner stream:   gather(0) xchg rows(0) [E_rows 0]  gather(1) xchg rows(1) [E_rows 1]
//                   then per k: wait E_k2 k, xchg grads(k), apply(k), gather(k+2), xchg rows(k+2)
//                   [E_rows k+2]
//   compute stream: per k: wait E_rows k, K1(k) on rows parity k & 1, K2(k) -> grads parity
//                   k & 1 [E_k2 k]
// So step k+2 reads the rows after apply(k), brought to its step t-1 by weight decay alone
// (owner_gather_body): one step stale, where the exact runner's gather waits for apply(k+1).
// Hazards: rows(k+2) lands in parity k & 1 after K1(k) has read it (the owner stream waited for
// K2(k), which follows K1(k)); K2(k+2) rewrites gradient parity k & 1 only after its K1 waited
// for E_rows(k+2), which the owner stream records after it sent grads(k) from there; grads_recv,
// rows_send and the table itself are touched by the owner stream alone, user rows and the step
// buffers by the compute stream alone.  Exchanges run with h->stream switched to the owner
// stream (the transports enqueue on h->stream).  hipGraph capture works as for the exact runner:
// the owner stream forks from and joins the capturing stream through events.
static int enqueue_stale1(bprmf_handle* h, int64_t n, int cap, const int32_t* ids_recv,
                          const int32_t* aplan) {
  DistState* d = h->dist;
  const int B = h->cfg.batch_size, W = h->cfg.world;
  const int ld = h->geom.ld;
  const BatchBuf bb{h->d_batch, B};
  const int self = d->tr->self_exchange ? -1 : h->cfg.rank;
  const int64_t R = h->cfg.rank;
  const size_t row_bytes = sizeof(float) * (size_t)cap * ld;
  hipStream_t cs = h->stream, xs = d->xs;
  float* rows_par[2] = {d->rows_recv, d->rows_recv1};
  float* grads_par[2] = {d->grads_send, d->grads_send1};
  std::vector<const void*> sp(W);
  std::vector<void*> rp(W);
  struct Restore {  // h->stream back to the compute stream on every exit
    bprmf_handle* h;
    hipStream_t s;
    ~Restore() { h->stream = s; }
  } restore{h, cs};
  auto gather_and_send = [&](int64_t k) -> int {  // on the owner stream
    float* rin = rows_par[k & 1];
    PushArgs gd{};
    for (int p = 0; p < W; ++p)
      gd.dst[p] = p == self ? rin + R * d->S * ld : d->rows_send + (int64_t)p * cap * ld;
    HIPCHK(dist_owner_gather(h->geom, h->Q, ids_recv, n, W, cap, (int)k, h->hp, h->d_tbase, gd,
                             nullptr, h->d_err, kBoardMax, xs));
    for (int p = 0; p < W; ++p) {
      sp[p] = p == self ? nullptr : d->rows_send + (int64_t)p * cap * ld;
      rp[p] = rin + (int64_t)p * d->S * ld;
    }
    h->stream = xs;
    const int r = d->tr->exchange(h, Xchg{X_ROWS, sp.data(), rp.data(), row_bytes, h->d_tbase, (int)k, 0});
    h->stream = cs;
    if (r) return r;
    HIPCHK(hipEventRecord(d->ev_rows[k & 3], xs));
    return 0;
  };
  HIPCHK(hipEventRecord(d->ev_fork, cs));  // the chunk's batches, plan and cursor are in place
  HIPCHK(hipStreamWaitEvent(xs, d->ev_fork, 0));
  for (int64_t k = 0; k < std::min<int64_t>(2, n); ++k)
    if (int r = gather_and_send(k)) return r;
  for (int64_t k = 0; k < n; ++k) {
    const BatchView v = bb.view(k);
    float* gs = grads_par[k & 1];
    HIPCHK(hipStreamWaitEvent(cs, d->ev_rows[k & 3], 0));
    HIPCHK(user_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_xloss, h->d_contrib,
                     h->d_ugrad, rows_par[k & 1], cs));
    HIPCHK(item_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib, h->d_ugrad,
                     gs, cs, h->d_xloss, h->d_loss));
    HIPCHK(hipEventRecord(d->ev_k2[k & 3], cs));
    HIPCHK(hipStreamWaitEvent(xs, d->ev_k2[k & 3], 0));
    for (int p = 0; p < W; ++p) {
      sp[p] = p == self ? nullptr : gs + (int64_t)p * d->S * ld;
      rp[p] = d->grads_recv + (int64_t)p * cap * ld;
    }
    h->stream = xs;
    const int r = d->tr->exchange(h, Xchg{X_GRADS, sp.data(), rp.data(), row_bytes, h->d_tbase, (int)k, 0});
    h->stream = cs;
    if (r) return r;
    HIPCHK(dist_owner_apply(h->geom, h->Q, ids_recv, aplan, n, W, cap, (int)k, h->hp, h->d_tbase,
                            d->grads_recv, self, gs + R * d->S * ld, nullptr, h->d_err, xs));
    if (k + 2 < n)
      if (int r2 = gather_and_send(k + 2)) return r2;
  }
  HIPCHK(hipEventRecord(d->ev_join, xs));  // the last apply before anything after the chunk
  HIPCHK(hipStreamWaitEvent(cs, d->ev_join, 0));
  return 0;
}

// Stale-1 over the IPC transport (the device-flag form): two launches per step on
// one stream, no cross-stream events.
//   front(k): owner phase [k = 0: gather steps 0 and 1 from the current table; k > 0: wait for
//             the gradients of step k-1, apply them, gather step k+1 (rows of the table after step
//             k-1, decayed to step k+1's t-1; none past the chunk)] beside K1(k), which waits for
//             the row flags of step k (pushed by front(k-1), so it never waits on its own launch's
//             owner workgroups except at k = 0);
//   back(k):  K2(k), its gradients straight into the owners' landing buffers;
//   after the chunk: the apply of step n-1.
// Rows and gradients land in two parities (step k: parity k & 1).  Hazards: rows(k+2) can land
// in parity k & 1 only after its owner applied step k, which needs this rank's gradients of step
// k, pushed by back(k) after K1(k) read parity k & 1; gradients(k+2) can land in parity k & 1
// only after their sender's K1(k+2) saw the row flags of step k+2, which every owner raises after
// applying step k (the gradients in parity k & 1).  Flags and boards carry step numbers, so the
// single flag word per peer serves both parities.
static int enqueue_stale1_ipc(bprmf_handle* h, int64_t n, int cap, const int32_t* ids_recv,
                              const int32_t* aplan, bool prof_kernels) {
  DistState* d = h->dist;
  auto* ipc = dynamic_cast<IpcTransport*>(d->tr);
  const int B = h->cfg.batch_size, W = h->cfg.world;
  const int ld = h->geom.ld;
  const BatchBuf bb{h->d_batch, B};
  const int64_t R = h->cfg.rank;
  const int64_t par_rows = (int64_t)W * d->S * ld;  // floats of one landing parity
  float* rows_land[2] = {ipc->landing(X_ROWS), ipc->landing(X_ROWS) + par_rows};
  float* grads_land[2] = {d->grads_recv, d->grads_recv + par_rows};
  float* grads_own[2] = {d->grads_send, d->grads_send1};
  auto row_dst = [&](int par) {  // where the owners' gather puts the rows of a step of parity par
    PushArgs gd{};
    for (int p = 0; p < W; ++p) {
      if (p == R) {
        gd.dst[p] = rows_land[par] + R * d->S * ld;
        gd.flag[p] = const_cast<int32_t*>(ipc->my_flags(X_ROWS)) + R;  // K1 waits on its own too
      } else {
        gd.dst[p] = static_cast<float*>(ipc->peer_landing(X_ROWS, p)) + par * par_rows + R * d->S * ld;
        gd.flag[p] = ipc->peer_flag(X_ROWS, p);
      }
    }
    return gd;
  };
  const PeerWait pw{ipc->my_flags(X_ROWS), W, (int)R, h->d_err};
  const int64_t WC0 = (int64_t)W * cap;
  OwnerArgs oa;
  oa.ids_recv = ids_recv;
  oa.aplan = aplan;
  oa.gdep = aplan + n * WC0 * W;
  oa.gfree = oa.gdep + n * WC0 * W;
  oa.n = n;
  oa.world = W;
  oa.cap = cap;
  oa.self = (int)R;
  oa.wait_flags = ipc->my_flags(X_GRADS);
  oa.mark = ipc->board(IpcTransport::kBoardOwner);
  oa.max_blocks = ipc->owner_blocks();
  oa.lag = 2;
  GradRoute gr[2];
  for (int par = 0; par < 2; ++par) {
    for (int p = 0; p < W; ++p) {
      gr[par].dst[p] = p == R ? grads_own[par] + R * d->S * ld
                              : static_cast<float*>(ipc->peer_landing(X_GRADS, p)) + par * par_rows +
                                    R * (int64_t)cap * ld;
      gr[par].flag[p] = p == R ? nullptr : ipc->peer_flag(X_GRADS, p);
    }
    gr[par].S = d->S;
    gr[par].world = W;
    gr[par].mark = ipc->board(IpcTransport::kBoardK2);
    gr[par].err = h->d_err;
  }
  for (int64_t k = 0; k < n; ++k) {
    const BatchView v = bb.view(k);
    const bool sampled = prof_kernels && ((h->t + k) % kProfStride) == 0;
    const int pk = (int)(k & 1), pa = (int)((k + 1) & 1);  // this step's parity, the other one
    oa.dst = row_dst(k == 0 ? 0 : pa);
    oa.dst1 = row_dst(1);
    oa.grads_recv = grads_land[pa];  // step k-1's gradients (k > 0)
    oa.self_grads = grads_own[pa] + R * d->S * ld;
    {
      ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER, sampled);
      HIPCHK(dist_front(h->geom, oa, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                        h->d_ugrad, h->d_xloss, rows_land[pk], pw, h->stream));
    }
    {
      ProfScope ps(h, BPRMF_KPROF_APPLY, sampled);
      HIPCHK(item_step_push(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                            h->d_ugrad, h->d_xloss, h->d_loss, gr[pk], h->stream));
    }
  }
  const int pl = (int)((n - 1) & 1);
  ProfScope ps(h, BPRMF_KPROF_OWNER, prof_kernels && ((h->t + n - 1) % kProfStride) == 0);
  HIPCHK(dist_owner_apply(h->geom, h->Q, ids_recv, aplan, n, W, cap, (int)(n - 1), h->hp, h->d_tbase,
                          grads_land[pl], (int)R, grads_own[pl] + R * d->S * ld, ipc->my_flags(X_GRADS),
                          h->d_err, h->stream));
  return 0;
}

// The per-step launches and exchanges of a chunk of n steps (plan of `cap` rows per peer):
// enqueued eagerly or captured into a hipGraph by dist_chunk.
static int enqueue_steps(bprmf_handle* h, int64_t n, int cap, const int32_t* ids_recv,
                         const int32_t* aplan, bool prof_kernels) {
  if (h->semantics == BPRMF_SEM_STALE1) {
    auto* ipc = dynamic_cast<IpcTransport*>(h->dist->tr);
    if (!ipc) return enqueue_stale1(h, n, cap, ids_recv, aplan);
    // the device-flag form needs one rank per GPU: its kernels wait inside the launches
    if (!ipc->device_flags())
      return fail(BPRMF_E_UNSUPPORTED, "stale1 semantics over the IPC transport run the device-flag form, "
                                       "which needs one rank per GPU (or BPRMF_DIST_FUSE=1); attach the "
                                       "rccl or loopback transport");
    // (a chunk with nothing to exchange reads no item row: the exact launch sequence below is it)
    if (cap > 0) return enqueue_stale1_ipc(h, n, cap, ids_recv, aplan, prof_kernels);
  }
  DistState* d = h->dist;
  const int B = h->cfg.batch_size, W = h->cfg.world;
  const int ld = h->geom.ld;
  const BatchBuf bb{h->d_batch, B};
  // this rank's own requests bypass the transport (gather into its slots, apply in place)
  const int self = d->tr->self_exchange ? -1 : h->cfg.rank;
  const int64_t R = h->cfg.rank;
  const size_t row_bytes = sizeof(float) * (size_t)cap * ld;
  auto* ipc = dynamic_cast<IpcTransport*>(d->tr);
  const bool fused = ipc && ipc->fused();
  float* rows_in = fused ? ipc->landing(X_ROWS) : d->rows_recv;  // what K1 reads, by slot
  PushArgs gd{};  // where the gather puts the row of position (p, idx): gd.dst[p] + idx * ld
  for (int p = 0; p < W; ++p) {
    if (p == self || (fused && p == R)) {
      gd.dst[p] = rows_in + R * d->S * ld;  // this rank's own slots
    } else if (fused) {
      gd.dst[p] = static_cast<float*>(ipc->peer_landing(X_ROWS, p)) + R * d->S * ld;
      gd.flag[p] = ipc->peer_flag(X_ROWS, p);
    } else {
      gd.dst[p] = d->rows_send + (int64_t)p * cap * ld;
    }
  }
  const PeerWait pw{fused ? ipc->my_flags(X_ROWS) : nullptr, W, (int)R, h->d_err};
  if (fused && cap > 0) {
    // two launches per step: [owner phase of step k | K1(k)], [K2(k) -> owners' landing buffers]
    const int64_t WC0 = (int64_t)W * cap;
    OwnerArgs oa;
    oa.ids_recv = ids_recv;
    oa.aplan = aplan;
    oa.gdep = aplan + n * WC0 * W;
    oa.gfree = oa.gdep + n * WC0 * W;
    oa.n = n;
    oa.world = W;
    oa.cap = cap;
    oa.self = (int)R;
    oa.grads_recv = d->grads_recv;
    oa.self_grads = d->grads_send + R * d->S * ld;
    oa.wait_flags = ipc->my_flags(X_GRADS);
    oa.dst = gd;
    oa.dst.flag[R] = const_cast<int32_t*>(ipc->my_flags(X_ROWS)) + R;  // K1 waits on its own too
    oa.mark = ipc->board(IpcTransport::kBoardOwner);
    oa.max_blocks = ipc->owner_blocks();
    GradRoute gr;
    for (int p = 0; p < W; ++p) {
      gr.dst[p] = p == R ? d->grads_send + R * d->S * ld
                         : static_cast<float*>(ipc->peer_landing(X_GRADS, p)) + R * (int64_t)cap * ld;
      gr.flag[p] = p == R ? nullptr : ipc->peer_flag(X_GRADS, p);
    }
    gr.S = d->S;
    gr.world = W;
    gr.mark = ipc->board(IpcTransport::kBoardK2);
    gr.err = h->d_err;
    for (int64_t k = 0; k < n; ++k) {
      const BatchView v = bb.view(k);
      const bool sampled = prof_kernels && ((h->t + k) % kProfStride) == 0;
      {
        ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER, sampled);
        HIPCHK(dist_front(h->geom, oa, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                          h->d_ugrad, h->d_xloss, rows_in, pw, h->stream));
      }
      {
        ProfScope ps(h, BPRMF_KPROF_APPLY, sampled);
        HIPCHK(item_step_push(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                              h->d_ugrad, h->d_xloss, h->d_loss, gr, h->stream));
      }
    }
    ProfScope ps(h, BPRMF_KPROF_OWNER, prof_kernels && ((h->t + n - 1) % kProfStride) == 0);
    HIPCHK(dist_owner_apply(h->geom, h->Q, ids_recv, aplan, n, W, cap, (int)(n - 1), h->hp, h->d_tbase,
                            d->grads_recv, (int)R, oa.self_grads, ipc->my_flags(X_GRADS), h->d_err,
                            h->stream));
    return 0;
  }
  std::vector<const void*> sp(W);
  std::vector<void*> rp(W);
  const int64_t WC = (int64_t)W * cap;
  const int32_t* gdep = aplan + n * WC * W;
  const int32_t* gfree = gdep + n * WC * W;
  {  // the chunk's first rows; later steps' rows come with the previous step's apply
    ProfScope ps(h, BPRMF_KPROF_OWNER, prof_kernels && (h->t % kProfStride) == 0);
    HIPCHK(dist_owner_gather(h->geom, h->Q, ids_recv, n, W, cap, 0, h->hp, h->d_tbase, gd,
                             fused ? ipc->board(IpcTransport::kBoardOwner) : nullptr, h->d_err,
                             fused ? ipc->owner_blocks() : kBoardMax, h->stream));
  }
  for (int64_t k = 0; k < n; ++k) {
    const BatchView v = bb.view(k);
    const bool sampled = prof_kernels && ((h->t + k) % kProfStride) == 0;
    if (!fused) {
      for (int p = 0; p < W; ++p) {
        sp[p] = p == self ? nullptr : d->rows_send + (int64_t)p * cap * ld;
        rp[p] = d->rows_recv + (int64_t)p * d->S * ld;
      }
      if (int r = d->tr->exchange(h, Xchg{X_ROWS, sp.data(), rp.data(), row_bytes, h->d_tbase, (int)k, 0}))
        return r;
    }
    {
      ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER, sampled);
      HIPCHK(user_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_xloss,
                       h->d_contrib, h->d_ugrad, rows_in, h->stream, pw));
    }
    {
      ProfScope ps(h, BPRMF_KPROF_APPLY, sampled);
      HIPCHK(item_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                       h->d_ugrad, d->grads_send, h->stream, h->d_xloss, h->d_loss));
    }
    for (int p = 0; p < W; ++p) {
      sp[p] = p == self ? nullptr : d->grads_send + (int64_t)p * d->S * ld;
      rp[p] = d->grads_recv + (int64_t)p * cap * ld;
    }
    const Xchg xg{X_GRADS, sp.data(), rp.data(), row_bytes, h->d_tbase, (int)k, 0};
    if (int r = fused ? (row_bytes ? ipc->push(h, xg) : 0) : d->tr->exchange(h, xg)) return r;
    {
      ProfScope ps(h, BPRMF_KPROF_OWNER, sampled);
      const int32_t* wf = fused ? ipc->my_flags(X_GRADS) : nullptr;
      const float* own = d->grads_send + R * d->S * ld;
      if (k + 1 < n)  // apply step k, gather step k+1
        HIPCHK(dist_owner_step(h->geom, h->Q, ids_recv, aplan, gdep, gfree, n, W, cap, (int)k, h->hp,
                               h->d_tbase, d->grads_recv, self, own, wf, h->d_err, gd,
                               fused ? ipc->board(IpcTransport::kBoardOwner) : nullptr,
                               fused ? ipc->owner_blocks() : kBoardMax, h->stream));
      else
        HIPCHK(dist_owner_apply(h->geom, h->Q, ids_recv, aplan, n, W, cap, (int)k, h->hp, h->d_tbase,
                                d->grads_recv, self, own, wf, h->d_err, h->stream));
    }
  }
  return 0;
}

// A chunk shape (n, cap, buffers) is captured the second time it is seen and replayed from then
// on; the first time its steps are launched eagerly (each step is several kernels of several us,
// so the host keeps ahead): a short run of odd-length chunks (a benchmark's warm-up and timed
// calls) then never pays a capture inside a call, and a long run replays graphs.
// Returns 1 when the caller should enqueue the steps eagerly instead.
static int launch_dist_graph(bprmf_handle* h, int64_t n, int cap, const int32_t* ids_recv,
                             const int32_t* aplan, bool* eager) {
  DistState* d = h->dist;
  const void* bufs[4] = {h->d_batch, ids_recv, aplan, h->d_contrib};
  DistGraph* ge = nullptr;
  for (auto& g : d->graphs)
    if (g.n == n && g.cap == cap && std::equal(bufs, bufs + 4, g.bufs)) ge = &g;
  *eager = false;
  if (!ge) {  // first sighting: remember the shape, run eagerly
    if (d->graphs.size() >= 16) drop_dist_graphs(d);
    DistGraph ng;
    ng.n = n;
    ng.cap = cap;
    std::copy(bufs, bufs + 4, ng.bufs);
    d->graphs.push_back(ng);
    *eager = true;
    return 0;
  }
  if (!ge->exec) {
    HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_steps(h, n, cap, ids_recv, aplan, false);
    hipGraph_t graph = nullptr;
    const hipError_t e2 = hipStreamEndCapture(h->stream, &graph);
    if (rc || e2 != hipSuccess) {
      if (graph) (void)!hipGraphDestroy(graph);
      return rc ? rc : fail(BPRMF_E_HIP, "sharded step graph capture: %s", hipGetErrorString(e2));
    }
    const hipError_t e = hipGraphInstantiate(&ge->exec, graph, nullptr, nullptr, 0);
    (void)!hipGraphDestroy(graph);
    if (e != hipSuccess) {
      ge->exec = nullptr;
      return fail(BPRMF_E_HIP, "sharded step graph instantiate: %s", hipGetErrorString(e));
    }
    const hipError_t eu = hipGraphUpload(ge->exec, h->stream);  // device-side setup before its first replay
    if (eu != hipSuccess) {
      (void)!hipGraphExecDestroy(ge->exec);
      ge->exec = nullptr;
      return fail(BPRMF_E_HIP, "sharded step graph upload: %s", hipGetErrorString(eu));
    }
  }
  HIPCHK(hipGraphLaunch(ge->exec, h->stream));
  return 0;
}

// n steps from the device sampler (ru == null: steps [first_step, first_step + n) of `epoch`) or
// from device triplets ru/ri/rj[n * B] (this shard's users, u < 0 = empty slot)
static int dist_chunk(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n,
                      const int32_t* ru, const int32_t* ri, const int32_t* rj) {
  DistState* d = h->dist;
  const int B = h->cfg.batch_size, W = h->cfg.world;
  if (n > d->nmax) return fail(BPRMF_E_INVALID, "chunk of %lld steps > %lld", (long long)n, (long long)d->nmax);
  if ((int64_t)h->t + n >= INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  if (int r = ensure_seg(h, n)) return r;
  const BatchBuf bb{h->d_batch, B};
  const int par = (int)(d->chunks & 1);
  const int32_t seq = (int32_t)(d->chunks + 1);
  // the cursor, the call's loss slots and the chunk's capacity max: the builder's first workgroup
  // and its item parts (one launch fewer each), or their own launches (every per-wave loss slot to
  // zero; the one-workgroup build)
  CursorInit ci;
  ci.cursor = h->d_tbase;
  ci.t = h->t;
  ci.loss = h->d_loss;
  ci.nloss = loss_zero_slots(h);
  ci.own_max = d->d_cap;  // zero: the previous chunk's pair_out (or the allocation) cleared it
  if (ci.nloss > kSegLossSlots) {
    HIPCHK(set_cursor(h->d_tbase, h->t, 0, h->stream, h->d_loss, ci.nloss));
    ci.cursor = nullptr;
    ci.loss = nullptr;
    ci.nloss = 0;
  }
  bool own_max_done = false;
  int64_t first_slot = 0, n_slots = n * B;
  if (!ru) {
    int64_t N;
    bprmf_epoch_size(h, &N, nullptr);
    first_slot = first_step * B;
    n_slots = std::max<int64_t>(0, std::min(N - first_slot, n * B));
  }
  {
    ProfScope ps(h, BPRMF_KPROF_SAMPLE);
    if (!ru && n_slots > 0 && split_build(n)) {  // short chunk: grid-wide sampler first
      if (int r = ensure_trip(h, n_slots)) return r;
      int32_t* tu = h->d_trip;
      // sampled inside the split builder's launch on one rank per GPU, else by k_sample first
      const bool in_launch = !d->tr->shares_device();
      if (!in_launch)
        HIPCHK(sample(sampler_args(h), epoch, first_slot, n_slots, tu, tu + h->trip_cap,
                      tu + 2 * h->trip_cap, h->d_err, h->stream));
      HIPCHK(build_batches(sampler_args(h), epoch, in_launch ? first_slot : 0, n_slots, B, tu,
                           tu + h->trip_cap, tu + 2 * h->trip_cap, h->U, h->cfg.item_num, W, true,
                           d->S, n, bb, h->d_err, h->stream, k1_triplets_per_block(h->geom), ci,
                           &own_max_done, in_launch));
    } else {
      HIPCHK(build_batches(sampler_args(h), epoch, first_slot, n_slots, B, ru, ri, rj, h->U,
                           h->cfg.item_num, W, true, d->S, n, bb, h->d_err, h->stream,
                           k1_triplets_per_block(h->geom), ci, &own_max_done));
    }
  }
  // exchange capacity of the chunk: the largest request count of any (rank, step, owner)
  if (!own_max_done) HIPCHK(dist_own_max(bb, n, W, d->d_cap, h->stream));
  if (int r = d->tr->max_i32(h, d->d_cap, d->vals + par * W, seq)) return r;
  // cap and the error word back in one wait: a tiny kernel writes them and then a sequence
  // number into the mapped status block, and the host spins on that number
  volatile int32_t* hv = reinterpret_cast<volatile int32_t*>(h->h_status + 8);
  const uint64_t cseq = ++h->status_seq;
  HIPCHK(pair_out(d->d_cap, h->d_err, h->h_status_dev + 8, h->h_status_dev + kSeqCapOff, cseq, h->stream,
                  d->d_cap));
  if (int r = wait_mapped_seq(h, kSeqCapOff, cseq)) return r;
  int32_t cap = hv[0];
  if (hv[1]) {
    if (int r = check_err_flag(h)) return r;
  }
  const bool graph = h->use_graphs && d->tr->capturable() && cap > 0;
  const int raw = cap;
  cap = exchange_capacity(raw, d->S, graph);  // graphs: rounded to 64 rows, so plans get reused
  if (cap < 0) return fail(BPRMF_E_STATE, "exchange capacity %d outside [0, %d]", raw, d->S);
  d->cap = cap;
  if (int r = ensure_aplan(h, par, n, cap)) return r;
  {
    const int64_t peers = W - 1, rowb = (int64_t)cap * h->geom.ld * (int64_t)sizeof(float);
    d->x_steps += n;
    d->x_rows += n * peers * rowb;
    d->x_grads += n * peers * rowb;
    d->x_ids += cap > 0 ? peers * n * cap * (int64_t)sizeof(int32_t) : 0;
  }
  int32_t* ids_recv = d->ids_recv + (int64_t)par * W * d->nmax * d->S;
  int32_t* aplan = d->aplan[par];
  if (cap > 0) {
    std::vector<const void*> sp(W);
    std::vector<void*> rp(W);
    HIPCHK(dist_pack_ids(bb, n, W, cap, d->ids_send, h->stream));
    for (int p = 0; p < W; ++p) {
      sp[p] = d->ids_send + (int64_t)p * n * cap;
      rp[p] = ids_recv + (int64_t)p * n * cap;
    }
    const bool se = d->tr->self_exchange;
    d->tr->self_exchange = false;  // the request lists always include the self block
    const int r = d->tr->exchange(h, Xchg{X_IDS, sp.data(), rp.data(), sizeof(int32_t) * n * cap,
                                          nullptr, 0, seq});
    d->tr->self_exchange = se;
    if (r) return r;
    HIPCHK(dist_owner_plan(ids_recv, n, W, cap, h->semantics == BPRMF_SEM_STALE1 ? 2 : 1, aplan,
                           aplan + n * W * (int64_t)cap * W,
                           aplan + 2 * n * W * (int64_t)cap * W, h->stream));
  }
  hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;
  if (ea) HIPCHK(hipEventRecord(ea, h->stream));
  bool eager = !graph;
  if (graph)
    if (int r = launch_dist_graph(h, n, cap, ids_recv, aplan, &eager)) return r;
  if (eager)
    if (int r = enqueue_steps(h, n, cap, ids_recv, aplan, !ea)) return r;
  if (ea) {
    hipEvent_t eb = prof_event(h);
    if (eb) {
      HIPCHK(hipEventRecord(eb, h->stream));
      h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
      h->prof_weight[BPRMF_KPROF_STEPS] += n - 1;
    }
  }
  h->t += (int32_t)n;
  ++d->chunks;
  return 0;
}

// ---- semantics LOCAL at world > 1: the item table replicated, merged across ranks ------------
// (include/bprmf.h BPRMF_SEM_LOCAL.)  Every rank trains its own users' triplets
// with the single-GPU local step (hogwild.hip, hot items in per-XCD replicas) on its own copy of
// the whole item table; a merge brings every rank's copy to base + the sum of the ranks' changes.
int dp_quiesce(bprmf_handle* h) {
  if (!h->dp_pending) return 0;
  h->dp_pending = false;
  if (h->dist)
    if (int r = h->dist->tr->allreduce_wait(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

// dp_overlap and not the call's last merge: the all-reduce is only started (beside the next
// period), and lands at the next merge.  Otherwise blocking: every rank leaves with base + sum.
static int dp_merge(bprmf_handle* h, bool last) {
  Transport* tr = h->dist->tr;
  const bool pend = h->dp_pending;
  if (pend)
    if (int r = tr->allreduce_wait(h)) return r;
  const int32_t tp = pend ? h->dp_tp : h->dp_t;
  const bool start = h->dp_overlap && !last;
  // the hot items' XCD replicas are merged inside the delta pass (k_local_merge's rule)
  const LocalArgs la = local_args(h);
  HIPCHK(dp_delta(h->Q, h->d_qbase, h->d_qdelta, pend ? h->dp_sum : nullptr, h->geom.ld, h->hp, h->dp_t, tp,
                  h->t, la, h->rep_t, start, h->stream));
  h->dp_t = tp;  // the base is current at tp now
  h->dp_pending = false;
  const int64_t n = h->I * (int64_t)h->geom.ld;
  // what a ring all-reduce moves per rank (reduce-scatter + all-gather): 2 (W-1)/W of the table
  const int64_t W = h->cfg.world;
  h->dist->x_grads += 2 * (W - 1) * (n * (int64_t)sizeof(float)) / W;
  if (start) {
    if (int r = tr->allreduce_start(h, h->d_qdelta, h->d_qsum, n, &h->dp_sum)) return r;
    h->dp_pending = true;
    h->dp_tp = h->t;
    h->rep_t = h->t;  // the rows and replicas went on from this rank's own result
    return 0;
  }
  const float* sum = nullptr;
  if (int r = tr->allreduce_sum(h, h->d_qdelta, n, &sum)) return r;
  // the merged rows, and the hot items' replicas restart from them (in the same pass)
  HIPCHK(dp_apply(h->Q, h->d_qbase, sum, h->geom.ld, h->hp, h->dp_t, h->t, la, h->stream));
  h->rep_t = h->dp_t = h->t;
  return 0;
}

// steps [first_step, first_step + n_steps) of this rank's epoch (sampled; slots past the rank's
// own epoch are empty, so every rank takes the same steps and merges) or n_steps * B replayed
// device ids ru/ri/rj (global ids, u < 0: empty slot).  The call ends merged.
// final: this is the call's last run of steps, which ends with a blocking merge (the host then
// sees the same table on every rank).  A replay call runs its chunks with final = false but for
// the last, so its merges follow dp_steps like a sampled call's do.
static int dp_run(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                  const int32_t* ru, const int32_t* ri, const int32_t* rj, int64_t* triplets,
                  bool final = true) {
  const int64_t B = h->cfg.batch_size;
  if ((int64_t)h->t + n_steps >= INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  int64_t N = 0;
  bprmf_epoch_size(h, &N, nullptr);
  if (int z = loss_zero_slots(h)) HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * z, h->stream));
  const SamplerArgs sa = sampler_args(h);
  const LocalArgs la = local_args(h);
  hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;  // one pair: the periods and the merges
  if (ea) HIPCHK(hipEventRecord(ea, h->stream));
  h->dist->x_steps += n_steps;
  for (int64_t s = 0; s < n_steps;) {
    int64_t m = n_steps - s;
    if (la.H > 0) m = std::min<int64_t>(m, std::max<int64_t>(1, h->local_steps - (h->t - h->rep_t)));
    m = std::min<int64_t>(m, std::max<int64_t>(1, h->dp_steps - (h->t - (h->dp_pending ? h->dp_tp : h->dp_t))));
    int64_t a0 = s * B, a1 = (s + m) * B;  // replay: positions in ru/ri/rj
    if (!ru) {
      a0 = std::min(N, (first_step + s) * B);
      a1 = std::min(N, (first_step + s + m) * B);
    }
    if (a1 > a0) {
      HIPCHK(hogwild(h->geom, ru ? nullptr : &sa, epoch, a0, ru ? ru + a0 : nullptr, ri ? ri + a0 : nullptr,
                     rj ? rj + a0 : nullptr, a1 - a0, h->P, h->Q, h->hp, h->t, (int)B, h->d_loss, h->d_err,
                     h->stream, la.H > 0 ? &la : nullptr, h->cfg.world));
      if (!ru) *triplets += a1 - a0;
    }
    h->t += (int32_t)m;
    s += m;
    const int32_t since = h->t - (h->dp_pending ? h->dp_tp : h->dp_t);  // steps since the last merge
    if (since >= h->dp_steps || (final && s >= n_steps)) {
      if (int r = dp_merge(h, final && s >= n_steps)) return r;
    } else if (la.H > 0 && h->t - h->rep_t >= h->local_steps) {
      HIPCHK(local_merge(h->geom, h->Q, la, h->d_hot_rows, h->hp, h->rep_t, h->t, false, h->stream));
      h->rep_t = h->t;
    }
  }
  if (ea) {
    hipEvent_t eb = prof_event(h);
    if (eb) {
      HIPCHK(hipEventRecord(eb, h->stream));
      h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
      h->prof_weight[BPRMF_KPROF_STEPS] += n_steps - 1;
    }
  }
  return 0;
}

}  // namespace bprmf

using namespace bprmf;

extern "C" {

int bprmf_dist_unique_id(uint8_t* id) {
  if (!id) return fail(BPRMF_E_INVALID, "null argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return 0;
}

int bprmf_dist_init_rccl(bprmf_handle* h, const uint8_t* id) {
  if (!h || !id) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = set_dev(h)) return r;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  auto* tr = new RcclTransport();
  const ncclResult_t e = ncclCommInitRank(&tr->comm, h->cfg.world, u, h->cfg.rank);
  if (e != ncclSuccess) {
    tr->comm = nullptr;
    delete tr;
    return fail(BPRMF_E_HIP, "ncclCommInitRank: %s", ncclGetErrorString(e));
  }
  return dist_attach(h, tr);
}

int bprmf_dist_ipc_export(bprmf_handle* h, uint8_t* blob) {
  if (!h || !blob) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = set_dev(h)) return r;
  static_assert(sizeof(hipIpcMemHandle_t) * kIpcHandles <= BPRMF_IPC_BLOB_BYTES, "blob size");
  auto* tr = new IpcTransport();
  tr->world = h->cfg.world;
  tr->rank = h->cfg.rank;
  const size_t flag_bytes = sizeof(int32_t) * X_KINDS * kMaxWorld;
  hipError_t e = hipExtMallocWithFlags(&tr->local[X_KINDS], flag_bytes, hipDeviceMallocUncached);
  const size_t board_bytes = sizeof(int32_t) * IpcTransport::kBoards * kBoardMax;
  if (e == hipSuccess) e = hipMalloc((void**)&tr->boards, board_bytes);
  if (e == hipSuccess) e = hipMemset(tr->local[X_KINDS], 0, flag_bytes);
  if (e == hipSuccess) e = hipMemset(tr->boards, 0, board_bytes);
  if (e != hipSuccess) {
    delete tr;
    return fail(BPRMF_E_HIP, "ipc transport buffers: %s", hipGetErrorString(e));
  }
  if (int r = dist_attach(h, tr)) return r;
  memset(blob, 0, BPRMF_IPC_BLOB_BYTES);
  for (int b = 0; b < kIpcHandles; ++b) {
    hipIpcMemHandle_t hd;
    HIPCHK(hipIpcGetMemHandle(&hd, tr->local[b]));
    memcpy(blob + b * sizeof hd, &hd, sizeof hd);
  }
  // this rank's physical device (PCI bus id) after the handles: peers on the same GPU are seen
  static_assert(sizeof(hipIpcMemHandle_t) * kIpcHandles + kBusIdBytes <= BPRMF_IPC_BLOB_BYTES, "blob");
  HIPCHK(hipDeviceGetPCIBusId(reinterpret_cast<char*>(blob) + kIpcHandles * sizeof(hipIpcMemHandle_t),
                              kBusIdBytes - 1, h->cfg.device));
  return 0;
}

int bprmf_dist_init_ipc(bprmf_handle* h, const uint8_t* blobs) {
  if (!h || !blobs) return fail(BPRMF_E_INVALID, "null argument");
  auto* tr = h->dist ? dynamic_cast<IpcTransport*>(h->dist->tr) : nullptr;
  if (!tr) return fail(BPRMF_E_STATE, "call bprmf_dist_ipc_export first");
  if (tr->opened) return fail(BPRMF_E_STATE, "ipc transport already initialised");
  if (int r = set_dev(h)) return r;
  for (int b = 0; b < kIpcHandles; ++b) tr->remote[b].assign(tr->world, nullptr);
  tr->shared_device = ipc_shares_device(blobs, tr->world, tr->rank, BPRMF_IPC_BLOB_BYTES,
                                        kIpcHandles * sizeof(hipIpcMemHandle_t), kBusIdBytes);
  for (int p = 0; p < tr->world; ++p)
    for (int b = 0; b < kIpcHandles; ++b) {
      if (p == tr->rank) {
        tr->remote[b][p] = tr->local[b];
        continue;
      }
      hipIpcMemHandle_t hd;
      memcpy(&hd, blobs + (size_t)p * BPRMF_IPC_BLOB_BYTES + b * sizeof hd, sizeof hd);
      HIPCHK(hipIpcOpenMemHandle(&tr->remote[b][p], hd, hipIpcMemLazyEnablePeerAccess));
    }
  tr->opened = true;
  return 0;
}

int bprmf_dist_init_loopback(bprmf_handle* h, int64_t group) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = set_dev(h)) return r;
  auto* tr = new LoopTransport();
  {
    std::lock_guard<std::mutex> l(g_loops_m);
    LoopGroup*& g = g_loops[group];
    if (!g) {
      g = new LoopGroup();
      g->world = h->cfg.world;
      g->send.assign(h->cfg.world, nullptr);
      g->val.assign(h->cfg.world, 0);
      g->fbuf.assign(h->cfg.world, nullptr);
    }
    if (g->world != h->cfg.world) {
      delete tr;
      return fail(BPRMF_E_INVALID, "loopback group %lld has world %d", (long long)group, g->world);
    }
    ++g->refs;
    tr->key = group;
    tr->g = g;
  }
  return dist_attach(h, tr);
}

int bprmf_dist_exchange_stats(bprmf_handle* h, int64_t* steps, int64_t* row_bytes,
                              int64_t* grad_bytes, int64_t* id_bytes) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  const DistState* d = h->dist;
  if (steps) *steps = d ? d->x_steps : 0;
  if (row_bytes) *row_bytes = d ? d->x_rows : 0;
  if (grad_bytes) *grad_bytes = d ? d->x_grads : 0;
  if (id_bytes) *id_bytes = d ? d->x_ids : 0;
  return 0;
}

int bprmf_dist_train_steps(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                           bprmf_stats* st) {
  if (!h || first_step < 0 || n_steps < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->dist || !h->dist->tr->ready())
    return fail(BPRMF_E_STATE, "attach a transport first (bprmf_dist_init_*)");
  if (!h->d_pos_u) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
  if (h->dp_mode) {  // LOCAL at world > 1
    if (int r = begin_call(h)) return r;
    int64_t trip = 0;
    if (int r = dp_run(h, epoch, first_step, n_steps, nullptr, nullptr, nullptr, &trip)) return r;
    return end_call(h, st, trip, n_steps);
  }
  // one rank: nothing to exchange, so the single-GPU fused step runs (the same sampler stream,
  // the same step; BPRMF_DIST_W1_RUNNER=1 keeps the runner, to measure it).  STALE1 keeps the
  // runner (its rows are stale at one rank too).
  if (h->cfg.world == 1 && !h->dist->tr->self_exchange && h->semantics != BPRMF_SEM_STALE1) {
    const char* e = getenv("BPRMF_DIST_W1_RUNNER");
    if (!(e && e[0] == '1')) return bprmf_train_steps(h, epoch, first_step, n_steps, st);
  }
  if (int r = begin_call(h)) return r;
  const int64_t chunk = dist_chunk_steps(h);
  for (int64_t s = 0; s < n_steps; s += chunk)
    if (int r = dist_chunk(h, epoch, first_step + s, std::min(chunk, n_steps - s), nullptr, nullptr,
                           nullptr))
      return r;
  int64_t N;
  bprmf_epoch_size(h, &N, nullptr);
  const int64_t B = h->cfg.batch_size;
  const int64_t trip = std::max<int64_t>(0, std::min(N, (first_step + n_steps) * B) - first_step * B);
  return end_call(h, st, trip, n_steps);
}

int bprmf_dist_train_replay(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                            int64_t n_steps, bprmf_stats* st) {
  if (!h || n_steps < 0 || (n_steps > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->dist || !h->dist->tr->ready())
    return fail(BPRMF_E_STATE, "attach a transport first (bprmf_dist_init_*)");
  const int64_t B = h->cfg.batch_size, n = n_steps * B, W = h->cfg.world, R = h->cfg.rank;
  int64_t valid = 0;
  for (int64_t k = 0; k < n; ++k) {
    if (u[k] < 0) continue;  // empty slot
    if (u[k] >= h->cfg.user_num || u[k] % W != R)
      return fail(BPRMF_E_RANGE, "user %d at %lld is not a user of shard %lld", u[k], (long long)k, (long long)R);
    if (i[k] < 0 || i[k] >= h->cfg.item_num || j[k] < 0 || j[k] >= h->cfg.item_num)
      return fail(BPRMF_E_RANGE, "item id at %lld out of range", (long long)k);
    ++valid;
  }
  if (int r = set_dev(h)) return r;
  if (int r = begin_call(h)) return r;
  const int64_t chunk = dist_chunk_steps(h);
  if (int r = ensure_trip(h, std::min(chunk, std::max<int64_t>(n_steps, 1)) * B)) return r;
  for (int64_t s = 0; s < n_steps; s += chunk) {
    const int64_t m = std::min(chunk, n_steps - s);
    int32_t* tu = h->d_trip;
    int32_t* ti = tu + h->trip_cap;
    int32_t* tj = ti + h->trip_cap;
    HIPCHK(hipMemcpyAsync(tu, u + s * B, 4 * m * B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(ti, i + s * B, 4 * m * B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(tj, j + s * B, 4 * m * B, hipMemcpyHostToDevice, h->stream));
    if (h->dp_mode) {
      int64_t unused = 0;
      if (int r = dp_run(h, 0, 0, m, tu, ti, tj, &unused, s + m >= n_steps)) return r;
    } else if (int r = dist_chunk(h, 0, 0, m, tu, ti, tj)) {
      return r;
    }
    HIPCHK(hipStreamSynchronize(h->stream));  // the next chunk's copies reuse d_trip
  }
  return end_call(h, st, valid, n_steps);
}

}  // extern "C"
