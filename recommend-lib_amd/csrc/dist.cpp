// dist.cpp — the sharded multi-GPU runner behind bprmf_dist_train_* (include/bprmf.h).
//
// One handle per GPU (one process per GPU under torch.distributed.run).  The runner drives whole
// chunks of steps from C++: no Python per step.  Transports:
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
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <vector>

#include "handle.h"

namespace bprmf {

struct Transport {
  virtual ~Transport() = default;
  // all-to-all of per-peer blocks of `bytes`: send[p] goes to rank p, recv[p] comes from rank p;
  // send[rank] == nullptr: no self block (the caller placed it already)
  virtual int exchange(bprmf_handle* h, const void* const* send, void* const* recv, size_t bytes) = 0;
  // in-place max over ranks of one device int32
  virtual int max_i32(bprmf_handle* h, int32_t* dev) = 0;
};

#define NCCLCHK(x)                                                                      \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) return fail(BPRMF_E_HIP, "%s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

struct RcclTransport final : Transport {
  ncclComm_t comm = nullptr;
  ~RcclTransport() override {
    if (comm) ncclCommDestroy(comm);
  }
  int exchange(bprmf_handle* h, const void* const* send, void* const* recv, size_t bytes) override {
    if (!bytes) return 0;
    const int W = h->cfg.world, R = h->cfg.rank;
    if (send[R]) HIPCHK(hipMemcpyAsync(recv[R], send[R], bytes, hipMemcpyDeviceToDevice, h->stream));
    if (W == 1) return 0;
    NCCLCHK(ncclGroupStart());
    for (int p = 0; p < W; ++p) {
      if (p == R) continue;
      NCCLCHK(ncclSend(send[p], bytes, ncclUint8, p, comm, h->stream));
      NCCLCHK(ncclRecv(recv[p], bytes, ncclUint8, p, comm, h->stream));
    }
    NCCLCHK(ncclGroupEnd());
    return 0;
  }
  int max_i32(bprmf_handle* h, int32_t* dev) override {
    if (h->cfg.world == 1) return 0;
    NCCLCHK(ncclAllReduce(dev, dev, 1, ncclInt32, ncclMax, comm, h->stream));
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
  int64_t key = 0;
  LoopGroup* g = nullptr;
  ~LoopTransport() override {
    std::lock_guard<std::mutex> l(g_loops_m);
    if (g && --g->refs == 0) {
      g_loops.erase(key);
      delete g;
    }
  }
  int exchange(bprmf_handle* h, const void* const* send, void* const* recv, size_t bytes) override {
    const int W = h->cfg.world, R = h->cfg.rank;
    HIPCHK(hipStreamSynchronize(h->stream));  // this shard's blocks are complete
    g->send[R] = send;
    g->barrier();
    int rc = 0;
    for (int p = 0; p < W && !rc && bytes; ++p) {
      if (!g->send[p][R]) continue;
      const hipError_t e = hipMemcpyAsync(recv[p], g->send[p][R], bytes, hipMemcpyDeviceToDevice, h->stream);
      if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback copy: %s", hipGetErrorString(e));
    }
    const hipError_t e = hipStreamSynchronize(h->stream);
    if (!rc && e != hipSuccess) rc = fail(BPRMF_E_HIP, "loopback sync: %s", hipGetErrorString(e));
    g->barrier();  // every peer has read this shard's send blocks
    return rc;
  }
  int max_i32(bprmf_handle* h, int32_t* dev) override {
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

struct DistState {
  Transport* tr = nullptr;
  int S = 0;             // requester-side slot stride per owner (rows)
  int cap = 0;           // rows per peer per step of the current chunk
  int64_t ids_n = 0, aplan_n = 0;
  int32_t* ids_send = nullptr;  // [W][n][cap]
  int32_t* ids_recv = nullptr;  // [W][n][cap]
  int32_t* aplan = nullptr;     // [n][W][cap][W]
  int32_t* d_cap = nullptr;
  float* rows_send = nullptr;   // owner:     [W][cap][ld]
  float* rows_recv = nullptr;   // requester: [W][S][ld] (slot order)
  float* grads_send = nullptr;  // requester: [W][S][ld]
  float* grads_recv = nullptr;  // owner:     [W][cap][ld]
};

void dist_free(DistState* d) {
  if (!d) return;
  delete d->tr;
  void* ptrs[] = {d->ids_send, d->ids_recv, d->aplan, d->d_cap, d->rows_send, d->rows_recv,
                  d->grads_send, d->grads_recv};
  for (void* p : ptrs)
    if (p) hipFree(p);
  delete d;
}

static int dist_attach(bprmf_handle* h, Transport* tr) {
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
  h->dist = d;
  const int64_t W = h->cfg.world, B = h->cfg.batch_size;
  const int64_t iloc = (h->cfg.item_num + W - 1) / W;
  d->S = (int)std::min<int64_t>(2 * B, iloc);
  const int64_t rows = W * d->S * h->geom.ld;
  if (int r = dalloc(&d->d_cap, 1)) return r;
  if (int r = dalloc(&d->rows_send, rows)) return r;
  if (int r = dalloc(&d->rows_recv, rows)) return r;
  if (int r = dalloc(&d->grads_send, rows)) return r;
  if (int r = dalloc(&d->grads_recv, rows)) return r;
  // rows past a peer's request count are sent but never read; keep them finite
  HIPCHK(hipMemsetAsync(d->rows_send, 0, sizeof(float) * rows, h->stream));
  HIPCHK(hipMemsetAsync(d->grads_send, 0, sizeof(float) * rows, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

static int ensure_plan_bufs(bprmf_handle* h, int64_t n, int cap) {
  DistState* d = h->dist;
  const int64_t W = h->cfg.world;
  const int64_t ids = W * n * cap, ap = ids * W;
  if (ids > d->ids_n) {
    if (d->ids_send) HIPCHK(hipFree(d->ids_send));
    if (d->ids_recv) HIPCHK(hipFree(d->ids_recv));
    d->ids_send = d->ids_recv = nullptr;
    d->ids_n = 0;
    if (int r = dalloc(&d->ids_send, ids)) return r;
    if (int r = dalloc(&d->ids_recv, ids)) return r;
    d->ids_n = ids;
  }
  if (ap > d->aplan_n) {
    if (d->aplan) HIPCHK(hipFree(d->aplan));
    d->aplan = nullptr;
    d->aplan_n = 0;
    if (int r = dalloc(&d->aplan, ap)) return r;
    d->aplan_n = ap;
  }
  return 0;
}

// n steps from the device sampler (ru == null: steps [first_step, first_step + n) of `epoch`) or
// from device triplets ru/ri/rj[n * B] (this shard's users, u < 0 = empty slot)
static int dist_chunk(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n,
                      const int32_t* ru, const int32_t* ri, const int32_t* rj) {
  DistState* d = h->dist;
  const int B = h->cfg.batch_size, W = h->cfg.world, R = h->cfg.rank;
  const int ld = h->geom.ld;
  if ((int64_t)h->t + n >= INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  if (int r = ensure_seg(h, n)) return r;
  const BatchBuf bb{h->d_batch, B};
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->d_tbase, h->t, 1, h->stream));
  int64_t first_slot = 0, n_slots = n * B;
  if (!ru) {
    int64_t N;
    bprmf_epoch_size(h, &N, nullptr);
    first_slot = first_step * B;
    n_slots = std::max<int64_t>(0, std::min(N - first_slot, n * B));
  }
  {
    ProfScope ps(h, BPRMF_KPROF_SAMPLE);
    HIPCHK(build_batches(sampler_args(h), epoch, first_slot, n_slots, B, ru, ri, rj, h->U,
                         h->cfg.item_num, W, true, d->S, n, bb, h->d_err, h->stream));
  }
  // exchange capacity of the chunk: the largest request count of any (rank, step, owner)
  HIPCHK(hipMemsetAsync(d->d_cap, 0, 4, h->stream));
  HIPCHK(dist_own_max(bb, n, W, d->d_cap, h->stream));
  if (int r = d->tr->max_i32(h, d->d_cap)) return r;
  int32_t cap = 0;
  HIPCHK(hipMemcpyAsync(&cap, d->d_cap, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (cap < 0 || cap > d->S) return fail(BPRMF_E_STATE, "exchange capacity %d outside [0, %d]", cap, d->S);
  d->cap = cap;
  if (int r = ensure_plan_bufs(h, n, std::max(cap, 1))) return r;
  std::vector<const void*> sp(W);
  std::vector<void*> rp(W);
  if (cap > 0) {
    HIPCHK(dist_pack_ids(bb, n, W, cap, d->ids_send, h->stream));
    for (int p = 0; p < W; ++p) {
      sp[p] = d->ids_send + (int64_t)p * n * cap;
      rp[p] = d->ids_recv + (int64_t)p * n * cap;
    }
    if (int r = d->tr->exchange(h, sp.data(), rp.data(), sizeof(int32_t) * n * cap)) return r;
    HIPCHK(dist_owner_plan(d->ids_recv, n, W, cap, d->aplan, h->stream));
  }
  hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;
  if (ea) HIPCHK(hipEventRecord(ea, h->stream));
  const size_t row_bytes = sizeof(float) * (size_t)cap * ld;
  for (int64_t k = 0; k < n; ++k) {
    const BatchView v = bb.view(k);
    const bool sampled = ((h->t + k) % kProfStride) == 0;
    {
      ProfScope ps(h, BPRMF_KPROF_OWNER, sampled && !ea);
      HIPCHK(dist_owner_gather(h->geom, h->Q, d->ids_recv, n, W, cap, (int)k, h->hp, h->d_tbase,
                               d->rows_send, R, d->rows_recv + (int64_t)R * d->S * ld, h->stream));
    }
    for (int p = 0; p < W; ++p) {
      sp[p] = p == R ? nullptr : d->rows_send + (int64_t)p * cap * ld;
      rp[p] = d->rows_recv + (int64_t)p * d->S * ld;
    }
    if (int r = d->tr->exchange(h, sp.data(), rp.data(), row_bytes)) return r;
    {
      ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER, sampled && !ea);
      HIPCHK(user_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_loss,
                       h->d_contrib, h->d_ugrad, d->rows_recv, h->stream));
    }
    {
      ProfScope ps(h, BPRMF_KPROF_APPLY, sampled && !ea);
      HIPCHK(item_step(h->geom, v, B, h->P, h->Q, h->hp, h->d_tbase, (int)k, h->d_contrib,
                       h->d_ugrad, d->grads_send, h->stream));
    }
    for (int p = 0; p < W; ++p) {
      sp[p] = p == R ? nullptr : d->grads_send + (int64_t)p * d->S * ld;
      rp[p] = d->grads_recv + (int64_t)p * cap * ld;
    }
    if (int r = d->tr->exchange(h, sp.data(), rp.data(), row_bytes)) return r;
    {
      ProfScope ps(h, BPRMF_KPROF_OWNER, sampled && !ea);
      HIPCHK(dist_owner_apply(h->geom, h->Q, d->ids_recv, d->aplan, n, W, cap, (int)k, h->hp,
                              h->d_tbase, d->grads_recv, R, d->grads_send + (int64_t)R * d->S * ld,
                              h->stream));
    }
  }
  if (ea) {
    hipEvent_t eb = prof_event(h);
    if (eb) {
      HIPCHK(hipEventRecord(eb, h->stream));
      h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
      h->prof_weight[BPRMF_KPROF_STEPS] += n - 1;
    }
  }
  h->t += (int32_t)n;
  return 0;
}

static int64_t dist_chunk_steps(const bprmf_handle* h) {
  return std::max<int64_t>(1, (int64_t(1) << 20) / h->cfg.batch_size);
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

int bprmf_dist_train_steps(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                           bprmf_stats* st) {
  if (!h || first_step < 0 || n_steps < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->dist) return fail(BPRMF_E_STATE, "attach a transport first (bprmf_dist_init_*)");
  if (!h->d_pos_u) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
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
  if (!h->dist) return fail(BPRMF_E_STATE, "attach a transport first (bprmf_dist_init_*)");
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
    if (int r = dist_chunk(h, 0, 0, m, tu, ti, tj)) return r;
    HIPCHK(hipStreamSynchronize(h->stream));  // the next chunk's copies reuse d_trip
  }
  return end_call(h, st, valid, n_steps);
}

}  // extern "C"
