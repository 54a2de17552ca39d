// capi.cpp — C ABI (include/bprmf.h) over the gfx950 kernels of kernels.hip.
//
// One handle = one GPU = one shard (rank of world).  The handle owns, in HBM:
//   P  [local users, ld] fp32 + grad accumulator + int32 stamp      (embed_user.weight)
//   Q  [local items, ld] fp32 + grad accumulator + int32 stamp      (embed_item.weight)
//   positives of its users (features order) and their sorted CSR     (BPRData.features / train_mat)
//   a triplet chunk buffer [chunk, 3] int32 filled by the sampler    (BPRData.features_fill)
// Training runs in chunks of steps: one k_build_batches launch lays out every batch of the chunk
// (segment.hip), then each step is k_user_step + k_item_step (step.hip), replayed from a captured
// hipGraph.  Batches above kMaxSegBatch use the f32-atomic pair fwd_scatter + apply_refs.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <string>
#include <vector>

#include "handle.h"
#include "host_plan.h"

using namespace bprmf;

static void drop_graphs(bprmf_handle* h);
static int ensure_step_graphs(bprmf_handle* h);

// Profiling events skip the system-scope fence a default event record performs (an L2 write-back
// that would otherwise land inside the measured interval: +2 us per kernel measured on gfx950).
hipEvent_t bprmf::prof_event(bprmf_handle* h) {
  if (h->prof_used == h->prof_pool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    h->prof_pool.push_back(e);
  }
  return h->prof_pool[h->prof_used++];
}

int bprmf::set_dev(bprmf_handle* h) {
  HIPCHK(hipSetDevice(h->cfg.device));
  return 0;
}

static int64_t chunk_triplets(const bprmf_handle* h) {
  // sample up to ~4M triplets (48 MB of ids) per sampler launch, whole steps only
  const int64_t B = h->cfg.batch_size;
  int64_t steps = std::max<int64_t>(1, (int64_t(1) << 22) / B);
  return steps * B;
}

int bprmf::ensure_trip(bprmf_handle* h, int64_t n) {
  if (n <= h->trip_cap) return 0;
  if (h->d_trip) HIPCHK(hipFree(h->d_trip));
  h->d_trip = nullptr;
  h->trip_cap = 0;
  if (int r = dalloc(&h->d_trip, 3 * n)) return r;
  h->trip_cap = n;
  return 0;
}

// after a timed-out build (err bit 16): the batch buffer back to zeros, as allocated, so no
// batch keeps its dead mark (kernels.h kMetaDead) or the unfinished build's exchange words
static hipError_t clear_batches(bprmf_handle* h) {
  if (!h->d_batch || !h->batch_cap) return hipSuccess;
  return hipMemsetAsync(h->d_batch, 0,
                        sizeof(int32_t) * h->batch_cap * BatchBuf::stride_for(h->cfg.batch_size), h->stream);
}

int bprmf::check_err_flag(bprmf_handle* h) {
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d_err, sizeof e, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (e) {
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int32_t), h->stream));
    if (e & 16) HIPCHK(clear_batches(h));
    if (e & 4) return fail(BPRMF_E_HIP, "sharded exchange timed out: a peer stopped signalling");
    if (e & 16) return fail(BPRMF_E_HIP, "batch builder: an item part never published its counts (wait timed out)");
    if (e & 2) return fail(BPRMF_E_NO_NEGATIVE, "a user has every item as a positive: no negative to sample");
    return fail(BPRMF_E_RANGE, "user/item id out of range (device check)");
  }
  return 0;
}

extern "C" {

int bprmf_version(void) { return 1; }

int bprmf_create(const bprmf_config* cfg, bprmf_handle** out) {
  if (!cfg || !out) return fail(BPRMF_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->user_num <= 0 || cfg->item_num <= 0)
    return fail(BPRMF_E_INVALID, "user_num and item_num must be positive");
  if (cfg->user_num > INT32_MAX || cfg->item_num > INT32_MAX)
    return fail(BPRMF_E_INVALID, "ids are int32: user_num/item_num must be < 2^31");
  if (cfg->batch_size <= 0 || cfg->num_ng <= 0)
    return fail(BPRMF_E_INVALID, "batch_size and num_ng must be positive");
  if (cfg->world <= 0 || cfg->rank < 0 || cfg->rank >= cfg->world)
    return fail(BPRMF_E_INVALID, "need 0 <= rank < world");
  if (cfg->world > kMaxWorld)
    return fail(BPRMF_E_UNSUPPORTED, "world %d > %d ranks", cfg->world, kMaxWorld);
  if (!(cfg->lr >= 0.f) || !(cfg->weight_decay >= 0.f) || !(cfg->init_std >= 0.f))
    return fail(BPRMF_E_INVALID, "lr, weight_decay and init_std must be >= 0");
  Geom g;
  if (!make_geom(cfg->factor_num, &g)) return fail(BPRMF_E_UNSUPPORTED, "factor_num must be in [1, 1024]");
  if (cfg->semantics != BPRMF_SEM_EXACT && cfg->semantics != BPRMF_SEM_HOGWILD &&
      cfg->semantics != BPRMF_SEM_LOCAL && cfg->semantics != BPRMF_SEM_STALE1)
    return fail(BPRMF_E_INVALID,
                "semantics must be BPRMF_SEM_EXACT (0), _HOGWILD (1), _LOCAL (2) or _STALE1 (3)");
  if (cfg->semantics == BPRMF_SEM_STALE1 &&
      (cfg->step_mode != BPRMF_STEP_SEGMENTED || cfg->batch_size > kMaxSegBatch))
    return fail(BPRMF_E_UNSUPPORTED, "stale1 semantics: the segmented sharded step (batch_size <= %d)",
                kMaxSegBatch);
  if (cfg->semantics == BPRMF_SEM_HOGWILD && cfg->world != 1)
    return fail(BPRMF_E_UNSUPPORTED, "hogwild semantics: single-GPU handles only");
  if (cfg->local_steps < 0 || cfg->dp_steps < 0)
    return fail(BPRMF_E_INVALID, "local_steps and dp_steps must be >= 0");
  if (cfg->dp_overlap != 0 && cfg->dp_overlap != 1) return fail(BPRMF_E_INVALID, "dp_overlap must be 0 or 1");
  if (cfg->step_mode != BPRMF_STEP_SEGMENTED && cfg->step_mode != BPRMF_STEP_ATOMIC)
    return fail(BPRMF_E_INVALID, "step_mode must be BPRMF_STEP_SEGMENTED (0) or BPRMF_STEP_ATOMIC (1)");
  if (cfg->step_mode == BPRMF_STEP_ATOMIC && cfg->world != 1)
    return fail(BPRMF_E_UNSUPPORTED, "the atomic step: single-GPU handles only (the sharded runner sums by segments)");
  auto* h = new bprmf_handle();
  h->cfg = *cfg;
  h->semantics = cfg->semantics;
  if (cfg->local_steps > 0) h->local_steps = cfg->local_steps;
  if (cfg->dp_steps > 0) h->dp_steps = cfg->dp_steps;
  h->dp_overlap = cfg->dp_overlap == 1;
  h->geom = g;
  h->hp.lr = cfg->lr;
  h->hp.wd = cfg->weight_decay;
  h->hp.alpha = 1.0 - (double)cfg->lr * (double)cfg->weight_decay;
  if (!(h->hp.alpha > 0.0)) {
    delete h;
    return fail(BPRMF_E_INVALID, "lr * weight_decay must be < 1 (weight decay would flip signs)");
  }
  h->hp.log2a = std::log2(h->hp.alpha);
  const int64_t W = cfg->world, R = cfg->rank;
  h->U = shard_rows(cfg->user_num, (int)W, (int)R);
  const bool dpi = dp_items(*cfg);  // LOCAL at world > 1: every item on every rank
  h->dp_mode = dpi;
  h->I = dpi ? cfg->item_num : shard_rows(cfg->item_num, (int)W, (int)R);
  const uint64_t shard_seed = cfg->seed + (uint64_t)cfg->rank * 0x9E3779B97F4A7C15ull;
  h->k0 = (uint32_t)shard_seed;
  h->k1 = (uint32_t)(shard_seed >> 32);
  int rc = 0;
#define TRY(x)            \
  do {                    \
    if ((rc = (x))) {     \
      bprmf_destroy(h);   \
      return rc;          \
    }                     \
  } while (0)
  TRY(set_dev(h));
  hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    bprmf_destroy(h);
    return fail(BPRMF_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  h->stream = h->own_stream;
  h->use_graphs = getenv("BPRMF_NO_GRAPH") == nullptr;
  {  // BPRMF_FUSED=0: K1 + K2 launch pairs instead of the fused launches (the bitwise A/B test)
    const char* f = getenv("BPRMF_FUSED");
    h->fused = !(f && f[0] == '0');
  }
  const int64_t ld = g.ld;
  if (dpi) {  // every rank holds the whole item table several times over: fail early and clearly
    // Q, its merge base, the delta table (padded to world slices), the overlap's sum buffer, and
    // the IPC transport's two exported [W * ceil(I / W)][ld] buffers (dist_attach); the hot
    // items' XCD replicas are at most 8 x 4096 rows on top
    const int64_t pad = W * ((h->I + W - 1) / W);
    const int64_t rows = h->U + h->I * 2 + pad * 3 + (h->dp_overlap ? h->I : 0) + 8 * 4096;
    const size_t need = sizeof(float) * (size_t)(rows * ld);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && need > fr) {
      bprmf_destroy(h);
      return fail(BPRMF_E_UNSUPPORTED,
                  "semantics local at world %lld replicates the %lld-row item table on every rank "
                  "(~%.1f GB with its merge buffers) but the device has %.1f GB free",
                  (long long)W, (long long)cfg->item_num, need / 1e9, fr / 1e9);
    }
  }
  TRY(dalloc(&h->P.W, h->U * ld));
  TRY(dalloc(&h->P.stamp, h->U));
  TRY(dalloc(&h->Q.W, h->I * ld));
  TRY(dalloc(&h->Q.stamp, h->I));
  if (dpi) {
    TRY(dalloc(&h->d_qbase, h->I * ld));
    // the delta table padded to world slices of ceil(I / world) rows (the IPC all-reduce pushes
    // whole slices; the padding stays zero)
    const int64_t pad_rows = W * ((h->I + W - 1) / W);
    TRY(dalloc(&h->d_qdelta, pad_rows * ld));
    if (h->dp_overlap) TRY(dalloc(&h->d_qsum, h->I * ld));
  }
  // {err, dist words, loss slots[kLossSlots], two call sequence numbers}
  const size_t status_bytes = kSeqCapOff + 8;
  TRY(dalloc(&h->d_status, (int64_t)status_bytes));
  if (hipHostMalloc((void**)&h->h_status, status_bytes, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->h_status_dev, h->h_status, 0) != hipSuccess) {
    if (h->h_status) (void)!hipHostFree(h->h_status);
    h->h_status = nullptr;
    bprmf_destroy(h);
    return fail(BPRMF_E_HIP, "hipHostMalloc (mapped status) failed");
  }
  memset(h->h_status, 0, status_bytes);  // no stale call sequence number
  h->d_err = reinterpret_cast<int32_t*>(h->d_status);
  h->d_loss = reinterpret_cast<double*>(h->d_status + 16);
  h->P.rows = h->U;
  h->Q.rows = h->I;
  auto memz = [&](void* p, size_t bytes) -> int {
    if (!p || !bytes) return 0;
    HIPCHK(hipMemsetAsync(p, 0, bytes, h->stream));
    return 0;
  };
  TRY(memz(h->P.stamp, sizeof(int32_t) * h->U));
  if (h->d_qdelta) TRY(memz(h->d_qdelta, sizeof(float) * (size_t)(W * ((h->I + W - 1) / W) * ld)));
  TRY(memz(h->Q.stamp, sizeof(int32_t) * h->I));
  TRY(memz(h->d_status, status_bytes));
  // init keyed by the global seed and GLOBAL row id: identical tables for any world size
  const uint32_t s0 = (uint32_t)cfg->seed, s1 = (uint32_t)(cfg->seed >> 32);
  e = init_normal(g, h->P.W, h->U, cfg->init_std, s0, s1, 0u, (int)W, (int)R, h->stream);
  if (e == hipSuccess)  // a replicated item table: every rank draws all of it
    e = init_normal(g, h->Q.W, h->I, cfg->init_std, s0, s1, 1u, dpi ? 1 : (int)W, dpi ? 0 : (int)R, h->stream);
  if (e == hipSuccess && dpi)
    e = hipMemcpyAsync(h->d_qbase, h->Q.W, sizeof(float) * h->I * ld, hipMemcpyDeviceToDevice, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    bprmf_destroy(h);
    return fail(BPRMF_E_HIP, "init: %s", hipGetErrorString(e));
  }
#undef TRY
  *out = h;
  return 0;
}

int bprmf_destroy(bprmf_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
  // a caller's stream is drained too before anything is freed
  if (h->stream && h->stream != h->own_stream) (void)hipStreamSynchronize(h->stream);
  void* ptrs[] = {h->P.W, h->P.G, h->P.stamp, h->Q.W, h->Q.G, h->Q.stamp, h->d_pos_u, h->d_pos_i,
                  h->d_indptr, h->d_indices, h->d_trip, h->d_status,
                  h->d_batch, h->d_contrib, h->d_ugrad, h->d_xloss, h->d_tbase,
                  h->d_pend_q, h->d_pend_p, h->d_hbits, h->d_hhash, h->d_hot, h->d_hot_rows, h->d_qrep, h->d_soff,
                  h->d_skeys, h->d_qbase, h->d_qdelta, h->d_qsum, h->d_pos2, h->d_urec,
                  h->d_pos4};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  drop_graphs(h);
  dist_free(h->dist);
  for (hipEvent_t e : h->prof_pool) (void)hipEventDestroy(e);
  if (h->h_status) (void)hipHostFree(h->h_status);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
  delete h;
  return 0;
}

int bprmf_set_stream(bprmf_handle* h, void* s) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  h->stream = s ? (hipStream_t)s : h->own_stream;
  return 0;
}

int bprmf_synchronize(bprmf_handle* h) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = set_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int bprmf_local_rows(bprmf_handle* h, int64_t* users, int64_t* items) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (users) *users = h->U;
  if (items) *items = h->I;
  return 0;
}

int bprmf_step_count(bprmf_handle* h, int64_t* steps) {
  if (!h || !steps) return fail(BPRMF_E_INVALID, "null argument");
  *steps = h->t;
  return 0;
}

int bprmf_row_stride(bprmf_handle* h, int32_t* ld) {
  if (!h || !ld) return fail(BPRMF_E_INVALID, "null argument");
  *ld = h->geom.ld;
  return 0;
}

extern "C++" LocalArgs bprmf::local_args(const bprmf_handle* h) {
  LocalArgs la;
  la.hot = h->d_hot;
  la.rep = h->d_qrep;
  la.H = h->hot_H;
  la.hbits = h->d_hbits;
  la.hhash = h->d_hhash;
  la.hlog = h->hot_hlog;
  return la;
}

// semantics LOCAL: the hot items (the most frequent positives; BPRMF_LOCAL_HOT overrides how many)
// get one replica row per XCD, filled from the base table (a refresh merge at the current step)
static int local_refresh(bprmf_handle* h) {
  if (!h->d_qrep) return 0;
  LocalArgs la = local_args(h);
  HIPCHK(local_merge(h->geom, h->Q, la, h->d_hot_rows, h->hp, h->t, h->t, true, h->stream));
  h->rep_t = h->t;
  return 0;
}

static int local_setup(bprmf_handle* h, const std::vector<int32_t>& pos_items) {
  const int64_t I = h->I;
  int64_t H = std::min<int64_t>(4096, std::max<int64_t>(1, I / 4));
  if (const char* e = getenv("BPRMF_LOCAL_HOT")) H = std::max<int64_t>(0, std::min<int64_t>(I, atoll(e)));
  std::vector<int64_t> cnt(I, 0);
  for (int32_t i : pos_items) ++cnt[i];
  std::vector<int32_t> order(I);
  for (int64_t i = 0; i < I; ++i) order[i] = (int32_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return cnt[a] > cnt[b]; });
  std::vector<int32_t> hot(I, -1), rows(std::max<int64_t>(H, 1));
  for (int64_t k = 0; k < H; ++k) {
    rows[k] = order[k];
    hot[order[k]] = (int32_t)k;
  }
  const size_t rep_bytes = sizeof(float) * (size_t)kLocalXcds * H * h->geom.ld;
  for (void* p : {(void*)h->d_hot, (void*)h->d_hot_rows, (void*)h->d_qrep, (void*)h->d_hbits, (void*)h->d_hhash})
    if (p) HIPCHK(hipFree(p));
  h->d_hot = h->d_hot_rows = nullptr;
  h->d_qrep = nullptr;
  h->d_hbits = nullptr;
  h->d_hhash = nullptr;
  h->hot_hlog = 0;
  h->hot_H = H;
  if (int r = dalloc(&h->d_hot, I)) return r;
  if (int r = dalloc(&h->d_hot_rows, std::max<int64_t>(H, 1))) return r;
  if (H > 0) HIPCHK(hipMalloc((void**)&h->d_qrep, rep_bytes));
  HIPCHK(hipMemcpy(h->d_hot, hot.data(), 4 * I, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->d_hot_rows, rows.data(), 4 * rows.size(), hipMemcpyHostToDevice));
  // a catalogue whose hot[] (4 B per item) is past the caches: the kernels' per-triplet lookup
  // reads a bit per item instead (I / 8 bytes, mostly cache-resident) and, for the hot items
  // alone, a small open-addressing table (BPRMF_LOCAL_HOT_BITS: the item count from which the
  // bits are used; 0 = always, default 16M items = a 64 MB hot[])
  int64_t bits_from = 16LL << 20;
  if (const char* e = getenv("BPRMF_LOCAL_HOT_BITS")) bits_from = std::max<int64_t>(0, atoll(e));
  if (H > 0 && I >= bits_from) {
    int hlog = 1;
    while ((1LL << hlog) < 2 * H) ++hlog;
    std::vector<uint32_t> bits((I + 31) / 32, 0u);
    std::vector<int2> tab((size_t)1 << hlog, int2{-1, -1});
    for (int64_t k = 0; k < H; ++k) {
      const uint32_t it = (uint32_t)rows[k];
      bits[it >> 5] |= 1u << (it & 31);
      uint32_t q = (it * 0x9E3779B1u) >> (32 - hlog);  // hogwild.hip hot_probe's hash
      while (tab[q].x >= 0) q = (q + 1) & ((1u << hlog) - 1);
      tab[q] = int2{(int32_t)it, (int32_t)k};
    }
    if (int r = dalloc(&h->d_hbits, (int64_t)bits.size())) return r;
    if (int r = dalloc(&h->d_hhash, (int64_t)tab.size())) return r;
    HIPCHK(hipMemcpy(h->d_hbits, bits.data(), 4 * bits.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_hhash, tab.data(), sizeof(int2) * tab.size(), hipMemcpyHostToDevice));
    h->hot_hlog = hlog;
  }
  return local_refresh(h);
}

int bprmf_set_train(bprmf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz) {
  return bprmf_set_train_ex(h, users, items, nnz, nullptr, nullptr, 0);
}

int bprmf_set_train_ex(bprmf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz,
                       const int32_t* ex_users, const int32_t* ex_items, int64_t n_ex) {
  if (!h || (nnz > 0 && (!users || !items)) || nnz < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (n_ex < 0 || (n_ex > 0 && (!ex_users || !ex_items))) return fail(BPRMF_E_INVALID, "bad exclusions");
  if (int r = set_dev(h)) return r;
  ShardCsr csr;  // host_plan.cpp (sanitizer-tested host code)
  if (int r = build_shard_csr(users, items, nnz, ex_users, ex_items, n_ex, h->cfg.user_num,
                              h->cfg.item_num, h->cfg.world, h->cfg.rank, h->U, &csr))
    return r;
  const std::vector<int32_t>& pu = csr.pos_u;
  const std::vector<int32_t>& pi = csr.pos_i;
  const std::vector<int64_t>& indptr = csr.indptr;
  const std::vector<int32_t>& indices = csr.indices;
  const int64_t n = (int64_t)pu.size();
  void* olds[] = {h->d_pos_u, h->d_pos_i, h->d_indptr, h->d_indices, h->d_soff, h->d_skeys, h->d_pos2, h->d_urec,
                  h->d_pos4};
  for (void* p : olds)
    if (p) HIPCHK(hipFree(p));
  h->d_pos_u = h->d_pos_i = h->d_indices = h->d_skeys = nullptr;
  h->d_indptr = h->d_soff = nullptr;
  h->d_pos2 = h->d_urec = nullptr;
  h->d_pos4 = nullptr;
  // the sampler's search trees and packed records (one line per dependent level; the separate
  // arrays and the binary search remain for positive sets past 32-bit tree offsets)
  {
    SearchTree st;
    build_search_tree(indptr, indices, &st);
    if (int r = dalloc(&h->d_soff, (int64_t)st.soff.size())) return r;
    if (int r = dalloc(&h->d_skeys, std::max<int64_t>(16, (int64_t)st.keys.size()))) return r;
    HIPCHK(hipMemcpy(h->d_soff, st.soff.data(), 8 * st.soff.size(), hipMemcpyHostToDevice));
    if (!st.keys.empty())
      HIPCHK(hipMemcpy(h->d_skeys, st.keys.data(), 4 * st.keys.size(), hipMemcpyHostToDevice));
    if (st.soff.back() < INT32_MAX) {
      std::vector<int2> ur(h->U);
      for (int64_t lu = 0; lu < h->U; ++lu)
        ur[lu] = make_int2((int32_t)st.soff[lu], (int32_t)(indptr[lu + 1] - indptr[lu]));
      if (int r = dalloc(&h->d_urec, std::max<int64_t>(1, h->U))) return r;
      if (h->U) HIPCHK(hipMemcpy(h->d_urec, ur.data(), 8 * ur.size(), hipMemcpyHostToDevice));
    }
  }
  // a large positive set: its user records (40+ MB of random reads) join the positives' records,
  // one 16-byte line per draw instead of two lines (BPRMF_SAMPLE_POS4: the positive count from
  // which; 0 = always, default 64M)
  int64_t pos4_from = 64LL << 20;
  if (const char* e = getenv("BPRMF_SAMPLE_POS4")) pos4_from = std::max<int64_t>(0, atoll(e));
  if (h->d_urec && !pu.empty() && (int64_t)pu.size() >= pos4_from) {
    std::vector<int2> ur(h->U);
    HIPCHK(hipMemcpy(ur.data(), h->d_urec, 8 * ur.size(), hipMemcpyDeviceToHost));
    std::vector<int4> p4(pu.size());
    const int64_t W = h->cfg.world;
    for (size_t k = 0; k < pu.size(); ++k) {
      const int2 r = ur[pu[k] / W];
      p4[k] = make_int4(pu[k], pi[k], r.x, r.y);
    }
    if (int r = dalloc(&h->d_pos4, (int64_t)p4.size())) return r;
    HIPCHK(hipMemcpy(h->d_pos4, p4.data(), 16 * p4.size(), hipMemcpyHostToDevice));
  } else if (!pu.empty()) {
    std::vector<int2> p2(pu.size());
    for (size_t k = 0; k < pu.size(); ++k) p2[k] = make_int2(pu[k], pi[k]);
    if (int r = dalloc(&h->d_pos2, (int64_t)p2.size())) return r;
    HIPCHK(hipMemcpy(h->d_pos2, p2.data(), 8 * p2.size(), hipMemcpyHostToDevice));
  }
  if (int r = dalloc(&h->d_pos_u, n)) return r;
  if (int r = dalloc(&h->d_pos_i, n)) return r;
  if (int r = dalloc(&h->d_indptr, h->U + 1)) return r;
  if (int r = dalloc(&h->d_indices, (int64_t)indices.size())) return r;
  if (n) {
    HIPCHK(hipMemcpy(h->d_pos_u, pu.data(), 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_pos_i, pi.data(), 4 * n, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(h->d_indptr, indptr.data(), 8 * (h->U + 1), hipMemcpyHostToDevice));
  if (!indices.empty())
    HIPCHK(hipMemcpy(h->d_indices, indices.data(), 4 * indices.size(), hipMemcpyHostToDevice));
  h->npos = n;
  if (h->semantics == BPRMF_SEM_LOCAL)
    if (int r = local_setup(h, pi)) return r;
  const uint64_t N = (uint64_t)n * (uint64_t)h->cfg.num_ng;
  feistel_dims(N, &h->feistel_a, &h->feistel_c);
  // single GPU: the step buffers of a whole chunk and the step graphs, now rather than inside
  // the first calls (a larger chunk later would reallocate and recapture)
  if (seg_mode(h) && (h->semantics == BPRMF_SEM_EXACT || h->semantics == BPRMF_SEM_STALE1)) {
    const int64_t B = h->cfg.batch_size;
    const bool one = h->cfg.world == 1 && h->semantics == BPRMF_SEM_EXACT;  // the single-GPU step
    const int64_t steps = one ? chunk_triplets(h) / B : dist_chunk_steps(h);
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(steps, ((int64_t)N + B - 1) / B));
    if (int r = ensure_seg(h, nb)) return r;
    if (int r = ensure_trip(h, nb * B)) return r;
    if (one && h->use_graphs)
      if (int r = ensure_step_graphs(h)) return r;
  }
  return 0;
}

int bprmf_epoch_size(bprmf_handle* h, int64_t* n_triplets, int64_t* n_steps) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  const int64_t N = h->npos * h->cfg.num_ng;
  if (n_triplets) *n_triplets = N;
  if (n_steps) *n_steps = (N + h->cfg.batch_size - 1) / h->cfg.batch_size;
  return 0;
}

}  // extern "C"

SamplerArgs bprmf::sampler_args(bprmf_handle* h) {
  SamplerArgs a;
  a.pos_u = h->d_pos_u;
  a.pos_i = h->d_pos_i;
  a.indptr = h->d_indptr;
  a.indices = h->d_indices;
  a.npos = h->npos;
  a.item_num = h->cfg.item_num;
  a.num_ng = h->cfg.num_ng;
  a.world = h->cfg.world;
  a.feistel_a = h->feistel_a;
  a.feistel_c = h->feistel_c;
  a.k0 = h->k0;
  a.k1 = h->k1;
  a.skeys = h->d_skeys;
  a.soff = h->d_soff;
  a.pos2 = h->d_pos2;
  a.urec = h->d_urec;
  a.pos4 = h->d_pos4;
  return a;
}

static double host_seconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// diagnostic build only (-DBPRMF_HOST_TRACE, tools/gpu/host_trace.sh): host timestamps of a
// thread's first calls' phases, to stderr
static bool trace_on() {
#ifdef BPRMF_HOST_TRACE
  return true;
#else
  return false;
#endif
}
static thread_local int g_trace_calls = 0;
static thread_local double g_trace_t[8];
static thread_local int g_trace_n = 0;
static void trace_mark() {
  if (trace_on() && g_trace_calls < 12 && g_trace_n < 8) g_trace_t[g_trace_n++] = host_seconds();
}
static void trace_flush() {
  if (!trace_on() || g_trace_calls >= 12 || g_trace_n == 0) return;
  fprintf(stderr, "host trace call %d:", g_trace_calls);
  for (int k = 1; k < g_trace_n; ++k) fprintf(stderr, " %.1f", (g_trace_t[k] - g_trace_t[0]) * 1e6);
  fprintf(stderr, " us\n");
  ++g_trace_calls;
  g_trace_n = 0;
}

// sum of every per-wave loss slot (the Python-orchestrated sharded step)
int bprmf::read_loss(bprmf_handle* h, double* loss) {
  HIPCHK(hipMemcpyAsync(h->h_status + 16, h->d_loss, sizeof(double) * kLossSlots,
                        hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  const double* slots = reinterpret_cast<const double*>(h->h_status + 16);
  double s = 0;
  for (int k = 0; k < kLossSlots; ++k) s += slots[k];
  *loss = s;
  return 0;
}

int bprmf::loss_zero_slots(bprmf_handle* h) {
  if (!h->loss_pending) return 0;
  h->loss_pending = false;
  const int n = h->slots_dirty ? kLossSlots : kSegLossSlots;
  h->slots_dirty = false;
  return n;
}

// no GPU work here: the call's first launch zeroes the loss (set_cursor / loss_zero_slots)
int bprmf::begin_call(bprmf_handle* h) {
  if (int r = set_dev(h)) return r;
  h->loss_pending = true;
  h->call_slots = false;
  h->call_t0 = host_seconds();
  return 0;
}

// one status read per call: {err, loss} written into mapped host memory by one tiny kernel (the
// f32-atomic path's per-wave slots: one copy), then one stream synchronisation
int bprmf::wait_mapped_seq(bprmf_handle* h, size_t off, uint64_t seq) {
  const volatile uint64_t* hs = reinterpret_cast<const volatile uint64_t*>(h->h_status + off);
  for (uint32_t spin = 1;; ++spin) {
    if (*hs == seq) return 0;
    if ((spin & 4095) == 0 && hipStreamQuery(h->stream) != hipErrorNotReady && *hs != seq) break;
    __builtin_ia32_pause();
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int bprmf::end_call(bprmf_handle* h, bprmf_stats* st, int64_t triplets, int64_t steps) {
  const bool ran = !h->loss_pending;
  h->loss_pending = false;
  if (h->call_slots) {
    HIPCHK(hipMemcpyAsync(h->h_status, h->d_status, 16 + sizeof(double) * kLossSlots,
                          hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  } else {
    // the status words, then this call's sequence number, written into mapped host memory
    const uint64_t seq = ++h->status_seq;
    HIPCHK(status_out(h->d_status, h->h_status_dev, 2 + kSegLossSlots, h->stream,
                      h->h_status_dev + kSeqEndOff, seq));
    if (int r = wait_mapped_seq(h, kSeqEndOff, seq)) return r;
  }
  const int32_t e = *reinterpret_cast<const volatile int32_t*>(h->h_status);
  if (e) {
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int32_t), h->stream));
    if (e & 16) HIPCHK(clear_batches(h));
    if (e & 4) return fail(BPRMF_E_HIP, "sharded exchange timed out: a peer stopped signalling");
    if (e & 8) return fail(BPRMF_E_HIP, "fused step: a row's owner never published it (wait timed out)");
    if (e & 16) return fail(BPRMF_E_HIP, "batch builder: an item part never published its counts (wait timed out)");
    if (e & 2) return fail(BPRMF_E_NO_NEGATIVE, "a user has every item as a positive: no negative to sample");
    return fail(BPRMF_E_RANGE, "user/item id out of range (device check)");
  }
  const volatile double* slots = reinterpret_cast<const volatile double*>(h->h_status + 16);
  double loss = 0;
  if (ran)
    for (int k = 0; k < (h->call_slots ? kLossSlots : kSegLossSlots); ++k) loss += slots[k];
  if (st) {
    st->triplets = triplets;
    st->steps = steps;
    st->loss = loss;
    st->seconds = host_seconds() - h->call_t0;
  }
  return 0;
}

// sampled chunks of at most this many batches draw their triplets with the grid-wide sampler
// first and build from those (the builder then has no sampler latency: one workgroup per batch
// cannot hide it when a chunk is short); longer chunks sample inside the builder, whose
// workgroups then fill the chip anyway.  BPRMF_SPLIT_BUILD=0/1 forces either.
bool bprmf::split_build(int64_t nb) {
  const char* e = getenv("BPRMF_SPLIT_BUILD");
  if (e && *e) return e[0] != '0';
  return nb <= 512;
}

bool bprmf::seg_mode(const bprmf_handle* h) {
  return h->cfg.batch_size <= kMaxSegBatch && h->cfg.step_mode != BPRMF_STEP_ATOMIC;
}

int bprmf::ensure_seg(bprmf_handle* h, int64_t n_batches) {
  const int64_t B = h->cfg.batch_size;
  if (!h->d_contrib) {
    if (int r = dalloc(&h->d_contrib, 2 * B * h->geom.ld)) return r;
    if (int r = dalloc(&h->d_ugrad, 2 * B * h->geom.ld)) return r;
    if (int r = dalloc(&h->d_xloss, 2 * B)) return r;
    if (int r = dalloc(&h->d_pend_q, 2 * h->I)) return r;
    if (int r = dalloc(&h->d_pend_p, 2 * h->U)) return r;
    // no step has marked a row yet (steps are >= 1; -1 never matches)
    if (h->I) HIPCHK(hipMemsetAsync(h->d_pend_q, 0xFF, sizeof(int32_t) * 2 * h->I, h->stream));
    if (h->U) HIPCHK(hipMemsetAsync(h->d_pend_p, 0xFF, sizeof(int32_t) * 2 * h->U, h->stream));
    if (int r = dalloc(&h->d_tbase, 4)) return r;
  }
  if (n_batches <= h->batch_cap) return 0;
  drop_graphs(h);  // captured graphs point into the old batch buffer
  if (h->d_batch) HIPCHK(hipFree(h->d_batch));
  h->d_batch = nullptr;
  h->batch_cap = 0;
  if (int r = dalloc(&h->d_batch, n_batches * BatchBuf::stride_for((int)B))) return r;
  // zeroed once: the split builder's exchange and sampling-board words (segment.hip) must never
  // see an earlier allocation's ints (a recycled block holds another handle's records, and those
  // small numbers once matched a fresh process's first launch tags)
  HIPCHK(hipMemsetAsync(h->d_batch, 0, sizeof(int32_t) * n_batches * BatchBuf::stride_for((int)B),
                        h->stream));
  h->batch_cap = n_batches;
  return 0;
}

extern "C" int bprmf_debug_fail_build(bprmf_handle* h) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (!h->d_batch) return fail(BPRMF_E_STATE, "no batch buffer yet");
  if (int r = set_dev(h)) return r;
  // what a build whose wait timed out leaves (segment.hip): the dead mark in every batch's meta
  // word and err bit 16 (the builders never clear either: the host does, when it reports the error)
  const BatchBuf bb{h->d_batch, h->cfg.batch_size};
  for (int64_t k = 0; k < h->batch_cap; ++k)
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(bb.view(k).meta + kMetaDead), kDeadMark, 1, h->stream));
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->d_err, kErrBuild, 1, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int bprmf_debug_fill_batches(bprmf_handle* h, int32_t value) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (!h->d_batch) return fail(BPRMF_E_STATE, "no batch buffer yet");
  if (int r = set_dev(h)) return r;
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->d_batch, value,
                           (size_t)h->batch_cap * BatchBuf::stride_for(h->cfg.batch_size), h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

// gradient accumulators of the f32-atomic step (B > kMaxSegBatch) and of the Python-orchestrated
// sharded owner apply, allocated on first use: the segmented steps never touch them, and at the
// C5 shape (100M x 256 items) they would be another 102 GB of HBM
int bprmf::ensure_grad(bprmf_handle* h) {
  const int64_t ld = h->geom.ld;
  if (!h->P.G) {
    if (int r = dalloc(&h->P.G, h->U * ld)) return r;
    if (h->U) HIPCHK(hipMemsetAsync(h->P.G, 0, sizeof(float) * h->U * ld, h->stream));
  }
  if (!h->Q.G) {
    if (int r = dalloc(&h->Q.G, h->I * ld)) return r;
    if (h->I) HIPCHK(hipMemsetAsync(h->Q.G, 0, sizeof(float) * h->I * ld, h->stream));
  }
  return 0;
}

extern "C" {

static int run_steps(bprmf_handle* h, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                     int64_t n, int64_t* steps_done);

}  // extern "C"

StepBufs bprmf::step_bufs(const bprmf_handle* h) {
  StepBufs b;
  b.contrib = h->d_contrib;
  b.ugrad = h->d_ugrad;
  b.xloss = h->d_xloss;
  b.pstride = (int64_t)h->cfg.batch_size * h->geom.ld;
  b.pend_q = h->fused ? h->d_pend_q : nullptr;  // only the fused step reads the marks
  b.pend_p = h->fused ? h->d_pend_p : nullptr;
  b.qrows = h->I;
  b.prows = h->U;
  return b;
}

extern "C" {

// The step launches of a chunk of nb steps, all indexed by the device cursor d_tbase = {t, k}
// (kernels take batch 0's view plus the batch stride, and a step index relative to the cursor).
// A "unit" is one launch group at relative index r:
//   fused (default):  K2 of step r and K1 of step r + 1 in one launch (k_fused_step); the chunk
//                     is K1(0), units 0 .. nb-2, K2(nb-1): nb + 1 launches;
//   unfused:          K1(r) then K2(r): 2 nb launches.
// Chunks of 64 units or more run as replays of position-independent graphs of 64 and 16 units
// (captured once per batch buffer; every graph but the chunk's last ends by advancing the cursor)
// plus fewer than 16 eager units; the eager launches and the epilogue index the cursor as the
// graphs left it.  Shorter chunks launch every unit eagerly.
static void drop_graphs(bprmf_handle* h) {
  for (auto& ge : h->graphs)
    if (ge.exec) (void)hipGraphExecDestroy(ge.exec);
  h->graphs.clear();
}

static int launch_unit(bprmf_handle* h, int64_t r) {
  const int B = h->cfg.batch_size;
  const BatchView v0 = BatchBuf{h->d_batch, B}.view(0);
  const int64_t stride = BatchBuf::stride_for(B);
  const StepBufs sb = step_bufs(h);
  if (h->fused) {
    HIPCHK(fused_step(h->geom, v0, stride, B, h->P, h->Q, h->hp, h->d_tbase, (int)r, sb, h->d_loss,
                      h->d_err, h->stream));
    return 0;
  }
  HIPCHK(user_step(h->geom, v0, B, h->P, h->Q, h->hp, h->d_tbase, (int)r, nullptr, nullptr, nullptr,
                   nullptr, h->stream, PeerWait{}, stride, &sb));
  HIPCHK(item_step(h->geom, v0, B, h->P, h->Q, h->hp, h->d_tbase, (int)r, nullptr, nullptr, nullptr,
                   h->stream, nullptr, h->d_loss, stride, &sb));
  return 0;
}

static int capture_step_graph(bprmf_handle* h, int64_t n, bool advance, StepGraph* out) {
  HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  for (int64_t r = 0; r < n && !rc; ++r) rc = launch_unit(h, r);
  if (!rc && advance) {
    const hipError_t e = advance_cursor(h->d_tbase, (int32_t)n, h->stream);
    if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "step graph cursor: %s", hipGetErrorString(e));
  }
  hipGraph_t graph = nullptr;
  const hipError_t e2 = hipStreamEndCapture(h->stream, &graph);
  if (rc || e2 != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc ? rc : fail(BPRMF_E_HIP, "step graph capture: %s", hipGetErrorString(e2));
  }
  out->n = n;
  out->advance = advance;
  const hipError_t e = hipGraphInstantiate(&out->exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (e != hipSuccess) {
    out->exec = nullptr;
    return fail(BPRMF_E_HIP, "step graph instantiate: %s", hipGetErrorString(e));
  }
  // the executable graph's device-side setup now (set_train) rather than inside its first replay
  const hipError_t eu = hipGraphUpload(out->exec, h->stream);
  if (eu != hipSuccess) {  // the caller never keeps a failed graph: destroy it here
    (void)hipGraphExecDestroy(out->exec);
    out->exec = nullptr;
    return fail(BPRMF_E_HIP, "step graph upload: %s", hipGetErrorString(eu));
  }
  return 0;
}

// capture every graph once (batch buffer and step buffers must exist: ensure_seg)
static int ensure_step_graphs(bprmf_handle* h) {
  if ((int)h->graphs.size() == kGraphKinds) return 0;
  drop_graphs(h);
  for (int g = 0; g < kGraphKinds; ++g) {  // graphs[2 * size + advance]
    StepGraph sg;
    if (int r = capture_step_graph(h, kGraphSizes[g / 2], g & 1, &sg)) {
      drop_graphs(h);
      return r;
    }
    h->graphs.push_back(sg);
  }
  return 0;
}

// n units from the cursor: whole 64- and 16-unit graphs, then the rest eagerly (a graph replay
// costs a cursor launch and a graph-to-graph gap of ~13 us on the GPU, more than the host takes
// to launch a few units while the GPU is busy).  Returns the cursor's advance (*base).
static int run_units(bprmf_handle* h, int64_t n, int64_t* base) {
  *base = 0;
  int64_t done = 0;
  // short chunks launch eagerly: a graph's end costs ~8 us before the next launch starts, more
  // than the host needs per launch (~4 us) while each fused launch runs ~10 us on the GPU
  if (h->use_graphs && n >= kGraphSizes[0]) {
    if (int r = ensure_step_graphs(h)) return r;
    const int64_t n64 = n / kGraphSizes[0], n16 = (n % kGraphSizes[0]) / kGraphSizes[1];
    const int64_t ng = n64 + n16;
    for (int64_t q = 0; q < ng; ++q) {
      const int size = q < n64 ? 0 : 1;
      const bool adv = q + 1 < ng;
      const StepGraph& g = h->graphs[2 * size + (adv ? 1 : 0)];
      HIPCHK(hipGraphLaunch(g.exec, h->stream));
      done += g.n;
      if (adv) *base += g.n;
    }
  }
  for (int64_t k = done; k < n; ++k)
    if (int r = launch_unit(h, k - *base)) return r;
  return 0;
}

// the chunk's nb steps (cursor {h->t, 0}, batches built)
static int launch_steps(bprmf_handle* h, int64_t nb) {
  int64_t base = 0;
  if (!h->fused) return run_units(h, nb, &base);
  const int B = h->cfg.batch_size;
  const BatchView v0 = BatchBuf{h->d_batch, B}.view(0);
  const int64_t stride = BatchBuf::stride_for(B);
  const StepBufs sb = step_bufs(h);
  HIPCHK(user_step(h->geom, v0, B, h->P, h->Q, h->hp, h->d_tbase, 0, nullptr, nullptr, nullptr,
                   nullptr, h->stream, PeerWait{}, stride, &sb));
  if (int r = run_units(h, nb - 1, &base)) return r;
  HIPCHK(item_step(h->geom, v0, B, h->P, h->Q, h->hp, h->d_tbase, (int)(nb - 1 - base), nullptr,
                   nullptr, nullptr, h->stream, nullptr, h->d_loss, stride, &sb));
  return 0;
}

// One chunk of whole steps: slots [first_slot, first_slot + n) of `epoch` from the device sampler
// (ru == nullptr) or replayed device ids ru/ri/rj[0..n).  Segmented path for B <= kMaxSegBatch:
// one build launch for the chunk, then two launches per step; otherwise the atomic path.
static int run_chunk(bprmf_handle* h, uint32_t epoch, int64_t first_slot, int64_t n,
                     const int32_t* ru, const int32_t* ri, const int32_t* rj, int64_t* steps_done) {
  if (n <= 0) return 0;
  const int64_t B = h->cfg.batch_size;
  const int64_t nb = (n + B - 1) / B;
  if ((int64_t)h->t + nb >= INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  if (h->semantics == BPRMF_SEM_STALE1)
    return fail(BPRMF_E_UNSUPPORTED, "stale1 semantics run through the sharded runner "
                                     "(bprmf_dist_init_* + bprmf_dist_train_*)");
  if (h->semantics == BPRMF_SEM_LOCAL) {
    // periods of local_steps steps: one hogwild launch (hot items in the XCD replicas), then the
    // merge; the call's last period is merged too, so the base table is current when it returns
    if (int z = loss_zero_slots(h)) HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * z, h->stream));
    const SamplerArgs sa = sampler_args(h);
    const LocalArgs la = local_args(h);
    hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;
    if (ea) HIPCHK(hipEventRecord(ea, h->stream));
    for (int64_t s0 = 0; s0 < n;) {
      const int64_t left = h->local_steps - (h->t - h->rep_t);  // steps left in this period
      const int64_t m = std::min<int64_t>(n - s0, std::max<int64_t>(1, left) * B);
      const int64_t mb = (m + B - 1) / B;
      HIPCHK(hogwild(h->geom, ru ? nullptr : &sa, epoch, first_slot + s0, ru ? ru + s0 : nullptr,
                     ri ? ri + s0 : nullptr, rj ? rj + s0 : nullptr, m, h->P, h->Q, h->hp, h->t, (int)B,
                     h->d_loss, h->d_err, h->stream, la.H > 0 ? &la : nullptr));
      h->t += (int32_t)mb;
      *steps_done += mb;
      s0 += m;
      if (la.H > 0 && (h->t - h->rep_t >= h->local_steps || s0 >= n)) {
        HIPCHK(local_merge(h->geom, h->Q, la, h->d_hot_rows, h->hp, h->rep_t, h->t, false, h->stream));
        h->rep_t = h->t;
      }
    }
    if (ea) {
      hipEvent_t eb = prof_event(h);
      if (eb) {
        HIPCHK(hipEventRecord(eb, h->stream));
        h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
        h->prof_weight[BPRMF_KPROF_STEPS] += nb - 1;
      }
    }
    return 0;
  }
  if (h->semantics == BPRMF_SEM_HOGWILD) {
    // one launch for the chunk: triplets sampled in the kernel (or replayed), each applied on its
    // own (hogwild.hip); the loss goes to the segmented path's kSegLossSlots slots
    if (int z = loss_zero_slots(h)) HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * z, h->stream));
    const SamplerArgs sa = sampler_args(h);
    {
      hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;
      if (ea) HIPCHK(hipEventRecord(ea, h->stream));
      HIPCHK(hogwild(h->geom, ru ? nullptr : &sa, epoch, first_slot, ru, ri, rj, n, h->P, h->Q, h->hp,
                     h->t, (int)B, h->d_loss, h->d_err, h->stream));
      if (ea) {
        hipEvent_t eb = prof_event(h);
        if (eb) {
          HIPCHK(hipEventRecord(eb, h->stream));
          h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
          h->prof_weight[BPRMF_KPROF_STEPS] += nb - 1;  // one pair covers nb steps
        }
      }
    }
    h->t += (int32_t)nb;
    *steps_done += nb;
    return 0;
  }
  if (!seg_mode(h)) {
    if (!ru) {
      if (int r = ensure_trip(h, n)) return r;
      int32_t* tu = h->d_trip;
      int32_t* ti = tu + h->trip_cap;
      int32_t* tj = ti + h->trip_cap;
      {
        ProfScope ps(h, BPRMF_KPROF_SAMPLE);
        HIPCHK(sample(sampler_args(h), epoch, first_slot, n, tu, ti, tj, h->d_err, h->stream));
      }
      return run_steps(h, tu, ti, tj, n, steps_done);
    }
    return run_steps(h, ru, ri, rj, n, steps_done);
  }
  if (int r = ensure_seg(h, nb)) return r;
  BatchBuf bb{h->d_batch, (int)B};
  // the cursor and the call's loss slots: set by the builder's first workgroup (one launch fewer
  // per call), or by their own launch when every per-wave slot needs zeroing
  CursorInit ci;
  ci.cursor = h->d_tbase;
  ci.t = h->t;
  ci.loss = h->d_loss;
  ci.nloss = loss_zero_slots(h);
  if (ci.nloss > kSegLossSlots) {
    HIPCHK(set_cursor(h->d_tbase, h->t, 0, h->stream, h->d_loss, ci.nloss));
    ci = CursorInit{};
  }
  {
    ProfScope ps(h, BPRMF_KPROF_SAMPLE);
    if (!ru && split_build(nb)) {
      if (int r = ensure_trip(h, n)) return r;
      int32_t* tu = h->d_trip;
      trace_mark();
      // the grid-wide sampler's triplets staged in d_trip: sampled inside the split builder's
      // launch, or by k_sample before the build
      HIPCHK(build_batches(sampler_args(h), epoch, first_slot, n, (int)B, tu, tu + h->trip_cap,
                           tu + 2 * h->trip_cap, h->U, h->cfg.item_num, 1, false, 0, nb, bb,
                           h->d_err, h->stream, k1_triplets_per_block(h->geom), ci, nullptr, true));
      trace_mark();
    } else {
      HIPCHK(build_batches(sampler_args(h), epoch, first_slot, n, (int)B, ru, ri, rj, h->U,
                           h->cfg.item_num, 1, false, 0, nb, bb, h->d_err, h->stream,
                           k1_triplets_per_block(h->geom), ci));
    }
  }
  {
    // profiling: one event pair around the chunk's step launches (GPU-bound, so the pair brackets
    // the step kernels and their gaps; per-kernel splits come from rocprofv3)
    hipEvent_t ea = h->prof_on ? prof_event(h) : nullptr;
    if (ea) HIPCHK(hipEventRecord(ea, h->stream));
#if defined(BPRMF_BUILD_STAMPS) && defined(BPRMF_DIAG_BUILD_ONLY)
    // diagnostic builder builds (tools/ubench_build.py) may write wrong batches on purpose: the
    // step kernels must never index rows with them
    h->t += (int32_t)nb;
    *steps_done += nb;
    return 0;
#endif
    if (int r = launch_steps(h, nb)) return r;
    if (ea) {
      hipEvent_t eb = prof_event(h);
      if (eb) {
        HIPCHK(hipEventRecord(eb, h->stream));
        h->prof_rec[BPRMF_KPROF_STEPS].push_back({ea, eb});
        h->prof_weight[BPRMF_KPROF_STEPS] += nb - 1;  // one pair covers nb steps
      }
    }
  }
  h->t += (int32_t)nb;
  *steps_done += nb;
  return 0;
}

static int run_steps(bprmf_handle* h, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                     int64_t n, int64_t* steps_done) {
  const int64_t B = h->cfg.batch_size;
  if (int r = ensure_grad(h)) return r;
  if (int z = loss_zero_slots(h)) HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * z, h->stream));
  h->slots_dirty = true;
  h->call_slots = true;
  for (int64_t off = 0; off < n; off += B) {
    const int64_t nb = std::min(B, n - off);
    if (h->t == INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
    const int32_t t = h->t + 1;
    {
      ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER);
      HIPCHK(fwd_scatter(h->geom, tu + off, ti + off, tj + off, nb, h->P, h->Q, h->hp, t, h->d_loss,
                         h->d_err, h->stream));
    }
    {
      ProfScope ps(h, BPRMF_KPROF_APPLY);
      HIPCHK(apply_refs(h->geom, tu + off, ti + off, tj + off, nb, h->P, h->Q, h->hp, t, h->stream));
    }
    h->t = t;
    ++*steps_done;
  }
  return 0;
}

int bprmf_train_steps(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                      bprmf_stats* st) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (h->cfg.world != 1)
    return fail(BPRMF_E_STATE, "sharded handle: drive steps with the bprmf_dist_* phases");
  if (!h->d_pos_u || h->npos == 0) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
  int64_t N, S;
  bprmf_epoch_size(h, &N, &S);
  if (first_step < 0 || n_steps < 0 || first_step + n_steps > S)
    return fail(BPRMF_E_INVALID, "steps [%lld, %lld) outside the epoch's %lld steps",
                (long long)first_step, (long long)(first_step + n_steps), (long long)S);
  const int64_t B = h->cfg.batch_size;
  const int64_t chunk = chunk_triplets(h);
  const int64_t beg = first_step * B, end = std::min(N, (first_step + n_steps) * B);
  g_trace_n = 0;  // a failed earlier call may have left marks
  trace_mark();
  if (int r = begin_call(h)) return r;
  int64_t steps = 0;
  for (int64_t off = beg; off < end; off += chunk)
    if (int r = run_chunk(h, epoch, off, std::min(chunk, end - off), nullptr, nullptr, nullptr, &steps))
      return r;
  trace_mark();
  const int rc_end = end_call(h, st, end - beg, steps);
  trace_mark();
  trace_flush();
  return rc_end;
}

int bprmf_train_epoch(bprmf_handle* h, uint32_t epoch, bprmf_stats* st) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  int64_t N, S;
  bprmf_epoch_size(h, &N, &S);
  return bprmf_train_steps(h, epoch, 0, S, st);
}

int bprmf_train_triplets_dev(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                             int64_t n, bprmf_stats* st) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_STATE, "sharded handle: use the bprmf_dist_* phases");
  if (int r = begin_call(h)) return r;
  const int64_t chunk = chunk_triplets(h);
  int64_t steps = 0;
  for (int64_t off = 0; off < n; off += chunk) {
    const int64_t m = std::min(chunk, n - off);
    if (int r = run_chunk(h, 0, 0, m, u + off, i + off, j + off, &steps)) return r;
  }
  return end_call(h, st, n, steps);
}

int bprmf_train_triplets(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                         int64_t n, bprmf_stats* st) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_STATE, "sharded handle: use the bprmf_dist_* phases");
  for (int64_t k = 0; k < n; ++k) {
    if (u[k] < 0 || u[k] >= h->cfg.user_num)
      return fail(BPRMF_E_RANGE, "user id %d at %lld out of range [0, %lld)", u[k], (long long)k,
                  (long long)h->cfg.user_num);
    if (i[k] < 0 || i[k] >= h->cfg.item_num || j[k] < 0 || j[k] >= h->cfg.item_num)
      return fail(BPRMF_E_RANGE, "item id at %lld out of range [0, %lld)", (long long)k,
                  (long long)h->cfg.item_num);
  }
  if (int r = set_dev(h)) return r;
  const int64_t chunk = chunk_triplets(h);  // whole batches
  if (int r = ensure_trip(h, std::min(chunk, std::max<int64_t>(n, 1)))) return r;
  if (int r = begin_call(h)) return r;
  int64_t steps = 0;
  for (int64_t off = 0; off < n; off += chunk) {
    const int64_t m = std::min(chunk, n - off);
    int32_t* tu = h->d_trip;
    int32_t* ti = tu + h->trip_cap;
    int32_t* tj = ti + h->trip_cap;
    HIPCHK(hipMemcpyAsync(tu, u + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(ti, i + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(tj, j + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    if (int r = run_chunk(h, 0, 0, m, tu, ti, tj, &steps)) return r;
    HIPCHK(hipStreamSynchronize(h->stream));  // host buffers reused by the next chunk's copies
  }
  return end_call(h, st, n, steps);
}

int bprmf_sample(bprmf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u, int32_t* i,
                 int32_t* j) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->d_pos_u || h->npos == 0) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
  int64_t N;
  bprmf_epoch_size(h, &N, nullptr);
  if (first < 0 || first + n > N) return fail(BPRMF_E_INVALID, "slots outside the epoch");
  if (int r = set_dev(h)) return r;
  if (n == 0) return 0;
  int32_t* buf = nullptr;
  if (int r = dalloc(&buf, 3 * n)) return r;
  int rc = 0;
  hipError_t e = sample(sampler_args(h), epoch, first, n, buf, buf + n, buf + 2 * n, h->d_err, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(u, buf, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(i, buf + n, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(j, buf + 2 * n, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "sample: %s", hipGetErrorString(e));
  (void)hipFree(buf);
  if (rc) return rc;
  return check_err_flag(h);
}

int bprmf_dist_sample_dev(bprmf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u,
                          int32_t* i, int32_t* j) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->d_pos_u || h->npos == 0) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
  int64_t N;
  bprmf_epoch_size(h, &N, nullptr);
  if (first < 0 || first + n > N) return fail(BPRMF_E_INVALID, "slots outside the epoch");
  if (int r = set_dev(h)) return r;
  HIPCHK(sample(sampler_args(h), epoch, first, n, u, i, j, h->d_err, h->stream));
  return 0;
}

int bprmf_set_weights(bprmf_handle* h, const float* P, const float* Q) {
  if (!h || !P || !Q) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = set_dev(h)) return r;
  const size_t D = h->geom.D, ld = h->geom.ld;
  if (int r = dp_quiesce(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemset(h->P.W, 0, sizeof(float) * h->U * ld));
  HIPCHK(hipMemset(h->Q.W, 0, sizeof(float) * h->I * ld));
  if (h->U) HIPCHK(hipMemcpy2D(h->P.W, ld * 4, P, D * 4, D * 4, h->U, hipMemcpyHostToDevice));
  if (h->I) HIPCHK(hipMemcpy2D(h->Q.W, ld * 4, Q, D * 4, D * 4, h->I, hipMemcpyHostToDevice));
  // rows are now current at step t; grads are zero between steps
  std::vector<int32_t> st(std::max(h->U, h->I), h->t);
  if (h->U) HIPCHK(hipMemcpy(h->P.stamp, st.data(), 4 * h->U, hipMemcpyHostToDevice));
  if (h->I) HIPCHK(hipMemcpy(h->Q.stamp, st.data(), 4 * h->I, hipMemcpyHostToDevice));
  if (h->d_qbase) {  // LOCAL at world > 1: the next merge's base (every rank sets the same Q)
    HIPCHK(hipMemcpy(h->d_qbase, h->Q.W, sizeof(float) * h->I * ld, hipMemcpyDeviceToDevice));
    h->dp_t = h->t;
  }
  return local_refresh(h);  // LOCAL: the replicas start from the new rows
}

int bprmf_get_weights(bprmf_handle* h, float* P, float* Q) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = set_dev(h)) return r;
  HIPCHK(flush(h->geom, h->P, h->hp, h->t, h->stream));
  HIPCHK(flush(h->geom, h->Q, h->hp, h->t, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  const size_t D = h->geom.D, ld = h->geom.ld;
  if (P && h->U) HIPCHK(hipMemcpy2D(P, D * 4, h->P.W, ld * 4, D * 4, h->U, hipMemcpyDeviceToHost));
  if (Q && h->I) HIPCHK(hipMemcpy2D(Q, D * 4, h->Q.W, ld * 4, D * 4, h->I, hipMemcpyDeviceToHost));
  return 0;
}

int bprmf_get_rows(bprmf_handle* h, int32_t table, const int32_t* rows, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!rows || !out)) || (table != 0 && table != 1))
    return fail(BPRMF_E_INVALID, "bad arguments");
  const Table& W = table == 0 ? h->P : h->Q;
  for (int64_t k = 0; k < n; ++k)
    if (rows[k] < 0 || rows[k] >= W.rows)
      return fail(BPRMF_E_RANGE, "row %d at %lld out of range [0, %lld)", rows[k], (long long)k,
                  (long long)W.rows);
  if (n == 0) return 0;
  if (int r = set_dev(h)) return r;
  const size_t D = h->geom.D, ld = h->geom.ld;
  int32_t* buf = nullptr;
  if (int r = dalloc(&buf, n + n * (int64_t)ld)) return r;
  float* o = reinterpret_cast<float*>(buf + n);
  int rc = 0;
  // gather_rows(t) brings a row to step t - 1: the rows as of the step count h->t
  hipError_t e = hipMemcpyAsync(buf, rows, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = gather_rows(h->geom, W, buf, n, h->hp, h->t + 1, o, h->d_err, h->stream);
  if (e == hipSuccess) e = hipMemcpy2DAsync(out, D * 4, o, ld * 4, D * 4, n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "get_rows: %s", hipGetErrorString(e));
  (void)hipFree(buf);
  if (rc) return rc;
  return check_err_flag(h);
}

int bprmf_score(bprmf_handle* h, const int32_t* u, const int32_t* i, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !out))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_UNSUPPORTED, "score needs an unsharded handle");
  for (int64_t k = 0; k < n; ++k) {
    if (u[k] < 0 || u[k] >= h->cfg.user_num) return fail(BPRMF_E_RANGE, "Invalid user code");
    if (i[k] < 0 || i[k] >= h->cfg.item_num) return fail(BPRMF_E_RANGE, "Invalid item code");
  }
  if (n == 0) return 0;
  if (int r = set_dev(h)) return r;
  int32_t* buf = nullptr;
  if (int r = dalloc(&buf, 3 * n)) return r;
  float* o = (float*)(buf + 2 * n);
  int rc = 0;
  hipError_t e = hipMemcpyAsync(buf, u, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(buf + n, i, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = score(h->geom, buf, buf + n, n, h->P, h->Q, h->hp, h->t, o, h->d_err, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, o, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "score: %s", hipGetErrorString(e));
  (void)hipFree(buf);
  if (rc) return rc;
  return check_err_flag(h);
}

int bprmf_forward_dev(bprmf_handle* h, const int64_t* u, const int64_t* i, const int64_t* j,
                      int64_t n, float* pred_i, float* pred_j) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !pred_i))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_UNSUPPORTED, "forward needs an unsharded handle");
  if (n == 0) return 0;
  if (int r = set_dev(h)) return r;
  HIPCHK(forward64(h->geom, u, i, j, n, h->P, h->Q, h->hp, h->t, pred_i, j ? pred_j : nullptr,
                   h->d_err, h->stream));
  return check_err_flag(h);
}

int bprmf_topk_lists(bprmf_handle* h, const int32_t* users, const int64_t* offsets,
                     const int32_t* items, int64_t n_users, int32_t k, int32_t* out_pos,
                     float* out_score) {
  if (!h || n_users < 0 || k <= 0 || (n_users > 0 && (!users || !offsets || !items || !out_pos || !out_score)))
    return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_UNSUPPORTED, "top-k needs an unsharded handle");
  if (k > 256) return fail(BPRMF_E_UNSUPPORTED, "k must be <= 256");
  if (n_users == 0) return 0;
  if (offsets[0] != 0) return fail(BPRMF_E_INVALID, "offsets[0] must be 0");
  for (int64_t r = 0; r < n_users; ++r) {
    if (offsets[r + 1] < offsets[r]) return fail(BPRMF_E_INVALID, "offsets must be non-decreasing");
    if (users[r] < 0 || users[r] >= h->cfg.user_num) return fail(BPRMF_E_RANGE, "Invalid user code");
  }
  const int64_t m = offsets[n_users];
  for (int64_t x = 0; x < m; ++x)
    if (items[x] < 0 || items[x] >= h->cfg.item_num) return fail(BPRMF_E_RANGE, "Invalid item code");
  if (int r = set_dev(h)) return r;
  // one device block: users | offsets (8-aligned) | items | out_pos | out_score
  const int64_t w_users = (n_users + 1) & ~1LL, w_offs = 2 * (n_users + 1);
  const int64_t words = w_users + w_offs + m + 2 * n_users * (int64_t)k;
  int32_t* buf = nullptr;
  if (int r = dalloc(&buf, words)) return r;
  int32_t* d_users = buf;
  int64_t* d_offs = reinterpret_cast<int64_t*>(buf + w_users);
  int32_t* d_items = buf + w_users + w_offs;
  int32_t* d_pos = d_items + m;
  float* d_score = reinterpret_cast<float*>(d_pos + n_users * (int64_t)k);
  int rc = 0;
  hipError_t e = hipMemcpyAsync(d_users, users, 4 * n_users, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_offs, offsets, 8 * (n_users + 1), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && m) e = hipMemcpyAsync(d_items, items, 4 * m, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess)
    e = topk_lists(h->geom, d_users, d_offs, d_items, n_users, k, h->P, h->Q, h->hp, h->t, d_pos,
                   d_score, h->d_err, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_pos, d_pos, 4 * n_users * (int64_t)k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_score, d_score, 4 * n_users * (int64_t)k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "topk_lists: %s", hipGetErrorString(e));
  (void)hipFree(buf);
  if (rc) return rc;
  return check_err_flag(h);
}

int bprmf_topk_all(bprmf_handle* h, const int32_t* users, int64_t n_users, int32_t k,
                   int32_t exclude_train, int32_t* out_items, float* out_scores) {
  if (!h || n_users < 0 || k <= 0 || (n_users > 0 && (!users || !out_items || !out_scores)))
    return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.world != 1) return fail(BPRMF_E_UNSUPPORTED, "top-k needs an unsharded handle");
  if (k > 32) return fail(BPRMF_E_UNSUPPORTED, "k must be <= 32");
  if (h->geom.ld > 128) return fail(BPRMF_E_UNSUPPORTED, "full-catalogue top-k supports factor_num <= 128");
  if (exclude_train && !h->d_indptr) return fail(BPRMF_E_STATE, "exclude_train needs bprmf_set_train");
  for (int64_t r = 0; r < n_users; ++r)
    if (users[r] < 0 || users[r] >= h->cfg.user_num) return fail(BPRMF_E_RANGE, "Invalid user code");
  if (n_users == 0) return 0;
  if (int r = set_dev(h)) return r;
  const int64_t words = ((n_users + 3) & ~3LL) + 2 * n_users * (int64_t)k;
  int32_t* buf = nullptr;
  if (int r = dalloc(&buf, words)) return r;
  int32_t* d_users = buf;
  int32_t* d_items = buf + ((n_users + 3) & ~3LL);
  float* d_scores = reinterpret_cast<float*>(d_items + n_users * (int64_t)k);
  int rc = 0;
  hipError_t e = hipMemcpyAsync(d_users, users, 4 * n_users, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    ProfScope ps(h, BPRMF_KPROF_TOPK);
    e = topk_all(h->geom, d_users, n_users, k, h->P, h->Q, h->hp, h->t,
                 exclude_train ? h->d_indptr : nullptr, exclude_train ? h->d_indices : nullptr,
                 d_items, d_scores, h->stream);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out_items, d_items, 4 * n_users * (int64_t)k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_scores, d_scores, 4 * n_users * (int64_t)k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "topk_all: %s", hipGetErrorString(e));
  (void)hipFree(buf);
  return rc;
}

int bprmf_profile(bprmf_handle* h, int32_t enable) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = set_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  h->prof_on = enable != 0;
  h->prof_used = 0;
  for (auto& w : h->prof_weight) w = 0;
  for (auto& v : h->prof_rec) v.clear();
  return 0;
}

int bprmf_profile_read(bprmf_handle* h, bprmf_kprof* out) {
  if (!h || !out) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = set_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  memset(out, 0, sizeof *out);
  for (int k = 0; k < BPRMF_KPROF_KINDS; ++k) {
    double total = 0;
    for (auto& pr : h->prof_rec[k]) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
      total += ms;
    }
    out->count[k] = (int64_t)h->prof_rec[k].size() + h->prof_weight[k];
    out->ms[k] = total;
  }
  return 0;
}

// ---- sharded steps (one process per GPU; the caller moves the buffers over RCCL) ------------
// Users u live on rank u % world, items i on rank i % world.  A step of this shard:
//   request_ids -> [all-to-all ids] -> gather_items (owner) -> [all-to-all rows back]
//   -> user_step (K1: local users vs received rows) -> item_grads (K2: per requested item)
//   -> [all-to-all grads to owners] -> apply_items (owner) -> end_step.
static int dist_counts(bprmf_handle* h, int64_t n_steps, int32_t* owner_counts) {
  const int64_t stride = BatchBuf::stride_for(h->cfg.batch_size);
  const BatchBuf bb{h->d_batch, h->cfg.batch_size};
  HIPCHK(hipMemcpy2DAsync(owner_counts, sizeof(int32_t) * h->cfg.world, bb.view(0).own,
                          sizeof(int32_t) * stride, sizeof(int32_t) * h->cfg.world, n_steps,
                          hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->plan_steps = n_steps;
  return check_err_flag(h);
}

// semantics LOCAL at world > 1 keeps the WHOLE item table on every rank (Q indexed by global id):
// the per-step sharded calls address items by owner (i % world, local row i / world) and would
// read and update the wrong rows of it.  Only the runner (bprmf_dist_train_*) runs
// that mode.
static int dist_per_step_ok(bprmf_handle* h) {
  if (h && h->dp_mode)
    return fail(BPRMF_E_UNSUPPORTED,
                "the per-step sharded calls address items by owner; semantics local at world > 1 "
                "replicates the item table: use bprmf_dist_train_steps / bprmf_dist_train_replay");
  if (h && h->semantics == BPRMF_SEM_STALE1)  // its staleness is the runner's two-stream schedule
    return fail(BPRMF_E_UNSUPPORTED,
                "semantics stale1 runs through the runner: use bprmf_dist_train_steps / _replay");
  return 0;
}

int bprmf_dist_plan(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                    int32_t* owner_counts) {
  if (!h || first_step < 0 || n_steps <= 0 || !owner_counts) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = dist_per_step_ok(h)) return r;
  if (!seg_mode(h)) return fail(BPRMF_E_UNSUPPORTED, "sharded steps need batch_size <= %d", kMaxSegBatch);
  if (!h->d_pos_u) return fail(BPRMF_E_STATE, "call bprmf_set_train first");
  if (int r = set_dev(h)) return r;
  if (int r = ensure_seg(h, n_steps)) return r;
  int64_t N;
  bprmf_epoch_size(h, &N, nullptr);
  const int64_t B = h->cfg.batch_size;
  const int64_t first_slot = first_step * B;
  const int64_t n_slots = std::max<int64_t>(0, std::min(N - first_slot, n_steps * B));
  const BatchBuf bb{h->d_batch, (int)B};
  {
    ProfScope ps(h, BPRMF_KPROF_SAMPLE);
    HIPCHK(build_batches(sampler_args(h), epoch, first_slot, n_slots, (int)B, nullptr, nullptr,
                         nullptr, h->U, h->cfg.item_num, h->cfg.world, true, 0, n_steps, bb, h->d_err,
                         h->stream, k1_triplets_per_block(h->geom)));
  }
  return dist_counts(h, n_steps, owner_counts);
}

int bprmf_dist_plan_replay(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                           int64_t n_steps, int32_t* owner_counts) {
  if (!h || n_steps <= 0 || !u || !i || !j || !owner_counts) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = dist_per_step_ok(h)) return r;
  if (!seg_mode(h)) return fail(BPRMF_E_UNSUPPORTED, "sharded steps need batch_size <= %d", kMaxSegBatch);
  const int64_t B = h->cfg.batch_size, n = n_steps * B, W = h->cfg.world, R = h->cfg.rank;
  for (int64_t k = 0; k < n; ++k) {
    if (u[k] < 0) continue;  // padding slot
    if (u[k] >= h->cfg.user_num || u[k] % W != R)
      return fail(BPRMF_E_RANGE, "user %d at %lld is not a user of shard %lld", u[k], (long long)k, (long long)R);
    if (i[k] < 0 || i[k] >= h->cfg.item_num || j[k] < 0 || j[k] >= h->cfg.item_num)
      return fail(BPRMF_E_RANGE, "item id at %lld out of range", (long long)k);
  }
  if (int r = set_dev(h)) return r;
  if (int r = ensure_seg(h, n_steps)) return r;
  if (int r = ensure_trip(h, n)) return r;
  int32_t* tu = h->d_trip;
  int32_t* ti = tu + h->trip_cap;
  int32_t* tj = ti + h->trip_cap;
  HIPCHK(hipMemcpyAsync(tu, u, 4 * n, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(ti, i, 4 * n, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(tj, j, 4 * n, hipMemcpyHostToDevice, h->stream));
  const BatchBuf bb{h->d_batch, (int)B};
  HIPCHK(build_batches(sampler_args(h), 0, 0, n, (int)B, tu, ti, tj, h->U, h->cfg.item_num,
                       h->cfg.world, true, 0, n_steps, bb, h->d_err, h->stream, k1_triplets_per_block(h->geom)));
  return dist_counts(h, n_steps, owner_counts);
}

static int dist_step_ok(bprmf_handle* h, int64_t k) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = dist_per_step_ok(h)) return r;
  if (k < 0 || k >= h->plan_steps) return fail(BPRMF_E_STATE, "step %lld is not in the current plan", (long long)k);
  return set_dev(h);
}

int bprmf_dist_request_ids(bprmf_handle* h, int64_t k, int32_t* ids, int64_t n) {
  if (int r = dist_step_ok(h, k)) return r;
  if (n < 0 || (n > 0 && !ids) || n > 2LL * h->cfg.batch_size) return fail(BPRMF_E_INVALID, "bad arguments");
  const BatchBuf bb{h->d_batch, h->cfg.batch_size};
  if (n) HIPCHK(hipMemcpyAsync(ids, bb.view(k).ukey, 4 * n, hipMemcpyDeviceToDevice, h->stream));
  return 0;
}

int bprmf_dist_gather_items(bprmf_handle* h, const int32_t* rows, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!rows || !out))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = dist_per_step_ok(h)) return r;
  if (int r = set_dev(h)) return r;
  HIPCHK(gather_rows(h->geom, h->Q, rows, n, h->hp, h->t + 1, out, h->d_err, h->stream));
  return 0;
}

int bprmf_dist_user_step(bprmf_handle* h, int64_t k, const float* item_rows) {
  if (int r = dist_step_ok(h, k)) return r;
  if (!item_rows) return fail(BPRMF_E_INVALID, "null item_rows");
  const BatchBuf bb{h->d_batch, h->cfg.batch_size};
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->d_tbase, h->t, 1, h->stream));
  ProfScope ps(h, BPRMF_KPROF_FWD_SCATTER);
  HIPCHK(user_step(h->geom, bb.view(k), h->cfg.batch_size, h->P, h->Q, h->hp, h->d_tbase, 0,
                   h->d_xloss, h->d_contrib, h->d_ugrad, item_rows, h->stream));
  return 0;
}

int bprmf_dist_item_grads(bprmf_handle* h, int64_t k, float* grads) {
  if (int r = dist_step_ok(h, k)) return r;
  if (!grads) return fail(BPRMF_E_INVALID, "null grads");
  const BatchBuf bb{h->d_batch, h->cfg.batch_size};
  ProfScope ps(h, BPRMF_KPROF_APPLY);
  HIPCHK(item_step(h->geom, bb.view(k), h->cfg.batch_size, h->P, h->Q, h->hp, h->d_tbase, 0,
                   h->d_contrib, h->d_ugrad, grads, h->stream, h->d_xloss, h->d_loss));
  return 0;
}

int bprmf_dist_apply_items(bprmf_handle* h, const int32_t* rows, const float* grads, int64_t n) {
  if (!h || n < 0 || (n > 0 && (!rows || !grads))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = dist_per_step_ok(h)) return r;
  if (int r = set_dev(h)) return r;
  if (int r = ensure_grad(h)) return r;
  ProfScope ps(h, BPRMF_KPROF_OWNER);
  HIPCHK(add_rows(h->geom, h->Q, rows, grads, n, h->d_err, h->stream));
  HIPCHK(apply_rows(h->geom, h->Q, rows, n, h->hp, h->t + 1, h->stream));
  return 0;
}

int bprmf_dist_end_step(bprmf_handle* h, double* loss) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = set_dev(h)) return r;
  if (h->t == INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  h->t += 1;
  if (loss) {  // loss since the last read; resets the accumulator
    if (int r = read_loss(h, loss)) return r;
    HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * kLossSlots, h->stream));
    return check_err_flag(h);
  }
  return 0;
}

}  // extern "C"
