// kernels.h — host-side launchers of the gfx950 BPR-MF kernels (kernels.hip).
// Internal to libbprmf_amd.so; the public ABI is include/bprmf.h.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace bprmf {

// Row geometry: a row of D floats is stored with stride ld (zero padded).  Two lane layouts share
// that stride: float4 (segmented step, step.hip): G4 = next_pow2(ceil(D/4)) <= 64 lanes per row,
// S stripes, ld = 4*G4*S; dword (atomic path, owner-side kernels, kernels.hip): G lanes per row,
// lane `sub` holds elements sub + G*k, k < EPL, with G*EPL = ld.
// per-wave loss partial slots of the step kernels: grid <= kMaxGridBlocks blocks of 4 waves
constexpr int kMaxGridBlocks = 256 * 8;
constexpr int kLossSlots = kMaxGridBlocks * 4;
constexpr int kSegLossSlots = 32;  // loss slots of the segmented step (item_step's loss workgroups)

struct Geom {
  int D, G, EPL, ld;
  int G4, S;  // float4 layout: G4 lanes per row, lane `sub` holds floats 4*sub + 4*G4*s, s < S
};
bool make_geom(int D, Geom* g);

// One factor table (user or item side) resident in HBM.
struct Table {
  float* W;        // [rows, ld] weights, value valid at step stamp[row]
  float* G;        // [rows, ld] gradient accumulator, zero outside a step
  int32_t* stamp;  // [rows] step at which W[row] is current (lazy dense weight decay)
  int64_t rows;
};

// One batch of a step, as laid out by k_build_batches (int32, positions within the batch).  Every
// step kernel reaches its rows after ONE dependent load of a 16- or 32-byte record:
//   trec  [B][4]    per triplet, sorted by (local) user row: {i, j, u, w}; bit 31 of i (of j): this
//                   triplet holds the item's first reference in the batch; w = 1: the user has no
//                   other triplet in the batch (K1 updates the user row itself); w >= 2: head of the
//                   user's segment of w triplets, all in one K1 workgroup (K1 sums it in LDS and
//                   updates the row); w = -1: another member of such a segment; w = 0: a segment
//                   spanning K1 workgroups (K2 finishes it)
//   mrec  [B/2][8]  the w = 0 user segments: {u, beg, end, 0...} (meta[4] of them; K2 sums their
//                   per-triplet user gradients in position order)
//   irec  [2B][8]   item segment s: {item, beg | len << 15 | long << 30, refs 0..11 two per int
//                   (16-bit halves, low first)}                                 (meta[2] of them)
//                   (sharded mode: item = the segment's slot)
//   lrec  [B/8][8]  copies of the records of item segments with > kLongSeg references (meta[3];
//                   at most 2B/(kLongSeg+1) < B/8 of them)
//   refs  [2B]      (triplet position << 1) | (1 if the item is the negative j, 0 if the positive i),
//                   sorted by item then position (fixed summation order)
//   useg  [B+1], ioff [2B+1]   builder scratch (ioff: the radix build's item segment starts;
//                   the bucket build keeps both in LDS and stores neither)
//   ukey  [2B]      sharded mode: the distinct items as the owner's local row, segment order
//   meta  [8]       {triplets, user segments, item segments, long item segments, multi user segs}
//   own   [64]      sharded mode: item segments per owner rank (segments are owner-major)
// Item segments are ordered by key = (item % world) * iloc + item / world (= item when world 1).
// In sharded mode trec holds item SLOTS (rows of the exchange buffers) instead of item rows.
constexpr int kRec = 8;
constexpr int kLongSeg = 16;
constexpr int kInlineRefs = 12;  // refs held in an item segment's record (B <= 8192: 14-bit refs)
constexpr int kMaxLongItems = 64;  // hot items per batch given a whole workgroup in K2
// ranks of a sharded run at most: the per-peer tables (PushArgs, GradRoute) travel as kernel
// arguments every step, and their size is what a launch costs on the host (one node's 8 GPUs,
// with room to spare)
constexpr int kMaxWorld = 16;
constexpr int kBoardMax = 16384;  // producing workgroups one completion board tracks
struct BatchView {
  int32_t *trec, *mrec, *irec, *lrec, *refs, *useg, *ioff, *ukey, *meta, *own;
  __host__ __device__ BatchView shifted(int64_t off) const {
    return BatchView{trec + off, mrec + off, irec + off, lrec + off, refs + off,
                     useg + off, ioff + off, ukey + off, meta + off, own + off};
  }
};
struct BatchBuf {
  int32_t* base;
  int B;
  // a multiple of 4 ints: every batch (and its int4 records) stays 16-byte aligned
  __host__ __device__ static int64_t stride_for(int B) { return 32LL * B + 76; }
  __host__ __device__ BatchView view(int64_t k) const {
    int32_t* p = base + k * stride_for(B);
    BatchView v;
    v.trec = p;
    v.mrec = p + 4LL * B;
    v.irec = p + 8LL * B;
    v.lrec = p + 24LL * B;
    v.refs = p + 25LL * B;
    v.useg = p + 27LL * B;
    v.ioff = p + 28LL * B + 1;
    v.ukey = p + 30LL * B + 2;
    v.meta = p + 32LL * B + 4;
    v.own = p + 32LL * B + 12;
    return v;
  }
};
constexpr int kMaxSegBatch = 8192;  // largest batch the one-workgroup builder handles
// The record packing above depends on kMaxSegBatch (segment.hip writes, step.hip reads):
// item records hold beg and len in 15 bits each; inline refs ((pos << 1) | is_j) are 16-bit
// halves; the builder's packed scan (heads << 16) | valid needs B < 2^16; K2's loss workgroups
// (one per 256 triplets) each own one of kSegLossSlots slots, all summed by the call's end.
static_assert(2 * kMaxSegBatch < (1 << 15), "item record beg/len fields are 15 bits");
static_assert(((2 * kMaxSegBatch - 1) << 1 | 1) <= 0xFFFF, "inline refs are 16-bit halves");
static_assert(kMaxSegBatch < (1 << 16), "builder packed scan keeps counts in 16 bits");
static_assert((kMaxSegBatch + 255) / 256 <= kSegLossSlots, "a loss slot per K2 loss workgroup");

struct Hyper {
  float lr, wd;
  double alpha;  // 1 - lr*wd in double: per-step decay factor of untouched rows
  double log2a;  // log2(alpha): decay over k steps = exp2(k * log2a)
};

// domain Z_a x Z_c of the sampler's Feistel permutation (device_common.h permute) for n items:
// c = ceil(sqrt(n)), a = ceil(n / c), so a*c >= n and a*c - n < c
inline void feistel_dims(uint64_t n, uint32_t* a, uint32_t* c) {
  if (n <= 1) {
    *a = *c = 1;
    return;
  }
  uint64_t r = (uint64_t)sqrt((double)n);
  while (r * r > n) --r;
  while ((r + 1) * (r + 1) <= n) ++r;  // r = isqrt(n)
  const uint64_t cc = r * r == n ? r : r + 1;
  *c = (uint32_t)cc;
  *a = (uint32_t)((n + cc - 1) / cc);
}

struct SamplerArgs {
  const int32_t* pos_u;   // [npos] global user id, features order
  const int32_t* pos_i;   // [npos] global item id
  const int64_t* indptr;  // [local_users+1]
  const int32_t* indices; // sorted positives per local user
  int64_t npos, item_num;
  int32_t num_ng, world;
  uint32_t feistel_a, feistel_c;  // permute's domain Z_a x Z_c (feistel_dims)
  uint32_t k0, k1;        // Philox key (shard seed)
  // the k-th non-member search's 16-ary trees (host_plan.h SearchTree; null: binary search)
  const int32_t* skeys = nullptr;
  const int64_t* soff = nullptr;
  // the same data packed so each dependent level is one line (null: the arrays above):
  // pos2[p] = {pos_u[p], pos_i[p]}; urec[local user] = {its first tree key, its positive count}
  const int2* pos2 = nullptr;
  const int2* urec = nullptr;
  // large positive sets: pos4[p] = {pos_u, pos_i, urec[local user]}, the positive's record and its
  // user's in ONE line (null: pos2 + urec)
  const int4* pos4 = nullptr;
};

// --- launches (all asynchronous on `s`) ---
// step cursor c = {t, k}: the step kernels of a position-independent graph run batch c[1] + r at
// optimizer step c[0] + r + 1 (r = the launch's index in the graph); advance adds n to both
// (loss != null: also zero loss[0 .. nloss))
hipError_t set_cursor(int32_t* cursor, int32_t t, int32_t k, hipStream_t s, double* loss = nullptr,
                      int nloss = 0);
// copy `words` (<= 64) 8-byte words of device memory into mapped host memory (one tiny kernel);
// seq_dev != null: then store seq there (mapped host memory) after those words are written
hipError_t status_out(const void* d_status, void* h_status_dev, int words, hipStream_t s,
                      void* seq_dev = nullptr, uint64_t seq = 0);
hipError_t advance_cursor(int32_t* cursor, int32_t n, hipStream_t s);
// a[0] and b[0] into mapped host memory dst[0..1], then seq into seq_dev (mapped); zero != null:
// then *zero = 0 (the sharded runner's capacity word, ready for the next chunk's builder)
hipError_t pair_out(const int32_t* a, const int32_t* b, void* dst_dev, void* seq_dev, uint64_t seq,
                    hipStream_t s, int32_t* zero = nullptr);
hipError_t init_normal(const Geom& g, float* W, int64_t rows, float std, uint32_t k0, uint32_t k1,
                       uint32_t table_tag, int world, int rank, hipStream_t s);
hipError_t sample(const SamplerArgs& a, uint32_t epoch, int64_t first, int64_t count, int32_t* ou,
                  int32_t* oi, int32_t* oj, int32_t* err, hipStream_t s);
// single-GPU step t (1-based): K1 forward + grad scatter, K2 claim + apply
hipError_t fwd_scatter(const Geom& g, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                       int64_t n, Table P, Table Q, const Hyper& hp, int32_t t, double* loss,
                       int32_t* err, hipStream_t s);
hipError_t apply_refs(const Geom& g, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                      int64_t n, Table P, Table Q, const Hyper& hp, int32_t t, hipStream_t s);
// segmented step: build `n_batches` batches of B (<= kMaxSegBatch) from the sampler (ru == null)
// or from replayed ids; then per batch k: user_step (K1) and item_step (K2) with t = *tbase+k+1.
// ru/ri/rj are GLOBAL ids (users are mapped to local rows u / world).  i_rows = global item count.
// slots: write item slots (sharded exchange) instead of item rows into ij/urec and irec/lrec:
// the item segment index (slot_stride 0) or owner * slot_stride + index within the owner's range.
// cursor != null: the builder's first workgroup also does set_cursor's work (one launch fewer)
struct CursorInit {
  int32_t* cursor = nullptr;
  int32_t t = 0, k = 0;
  double* loss = nullptr;
  int nloss = 0;
  // sharded runner: the split builder raises *own_max (zero before the launch) to the chunk's
  // largest per-owner segment count (dist_own_max's result), and says so in *own_max_done
  int32_t* own_max = nullptr;
};
hipError_t build_batches(const SamplerArgs& a, uint32_t epoch, int64_t first_slot, int64_t n_slots,
                         int B, const int32_t* ru, const int32_t* ri, const int32_t* rj,
                         int64_t u_rows, int64_t i_rows, int world, bool slots, int slot_stride,
                         int64_t n_batches, BatchBuf bb, int32_t* err, hipStream_t s, int tpb,
                         const CursorInit& ci = CursorInit{}, bool* own_max_done = nullptr,
                         bool sample_first = false);
// (sample_first: ru/ri/rj are staging arrays [n_slots] the call fills with the device sampler's
// triplets of slots first_slot.. of `epoch` before building from them: inside the split builder's
// launch where it applies, else by a k_sample launch)
// triplets per K1 workgroup for a geometry (the builder marks user segments that lie in one)
int k1_triplets_per_block(const Geom& g);
// Per-step buffers of the step kernels.  pstride != 0 (single GPU): contrib / ugrad / xloss hold
// two halves, step t uses half t & 1 (contrib, ugrad: pstride floats each; xloss: B floats), so
// K1 of step t+1 can write while K2 of step t still reads (the fused step).  pend_q [2][qrows],
// pend_p [2][prows] (single GPU, fused step): K1 of step t marks half t & 1 of the rows step t
// updates with t.
struct StepBufs {
  float* contrib = nullptr;
  float* ugrad = nullptr;
  float* xloss = nullptr;
  int64_t pstride = 0;
  int32_t* pend_q = nullptr;
  int32_t* pend_p = nullptr;
  int64_t qrows = 0, prows = 0;
};
constexpr int32_t kErrBuild = 16;
// A batch whose build timed out (err bit 16, segment.hip) is left unfinished; the workgroup that
// gave up also stores kDeadMark into the batch's meta[kMetaDead], and every step workgroup of that
// batch returns without touching a row.  The word sits beside meta[0..4], which the step kernels
// load anyway (one line: no extra load level, where a check of the call's error word cost
// ~0.2 us per fused step, profiles/r05_ab_round4_additions.txt).  The batch buffer is zeroed when
// allocated and again by the host when it reports err bit 16 (capi.cpp), so the mark never
// outlives the failed call; no builder ever stores this value elsewhere in the buffer.
constexpr int kMetaDead = 7;
constexpr int32_t kDeadMark = (int32_t)0xDEADB175u;
// sharded K1 over the IPC transport: wait for the peers' row flags first (flags == null: none)
struct PeerWait {
  const int32_t* flags = nullptr;
  int world = 1, self = 0;
  int32_t* err = nullptr;
};
// K1, one lane group per triplet: c*P_u -> contrib[p]; single-triplet users updated in place,
// the others' per-triplet gradients -> ugrad[p]; x = <P_u,Q_i> - <P_u,Q_j> -> xloss[p] (if set).  item_rows != null: sharded K1 (item rows by
// slot from the exchange buffer)
// bstride != 0: bv is batch 0's view and the kernel runs batch tbase[1] + step (cursor graphs);
// bstride == 0: bv is the batch's own view.  Either way t = tbase[0] + step + 1.
hipError_t user_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, float* xloss, float* contrib, float* ugrad,
                     const float* item_rows, hipStream_t s, const PeerWait& pw = PeerWait{},
                     int64_t bstride = 0, const StepBufs* sb = nullptr);
// K2: item segments (fixed-order sums of contrib) and multi-triplet user segments (of ugrad).
// grads != null: sharded K2 (per-slot item gradients [slots, ld] instead of applying the items).
// loss != null: one more workgroup adds the step's loss, sum of log(1 + e^-x) over the x that K1
// x K1 left in xloss, to loss[0 .. ceil(B / 256)) (one slot per loss workgroup, fixed order;
// at most kSegLossSlots slots)
hipError_t item_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, const float* contrib, const float* ugrad,
                     float* grads, hipStream_t s, const float* xloss = nullptr,
                     double* loss = nullptr, int64_t bstride = 0, const StepBufs* sb = nullptr);
// (sb != null: its buffers replace contrib / ugrad / xloss)
// K2 of step t = tbase[0] + step + 1 on batch tbase[1] + step, and K1 of step t + 1 on the next
// batch, in one launch (bv0: batch 0's view; single GPU, sb with both halves and pend arrays)
hipError_t fused_step(const Geom& g, BatchView bv0, int64_t bstride, int B, Table P, Table Q,
                      const Hyper& hp, const int32_t* tbase, int step, const StepBufs& sb,
                      double* loss, int32_t* err, hipStream_t s);
int item_long_blocks(int B);
// relaxed-synchronisation (Hogwild) steps over n slots (hogwild.hip): triplets from the device
// sampler (sa != null: slots slot0 .. slot0+n of `epoch`) or replayed device ids tu/ti/tj; slot s
// belongs to step t0 + 1 + s / B; loss into kSegLossSlots slots
struct LocalArgs;
hipError_t hogwild(const Geom& g, const SamplerArgs* sa, uint32_t epoch, int64_t slot0,
                   const int32_t* tu, const int32_t* ti, const int32_t* tj, int64_t n, Table P,
                   Table Q, const Hyper& hp, int32_t t0, int B, double* loss, int32_t* err,
                   hipStream_t s, const LocalArgs* la = nullptr, int user_world = 1);
// semantics "local" (hogwild.hip): the hot items' rows in one replica per XCD
// (rep [8][H][ld]; hot[item] = replica slot or -1), merged every period: the base row (stamp
// t0) decayed to t1 plus every replica's change, then copied back into the replicas
struct LocalArgs {
  const int32_t* hot = nullptr;
  float* rep = nullptr;
  int64_t H = 0;
  // for a large catalogue (hot[] past the caches), the per-triplet lookup instead reads a bit
  // per item (hbits, I bits) and, for a hot item, an open-addressing table of {item, slot}
  // (hhash, 2^hlog entries, item -1 = empty); null: hot[] is read
  const uint32_t* hbits = nullptr;
  const int2* hhash = nullptr;
  int hlog = 0;
};
constexpr int kLocalXcds = 8;
hipError_t local_merge(const Geom& g, Table Q, const LocalArgs& la, const int32_t* rows,
                       const Hyper& hp, int32_t t0, int32_t t1, bool refresh, hipStream_t s);
// semantics "local" at world > 1 (hogwild.hip): every rank holds the whole item
// table; at a merge (steps tm -> t1) each rank's change is delta = row at t1 - base decayed to t1
// (base: the table at the last merge, current at tm), the ranks' deltas are summed, and every
// rank's row and base become base decayed to t1 + that sum (stamp t1).  Flat over [rows][ld].
// dp_delta also brings a hot row from its XCD replicas (la.H > 0, k_local_merge's rule over
// rep_t -> t1).  pend_sum (dp_overlap): the all-reduce started at the last merge (step tp) has
// landed: base becomes base decayed to tp + pend_sum, the row takes the other ranks' part
// (pend_sum - delta, decayed to t1), and delta is taken against the new base.  keep: the row
// (and a hot row's replicas) keep the result, current at t1 (the next period starts from it).
hipError_t dp_delta(Table Q, float* base, float* delta, const float* pend_sum, int ld, const Hyper& hp,
                    int32_t tm, int32_t tp, int32_t t1, const LocalArgs& la, int32_t rep_t, bool keep,
                    hipStream_t s);
hipError_t dp_apply(Table Q, float* base, const float* sum, int ld, const Hyper& hp, int32_t tm,
                    int32_t t1, const LocalArgs& la, hipStream_t s);  // la.H > 0: replicas too
struct DpSrcs {  // the ranks' delta tables, rank order (in-process transport)
  const float* p[kMaxWorld];
};
hipError_t dp_sum(const DpSrcs& src, int world, float* out, int64_t n, hipStream_t s);
// scoring of the current weights after T steps (reads apply the pending decay)
hipError_t score(const Geom& g, const int32_t* u, const int32_t* i, int64_t n, Table P, Table Q,
                 const Hyper& hp, int32_t T, float* out, int32_t* err, hipStream_t s);
hipError_t forward64(const Geom& g, const int64_t* u, const int64_t* i, const int64_t* j,
                     int64_t n, Table P, Table Q, const Hyper& hp, int32_t T, float* oi, float* oj,
                     int32_t* err, hipStream_t s);
// per-user top-k positions of candidate lists items[offs[r]..offs[r+1]) of users[r] (topk.hip)
hipError_t topk_lists(const Geom& g, const int32_t* users, const int64_t* offs, const int32_t* items,
                      int64_t n_users, int k, Table P, Table Q, const Hyper& hp, int32_t T,
                      int32_t* out_pos, float* out_score, int32_t* err, hipStream_t s);
// per-user top-k items of the whole catalogue (f32 MFMA scores), optionally skipping the user's
// training positives (indptr/indices: the handle's CSR); ld <= 128, k <= 32 (topk.hip)
hipError_t topk_all(const Geom& g, const int32_t* users, int64_t n_users, int k, Table P, Table Q,
                    const Hyper& hp, int32_t T, const int64_t* indptr, const int32_t* indices,
                    int32_t* out_items, float* out_scores, hipStream_t s);
// bring every row of a table to step T (before get_weights)
hipError_t flush(const Geom& g, Table W, const Hyper& hp, int32_t T, hipStream_t s);
// --- sharded step phases ---
hipError_t gather_rows(const Geom& g, Table W, const int32_t* rows, int64_t n, const Hyper& hp,
                       int32_t t, float* out, int32_t* err, hipStream_t s);
hipError_t add_rows(const Geom& g, Table W, const int32_t* rows, const float* grads, int64_t n,
                    int32_t* err, hipStream_t s);
hipError_t apply_rows(const Geom& g, Table W, const int32_t* rows, int64_t n, const Hyper& hp,
                      int32_t t, hipStream_t s);
// --- sharded runner (dist.hip; layouts in dist.hip's header comment) ---
struct PushArgs {  // one IPC exchange: per peer, source block, destination, flag to raise
  const void* src[kMaxWorld];
  void* dst[kMaxWorld];
  int32_t* flag[kMaxWorld];
};
// mark: the launch's completion board (device_common.h board_mark / board_finish), >= kBoardMax
// words, zero before first use
hipError_t ipc_push(const PushArgs& a, int world, int64_t bytes, const int32_t* tbase, int k,
                    int32_t seq, int32_t* mark, int32_t* err, hipStream_t s);
hipError_t ipc_wait(const int32_t* flags, int world, int self, const int32_t* tbase, int k,
                    int32_t seq, int32_t* err, hipStream_t s);
hipError_t ipc_recv(const PushArgs& a, int world, int self, int64_t bytes, const int32_t* flags,
                    const int32_t* tbase, int k, int32_t seq, int32_t* err, hipStream_t s);
hipError_t max_vals(const int32_t* vals, int world, int32_t* out, hipStream_t s);
hipError_t dist_own_max(BatchBuf bb, int64_t n, int world, int32_t* cap, hipStream_t s);
hipError_t dist_pack_ids(BatchBuf bb, int64_t n, int world, int cap, int32_t* ids_send,
                         hipStream_t s);
hipError_t dist_owner_plan(const int32_t* ids_recv, int64_t n, int world, int cap, int lag, int32_t* aplan,
                           int32_t* gdep, int32_t* gfree, hipStream_t s);
// ---- the fused sharded step over the IPC transport (step.hip; two launches per step) ----
// K2 whose per-slot gradients go straight to the owners: slot s of owner p = s / S lands at
// dst[p] + (s % S) * ld; once every workgroup's stores are acknowledged the launch's last
// workgroup (a finisher polling the others' completion marks) raises flag[p] (non-null) to the
// step number
struct GradRoute {
  float* dst[kMaxWorld];
  int32_t* flag[kMaxWorld];
  int S = 0, world = 1;
  int32_t* mark = nullptr;  // completion board, >= kBoardMax words
  int32_t* err = nullptr;
};
hipError_t item_step_push(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                          const int32_t* tbase, int step, float* contrib, float* ugrad, float* xloss,
                          double* loss, const GradRoute& gr, hipStream_t s);
// the owner phase's arguments (dist.hip k_owner_gather / k_owner_step)
struct OwnerArgs {
  const int32_t* ids_recv = nullptr;
  const int32_t* aplan = nullptr;
  const int32_t* gdep = nullptr;
  const int32_t* gfree = nullptr;
  int64_t n = 0;
  int world = 1, cap = 0, self = 0;
  int max_blocks = kBoardMax;  // owner workgroups at most (grid-stride beyond)
  const float* grads_recv = nullptr;
  const float* self_grads = nullptr;
  const int32_t* wait_flags = nullptr;
  PushArgs dst;
  int32_t* mark = nullptr;  // completion board of the owner workgroups, >= kBoardMax words
  // stale-1 (lag 2): front k applies step k-1 and gathers step k+1 (rows of the table after step
  // k-1); the chunk's first front gathers steps 0 (dst) and 1 (dst1, the other parity)
  int lag = 1;
  PushArgs dst1;
};
// owner phase of step `step` of the chunk (0: gather step 0; else apply step-1 and gather step,
// or step+1 for lag 2) in the first workgroups, K1 of `step` (sharded, waiting for every rank's
// row flags) in the rest
hipError_t dist_front(const Geom& g, const OwnerArgs& o, BatchView bv, int B, Table P, Table Q,
                      const Hyper& hp, const int32_t* tbase, int step, float* contrib, float* ugrad,
                      float* xloss, const float* item_rows, const PeerWait& pw, hipStream_t s);
// apply step k and gather step k+1 in one launch (dist.hip k_owner_step)
hipError_t dist_owner_step(const Geom& g, Table Q, const int32_t* ids_recv, const int32_t* aplan,
                           const int32_t* gdep, const int32_t* gfree, int64_t n, int world, int cap,
                           int k, const Hyper& hp, const int32_t* tbase, const float* grads_recv,
                           int self, const float* self_grads, const int32_t* wait_flags,
                           int32_t* err, const PushArgs& dst, int32_t* mark, int max_blocks,
                           hipStream_t s);
// row of position (p, idx) -> dst.dst[p] + idx * ld; mark != null (IPC): a finisher workgroup
// raises dst.flag[p] to the step number once every other workgroup's stores are acknowledged
hipError_t dist_owner_gather(const Geom& g, Table Q, const int32_t* ids_recv, int64_t n, int world,
                             int cap, int k, const Hyper& hp, const int32_t* tbase,
                             const PushArgs& dst, int32_t* mark, int32_t* err, int max_blocks,
                             hipStream_t s);
// wait_flags != null (IPC): every workgroup first waits for the peers' gradient flags
hipError_t dist_owner_apply(const Geom& g, Table Q, const int32_t* ids_recv, const int32_t* aplan,
                            int64_t n, int world, int cap, int k, const Hyper& hp,
                            const int32_t* tbase, const float* grads_recv, int self,
                            const float* self_grads, const int32_t* wait_flags, int32_t* err,
                            hipStream_t s);

}  // namespace bprmf
