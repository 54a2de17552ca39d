// step.hip — the two per-step kernels of the segmented (atomic-free, deterministic) BPR-MF step,
// over the batch layout built by k_build_batches (segment.hip).
//
//   k_user_step (K1) one lane group per triplet: gather P_u, Q_i, Q_j with their pending weight
//     decay, x = <P_u,Q_i> - <P_u,Q_j>, c = sigmoid(-x) = -dL/dx; c*P_u is stored for K2.  A
//     user with one triplet in the batch is updated right there, W = V - lr (g + wd V) with
//     g = -c (Q_i - Q_j) (no other read of P_u in the step); otherwise g goes to ugrad[p].
//   k_item_step (K2) one lane group per distinct item; items with more than kLongSeg references
//     get a whole workgroup and an LDS reduction in group order.  g = sum of -/+ c*P_u over the
//     item's references in a fixed order, then the same SGD + weight decay update.  The users with
//     several triplets are finished here too: g = their ugrad rows summed in position order.
// Every triplet is one group in K1 whatever its user's multiplicity, so no group walks a chain of
// dependent row loads (heavy users were K1's tail when a group owned a whole user segment).
// Reference semantics: BPRMFRecommender.py:172-176 (forward :42-50, loss :174, SGD(wd) :154).
//
// Row layout: G4 lanes per row, each lane one float4 per stripe (16 B/lane, whole 64..1024 B rows
// per wave instruction); 64/G4 rows per wave.  Nothing here is an atomic: every output row has
// exactly one writer, so the result does not depend on scheduling.
#include <stdlib.h>

#include <algorithm>

#include "device_common.h"
#include "dist_body.h"

BPRMF_CALL_STAMPS_DEF(step)

// The in-launch hand-off below uses gfx94x/gfx950 cache-policy bits (sc1 stores and loads) and
// the CDNA3/4 L2-per-XCD coherence model; no other target is built or supported.
#if defined(__HIP_DEVICE_COMPILE__) && !(defined(__gfx950__) || defined(__gfx942__))
#error "step.hip targets gfx950 (gfx942 also has the sc1 policy bits); build with --offload-arch=gfx950"
#endif

namespace bprmf {

// diagnostic build only (-DBPRMF_STEP_STAMPS, tools/ubench_step_stamps.py): per workgroup,
// s_memrealtime at entry, after its record load, after its row loads / sums, and after its stores
// drained (thread 0; the waits serialise that thread, so the stamps bound each phase from above).
#ifdef BPRMF_STEP_STAMPS
__device__ uint64_t g_step_stamps[2][8192][6];
#ifdef BPRMF_FUSED_STAMPS_ONLY  // only the fused launches stamp (the chunk's last K2 would overwrite)
constexpr bool kFusedStampsOnly = true;
#else
constexpr bool kFusedStampsOnly = false;
#endif
#define SSTAMP(kern, k)                                                           \
  do {                                                                            \
    if (kStampHere && threadIdx.x == 0) {                                         \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                            \
      g_step_stamps[kern][blk][k] = __builtin_amdgcn_s_memrealtime();             \
    }                                                                             \
  } while (0)
#define SROLE(kern, r)                                                            \
  do {                                                                            \
    if (kStampHere && threadIdx.x == 0) g_step_stamps[kern][blk][5] = (r);        \
  } while (0)
extern "C" int bprmf_debug_step_stamps(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_stamps), sizeof(g_step_stamps)) == hipSuccess ? 0 : -3;
}
#else
#define SSTAMP(kern, k) \
  do {                  \
  } while (0)
#define SROLE(kern, r) \
  do {                 \
  } while (0)
#endif

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// A row the NEXT kernel reads (or the next step's kernels), stored write-through (sc1): the line
// leaves the XCD's L2 as it is written instead of staying dirty there, so the kernel boundary has
// no L2 write-back of it to wait for (MI355X_MICROARCH.md: boundary + B / 6 TB/s of dirty bytes).
// Plain vector store form, one per lane (no scalar-cache store).
template <bool WT>
static __device__ __forceinline__ void st4o(float* p, float4 v) {
  if constexpr (WT) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = {v.x, v.y, v.z, v.w};
    // s_nop: the wait states the compiler inserts after its own >8-byte vector stores before a
    // VALU may overwrite their data registers (it cannot see inside the asm to do so)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
// a 4-byte word the next kernel reads: write-through (sc1) like st4o, so it leaves no dirty line
template <bool WT>
static __device__ __forceinline__ void st_word(int32_t* p, int32_t v) {
  if constexpr (WT)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
static __device__ __forceinline__ float4 scale4(float4 a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}
static __device__ __forceinline__ float dot4(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}
// a + s*b, per component, fused
static __device__ __forceinline__ float4 fma4(float s, float4 b, float4 a) {
  return make_float4(fmaf(s, b.x, a.x), fmaf(s, b.y, a.y), fmaf(s, b.z, a.z), fmaf(s, b.w, a.w));
}
static __device__ __forceinline__ float4 sub4(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
// W <- V - lr (g + wd V): torch SGD  d_p = grad.add(param, alpha=wd); param.add_(d_p, alpha=-lr)
static __device__ __forceinline__ float4 sgd4(float4 v, float4 g, float lr, float wd) {
  return make_float4(fmaf(-lr, fmaf(wd, v.x, g.x), v.x), fmaf(-lr, fmaf(wd, v.y, g.y), v.y),
                     fmaf(-lr, fmaf(wd, v.z, g.z), v.z), fmaf(-lr, fmaf(wd, v.w, g.w), v.w));
}

// One row segment (16 B per lane) read with sc1 loads: past this CU's L1, so a row another XCD
// just wrote is seen once its stamp is (the fused step's hand-off, MI355X_MICROARCH.md "Valid
// forms": sc1 payload stores + vmcnt(0) + sc1 flag store; sc1 poll + sc1 payload loads).
static __device__ __forceinline__ float4 ld4_sc1(const float* p) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)),
                     __uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}

// Wait (sc1 polls) until a row's stamp reaches step tp, i.e. its owner in the same launch has
// stored the row and then the stamp.  Bounded: after ~10 s err bit 8 is raised and the wait gives
// up (the call then fails) instead of hanging the queue.
static __device__ __forceinline__ void wait_stamp(const int32_t* stamp, int32_t tp, int32_t* err) {
  if (__hip_atomic_load(stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tp) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t polls = 0;
    while (__hip_atomic_load(stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tp) {
      __builtin_amdgcn_s_sleep(1);
      if ((++polls & 255) == 0) {  // a wait that already timed out elsewhere ends this one too
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 100 MHz: 10 s
          atomicOr(err, 8);
          break;
        }
      }
    }
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the row loads stay after the poll
}

// Publish a row's step stamp after the row: every lane's (write-through) row stores acknowledged,
// then an sc1 stamp store.  A lane group lies within one wave (G4 <= 64), so the wave's own wait
// covers the whole row.
template <bool PUB>
static __device__ __forceinline__ void put_stamp(int32_t* stamp, int32_t t, bool writer) {
  if constexpr (PUB) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (writer) __hip_atomic_store(stamp, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (writer) *stamp = t;
  }
}

// this batch's build timed out (kernels.h kMetaDead): the step leaves the tables alone
static __device__ __forceinline__ bool build_failed(const BatchView& bv) {
  return bv.meta[kMetaDead] == kDeadMark;
}

// K1 of step t, one lane group per triplet p (sorted by user).  SH (sharded): i/j are slots of
// item_rows, the rows the owners sent for this step, already brought to step t-1 by the owner (no
// stamps).  WAIT (fused step, k_fused_step): this K1 runs beside K2 of step t-1, so a row that
// step t-1 updates (pend[(t-1)&1][row] == t-1, written by K1 of step t-1 in the previous launch)
// is read only after its owner publishes stamp t-1.  pend (single GPU): every triplet marks its
// rows with t (users: only those K2 finishes), for K1 of step t+1.  pw (sharded, fused front
// launch): the record and the user row are loaded first, then the workgroup waits for the row
// flags, then the item rows are read.
template <int G4, int S, bool SH, bool WT, bool WAIT>
static __device__ __forceinline__ void k1_body(int blk, BatchView bv, const Table& P, const Table& Q,
                                               const Hyper& hp, int ld, int32_t t,
                                               const StepBufs& sb, const float* __restrict__ item_rows,
                                               int B, int32_t* err, const PeerWait* pw = nullptr) {
#ifdef BPRMF_STEP_STAMPS
  constexpr bool kStampHere = WAIT || !kFusedStampsOnly;
#endif
  SSTAMP(0, 0);
  const int sub = threadIdx.x & (G4 - 1);
  const int p = blk * (kBlock / G4) + threadIdx.x / G4;
  // independent loads: the record and the triplet count.  The grid covers B rounded up to whole
  // blocks: the index is clamped into the batch's B records (never read past them)
  const int4 r = reinterpret_cast<const int4*>(bv.trec)[min(p, B - 1)];
  const int n = bv.meta[0];
  const bool dead = build_failed(bv);  // the batch build failed
  const int64_t par = sb.pstride ? (int64_t)(t & 1) : 0;  // this step's half of the buffers
  float* contrib = sb.contrib + par * sb.pstride;
  float* ugrad = sb.ugrad + par * sb.pstride;
  float* xloss = sb.xloss ? sb.xloss + par * B : nullptr;
  SSTAMP(0, 1);
  // kept past the workgroup barrier for an in-workgroup segment head (w >= 2)
  float4 pu[S];
  float* prow = nullptr;
  int w = 0;
  int32_t u = 0;
  __shared__ float4 s_g[S * kBlock];  // per-triplet user gradients of in-workgroup segments
  if (pw) {  // the user row (this rank's, final since the previous launch) while the owners work
    if (p < n) {
      const float* pr = P.W + (int64_t)r.z * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) pu[k] = ld4(pr + 4 * G4 * k);
    }
    wait_peer_flags(pw->flags, pw->world, pw->self, t, pw->err);
  }
  if (p < n && !dead) {
    // bit 31: the item's first reference in the batch; bit 30 (single GPU): its ONLY reference,
    // so this triplet finishes the item (no contribution row, no K2 record)
    const int32_t i = r.x & 0x3FFFFFFF, j = r.y & 0x3FFFFFFF;
    const bool soli = !SH && (r.x & 0x40000000), solj = !SH && (r.y & 0x40000000);
    u = r.z;
    w = r.w;
    prow = P.W + (int64_t)u * ld + 4 * sub;
    if (sb.pend_q && sub == 0) {  // this step's rows, for the next step's fused K1
      // one mark per distinct item K2 updates (from the triplet holding its first reference) and
      // per user K2 finishes; write-through (sc1), so no dirty partial lines wait for the kernel
      // boundary.  Rows K1 finishes itself are final before the next launch: no mark.
      const int64_t o = (int64_t)(t & 1);
      if (r.x < 0 && !soli)
        __hip_atomic_store(sb.pend_q + o * sb.qrows + i, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r.y < 0 && !solj)
        __hip_atomic_store(sb.pend_q + o * sb.qrows + j, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0)
        __hip_atomic_store(sb.pend_p + o * sb.prows + u, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bool wi = false, wj = false, wu = false;
    const int32_t tp = t - 1;
    int32_t si = 0, sj = 0, su0 = 0;  // WAIT: the three stamps, loaded beside the marks
    const float* qbase = SH ? item_rows : Q.W;
    const float* qi = qbase + (int64_t)i * ld + 4 * sub;
    const float* qj = qbase + (int64_t)j * ld + 4 * sub;
    float4 vi[S], vj[S];
    if (WAIT) {
      // the user row too, speculatively in the same round (a user step t-1 does not update is
      // final here; a marked one is read again, sc1, once its stamp says it is published).  The
      // item rows wait for their marks: most triplets hold a marked item, whose speculative read
      // was wasted bytes in the launch's opening burst, and the triplets with unmarked items are
      // not the launch's tail (round 5 A/B: fused launch 9.45 -> 9.37 us by rocprofv3, 9.37-9.47
      // -> 9.21-9.24 us by events, profiles/r05_ab_k1_late_items.txt)
#pragma unroll
      for (int k = 0; k < S; ++k) pu[k] = ld4(prow + 4 * G4 * k);
      // marks and stamps in ONE round of loads (sc1 stamps: the first poll of a marked row); a
      // marked row whose stamp is not yet tp is then polled alone, so a triplet with two or three
      // rows already published pays one load latency here instead of one per row
      const int64_t o = (int64_t)(tp & 1);
      const int32_t mi = *(sb.pend_q + o * sb.qrows + i), mj = *(sb.pend_q + o * sb.qrows + j);
      const int32_t mu = *(sb.pend_p + o * sb.prows + u);
      si = __hip_atomic_load(Q.stamp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sj = __hip_atomic_load(Q.stamp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      su0 = __hip_atomic_load(P.stamp + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wi = mi == tp;
      wj = mj == tp;
      wu = mu == tp;
      if (wi && si != tp) wait_stamp(Q.stamp + i, tp, err);
      if (wj && sj != tp) wait_stamp(Q.stamp + j, tp, err);
      if (wu && su0 != tp) wait_stamp(P.stamp + u, tp, err);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the row loads stay after the stamp reads
    }
    SSTAMP(0, 4);
    if (WAIT) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        if (wu) pu[k] = ld4_sc1(prow + 4 * G4 * k);
        vi[k] = wi ? ld4_sc1(qi + 4 * G4 * k) : ld4(qi + 4 * G4 * k);
        vj[k] = wj ? ld4_sc1(qj + 4 * G4 * k) : ld4(qj + 4 * G4 * k);
      }
    } else {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        if (!pw) pu[k] = ld4(prow + 4 * G4 * k);
        vi[k] = ld4(qi + 4 * G4 * k);
        vj[k] = ld4(qj + 4 * G4 * k);
      }
    }
    // a row just published is current at tp (no pending decay); the others read their stamps
    // (WAIT: an unmarked row's stamp, read above, is stable in this launch)
    const int32_t su = wu ? tp : (WAIT ? su0 : P.stamp[u]);
    const float fi = SH ? 1.f : decay_pow(hp.log2a, t - 1 - (wi ? tp : (WAIT ? si : Q.stamp[i])));
    const float fj = SH ? 1.f : decay_pow(hp.log2a, t - 1 - (wj ? tp : (WAIT ? sj : Q.stamp[j])));
    const float fu = decay_pow(hp.log2a, t - 1 - su);
    float di = 0.f, dj = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      pu[k] = scale4(pu[k], fu);
      vi[k] = scale4(vi[k], fi);
      vj[k] = scale4(vj[k], fj);
      di = dot4(pu[k], vi[k], di);
      dj = dot4(pu[k], vj[k], dj);
    }
    di = group_sum<G4>(di);
    dj = group_sum<G4>(dj);
    const float x = di - dj;
    SSTAMP(0, 2);
    const float c = 1.0f / (1.0f + expf(x));  // sigmoid(-x) = -dL/dx
    if (sub == 0 && xloss) st_word<WT>(reinterpret_cast<int32_t*>(xloss) + p, __float_as_int(x));  // K2 sums the loss terms
    if (!(soli && solj)) {  // K2 reads c*P_u for the side(s) it serves
      float* cb = contrib + (int64_t)p * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) st4o<WT>(cb + 4 * G4 * k, scale4(pu[k], c));
    }
    // an item with this one reference: W = V - lr (g + wd V), g = -c P_u (i) / +c P_u (j), the
    // exact arithmetic of K2's one-term sum (fmaf(-/+1, c P_u, 0) is -/+ c P_u exactly)
    if (soli) {
      float* qw = Q.W + (int64_t)i * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) st4o<WT>(qw + 4 * G4 * k, sgd4(vi[k], scale4(scale4(pu[k], c), -1.f), hp.lr, hp.wd));
      if (sub == 0) st_word<WT>(Q.stamp + i, t);
    }
    if (solj) {
      float* qw = Q.W + (int64_t)j * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) st4o<WT>(qw + 4 * G4 * k, sgd4(vj[k], scale4(pu[k], c), hp.lr, hp.wd));
      if (sub == 0) st_word<WT>(Q.stamp + j, t);
    }
    if (w == 1) {  // the user's only triplet: W = V - lr (g + wd V) with g = -c (Q_i - Q_j)
#pragma unroll
      for (int k = 0; k < S; ++k)
        st4o<WT>(prow + 4 * G4 * k, sgd4(pu[k], scale4(sub4(vi[k], vj[k]), -c), hp.lr, hp.wd));
      if (sub == 0) st_word<WT>(P.stamp + u, t);
    } else if (w == 0) {  // a segment across workgroups: K2 sums its gradients in position order
      float* ub = ugrad + (int64_t)p * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) st4o<WT>(ub + 4 * G4 * k, scale4(sub4(vi[k], vj[k]), -c));
    } else {  // a segment inside this workgroup: its head finishes it below
#pragma unroll
      for (int k = 0; k < S; ++k) s_g[k * kBlock + threadIdx.x] = scale4(sub4(vi[k], vj[k]), -c);
    }
  }
  // The head of an in-workgroup segment adds its members' gradients in position order (K2's
  // order and arithmetic for the same segment) and applies SGD + decay: most users with several
  // triplets in a batch never wait for K2.
  __syncthreads();
  if (w >= 2) {
    const int q0 = threadIdx.x - sub;  // = (this triplet's slot in the workgroup) * G4
#pragma unroll
    for (int k = 0; k < S; ++k) {
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int m = 0; m < w; ++m) {
        const float4 x = s_g[k * kBlock + q0 + m * G4 + sub];
        g = make_float4(g.x + x.x, g.y + x.y, g.z + x.z, g.w + x.w);
      }
      st4o<WT>(prow + 4 * G4 * k, sgd4(pu[k], g, hp.lr, hp.wd));
    }
    if (sub == 0) st_word<WT>(P.stamp + u, t);
  }
  SSTAMP(0, 3);
}

template <int G4, int S, bool SH, bool WT>
__global__ __launch_bounds__(kBlock) void k_user_step(BatchView bv, Table P, Table Q, Hyper hp,
                                                      int ld, const int32_t* __restrict__ tbase,
                                                      int step, StepBufs sb,
                                                      const float* __restrict__ item_rows,
                                                      PeerWait pw, int64_t bstride, int B) {
  CsScope cs_(2);  // diagnostic builds only (BPRMF_CALL_STAMPS)
  if (bstride) bv = bv.shifted((int64_t)(tbase[1] + step) * bstride);
  if (SH) wait_peer_flags(pw.flags, pw.world, pw.self, *tbase + step + 1, pw.err);
  k1_body<G4, S, SH, WT, false>(blockIdx.x, bv, P, Q, hp, ld, *tbase + step + 1, sb, item_rows, B,
                                nullptr);
}

// an item row and its stamp, loaded as soon as the segment's record is known so the loads run
// alongside the contribution gathers instead of after them (single GPU only; sharded K2 emits the
// gradient and reads no item row)
template <int G4, int S, bool SH>
struct ItemRow {
  float4 x[S];
  int32_t stamp = 0;
  __device__ __forceinline__ void load(const Table& Q, int32_t item, int ld, int sub) {
    if (SH) return;
    const float* w = Q.W + (int64_t)item * ld + 4 * sub;
#pragma unroll
    for (int k = 0; k < S; ++k) x[k] = ld4(w + 4 * G4 * k);
    stamp = *(Q.stamp + item);
  }
};

template <int G4, int S>
static __device__ __forceinline__ void load_ref(float4 (&row)[S], const float* __restrict__ contrib,
                                                int32_t ref, int ld, int sub) {
  const float* cb = contrib + (int64_t)(ref >> 1) * ld + 4 * sub;
#pragma unroll
  for (int k = 0; k < S; ++k) row[k] = ld4(cb + 4 * G4 * k);
}

template <int S>
static __device__ __forceinline__ void acc_ref(float4 (&g)[S], const float4 (&row)[S], int32_t ref) {
  const float sgn = (ref & 1) ? 1.f : -1.f;  // j: +c P_u, i: -c P_u
#pragma unroll
  for (int k = 0; k < S; ++k) g[k] = fma4(sgn, row[k], g[k]);
}

// finish one item segment: apply W = V - lr (g + wd V) to the preloaded row (single GPU) or hand
// the gradient to the exchange (sharded)
template <int G4, int S, bool SH, bool WT, bool PUB>
static __device__ __forceinline__ void finish_item(Table Q, int32_t item, int slot,
                                                   const float4 (&g)[S], const ItemRow<G4, S, SH>& row,
                                                   const Hyper& hp, int ld, int32_t t, int sub,
                                                   float* __restrict__ grads,
                                                   const GradRoute* gr = nullptr) {
  if (SH) {
    // per-slot gradient: the exchange's send buffer, or (gr: fused IPC step) straight into its
    // owner's landing buffer
    float* o;
    if (gr) {
      const int p = slot / gr->S;
      o = gr->dst[p] + (int64_t)(slot - p * gr->S) * ld + 4 * sub;
    } else {
      o = grads + (int64_t)slot * ld + 4 * sub;
    }
#pragma unroll
    for (int k = 0; k < S; ++k) st4o<WT>(o + 4 * G4 * k, g[k]);
  } else {
    float* w = Q.W + (int64_t)item * ld + 4 * sub;
    const float f = decay_pow(hp.log2a, t - 1 - row.stamp);
#pragma unroll
    for (int k = 0; k < S; ++k) st4o<WT>(w + 4 * G4 * k, sgd4(scale4(row.x[k], f), g[k], hp.lr, hp.wd));
    put_stamp<PUB>(Q.stamp + item, t, sub == 0);
  }
}

// sum of the rows src[beg..end) in order (lanes fetch G4 indices at once, 8 rows in flight)
template <int G4, int S>
static __device__ __forceinline__ void sum_rows(float4 (&g)[S], const float* __restrict__ src,
                                                int beg, int end, int ld, int sub) {
#pragma unroll
  for (int k = 0; k < S; ++k) g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int m0 = beg; m0 < end; m0 += 8) {
    float4 rows[8][S];
#pragma unroll
    for (int m = 0; m < 8; ++m)
      if (m0 + m < end) {
        const float* rp = src + (int64_t)(m0 + m) * ld + 4 * sub;
#pragma unroll
        for (int k = 0; k < S; ++k) rows[m][k] = ld4(rp + 4 * G4 * k);
      }
#pragma unroll
    for (int m = 0; m < 8; ++m)
      if (m0 + m < end) {
#pragma unroll
        for (int k = 0; k < S; ++k)
          g[k] = make_float4(g[k].x + rows[m][k].x, g[k].y + rows[m][k].y, g[k].z + rows[m][k].z,
                             g[k].w + rows[m][k].w);
      }
  }
}

// item segments one K2 lane group serves at most (k2_grid sizes the item grid for it): 6 at one
// stripe (d <= 256); wider rows keep one per lane group (the rounds cost their registers 2-3 more
// VGPRs there, and one wave per SIMD fewer at d = 512)
template <int S>
constexpr int item_rounds() { return S == 1 ? 6 : 1; }
// one K2 item segment (record r0/r1): the sum of -/+ c P_u over its references in order, then the
// update (single GPU) or the per-slot gradient (sharded)
template <int G4, int S, bool SH, bool WT, bool PUB>
static __device__ __forceinline__ void k2_item_segment(int4 r0, int4 r1, const BatchView& bv,
                                                       const Table& Q, const Hyper& hp, int ld,
                                                       int32_t t, int sub,
                                                       const float* __restrict__ contrib,
                                                       float* __restrict__ grads, const GradRoute* gr,
                                                       int blk) {
#ifdef BPRMF_STEP_STAMPS
  constexpr bool kStampHere = PUB || !kFusedStampsOnly;
#endif
  (void)blk;
  // record {item, beg | len << 15 | long << 30, refs 0..11 as 16-bit halves} (segment.hip)
  if (r0.y >> 30) return;  // a workgroup-served hot item
  const int32_t item = r0.x;
  const int beg = r0.y & 0x7FFF, len = (r0.y >> 15) & 0x7FFF, end = beg + len;
#ifdef BPRMF_STEP_STAMPS
  if (kStampHere && threadIdx.x == 0) g_step_stamps[1][blk][4] = (uint64_t)len;
#endif
  ItemRow<G4, S, SH> row;
  row.load(Q, item, ld, sub);
  float4 g[S];
#pragma unroll
  for (int k = 0; k < S; ++k) g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (len <= kInlineRefs) {  // the common case: every ref inline, all rows requested at once
    const int32_t pk[6] = {r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    float4 rows[kInlineRefs][S];
    int32_t rf[kInlineRefs];
#pragma unroll
    for (int m = 0; m < kInlineRefs; ++m) {
      rf[m] = (pk[m >> 1] >> (16 * (m & 1))) & 0xFFFF;
      if (m < len) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
    }
#pragma unroll
    for (int m = 0; m < kInlineRefs; ++m)
      if (m < len) acc_ref<S>(g, rows[m], rf[m]);
  } else {  // lanes fetch G4 refs at once; rows requested F at a time before accumulating
    // (F = 16 at S = 1, as on the hot-item path: a 13..16-reference item, the slowest K2 lane
    // groups, then needs one round of row loads instead of two; the order of the sum is the same)
    constexpr int F = S == 1 ? 16 : 8;
    const int lane0 = (threadIdx.x & 63) - sub;
    for (int base = beg; base < end; base += G4) {
      const int32_t myref = base + sub < end ? bv.refs[base + sub] : 0;
      const int cnt = min(G4, end - base);
      for (int m0 = 0; m0 < cnt; m0 += F) {
        float4 rows[F][S];
        int32_t rf[F];
#pragma unroll
        for (int m = 0; m < F; ++m) {
          rf[m] = __shfl(myref, lane0 + ((m0 + m) & (G4 - 1)));
          if (m0 + m < cnt) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
        }
#pragma unroll
        for (int m = 0; m < F; ++m)
          if (m0 + m < cnt) acc_ref<S>(g, rows[m], rf[m]);
      }
    }
  }
  SSTAMP(1, 2);
  finish_item<G4, S, SH, WT, PUB>(Q, item, item, g, row, hp, ld, t, sub, grads, gr);  // SH: item field = slot
  SSTAMP(1, 3);
}
// K2 of step t, workgroup `blk` of its grid: loss workgroups, hot items (whole workgroups), item
// segments (one lane group each), user segments spanning K1 workgroups.  PUB (fused step): every
// updated row's stamp is published after the row (put_stamp), for K1 of step t+1 in the same
// launch.
template <int G4, int S, bool SH, int KB, bool WT, bool PUB>
static __device__ __forceinline__ void k2_body(int blk, BatchView bv, const Table& P, const Table& Q,
                                               const Hyper& hp, int ld, int32_t t,
                                               const StepBufs& sb, int long_blocks, int item_blocks,
                                               float* __restrict__ grads, double* __restrict__ loss,
                                               int B, const GradRoute* gr = nullptr) {
  constexpr int NG = KB / G4;
#ifdef BPRMF_STEP_STAMPS
  constexpr bool kStampHere = PUB || !kFusedStampsOnly;
#endif
  SSTAMP(1, 0);
  const int sub = threadIdx.x & (G4 - 1);
  const int grp = threadIdx.x / G4;
  const int64_t par = sb.pstride ? (int64_t)(t & 1) : 0;  // the half K1 of step t wrote
  const float* __restrict__ contrib = sb.contrib + par * sb.pstride;
  const float* __restrict__ ugrad = sb.ugrad + par * sb.pstride;
  const float* __restrict__ xloss = sb.xloss ? sb.xloss + par * B : nullptr;
  if (!xloss) loss = nullptr;
  const bool dead = build_failed(bv);  // the batch build failed
  // the step's loss: the first loss_blocks(B, KB) workgroups (dispatched first, off the tail) each
  // sum log(1 + e^-x) over KB triplets, one per thread, in a fixed tree, and add it to their own
  // slot loss[b] (one writer per slot per launch; the host adds the slots once per call)
  const int lb = loss ? (B + KB - 1) / KB : 0;
  if (blk < lb) {
    if (dead) return;
    __shared__ double red[KB / 64];
    const int n = bv.meta[0];
    const int p = blk * KB + threadIdx.x;
    double acc =
        p < n ? (double)softplus(-__int_as_float(*(reinterpret_cast<const int32_t*>(xloss) + p))) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);  // fixed butterfly
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double tot = 0.0;
      for (int w = 0; w < KB / 64; ++w) tot += red[w];
      loss[blk] += tot;
    }
    return;
  }
  const int bid = blk - lb;
  if (bid >= long_blocks + item_blocks) {  // users with several triplets
    const int m = (bid - long_blocks - item_blocks) * NG + grp;
    // indices clamped into the batch's record arrays (B/2 user records, 2B item records): the
    // groups past the count read a valid record and return
    const int4 r0 = reinterpret_cast<const int4*>(bv.mrec + (int64_t)min(m, max(B / 2 - 1, 0)) * kRec)[0];
    const int n_multi = bv.meta[4];
    SSTAMP(1, 1);
    SROLE(1, 3);
    if (m >= n_multi || dead) return;
    const int32_t u = r0.x;
    float* pw = P.W + (int64_t)u * ld + 4 * sub;
    float4 cur[S], g[S];
#pragma unroll
    for (int k = 0; k < S; ++k) cur[k] = ld4(pw + 4 * G4 * k);
    const int32_t su = *(P.stamp + u);
    sum_rows<G4, S>(g, ugrad, r0.y, r0.z, ld, sub);
    SSTAMP(1, 2);
    const float f = decay_pow(hp.log2a, t - 1 - su);
#pragma unroll
    for (int k = 0; k < S; ++k) st4o<WT>(pw + 4 * G4 * k, sgd4(scale4(cur[k], f), g[k], hp.lr, hp.wd));
    put_stamp<PUB>(P.stamp + u, t, sub == 0);
    SSTAMP(1, 3);
    return;
  }
  if (bid < long_blocks) {
    __shared__ float4 part[NG][G4 * S];
    const int4 r0 = reinterpret_cast<const int4*>(bv.lrec + (int64_t)bid * kRec)[0];
    const int n_long = bv.meta[3];
    SSTAMP(1, 1);
    SROLE(1, 1);
    if (bid >= n_long || dead) return;  // uniform over the block
    const int32_t item = r0.x;
    const int beg = r0.y, end = r0.z;
    ItemRow<G4, S, SH> row;
    if (grp == 0) row.load(Q, item, ld, sub);
    float4 g[S];
#pragma unroll
    for (int k = 0; k < S; ++k) g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    // group q owns refs beg + q + NG*m.  Its lanes fetch G4 of those refs at once; every row of a
    // chunk of 8 is requested before any is accumulated (accumulation order fixed: m ascending).
    const int lane0 = (threadIdx.x & 63) - sub;
    for (int base = beg + grp; base < end; base += NG * G4) {
      const int ridx = base + NG * sub;
      const int32_t myref = ridx < end ? bv.refs[ridx] : 0;
      const int cnt = min(G4, (end - base + NG - 1) / NG);
      constexpr int F = S == 1 ? 16 : 8;  // rows in flight per group (a hot item has ~80 refs)
      for (int m0 = 0; m0 < cnt; m0 += F) {
        float4 rows[F][S];
        int32_t rf[F];
#pragma unroll
        for (int m = 0; m < F; ++m) {
          rf[m] = __shfl(myref, lane0 + ((m0 + m) & (G4 - 1)));
          if (m0 + m < cnt) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
        }
#pragma unroll
        for (int m = 0; m < F; ++m)
          if (m0 + m < cnt) acc_ref<S>(g, rows[m], rf[m]);
      }
    }
    // fixed-shape tree over the groups' partial sums (deterministic order)
#pragma unroll
    for (int k = 0; k < S; ++k) part[grp][sub + G4 * k] = g[k];
    __syncthreads();
#pragma unroll
    for (int half = NG / 2; half >= 1; half >>= 1) {
      if (grp < half) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const float4 a = part[grp][sub + G4 * k], o = part[grp + half][sub + G4 * k];
          part[grp][sub + G4 * k] = make_float4(a.x + o.x, a.y + o.y, a.z + o.z, a.w + o.w);
        }
      }
      __syncthreads();
    }
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < S; ++k) g[k] = part[0][sub + G4 * k];
      SSTAMP(1, 2);
      finish_item<G4, S, SH, WT, PUB>(Q, item, r0.w, g, row, hp, ld, t, sub, grads, gr);
    }
    SSTAMP(1, 3);
    return;
  }
  // item segments: lane group g of the item workgroups takes segments g, g + G, g + 2G, ... (G =
  // item_blocks * NG lane groups).  The single-GPU step caps item_blocks (k2_grid): ~1,000 of a
  // batch's ~5,700 items reach K2 there, and a grid sized for the 2B possible segments held
  // ~900 workgroups that only loaded a record and left, dispatched ahead of K1 of the next step.
  // At most item_rounds<S>() segments per lane group (k2_grid keeps item_blocks * NG >= 2B /
  // rounds), in a fully unrolled sequence: a rolled loop here took 108 -> 162 VGPRs.
  const int s0 = (bid - long_blocks) * NG + grp;
  const int stride = item_blocks * NG;
  const int sc = min(s0, 2 * B - 1);
  int4 r0 = reinterpret_cast<const int4*>(bv.irec + (int64_t)sc * kRec)[0];
  int4 r1 = reinterpret_cast<const int4*>(bv.irec + (int64_t)sc * kRec)[1];
  const int n_iseg = bv.meta[2];
  SSTAMP(1, 1);
  SROLE(1, 2);
  if (dead) return;
#pragma unroll
  for (int round = 0; round < item_rounds<S>(); ++round) {
    const int s = s0 + round * stride;
    if (s >= n_iseg) break;  // past the batch's items
    if (round) {
      r0 = reinterpret_cast<const int4*>(bv.irec + (int64_t)s * kRec)[0];
      r1 = reinterpret_cast<const int4*>(bv.irec + (int64_t)s * kRec)[1];
    }
    k2_item_segment<G4, S, SH, WT, PUB>(r0, r1, bv, Q, hp, ld, t, sub, contrib, grads, gr, blk);
  }
}

template <int G4, int S, bool SH, int KB, bool WT>
__global__ __launch_bounds__(KB) void k_item_step(BatchView bv, Table P, Table Q, Hyper hp, int ld,
                                                  const int32_t* __restrict__ tbase, int step,
                                                  StepBufs sb, int long_blocks, int item_blocks,
                                                  float* __restrict__ grads, double* __restrict__ loss,
                                                  int64_t bstride, int B) {
  CsScope cs_(62);
  if (bstride) bv = bv.shifted((int64_t)(tbase[1] + step) * bstride);
  k2_body<G4, S, SH, KB, WT, false>(blockIdx.x, bv, P, Q, hp, ld, *tbase + step + 1, sb, long_blocks,
                                    item_blocks, grads, loss, B);
}

// The fused step: K2 of step t (batch c[1] + step) and K1 of step t + 1 (the next batch) in one
// launch.  K2's workgroups come first in the grid, so every one of them is dispatched before any
// K1 workgroup that may wait on it (bounded waits besides).  That relies on the command
// processor dispatching workgroups in blockIdx order, which CDNA hardware does (round-robin over
// the XCDs, ascending ids) but HIP does not promise: were it ever violated, a K1 wait would end
// after ~10 s with err bit 8 and the call would fail ("a row's owner never published it"), not
// hang.  A dynamic ticket (one same-address atomic per workgroup, ~1,700 per step at ~13 ns each
// when serialised) would cost more than the whole step.  K1 of step t+1 reads the rows step t
// does not touch at once and the others after their owners publish them; a chunk of n steps is
// then K1, n - 1 fused launches and K2: one kernel boundary per step instead of two.
template <int G4, int S, int KB>
__global__ __launch_bounds__(KB) void k_fused_step(BatchView bv0, Table P, Table Q, Hyper hp, int ld,
                                                   const int32_t* __restrict__ tbase, int step,
                                                   StepBufs sb, int long_blocks, int item_blocks,
                                                   int k2_blocks, double* __restrict__ loss,
                                                   int64_t bstride, int B, int32_t* err) {
  static_assert(KB == kBlock, "K1 and K2 workgroups share the launch's block size");
  CsScope cs_(3 + step);
  const int32_t t = tbase[0] + step + 1;
  const int64_t kb = (int64_t)tbase[1] + step;
  if ((int)blockIdx.x < k2_blocks)
    k2_body<G4, S, false, KB, true, true>(blockIdx.x, bv0.shifted(kb * bstride), P, Q, hp, ld, t, sb,
                                          long_blocks, item_blocks, nullptr, loss, B);
  else
    k1_body<G4, S, false, true, true>(blockIdx.x - k2_blocks, bv0.shifted((kb + 1) * bstride), P, Q,
                                      hp, ld, t + 1, sb, nullptr, B, err);
}

// ---- the fused sharded step over the IPC transport (dist.cpp enqueue_steps, two launches/step) ----
// Back: K2 of step t (sharded: per-slot gradients) written straight into the owners' landing
// buffers (GradRoute); each workgroup marks the completion board once its stores are acknowledged,
// and the grid's last workgroup (the finisher) raises each peer's gradient flag to t once every
// mark is in (the pattern of dist.hip k_ipc_push, with the push kernel gone).
template <int G4, int S, int KB>
__global__ __launch_bounds__(KB) void k_item_step_push(BatchView bv, Table P, Table Q, Hyper hp,
                                                       int ld, const int32_t* __restrict__ tbase,
                                                       int step, StepBufs sb, int long_blocks,
                                                       int item_blocks, double* __restrict__ loss,
                                                       int B, GradRoute gr) {
  const int32_t t = *tbase + step + 1;
  const int nprod = (int)gridDim.x - 1;
  if ((int)blockIdx.x == nprod) {
    board_finish(gr.mark, nprod, t, gr.flag, gr.world, gr.err);
    return;
  }
  k2_body<G4, S, true, KB, true, false>(blockIdx.x, bv, P, Q, hp, ld, t, sb, long_blocks,
                                        item_blocks, nullptr, loss, B, &gr);
  board_mark(gr.mark, blockIdx.x, t);
}

// Front: the owner phase of step t (k == 0 of a chunk: gather step 0's rows; else apply step k-1
// and gather step k, dist_body.h) in the first `ob` workgroups, K1 of step t in the others.  The
// owner workgroups come first in the grid (dispatched before any K1 workgroup that waits on them);
// every K1 workgroup waits for the row flags of EVERY rank, this one's own included (its own
// owner workgroups raise that flag once their stores into its landing slots are acknowledged).
template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_dist_front(OwnerArgs o, BatchView bv, Table P, Table Q,
                                                       Hyper hp, int ld, const int32_t* __restrict__ tbase,
                                                       int step, StepBufs sb,
                                                       const float* __restrict__ item_rows,
                                                       PeerWait pw, int ob, int B) {
  if ((int)blockIdx.x < ob) {
    if (step == 0) {
      owner_gather_body<G4, S>(blockIdx.x, ob, Q, o.ids_recv, o.n, o.world, o.cap, 0, hp, ld, tbase,
                               o.dst, o.mark);
      if (o.lag > 1 && o.n > 1)  // stale-1: step 1's rows from the same table, other parity
        owner_gather_body<G4, S>(blockIdx.x, ob, Q, o.ids_recv, o.n, o.world, o.cap, 1, hp, ld, tbase,
                                 o.dst1, o.mark);
    } else {
      owner_step_body<G4, S>(blockIdx.x, ob, Q, o.ids_recv, o.aplan, o.gdep, o.gfree, o.n, o.world,
                             o.cap, step - 1, hp, ld, tbase, o.grads_recv, o.self, o.self_grads,
                             o.wait_flags, pw.err, o.dst, o.mark, o.lag);
    }
    return;
  }
  if ((int)blockIdx.x == ob) {  // the owner workgroups' finisher: every rank's row flag for us
    // the last step whose rows this launch gathered (stale-1: one ahead; none at the chunk's end)
    const int rs = o.lag == 1 ? step : step == 0 ? (o.n > 1 ? 1 : 0) : step + 1;
    if (rs < o.n) board_finish(o.mark, ob, *tbase + rs + 1, o.dst.flag, o.world, pw.err);
    return;
  }
  const PeerWait all{pw.flags, pw.world, -1, pw.err};  // every rank's rows, this one's included
  k1_body<G4, S, true, true, false>(blockIdx.x - ob - 1, bv, P, Q, hp, ld, *tbase + step + 1, sb,
                                    item_rows, B, nullptr, &all);
}

static StepBufs plain_bufs(float* contrib, float* ugrad, float* xloss, const StepBufs* sb) {
  if (sb) return *sb;
  StepBufs b;
  b.contrib = contrib;
  b.ugrad = ugrad;
  b.xloss = xloss;
  return b;
}

hipError_t user_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, float* xloss, float* contrib, float* ugrad,
                     const float* item_rows, hipStream_t s, const PeerWait& pw,
                     int64_t bstride, const StepBufs* sbp) {
  const StepBufs sb = plain_bufs(contrib, ugrad, xloss, sbp);
  BPRMF_DISPATCH4(g, ({
    // every row and contribution store is write-through (sc1): the kernel boundary then has no
    // dirty-L2 write-back of them to wait for (WT = false builds remain for the template's sake)
    const unsigned blocks = (unsigned)((B + kBlock / G4_ - 1) / (kBlock / G4_));
    if (item_rows)
      k_user_step<G4_, S_, true, true><<<blocks, kBlock, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, sb,
                                                                 item_rows, pw, bstride, B);
    else
      k_user_step<G4_, S_, false, true><<<blocks, kBlock, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, sb,
                                                                  nullptr, pw, bstride, B);
  }));
  return hipGetLastError();
}

int k1_triplets_per_block(const Geom& g) { return kBlock / g.G4; }

int item_long_blocks(int B) { return std::min(kMaxLongItems, (2 * B) / (kLongSeg + 1)); }

// K2's grid: [loss workgroups][hot items][item segments][user segments spanning K1 workgroups]
struct K2Grid {
  int lb, long_blocks, item_blocks, user_blocks;
  int total() const { return lb + long_blocks + item_blocks + user_blocks; }
};
// item lane groups of the single-GPU step per 1024 triplets of the batch: K1 finishes the
// single-reference items, so ~1,000 of a 4,096-triplet batch's ~5,700 distinct items reach K2
// (ml-20m shape); 384 per 1024 gives those one lane group each, and a lane group loops when a
// batch has more (round 4 A/B against one lane group per possible segment: DESIGN.md §5)
constexpr int kK2ItemLg = 384;

template <int G4, int S, int KB>
static K2Grid k2_grid(int B, bool loss, bool capped = false) {
  constexpr int NG = KB / G4;
  constexpr int R = item_rounds<S>();
  K2Grid k;
  k.long_blocks = item_long_blocks(B);
  k.item_blocks = (int)((2LL * B + NG - 1) / NG);
  if (R > 1 && capped) {
    const int need = (int)((2LL * B + (int64_t)R * NG - 1) / ((int64_t)R * NG));
    k.item_blocks = std::min<int>(
        k.item_blocks, std::max<int>(need, (int)(((int64_t)B * kK2ItemLg / 1024 + NG - 1) / NG)));
  }
  // segments K2 finishes span K1 workgroups: at most one per workgroup boundary, and B/2
  const int tpb = kBlock / G4;
  const int k2_users = (int)std::min<int64_t>(B / 2, (B + tpb - 1) / tpb);
  k.user_blocks = (k2_users + NG - 1) / NG;
  k.lb = loss ? (B + KB - 1) / KB : 0;  // <= kSegLossSlots
  return k;
}

template <int G4, int S, int KB>
static hipError_t launch_item_step(const Geom& g, BatchView bv, int B, Table P, Table Q,
                                   const Hyper& hp, const int32_t* tbase, int step,
                                   const StepBufs& sb, float* grads, hipStream_t s, double* loss,
                                   int64_t bstride) {
  // single GPU: capped, when the items are many against the batch's 2B references (few items, as
  // at the ml-1m shape, send most of their segments to K2, which the capped grid serialises)
  const K2Grid k = k2_grid<G4, S, KB>(B, loss != nullptr, grads == nullptr && Q.rows >= 2LL * B);
  const unsigned blocks = (unsigned)k.total();
#define BPRMF_K2(SH_, WT_)                                                                        \
  k_item_step<G4, S, SH_, KB, WT_><<<blocks, KB, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, sb,       \
                                                        k.long_blocks, k.item_blocks, grads, loss, \
                                                        bstride, B)
  if (grads) BPRMF_K2(true, true);
  else BPRMF_K2(false, true);
#undef BPRMF_K2
  return hipGetLastError();
}

// K2 workgroups of 256 threads: a step's K2 dispatches ~1,300 of them in well under a microsecond,
// where 1024-thread workgroups (round 1) took ~2.4 us to be dispatched (per-workgroup stamps,
// tools/ubench_step_stamps.py); a hot item then has 8 lane groups (d <= 128), each keeping 8
// contribution rows in flight.
hipError_t item_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, const float* contrib, const float* ugrad,
                     float* grads, hipStream_t s, const float* xloss, double* loss,
                     int64_t bstride, const StepBufs* sbp) {
  const StepBufs sb = plain_bufs(const_cast<float*>(contrib), const_cast<float*>(ugrad),
                                 const_cast<float*>(xloss), sbp);
  if (!sb.xloss) loss = nullptr;
  BPRMF_DISPATCH4(g, ({
    return launch_item_step<G4_, S_, 256>(g, bv, B, P, Q, hp, tbase, step, sb, grads, s, loss,
                                          bstride);
  }));
  return hipGetLastError();
}

hipError_t fused_step(const Geom& g, BatchView bv0, int64_t bstride, int B, Table P, Table Q,
                      const Hyper& hp, const int32_t* tbase, int step, const StepBufs& sb,
                      double* loss, int32_t* err, hipStream_t s) {
  if (!sb.pend_q || !sb.pend_p || !sb.pstride || !bstride) return hipErrorInvalidValue;
  if (!sb.xloss) loss = nullptr;
  BPRMF_DISPATCH4(g, ({
    const K2Grid k = k2_grid<G4_, S_, kBlock>(B, loss != nullptr, Q.rows >= 2LL * B);
    const int k1_blocks = (B + kBlock / G4_ - 1) / (kBlock / G4_);
    k_fused_step<G4_, S_, kBlock><<<(unsigned)(k.total() + k1_blocks), kBlock, 0, s>>>(
        bv0, P, Q, hp, g.ld, tbase, step, sb, k.long_blocks, k.item_blocks, k.total(), loss,
        bstride, B, err);
  }));
  return hipGetLastError();
}

hipError_t item_step_push(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                          const int32_t* tbase, int step, float* contrib, float* ugrad, float* xloss,
                          double* loss, const GradRoute& gr, hipStream_t s) {
  const StepBufs sb = plain_bufs(contrib, ugrad, xloss, nullptr);
  if (!xloss) loss = nullptr;
  if (!gr.mark || gr.S <= 0) return hipErrorInvalidValue;
  BPRMF_DISPATCH4(g, ({
    const K2Grid k = k2_grid<G4_, S_, 256>(B, loss != nullptr);
    if (k.total() > kBoardMax) return hipErrorInvalidValue;
    k_item_step_push<G4_, S_, 256><<<(unsigned)k.total() + 1, 256, 0, s>>>(
        bv, P, Q, hp, g.ld, tbase, step, sb, k.long_blocks, k.item_blocks, loss, B, gr);
  }));
  return hipGetLastError();
}

hipError_t dist_front(const Geom& g, const OwnerArgs& o, BatchView bv, int B, Table P, Table Q,
                      const Hyper& hp, const int32_t* tbase, int step, float* contrib, float* ugrad,
                      float* xloss, const float* item_rows, const PeerWait& pw, hipStream_t s) {
  const StepBufs sb = plain_bufs(contrib, ugrad, xloss, nullptr);
  if (!o.mark || o.cap <= 0) return hipErrorInvalidValue;
  BPRMF_DISPATCH4(g, ({
    // the owner grid of dist.hip's launches: one lane group per position (two per position for
    // the fused apply + gather), then the owners' finisher, then K1
    const int64_t units = (step == 0 ? 1 : 2) * (int64_t)o.world * o.cap * G4_;
    const int ob = (int)std::max<int64_t>(
        1, std::min<int64_t>(std::min(o.max_blocks, kBoardMax), (units + kBlock - 1) / kBlock));
    const int k1b = (B + kBlock / G4_ - 1) / (kBlock / G4_);
    k_dist_front<G4_, S_><<<(unsigned)(ob + 1 + k1b), kBlock, 0, s>>>(o, bv, P, Q, hp, g.ld, tbase, step,
                                                                     sb, item_rows, pw, ob, B);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
