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
#include <algorithm>

#include "device_common.h"

namespace bprmf {

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
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

// K1, one lane group per triplet p (sorted by user).  SH (sharded): i/j are slots of item_rows,
// the rows the owners sent for this step, already brought to step t-1 by the owner (no stamps).
template <int G4, int S, bool SH>
__global__ __launch_bounds__(kBlock) void k_user_step(BatchView bv, Table P, Table Q, Hyper hp,
                                                      int ld, const int32_t* __restrict__ tbase,
                                                      int step, float* __restrict__ xloss,
                                                      float* __restrict__ contrib,
                                                      float* __restrict__ ugrad,
                                                      const float* __restrict__ item_rows,
                                                      PeerWait pw, int64_t bstride, int B) {
  const int sub = threadIdx.x & (G4 - 1);
  const int p = blockIdx.x * (kBlock / G4) + threadIdx.x / G4;
  if (bstride) bv = bv.shifted((int64_t)(tbase[1] + step) * bstride);
  if (SH) wait_peer_flags(pw.flags, pw.world, pw.self, *tbase + step + 1, pw.err);
  // independent loads: the record, the triplet count, the step base.  The grid covers B rounded
  // up to whole blocks: the index is clamped into the batch's B records (never read past them)
  const int4 r = reinterpret_cast<const int4*>(bv.trec)[min(p, B - 1)];
  const int n = bv.meta[0];
  const int32_t t = *tbase + step + 1;
  if (p < n) {
    const int32_t i = r.x, j = r.y, u = r.z;
    float* pw = P.W + (int64_t)u * ld + 4 * sub;
    const float* qbase = SH ? item_rows : Q.W;
    const float* qi = qbase + (int64_t)i * ld + 4 * sub;
    const float* qj = qbase + (int64_t)j * ld + 4 * sub;
    float4 pu[S], vi[S], vj[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      pu[k] = ld4(pw + 4 * G4 * k);
      vi[k] = ld4(qi + 4 * G4 * k);
      vj[k] = ld4(qj + 4 * G4 * k);
    }
    const int32_t su = P.stamp[u];
    const float fi = SH ? 1.f : decay_pow(hp.log2a, t - 1 - Q.stamp[i]);
    const float fj = SH ? 1.f : decay_pow(hp.log2a, t - 1 - Q.stamp[j]);
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
    const float c = 1.0f / (1.0f + expf(x));  // sigmoid(-x) = -dL/dx
    if (sub == 0 && xloss) xloss[p] = x;  // K2 sums the loss terms
    float* cb = contrib + (int64_t)p * ld + 4 * sub;
#pragma unroll
    for (int k = 0; k < S; ++k) st4(cb + 4 * G4 * k, scale4(pu[k], c));
    if (r.w) {  // the user's only triplet: W = V - lr (g + wd V) with g = -c (Q_i - Q_j)
#pragma unroll
      for (int k = 0; k < S; ++k)
        st4(pw + 4 * G4 * k, sgd4(pu[k], scale4(sub4(vi[k], vj[k]), -c), hp.lr, hp.wd));
      if (sub == 0) P.stamp[u] = t;
    } else {  // K2 sums the segment's gradients in position order
      float* ub = ugrad + (int64_t)p * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) st4(ub + 4 * G4 * k, scale4(sub4(vi[k], vj[k]), -c));
    }
  }
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
    stamp = Q.stamp[item];
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
template <int G4, int S, bool SH>
static __device__ __forceinline__ void finish_item(Table Q, int32_t item, int slot,
                                                   const float4 (&g)[S], const ItemRow<G4, S, SH>& row,
                                                   const Hyper& hp, int ld, int32_t t, int sub,
                                                   float* __restrict__ grads) {
  if (SH) {
    float* o = grads + (int64_t)slot * ld + 4 * sub;
#pragma unroll
    for (int k = 0; k < S; ++k) st4(o + 4 * G4 * k, g[k]);
  } else {
    float* w = Q.W + (int64_t)item * ld + 4 * sub;
    const float f = decay_pow(hp.log2a, t - 1 - row.stamp);
#pragma unroll
    for (int k = 0; k < S; ++k) st4(w + 4 * G4 * k, sgd4(scale4(row.x[k], f), g[k], hp.lr, hp.wd));
    if (sub == 0) Q.stamp[item] = t;
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

// KB threads per block: 1024 (512 for rows over 1 KB) so a hot item's workgroup has 16-32 lane
// groups fetching its references in parallel
template <int G4, int S, bool SH, int KB>
__global__ __launch_bounds__(KB) void k_item_step(BatchView bv, Table P, Table Q, Hyper hp, int ld,
                                                  const int32_t* __restrict__ tbase, int step,
                                                  const float* __restrict__ contrib,
                                                  const float* __restrict__ ugrad, int long_blocks,
                                                  int item_blocks, float* __restrict__ grads,
                                                  const float* __restrict__ xloss,
                                                  double* __restrict__ loss, int64_t bstride,
                                                  int B) {
  constexpr int NG = KB / G4;
  if (bstride) bv = bv.shifted((int64_t)(tbase[1] + step) * bstride);
  const int sub = threadIdx.x & (G4 - 1);
  const int grp = threadIdx.x / G4;
  const int32_t t = *tbase + step + 1;
  if (loss && blockIdx.x == 0) {  // the step's loss (first block: dispatched first, off the tail)
    __shared__ double red[KB / 64];
    const int n = bv.meta[0];
    double acc = 0.0;
    for (int p = threadIdx.x; p < n; p += KB) acc += (double)softplus(-xloss[p]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);  // fixed butterfly
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {  // the only writer of this slot in the launch
      double tot = 0.0;
      for (int w = 0; w < KB / 64; ++w) tot += red[w];
      loss[0] += tot;
    }
    return;
  }
  const int bid = (int)blockIdx.x - (loss ? 1 : 0);
  if (bid >= long_blocks + item_blocks) {  // users with several triplets
    const int m = (bid - long_blocks - item_blocks) * NG + grp;
    // indices clamped into the batch's record arrays (B/2 user records, 2B item records): the
    // groups past the count read a valid record and return
    const int4 r0 = reinterpret_cast<const int4*>(bv.mrec + (int64_t)min(m, max(B / 2 - 1, 0)) * kRec)[0];
    const int n_multi = bv.meta[4];
    if (m >= n_multi) return;
    const int32_t u = r0.x;
    float* pw = P.W + (int64_t)u * ld + 4 * sub;
    float4 cur[S], g[S];
#pragma unroll
    for (int k = 0; k < S; ++k) cur[k] = ld4(pw + 4 * G4 * k);
    const int32_t su = P.stamp[u];
    sum_rows<G4, S>(g, ugrad, r0.y, r0.z, ld, sub);
    const float f = decay_pow(hp.log2a, t - 1 - su);
#pragma unroll
    for (int k = 0; k < S; ++k) st4(pw + 4 * G4 * k, sgd4(scale4(cur[k], f), g[k], hp.lr, hp.wd));
    if (sub == 0) P.stamp[u] = t;
    return;
  }
  if (bid < long_blocks) {
    __shared__ float4 part[NG][G4 * S];
    const int4 r0 = reinterpret_cast<const int4*>(bv.lrec + (int64_t)bid * kRec)[0];
    const int n_long = bv.meta[3];
    if (bid >= n_long) return;  // uniform over the block
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
      for (int m0 = 0; m0 < cnt; m0 += 8) {
        float4 rows[8][S];
        int32_t rf[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          rf[m] = __shfl(myref, lane0 + ((m0 + m) & (G4 - 1)));
          if (m0 + m < cnt) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
        }
#pragma unroll
        for (int m = 0; m < 8; ++m)
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
      finish_item<G4, S, SH>(Q, item, r0.w, g, row, hp, ld, t, sub, grads);
    }
    return;
  }
  const int s = (bid - long_blocks) * NG + grp;
  const int sc = min(s, 2 * B - 1);
  const int4 r0 = reinterpret_cast<const int4*>(bv.irec + (int64_t)sc * kRec)[0];
  const int4 r1 = reinterpret_cast<const int4*>(bv.irec + (int64_t)sc * kRec)[1];
  const int n_iseg = bv.meta[2];
  if (s >= n_iseg || r1.w) return;  // past the batch's items, or a workgroup-served hot item
  const int32_t item = r0.x;
  const int beg = r0.y, end = r0.z, len = end - beg;
  ItemRow<G4, S, SH> row;
  row.load(Q, item, ld, sub);
  float4 g[S];
#pragma unroll
  for (int k = 0; k < S; ++k) g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (len <= 4) {  // the common case: every ref inline, all rows requested before accumulating
    float4 rows[4][S];
    const int32_t rf[4] = {r0.w, r1.x, r1.y, r1.z};
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (m < len) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (m < len) acc_ref<S>(g, rows[m], rf[m]);
  } else {  // lanes fetch G4 refs at once; rows requested 8 at a time before accumulating
    const int lane0 = (threadIdx.x & 63) - sub;
    for (int base = beg; base < end; base += G4) {
      const int32_t myref = base + sub < end ? bv.refs[base + sub] : 0;
      const int cnt = min(G4, end - base);
      for (int m0 = 0; m0 < cnt; m0 += 8) {
        float4 rows[8][S];
        int32_t rf[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          rf[m] = __shfl(myref, lane0 + ((m0 + m) & (G4 - 1)));
          if (m0 + m < cnt) load_ref<G4, S>(rows[m], contrib, rf[m], ld, sub);
        }
#pragma unroll
        for (int m = 0; m < 8; ++m)
          if (m0 + m < cnt) acc_ref<S>(g, rows[m], rf[m]);
      }
    }
  }
  finish_item<G4, S, SH>(Q, item, item, g, row, hp, ld, t, sub, grads);  // SH: item field = slot
}

// Expand BODY for every instantiated float4 geometry (G4_, S_).
#define BPRMF_DISPATCH4(geom, BODY)                                \
  switch ((geom).G4 * 10 + (geom).S) {                             \
    case 11: { constexpr int G4_ = 1, S_ = 1; BODY; } break;       \
    case 21: { constexpr int G4_ = 2, S_ = 1; BODY; } break;       \
    case 41: { constexpr int G4_ = 4, S_ = 1; BODY; } break;       \
    case 81: { constexpr int G4_ = 8, S_ = 1; BODY; } break;       \
    case 161: { constexpr int G4_ = 16, S_ = 1; BODY; } break;     \
    case 321: { constexpr int G4_ = 32, S_ = 1; BODY; } break;     \
    case 641: { constexpr int G4_ = 64, S_ = 1; BODY; } break;     \
    case 642: { constexpr int G4_ = 64, S_ = 2; BODY; } break;     \
    case 643: { constexpr int G4_ = 64, S_ = 3; BODY; } break;     \
    case 644: { constexpr int G4_ = 64, S_ = 4; BODY; } break;     \
    default: return hipErrorInvalidValue;                          \
  }

hipError_t user_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, float* xloss, float* contrib, float* ugrad,
                     const float* item_rows, hipStream_t s, const PeerWait& pw,
                     int64_t bstride) {
  BPRMF_DISPATCH4(g, ({
    const unsigned blocks = (unsigned)((B + kBlock / G4_ - 1) / (kBlock / G4_));
    if (item_rows)
      k_user_step<G4_, S_, true><<<blocks, kBlock, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, xloss,
                                                           contrib, ugrad, item_rows, pw,
                                                           bstride, B);
    else
      k_user_step<G4_, S_, false><<<blocks, kBlock, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, xloss,
                                                            contrib, ugrad, nullptr, pw,
                                                            bstride, B);
  }));
  return hipGetLastError();
}

int item_long_blocks(int B) { return std::min(kMaxLongItems, (2 * B) / (kLongSeg + 1)); }

hipError_t item_step(const Geom& g, BatchView bv, int B, Table P, Table Q, const Hyper& hp,
                     const int32_t* tbase, int step, const float* contrib, const float* ugrad,
                     float* grads, hipStream_t s, const float* xloss, double* loss,
                     int64_t bstride) {
  const int long_blocks = item_long_blocks(B);
  if (!xloss) loss = nullptr;
  BPRMF_DISPATCH4(g, ({
    constexpr int KB = S_ == 1 ? 1024 : 512;
    constexpr int NG = KB / G4_;
    const int item_blocks = (int)((2LL * B + NG - 1) / NG);
    const int user_blocks = (int)((B / 2 + NG - 1) / NG);  // multi-triplet users <= B/2
    const unsigned blocks = (unsigned)(long_blocks + item_blocks + user_blocks + (loss ? 1 : 0));
    if (grads)
      k_item_step<G4_, S_, true, KB><<<blocks, KB, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step, contrib,
                                                           ugrad, long_blocks, item_blocks, grads,
                                                           xloss, loss, bstride, B);
    else
      k_item_step<G4_, S_, false, KB><<<blocks, KB, 0, s>>>(bv, P, Q, hp, g.ld, tbase, step,
                                                            contrib, ugrad, long_blocks,
                                                            item_blocks, nullptr, xloss, loss,
                                                            bstride, B);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
