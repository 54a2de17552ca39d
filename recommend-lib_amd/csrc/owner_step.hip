// owner_step.hip — DIAGNOSTIC timing prototype (-DBPRMF_DIAG_OWNER only; WRONG results): one
// launch per step in which every row's owner recomputes x for each of its references (users:
// one lane group per triplet as K1; items: one lane group per item segment, reading each
// reference's triplet record and the rows it needs), with no contribution round trip and no
// in-launch waits.  Rows are read and written in place here (racy), which a real form would
// replace with builder-assigned double buffers; this build measures the memory pattern only.
#include "device_common.h"

#ifdef BPRMF_DIAG_OWNER
namespace bprmf {

static __device__ __forceinline__ float4 o_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void o_st4(float* p, float4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
}
static __device__ __forceinline__ float4 o_scale(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }
static __device__ __forceinline__ float o_dot(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}
static __device__ __forceinline__ float4 o_fma(float s, float4 b, float4 a) {
  return make_float4(fmaf(s, b.x, a.x), fmaf(s, b.y, a.y), fmaf(s, b.z, a.z), fmaf(s, b.w, a.w));
}
static __device__ __forceinline__ float4 o_sgd(float4 v, float4 g, float lr, float wd) {
  return make_float4(fmaf(-lr, fmaf(wd, v.x, g.x), v.x), fmaf(-lr, fmaf(wd, v.y, g.y), v.y),
                     fmaf(-lr, fmaf(wd, v.z, g.z), v.z), fmaf(-lr, fmaf(wd, v.w, g.w), v.w));
}

// F references of one item at once: their triplet records, then their rows, then the sums
template <int G4, int S, int F>
static __device__ __forceinline__ void item_refs(float4 (&g)[S], const float4 (&own)[S], int32_t item,
                                                 const int32_t (&rf)[F], int cnt, const BatchView& bv,
                                                 const Table& P, const Table& Q, const Hyper& hp,
                                                 int ld, int32_t t, int sub) {
  int4 tr[F];
#pragma unroll
  for (int m = 0; m < F; ++m)
    if (m < cnt) tr[m] = reinterpret_cast<const int4*>(bv.trec)[rf[m] >> 1];
  float4 pu[F][S], vo[F][S];
  int32_t su[F], so[F];
#pragma unroll
  for (int m = 0; m < F; ++m)
    if (m < cnt) {
      const int32_t other = ((rf[m] & 1) ? tr[m].x : tr[m].y) & 0x3FFFFFFF;
      const float* pr = P.W + (int64_t)tr[m].z * ld + 4 * sub;
      const float* qr = Q.W + (int64_t)other * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        pu[m][k] = o_ld4(pr + 4 * G4 * k);
        vo[m][k] = o_ld4(qr + 4 * G4 * k);
      }
      su[m] = P.stamp[tr[m].z];
      so[m] = Q.stamp[other];
    }
#pragma unroll
  for (int m = 0; m < F; ++m) {
    if (m >= cnt) continue;
    const float fu = decay_pow(hp.log2a, t - 1 - su[m]), fo = decay_pow(hp.log2a, t - 1 - so[m]);
    float dn = 0.f, dt = 0.f;  // <P_u, own>, <P_u, other>
#pragma unroll
    for (int k = 0; k < S; ++k) {
      pu[m][k] = o_scale(pu[m][k], fu);
      dn = o_dot(pu[m][k], own[k], dn);
      dt = o_dot(pu[m][k], o_scale(vo[m][k], fo), dt);
    }
    dn = group_sum<G4>(dn);
    dt = group_sum<G4>(dt);
    const bool isj = rf[m] & 1;
    const float x = isj ? dt - dn : dn - dt;
    const float c = 1.0f / (1.0f + expf(x));
#pragma unroll
    for (int k = 0; k < S; ++k) g[k] = o_fma(isj ? 1.f : -1.f, o_scale(pu[m][k], c), g[k]);
  }
  (void)item;
}

template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_owner_diag(BatchView bv0, Table P, Table Q, Hyper hp, int ld,
                                                      const int32_t* __restrict__ tbase, int step,
                                                      int long_blocks, int item_blocks, int64_t bstride,
                                                      int B) {
  constexpr int NG = kBlock / G4;
  const int32_t t = tbase[0] + step + 1;
  const BatchView bv = bv0.shifted(((int64_t)tbase[1] + step) * bstride);
  const int sub = threadIdx.x & (G4 - 1);
  const int grp = threadIdx.x / G4;
  const int blk = blockIdx.x;
  if (blk < long_blocks) {  // hot item: 8 lane groups over its references, LDS tree
    __shared__ float4 part[NG][G4 * S];
    const int4 r0 = reinterpret_cast<const int4*>(bv.lrec + (int64_t)blk * kRec)[0];
    if (blk >= bv.meta[3]) return;
    const int32_t item = r0.x;
    const int beg = r0.y, end = r0.z;
    float4 own[S], g[S];
    const float* w = Q.W + (int64_t)item * ld + 4 * sub;
#pragma unroll
    for (int k = 0; k < S; ++k) own[k] = o_ld4(w + 4 * G4 * k);
    const float fw = decay_pow(hp.log2a, t - 1 - Q.stamp[item]);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      own[k] = o_scale(own[k], fw);
      g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    constexpr int F = 4;
    for (int b0 = beg + grp * F; b0 < end; b0 += NG * F) {
      int32_t rf[F];
#pragma unroll
      for (int m = 0; m < F; ++m) rf[m] = b0 + m < end ? bv.refs[b0 + m] : 0;
      item_refs<G4, S, F>(g, own, item, rf, min(F, end - b0), bv, P, Q, hp, ld, t, sub);
    }
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
      float* wo = Q.W + (int64_t)item * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) o_st4(wo + 4 * G4 * k, o_sgd(own[k], part[0][sub + G4 * k], hp.lr, hp.wd));
      if (sub == 0) __hip_atomic_store(Q.stamp + item, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (blk < long_blocks + item_blocks) {  // item segments: one lane group each, in rounds
    const int n_iseg = bv.meta[2];
    for (int s = (blk - long_blocks) * NG + grp; s < n_iseg; s += item_blocks * NG) {
      const int4 r0 = reinterpret_cast<const int4*>(bv.irec + (int64_t)s * kRec)[0];
      const int4 r1 = reinterpret_cast<const int4*>(bv.irec + (int64_t)s * kRec)[1];
      if (r0.y >> 30) continue;  // hot
      const int32_t item = r0.x;
      const int beg = r0.y & 0x7FFF, len = (r0.y >> 15) & 0x7FFF;
      float4 own[S], g[S];
      const float* w = Q.W + (int64_t)item * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) own[k] = o_ld4(w + 4 * G4 * k);
      const float fw = decay_pow(hp.log2a, t - 1 - Q.stamp[item]);
#pragma unroll
      for (int k = 0; k < S; ++k) {
        own[k] = o_scale(own[k], fw);
        g[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const int32_t pk[6] = {r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
      constexpr int F = 6;
      for (int m0 = 0; m0 < len; m0 += F) {
        int32_t rf[F];
#pragma unroll
        for (int m = 0; m < F; ++m) {
          const int q = m0 + m;
          rf[m] = q < kInlineRefs ? (pk[(q >> 1) % 6] >> (16 * (q & 1))) & 0xFFFF
                                  : (q < len ? bv.refs[beg + q] : 0);
        }
        item_refs<G4, S, F>(g, own, item, rf, min(F, len - m0), bv, P, Q, hp, ld, t, sub);
      }
      float* wo = Q.W + (int64_t)item * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) o_st4(wo + 4 * G4 * k, o_sgd(own[k], g[k], hp.lr, hp.wd));
      if (sub == 0) __hip_atomic_store(Q.stamp + item, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // users: one lane group per triplet (K1's shape), in-workgroup segments summed in LDS
  __shared__ float4 s_g[S * kBlock];
  const int p = (blk - long_blocks - item_blocks) * NG + grp;
  const int4 r = reinterpret_cast<const int4*>(bv.trec)[min(p, B - 1)];
  const int n = bv.meta[0];
  float4 pu[S];
  int w = 0;
  float* prow = nullptr;
  if (p < n) {
    const int32_t i = r.x & 0x3FFFFFFF, j = r.y & 0x3FFFFFFF;
    const bool soli = r.x & 0x40000000, solj = r.y & 0x40000000;
    w = r.w;
    prow = P.W + (int64_t)r.z * ld + 4 * sub;
    const float* qi = Q.W + (int64_t)i * ld + 4 * sub;
    const float* qj = Q.W + (int64_t)j * ld + 4 * sub;
    float4 vi[S], vj[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      pu[k] = o_ld4(prow + 4 * G4 * k);
      vi[k] = o_ld4(qi + 4 * G4 * k);
      vj[k] = o_ld4(qj + 4 * G4 * k);
    }
    const float fu = decay_pow(hp.log2a, t - 1 - P.stamp[r.z]);
    const float fi = decay_pow(hp.log2a, t - 1 - Q.stamp[i]);
    const float fj = decay_pow(hp.log2a, t - 1 - Q.stamp[j]);
    float di = 0.f, dj = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      pu[k] = o_scale(pu[k], fu);
      vi[k] = o_scale(vi[k], fi);
      vj[k] = o_scale(vj[k], fj);
      di = o_dot(pu[k], vi[k], di);
      dj = o_dot(pu[k], vj[k], dj);
    }
    di = group_sum<G4>(di);
    dj = group_sum<G4>(dj);
    const float x = di - dj;
    const float c = 1.0f / (1.0f + expf(x));
    if (soli) {
      float* qw = Q.W + (int64_t)i * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) o_st4(qw + 4 * G4 * k, o_sgd(vi[k], o_scale(pu[k], -c), hp.lr, hp.wd));
    }
    if (solj) {
      float* qw = Q.W + (int64_t)j * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) o_st4(qw + 4 * G4 * k, o_sgd(vj[k], o_scale(pu[k], c), hp.lr, hp.wd));
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const float4 d = make_float4(vi[k].x - vj[k].x, vi[k].y - vj[k].y, vi[k].z - vj[k].z, vi[k].w - vj[k].w);
      s_g[k * kBlock + threadIdx.x] = o_scale(d, -c);
    }
    if (w == 1 || w == 0) {
#pragma unroll
      for (int k = 0; k < S; ++k) o_st4(prow + 4 * G4 * k, o_sgd(pu[k], s_g[k * kBlock + threadIdx.x], hp.lr, hp.wd));
    }
  }
  __syncthreads();
  if (w >= 2) {
    const int q0 = threadIdx.x - sub;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int m = 0; m < w; ++m) {
        const float4 x = s_g[k * kBlock + q0 + m * G4 + sub];
        g = make_float4(g.x + x.x, g.y + x.y, g.z + x.z, g.w + x.w);
      }
      o_st4(prow + 4 * G4 * k, o_sgd(pu[k], g, hp.lr, hp.wd));
    }
  }
}

hipError_t owner_diag_step(const Geom& g, BatchView bv0, int64_t bstride, int B, Table P, Table Q,
                           const Hyper& hp, const int32_t* tbase, int step, hipStream_t s) {
  BPRMF_DISPATCH4(g, ({
    if (S_ != 1) return hipErrorInvalidValue;
    constexpr int NG = kBlock / G4_;
    const int long_blocks = item_long_blocks(B);
    const int item_blocks = (int)(((int64_t)B * 384 / 1024 + NG - 1) / NG);
    const int user_blocks = (B + NG - 1) / NG;
    k_owner_diag<G4_, S_><<<(unsigned)(long_blocks + item_blocks + user_blocks), kBlock, 0, s>>>(
        bv0, P, Q, hp, g.ld, tbase, step, long_blocks, item_blocks, bstride, B);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
#endif
