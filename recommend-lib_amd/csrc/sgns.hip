// sgns.hip — gfx950 kernels of the Item2Vec training step (include/sgns.h), SURVEY.md §8f row 4:
// SGNS.forward (Item2VecRecommender.py:82-97), its backward and Adam (:272, :282-286).
//
// Per example b (centre word i, C context words o_c, C * n negatives w):
//   loss = 1/(B C) sum_b [ sum_c softplus(-o_c . i) + sum_{c,k} softplus(w_ck . i) ]
//   d loss / d (o . i) = -(1 - sigma(o . i)) / (B C),   d loss / d (w . i) = sigma(w . i) / (B C)
// K1 (k_sgns_fwd): one wave per example, lane l holding factors l, l + 64, ... of the centre row in
// registers; the R = C (1 + n) ovectors rows are streamed U at a time (coalesced 256-byte row
// segments), each dot reduced across the wave; the centre row's gradient sum_r g_r o_r stays in
// registers and is added into GI with f32 atomics; g_r goes into S[word, b] after the loop.  The
// ovectors gradient is then a GEMM, GO [V, E] = S [V, B] x IB [B, E] (rocBLAS, split over B into
// partial products, sgns_capi.cpp), and k_sgns_post gives both tables a dense Adam sweep (rows
// never touched keep m = v = 0 and are skipped, exactly as torch leaves them), summing the
// partials on the way, clears S and adds the loss.
// Row 0 is nn.Embedding's padding_idx: it gets no gradient.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "device_common.h"
#include "ncf_kernels.h"
#include "sgns_kernels.h"

namespace bprmf {
namespace sgns {

constexpr int kT = 256;  // 4 waves, one example each
constexpr int kU = 8;    // ovectors rows in flight per wave (a multiple of 8: wave_sum8 groups)
constexpr int kMaxR = 1024;  // references per example (C (1 + n)), staged in LDS
constexpr uint32_t TAG_SGNS = 0x53474E00u;

static __device__ __forceinline__ int32_t draw_neg(const Args& a, int b, int k) {
  uint32_t c0 = (uint32_t)b, c1 = (uint32_t)k, c2 = (uint32_t)a.t, c3 = TAG_SGNS;
  philox10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  const float u = (float)(c0 >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  if (!a.cdf) {  // torch.FloatTensor(...).uniform_(0, V - 1).long(): [0, V - 2]
    const int64_t w = (int64_t)(u * (float)(a.V - 1));
    return (int32_t)std::min<int64_t>(w, a.V - 2 > 0 ? a.V - 2 : 0);
  }
  // torch.multinomial(weights, ..., replacement=True): first x with cdf[x] > u
  int64_t lo = 0, hi = a.V - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a.cdf[mid] > u) hi = mid;
    else lo = mid + 1;
  }
  return (int32_t)lo;
}

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// sum over the 64 lanes of 8 values at once (a transposed butterfly: 4 + 2 + 1 exchanges halve
// the values per lane, then 3 plain steps): on return lanes 8q .. 8q + 7 hold the total of p[q]
static __device__ __forceinline__ float wave_sum8(const float (&p)[8], int lane) {
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8;
  float q4[4], q2[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float send = h5 ? p[j] : p[j + 4];
    q4[j] = (h5 ? p[j + 4] : p[j]) + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float send = h4 ? q4[j] : q4[j + 2];
    q2[j] = (h4 ? q4[j + 2] : q4[j]) + __shfl_xor(send, 16);
  }
  float v = (h3 ? q2[1] : q2[0]) + __shfl_xor(h3 ? q2[0] : q2[1], 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

template <int M>
__global__ __launch_bounds__(kT) void k_sgns_fwd(Args a) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int b = blockIdx.x * (kT / 64) + wv;
  if (b >= a.B) return;  // whole waves
  const int64_t iw = a.iw[b];
  const int C = a.C, CN = a.C * a.n, R = C + CN;
  const float inv = 1.0f / ((float)a.B * (float)C);
  // the example's R words (contexts, then negatives: given, or drawn one per lane) and, after
  // the loop, their coefficients, in this wave's LDS slice
  __shared__ int32_t wsh[kT / 64][kMaxR];
  __shared__ float gsh[kT / 64][kMaxR];
  for (int r = lane; r < R; r += 64)
    wsh[wv][r] = r < C ? a.ow[(int64_t)b * C + r]
                : a.nw ? a.nw[(int64_t)b * CN + (r - C)] : draw_neg(a, b, r - C);
  float iv[M], gi[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int e = lane + 64 * m;
    iv[m] = e < a.E ? a.I[iw * a.ld + e] : 0.f;
    gi[m] = 0.f;
    if (e < a.E) a.IB[(int64_t)b * a.ld + e] = iv[m];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float lsum = 0.f;
  const int mine = lane >> 3;  // the reference of each group of 8 whose sum this lane holds
  for (int r0 = 0; r0 < R; r0 += kU) {
    int32_t w[kU];
    float ov[kU][M], p[kU];
    // the words are wave-uniform: scalar row addresses, unguarded loads (lanes past E read the
    // row's tail or the next row, or the table's padding row: they meet iv = 0 and are never
    // stored); past R, row 0 with a zero coefficient
#pragma unroll
    for (int u = 0; u < kU; ++u)
      w[u] = __builtin_amdgcn_readfirstlane(r0 + u < R ? wsh[wv][r0 + u] : 0);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const float* row = a.O + (int64_t)w[u] * a.ld;
#pragma unroll
      for (int m = 0; m < M; ++m) ov[u][m] = row[lane + 64 * m];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      p[u] = 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m) p[u] += iv[m] * ov[u][m];
    }
#pragma unroll
    for (int gg = 0; gg < kU / 8; ++gg) {
      float p8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) p8[j] = p[8 * gg + j];
      const float sdot = wave_sum8(p8, lane);  // o . i of reference r0 + 8 gg + mine
      const int r = r0 + 8 * gg + mine;
      float g = 0.f;
      if (r < R) {
        const bool ctx = r < C;
        const float sig = 1.0f / (1.0f + __expf(-sdot));
        g = ctx ? -(1.0f - sig) * inv : sig * inv;
        if ((lane & 7) == 0) {
          const float z = ctx ? -sdot : sdot;  // softplus(z) on the fast exp / log
          lsum += fmaxf(z, 0.f) + __logf(1.0f + __expf(-fabsf(z)));
          gsh[wv][r] = g;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), 8 * j));
#pragma unroll
        for (int m = 0; m < M; ++m) gi[m] += gu * ov[8 * gg + j][m];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // S and touch_o after the loop (gfx9 counts stores and atomics in vmcnt: issued inside the loop
  // they would hold the next iteration's row loads until they complete)
  for (int r = lane; r < R; r += 64) {
    const int32_t wr = wsh[wv][r];
    if (wr != 0) {
      atomicAdd(a.S + (int64_t)wr * a.B + b, gsh[wv][r]);
      a.touch_o[wr] = a.t;
    }
  }
  if (iw != 0) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int e = lane + 64 * m;
      if (e < a.E) atomicAdd(a.GI + iw * a.ld + e, gi[m]);
    }
    if (lane == 0) a.touch_i[iw] = a.t;
  }
  lsum = wave_sum(lsum);
  if (lane == 0) a.lbuf[b] = lsum * inv;
}

__global__ void k_sgns_negs(Args a, int32_t* __restrict__ out) {
  const int64_t CN = (int64_t)a.C * a.n, total = CN * a.B;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x)
    out[x] = draw_neg(a, (int)(x / CN), (int)(x % CN));
}

// Item2Vec.__init__ (:46-53): row 0 zeros, the rest uniform(-lim, lim); padding columns 0
__global__ void k_sgns_init(float* __restrict__ W, int64_t V, int E, int ld, float lim,
                            uint64_t seed, uint32_t tag) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < V * ld;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = x / ld;
    const int e = (int)(x % ld);
    float v = 0.f;
    if (row > 0 && e < E) {
      uint32_t c0 = (uint32_t)row, c1 = (uint32_t)(row >> 32), c2 = (uint32_t)e, c3 = tag;
      philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
      v = lim * (2.f * ((float)(c0 >> 8) * (1.0f / 16777216.0f)) - 1.f);
    }
    W[x] = v;
  }
}

__global__ void k_sgns_lookup(const float* __restrict__ W, int ld, int E,
                              const int32_t* __restrict__ idx, int64_t n, float* __restrict__ out) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n * E;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = x / E;
    out[x] = W[(int64_t)idx[q] * ld + (x % E)];
  }
}

// torch Adam (single-tensor form), as ncf.hip's adam_rows: m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)
static __device__ __forceinline__ void adam1(float& p, float& m, float& v, float g,
                                             const ncf::AdamArgs& ad) {
  m = m + ad.one_minus_b1 * (g - m);
  v = fmaf(ad.b2, v, ad.one_minus_b2 * g * g);
  p = p - ad.step_size * (m / (sqrtf(v) / ad.bc2_sqrt + ad.eps));
}

// everything after the GEMM in one launch, all of it elementwise: Adam on ivectors (gradient GI,
// re-zeroed) and on ovectors (gradient = the nsp GEMM partials summed in order, or GO itself),
// rows never touched skipped (m = v = 0: torch leaves them unchanged); S zeroed for the next
// step; the last workgroup adds the batch's loss.
__global__ __launch_bounds__(256) void k_sgns_post(Args a, const float* __restrict__ parts, int nsp,
                                                   ncf::AdamArgs ad, float* __restrict__ mI,
                                                   float* __restrict__ vI, float* __restrict__ mO,
                                                   float* __restrict__ vO) {
  if (blockIdx.x == gridDim.x - 1) {  // the loss, fixed order (block-uniform branch)
    constexpr int R = 16;
    __shared__ double red[256];
    double sum = 0.0;
    for (int t0 = 0; t0 < a.B; t0 += 256 * R) {
      float v[R];
#pragma unroll
      for (int m = 0; m < R; ++m) {
        const int t = t0 + m * 256 + threadIdx.x;
        v[m] = t < a.B ? a.lbuf[t] : 0.f;
      }
#pragma unroll
      for (int m = 0; m < R; ++m) sum += (double)v[m];
    }
    red[threadIdx.x] = sum;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) a.loss[0] += red[0];
  }
  // 4 elements (one float4, within one row: ld % 4 == 0) per thread and iteration
  const int64_t n = a.V * a.ld, n4 = n / 4, stride = (int64_t)gridDim.x * blockDim.x;
  const int ld4 = a.ld / 4;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < 2 * n4; x += stride) {
    const bool o = x >= n4;
    const int64_t y = o ? x - n4 : x;
    const int32_t row = (int32_t)((uint32_t)y / (uint32_t)ld4);
    const int32_t st = o ? a.touch_o[row] : a.touch_i[row];
    if (st < 0) continue;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (st == a.t) {
      if (o) {
        g = reinterpret_cast<const float4*>(parts)[y];
        for (int q = 1; q < nsp; ++q) {
          const float4 v = reinterpret_cast<const float4*>(parts)[q * n4 + y];
          g.x += v.x;
          g.y += v.y;
          g.z += v.z;
          g.w += v.w;
        }
      } else {
        g = reinterpret_cast<const float4*>(a.GI)[y];
        reinterpret_cast<float4*>(a.GI)[y] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    float4* P = reinterpret_cast<float4*>(o ? a.O : a.I) + y;
    float4* Mm = reinterpret_cast<float4*>(o ? mO : mI) + y;
    float4* Vv = reinterpret_cast<float4*>(o ? vO : vI) + y;
    float4 p = *P, m = *Mm, v = *Vv;
    adam1(p.x, m.x, v.x, g.x, ad);
    adam1(p.y, m.y, v.y, g.y, ad);
    adam1(p.z, m.z, v.z, g.z, ad);
    adam1(p.w, m.w, v.w, g.w, ad);
    *P = p;
    *Mm = m;
    *Vv = v;
  }
  const int64_t s4 = a.V * a.B / 4;  // S for the next step (V * B is a multiple of 4: B % 4 below)
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < s4; x += stride)
    reinterpret_cast<float4*>(a.S)[x] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t x = 4 * s4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < a.V * a.B; x += stride)
    a.S[x] = 0.f;
}

static unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

int lanes_elems(int E) { return (E + 63) / 64; }

hipError_t init_uniform(float* W, int64_t V, int E, int ld, float lim, uint64_t seed, uint32_t tag,
                        hipStream_t s) {
  if (V <= 0) return hipSuccess;
  k_sgns_init<<<grid_for(V * ld), 256, 0, s>>>(W, V, E, ld, lim, seed, tag);
  return hipGetLastError();
}

hipError_t forward_backward(const Args& a, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((a.B + kT / 64 - 1) / (kT / 64));
  switch (lanes_elems(a.E)) {
#define SG(M_) \
  case M_: k_sgns_fwd<M_><<<blocks, kT, 0, s>>>(a); break;
    SG(1) SG(2) SG(3) SG(4) SG(5) SG(6) SG(7) SG(8) SG(9) SG(10) SG(11) SG(12) SG(13) SG(14)
    SG(15) SG(16)
#undef SG
    default: return hipErrorInvalidValue;  // E > 1024
  }
  return hipGetLastError();
}

hipError_t post(const Args& a, const float* parts, int nsp, const ncf::AdamArgs& ad, float* mI,
                float* vI, float* mO, float* vO, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  const int64_t n = 2 * a.V * a.ld / 4;
  const unsigned blocks = (unsigned)std::max<int64_t>(2, std::min<int64_t>((n + 255) / 256, 4096));
  k_sgns_post<<<blocks, 256, 0, s>>>(a, parts, nsp, ad, mI, vI, mO, vO);
  return hipGetLastError();
}

hipError_t negatives(const Args& a, int32_t* out, hipStream_t s) {
  if (a.B <= 0 || a.C * a.n <= 0) return hipSuccess;
  k_sgns_negs<<<grid_for((int64_t)a.B * a.C * a.n), 256, 0, s>>>(a, out);
  return hipGetLastError();
}

hipError_t lookup(const float* W, int ld, int E, const int32_t* idx, int64_t n, float* out,
                  hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_sgns_lookup<<<grid_for(n * E), 256, 0, s>>>(W, ld, E, idx, n, out);
  return hipGetLastError();
}

}  // namespace sgns
}  // namespace bprmf
