// mf.hip — gfx950 kernels of the rating-SGD path (include/mf.h): the reference's Cython SVD and
// RSVD epochs (util/matrix_factorization.pyx:128-151, :40-61), bit-identical in double.
//
// A per-sample SGD epoch is a sequence; sample s can run as soon as the last earlier samples
// touching its user and its item have run.  The host assigns every sample its dependency level
// (mf_capi.cpp) and lays the samples out level by level; one workgroup of 1024 threads walks the
// levels, one lane group per sample, with a workgroup barrier between levels (the samples of a
// level touch disjoint rows, and the barrier orders a level's writes before the next level's
// reads on the workgroup's CU).  Each sample is evaluated with the reference's operations in the
// reference's order, in double, with no contraction into fused multiply-adds, so every value is
// rounded exactly as the Cython loop rounds it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "mf_kernels.h"

#pragma clang fp contract(off)

namespace bprmf {
namespace mf {

constexpr int kThreads = 1024;
constexpr int kPerLane = 16;  // factors held per lane (a lane group of G lanes covers k <= 16 G)

// One sample per lane group of G lanes (G = 64 / 2^n, k <= 16 G); lane l holds factors
// l, l + G, l + 2G, ... of the sample's two rows in registers, so each row load instruction
// reads whole cache lines.  The products go to LDS and the group's first lane sums them in factor
// order: the reference's strictly sequential dot product.  MODEL 0 = SVD.fit (:132-151),
// 1 = RSVD.fit (:42-61).
struct Rec {  // one sample's train row
  int32_t u = 0, i = 0;
  double r = 0.0;
};
static __device__ __forceinline__ Rec load_rec(const Args& a, int s, bool active) {
  Rec x;
  if (active) {
    x.u = a.su[s];
    x.i = a.si[s];
    x.r = a.sr[s];
  }
  return x;
}

template <int MODEL, int G>
static __device__ __forceinline__ void mf_sample(const Args& a, const Rec& rec, bool active,
                                                 int lane, double* __restrict__ prod) {
  const int64_t u = rec.u, i = rec.i;
  const double r = rec.r;
  const int k = a.k;
  double* pu = a.P + u * k;
  double* qi = a.Q + i * k;
  double p[kPerLane], q[kPerLane];
#pragma unroll
  for (int m = 0; m < kPerLane; ++m) {
    const int f = lane + G * m;
    if (active && f < k) {
      p[m] = pu[f];
      q[m] = qi[f];
    }
  }
  double b_u = 0.0, b_i = 0.0;
  if (active && lane == 0) {
    b_u = a.bu[u];
    b_i = a.bi[i];
  }
#pragma unroll
  for (int m = 0; m < kPerLane; ++m) {
    const int f = lane + G * m;
    if (active && f < k) prod[f] = MODEL == 0 ? q[m] * p[m] : p[m] * q[m];  // qi*pu (SVD), ui*vj
  }
  // the group's lanes share one wave: its LDS writes are complete once lgkmcnt drains
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double dot = 0.0;
  if (active && lane == 0) {  // LDS reads 16 at a time, then the adds in factor order
    int f = 0;
    for (; f + 16 <= k; f += 16) {
      double v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = prod[f + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) dot = dot + v[j];
    }
    for (; f < k; ++f) dot = dot + prod[f];
  }
  __builtin_amdgcn_wave_barrier();  // prod is rewritten by the group's next sample
  if (!active) return;
  const int leader = (threadIdx.x & 63) & ~(G - 1);
  double err = 0.0;
  if (MODEL == 0) {
    if (lane == 0) {
      err = r - (((a.gm + b_u) + b_i) + dot);
      if (a.variant) {
        a.bu[u] = b_u + a.lr[0] * (err - a.reg[0] * b_u);
        a.bi[i] = b_i + a.lr[1] * (err - a.reg[1] * b_i);
      }
    }
    err = __shfl(err, leader);
#pragma unroll
    for (int m = 0; m < kPerLane; ++m) {
      const int f = lane + G * m;
      if (f < k) {
        pu[f] = p[m] + a.lr[2] * (err * q[m] - a.reg[2] * p[m]);
        qi[f] = q[m] + a.lr[3] * (err * p[m] - a.reg[3] * q[m]);
      }
    }
  } else {
    const double lr = a.lr[0], reg = a.reg[0], reg2 = a.reg[1];
    if (lane == 0) {
      err = r - ((b_u + b_i) + dot);
      if (a.variant == 2) {
        a.bu[u] = b_u + lr * (err - reg2 * ((b_u + b_i) - a.gm));
        a.bi[i] = b_i + lr * (err - reg2 * ((b_u + b_i) - a.gm));
      }
    }
    err = __shfl(err, leader);
#pragma unroll
    for (int m = 0; m < kPerLane; ++m) {
      const int f = lane + G * m;
      if (f < k) {
        pu[f] = p[m] + lr * (err * q[m] - reg * p[m]);
        qi[f] = q[m] + lr * (err * p[m] - reg * q[m]);
      }
    }
  }
}

template <int MODEL, int G>
__global__ __launch_bounds__(kThreads) void k_mf_epoch(Args a) {
  constexpr int SPR = kThreads / G;  // samples per round
  __shared__ double prod[SPR * G * kPerLane];  // per sample slot: its k <= 16 G products
  const int lane = threadIdx.x & (G - 1);
  const int slot = threadIdx.x / G;
  double* my = prod + slot * G * kPerLane;
  // the first round's record of each level is loaded one level ahead (records do not depend on
  // the tables), so a level starts with its rows' loads
  int beg = a.loff[0], end = a.loff[1];
  Rec next = load_rec(a, beg + slot, beg + slot < end);
  for (int L = 0; L < a.levels; ++L) {
    const Rec cur = next;
    const int nbeg = end, nend = L + 1 < a.levels ? a.loff[L + 2] : end;
    next = load_rec(a, nbeg + slot, nbeg + slot < nend);
    mf_sample<MODEL, G>(a, cur, beg + slot < end, lane, my);
    for (int s0 = beg + SPR; s0 < end; s0 += SPR)
      mf_sample<MODEL, G>(a, load_rec(a, s0 + slot, s0 + slot < end), s0 + slot < end, lane, my);
    __threadfence_block();  // this level's row writes before the next level's reads
    __syncthreads();
    beg = nbeg;
    end = nend;
  }
}

// predict (:157-167 SVD, :67-78 RSVD) for n pairs; the dot product in sample order (numpy's dot
// may sum in another order: agreement to rounding)
__global__ void k_mf_predict(Args a, int model, const int32_t* __restrict__ us,
                             const int32_t* __restrict__ is, int64_t n, int64_t U, int64_t I,
                             double* __restrict__ out, int32_t* __restrict__ err) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = us[x], i = is[x];
    if (u < 0 || u >= U || i < 0 || i >= I) {
      atomicOr(err, 1);
      out[x] = 0.0;
      continue;
    }
    const double* p = a.P + u * a.k;
    const double* q = a.Q + i * a.k;
    double dot = 0.0;
    for (int f = 0; f < a.k; ++f) dot = dot + q[f] * p[f];
    double est;
    if (model == 0)
      est = a.variant ? ((a.gm + a.bu[u]) + a.bi[i]) + dot : dot;
    else
      est = a.variant == 2 ? (a.bu[u] + a.bi[i]) + dot : dot;
    out[x] = est;
  }
}

hipError_t epoch(const Args& a, int model, hipStream_t s) {
  if (a.levels <= 0) return hipSuccess;
  const int g = (a.k + kPerLane - 1) / kPerLane;  // lanes per sample
#define MF_LAUNCH(G_)                                                        \
  {                                                                          \
    if (model == 0) k_mf_epoch<0, G_><<<1, kThreads, 0, s>>>(a);             \
    else k_mf_epoch<1, G_><<<1, kThreads, 0, s>>>(a);                        \
  }
  if (g <= 1) MF_LAUNCH(1)
  else if (g <= 2) MF_LAUNCH(2)
  else if (g <= 4) MF_LAUNCH(4)
  else if (g <= 8) MF_LAUNCH(8)
  else if (g <= 16) MF_LAUNCH(16)
  else if (g <= 32) MF_LAUNCH(32)
  else if (g <= 64) MF_LAUNCH(64)
  else return hipErrorInvalidValue;  // k > 1024
#undef MF_LAUNCH
  return hipGetLastError();
}

hipError_t predict(const Args& a, int model, const int32_t* us, const int32_t* is, int64_t n,
                   int64_t U, int64_t I, double* out, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  k_mf_predict<<<(unsigned)blocks, 256, 0, s>>>(a, model, us, is, n, U, I, out, err);
  return hipGetLastError();
}

}  // namespace mf
}  // namespace bprmf
