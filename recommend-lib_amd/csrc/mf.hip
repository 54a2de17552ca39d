// mf.hip — gfx950 kernels of the rating-SGD path (include/mf.h): the reference's Cython SVD and
// RSVD epochs (util/matrix_factorization.pyx:128-151, :40-61), bit-identical in double.
//
// A per-sample SGD epoch is a sequence; sample s can run as soon as the last earlier samples
// touching its user and its item have run.  The host assigns every sample its dependency level
// (mf_capi.cpp) and lays the samples out level by level; one workgroup of 1024 threads walks the
// levels, one thread per sample, with a workgroup barrier between levels (the samples of a level
// touch disjoint rows, and the barrier orders a level's writes before the next level's reads on
// the workgroup's CU).  Each thread evaluates its sample with the reference's operations in the
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

// SVD.fit, one sample (:132-151)
static __device__ __forceinline__ void svd_sample(const Args& a, int64_t s) {
  const int64_t u = a.su[s], i = a.si[s];
  const double r = a.sr[s];
  double* pu = a.P + u * a.k;
  double* qi = a.Q + i * a.k;
  double dot = 0.0;
  for (int f = 0; f < a.k; ++f) dot = dot + qi[f] * pu[f];
  const double err = r - (((a.gm + a.bu[u]) + a.bi[i]) + dot);
  if (a.variant) {
    a.bu[u] = a.bu[u] + a.lr[0] * (err - a.reg[0] * a.bu[u]);
    a.bi[i] = a.bi[i] + a.lr[1] * (err - a.reg[1] * a.bi[i]);
  }
  for (int f = 0; f < a.k; ++f) {
    const double puf = pu[f], qif = qi[f];
    pu[f] = puf + a.lr[2] * (err * qif - a.reg[2] * puf);
    qi[f] = qif + a.lr[3] * (err * puf - a.reg[3] * qif);
  }
}

// RSVD.fit, one sample (:42-61)
static __device__ __forceinline__ void rsvd_sample(const Args& a, int64_t s) {
  const int64_t i = a.su[s], j = a.si[s];
  const double r = a.sr[s];
  double* ui = a.P + i * a.k;
  double* vj = a.Q + j * a.k;
  double dot = 0.0;
  for (int f = 0; f < a.k; ++f) dot = dot + ui[f] * vj[f];
  const double err = r - ((a.bu[i] + a.bi[j]) + dot);
  const double lr = a.lr[0], reg = a.reg[0], reg2 = a.reg[1];
  if (a.variant == 2) {
    const double cii = a.bu[i], djj = a.bi[j];
    a.bu[i] = cii + lr * (err - reg2 * ((cii + djj) - a.gm));
    a.bi[j] = djj + lr * (err - reg2 * ((cii + djj) - a.gm));
  }
  for (int f = 0; f < a.k; ++f) {
    const double uik = ui[f], vjk = vj[f];
    ui[f] = uik + lr * (err * vjk - reg * uik);
    vj[f] = vjk + lr * (err * uik - reg * vjk);
  }
}

template <int MODEL>
__global__ __launch_bounds__(kThreads) void k_mf_epoch(Args a) {
  for (int L = 0; L < a.levels; ++L) {
    const int beg = a.loff[L], end = a.loff[L + 1];
    for (int s = beg + (int)threadIdx.x; s < end; s += kThreads) {
      if (MODEL == 0) svd_sample(a, s);
      else rsvd_sample(a, s);
    }
    __threadfence_block();  // this level's row writes before the next level's reads
    __syncthreads();
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
  if (model == 0) k_mf_epoch<0><<<1, kThreads, 0, s>>>(a);
  else k_mf_epoch<1><<<1, kThreads, 0, s>>>(a);
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
