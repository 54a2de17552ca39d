// mf.hip — gfx950 kernels of the rating-SGD path (include/mf.h): the reference's Cython SVD,
// RSVD and SVDpp epochs (util/matrix_factorization.pyx:128-151, :40-61, :226-262), bit-identical
// in double.
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


// SVDpp.fit (:226-262), one sample after another: each sample reads the implicit rows y_j of all
// the items its user rated and writes them back, so two samples conflict whenever their users
// share an item and no parallel schedule keeps the reference's order.  One workgroup runs the
// samples in train order; within a sample it stages the user's y rows (and y / sqrt|Iu|, divided
// in parallel) in LDS in one round of loads, then
//   impl[f] = sum_j y[j,f] / sqrt|Iu|   thread f, j in the user's order (from LDS)
//   prod[f] = qi[f] (pu[f] + impl[f])   thread f; thread 0 adds them in factor order -> err
//   pu, qi updates                      thread f, values before the update
//   y[j,f] += lr_yj (err qi[f] / sqrt|Iu| - reg_yj y[j,f])   thread (j, f), from the staged rows
// A user whose list holds an item twice updates the staged rows sequentially per f, every position
// through the slot of its item's first occurrence (each thread owns its f, so the second update of
// a row sees the first); beyond one stage, the same through global memory.  Rows longer than the LDS
// stage are processed in chunks, in order.
constexpr int kStage = 7680;  // doubles of y staged per chunk (60 KB, and as many divided)
constexpr int kList = 2048;   // items of the user's list staged per chunk
// Thread t works on factor f = t % k of rows q = t / k, t / k + RS, ... (RS = 1024 / k rows at a
// time), four rows' loads in flight.
template <bool DIV>
static __device__ __forceinline__ void svdpp_stage(const Args& a, const int32_t* __restrict__ items,
                                                   int rows, double sqrt_Iu, double* ysh,
                                                   double* ydv) {
  const int k = a.k, t = threadIdx.x, RS = kThreads / k, f = t % k, q0 = t / k;
  if (q0 >= RS) return;
  int q = q0;
  for (; q + 3 * RS < rows; q += 4 * RS) {
    double y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = a.Y[(int64_t)items[q + j * RS] * k + f];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ysh[(q + j * RS) * k + f] = y[j];
      if (DIV) ydv[(q + j * RS) * k + f] = y[j] / sqrt_Iu;
    }
  }
  for (; q < rows; q += RS) {
    const double y = a.Y[(int64_t)items[q] * k + f];
    ysh[q * k + f] = y;
    if (DIV) ydv[q * k + f] = y / sqrt_Iu;
  }
}

__global__ __launch_bounds__(kThreads) void k_svdpp_epoch(Args a, int64_t n) {
  __shared__ double ysh[kStage], ydv[kStage];  // y rows of the chunk, and y / sqrt|Iu|
  __shared__ double impl[kThreads], prod[kThreads];
  __shared__ int32_t lst[kList], lslot[kList];
  __shared__ double sh_err;
  const int k = a.k, t = threadIdx.x;
  const int rows_per = min(kStage / k, kList);  // >= 8 for k <= 1024
  const int RS = kThreads / k, f_of = t % k, q_of = t / k;
  for (int64_t s = 0; s < n; ++s) {
    const int64_t u = a.su[s], i = a.si[s];
    const double r = a.sr[s];
    const int beg = a.uoff[u], end = a.uoff[u + 1], cnt = end - beg;
    const double sqrt_Iu = sqrt((double)cnt);
    double puf = 0.0, qif = 0.0;
    if (t < k) {
      puf = a.P[u * k + t];
      qif = a.Q[i * k + t];
    }
    // impl[f] = sum_j y[j,f] / sqrt|Iu|: the divisions in parallel while staging, then thread f
    // adds them in list order
    double acc = 0.0;
    const bool one_chunk = cnt <= rows_per;
    for (int c0 = 0; c0 < cnt; c0 += rows_per) {
      const int rows = min(cnt, c0 + rows_per) - c0;
      for (int x = t; x < rows; x += kThreads) lst[x] = a.uitems[beg + c0 + x];
      __syncthreads();
      svdpp_stage<true>(a, lst, rows, sqrt_Iu, ysh, ydv);
      __syncthreads();
      if (t < k) {
        int q = 0;
        for (; q + 8 <= rows; q += 8) {
          double v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = ydv[(q + j) * k + t];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc = acc + v[j];
        }
        for (; q < rows; ++q) acc = acc + ydv[q * k + t];
      }
      if (!one_chunk) __syncthreads();  // the next chunk overwrites the stage
    }
    if (t < k) {
      impl[t] = acc;
      prod[t] = qif * (puf + acc);
    }
    __syncthreads();
    if (t == 0) {
      double dot = 0.0;
      int f = 0;
      for (; f + 16 <= k; f += 16) {
        double v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = prod[f + j];
#pragma unroll
        for (int j = 0; j < 16; ++j) dot = dot + v[j];
      }
      for (; f < k; ++f) dot = dot + prod[f];
      const double b_u = a.bu[u], b_i = a.bi[i];
      const double err = r - (((a.gm + b_u) + b_i) + dot);
      a.bu[u] = b_u + a.lr[0] * (err - a.reg[0] * b_u);
      a.bi[i] = b_i + a.lr[1] * (err - a.reg[1] * b_i);
      sh_err = err;
    }
    __syncthreads();
    const double err = sh_err;
    if (t < k) {
      a.P[u * k + t] = puf + a.lr[2] * (err * qif - a.reg[2] * puf);
      a.Q[i * k + t] = qif + a.lr[3] * (err * (puf + impl[t]) - a.reg[3] * qif);
      prod[t] = err * qif / sqrt_Iu;  // the y update's gradient term of factor f (:261)
    }
    __syncthreads();
    if (a.udup[u] && one_chunk) {
      // the list holds an item twice: thread f applies the updates in list order to the staged
      // rows, each position through the slot of its item's first occurrence, then the first
      // occurrences go back to memory
      for (int x = t; x < cnt; x += kThreads) lslot[x] = a.uslot[beg + x];
      __syncthreads();
      if (t < k)
        for (int q = 0; q < cnt; ++q) {
          double* y = ysh + lslot[q] * k + t;
          *y = *y + a.lr_yj * (prod[t] - a.reg_yj * *y);
        }
      __syncthreads();
      if (q_of < RS)
        for (int q = q_of; q < cnt; q += RS)
          if (lslot[q] == q) a.Y[(int64_t)lst[q] * k + f_of] = ysh[q * k + f_of];
    } else if (a.udup[u]) {  // (longer lists) sequential per f through global memory
      if (t < k)
        for (int q = 0; q < cnt; ++q) {
          double* y = a.Y + (int64_t)a.uitems[beg + q] * k + t;
          *y = *y + a.lr_yj * (prod[t] - a.reg_yj * *y);
        }
    } else {
      for (int c0 = 0; c0 < cnt; c0 += rows_per) {
        const int rows = min(cnt, c0 + rows_per) - c0;
        if (!one_chunk) {
          __syncthreads();
          for (int x = t; x < rows; x += kThreads) lst[x] = a.uitems[beg + c0 + x];
          __syncthreads();
          svdpp_stage<false>(a, lst, rows, sqrt_Iu, ysh, ydv);
          __syncthreads();
        }
        if (q_of < RS) {
          const double g = prod[f_of];
          for (int q = q_of; q < rows; q += RS) {
            const double y = ysh[q * k + f_of];
            a.Y[(int64_t)lst[q] * k + f_of] = y + a.lr_yj * (g - a.reg_yj * y);
          }
        }
      }
    }
    __threadfence_block();  // this sample's writes before the next sample's reads
    __syncthreads();
  }
}

// SVDpp.predict (:274-287) for n pairs: gm + bu + bi + qi . (pu + sum_j y_j / sqrt|Iu|), the
// implicit sum in list order then divided (numpy's dot may sum in another order)
__global__ void k_svdpp_predict(Args a, const int32_t* __restrict__ us, const int32_t* __restrict__ is,
                                int64_t n, int64_t U, int64_t I, double* __restrict__ out,
                                int32_t* __restrict__ err) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = us[x], i = is[x];
    if (u < 0 || u >= U || i < 0 || i >= I) {
      atomicOr(err, 1);
      out[x] = 0.0;
      continue;
    }
    const int beg = a.uoff[u], cnt = a.uoff[u + 1] - beg;
    const double sq = sqrt((double)cnt);
    double dot = 0.0;
    for (int f = 0; f < a.k; ++f) {
      double impl = 0.0;
      for (int q = 0; q < cnt; ++q) impl = impl + a.Y[(int64_t)a.uitems[beg + q] * a.k + f];
      if (cnt) impl = impl / sq;
      dot = dot + a.Q[i * a.k + f] * (a.P[u * a.k + f] + impl);
    }
    out[x] = (a.gm + (a.bu[u] + a.bi[i])) + dot;  // est = gm; est += bu + bi; est += dot
  }
}

hipError_t epoch(const Args& a, int model, hipStream_t s) {
  if (model == 2) {
    if (a.levels <= 0) return hipSuccess;
    if (a.k > kThreads) return hipErrorInvalidValue;
    k_svdpp_epoch<<<1, kThreads, 0, s>>>(a, a.levels);
    return hipGetLastError();
  }
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
  if (model == 2)
    k_svdpp_predict<<<(unsigned)blocks, 256, 0, s>>>(a, us, is, n, U, I, out, err);
  else
    k_mf_predict<<<(unsigned)blocks, 256, 0, s>>>(a, model, us, is, n, U, I, out, err);
  return hipGetLastError();
}

}  // namespace mf
}  // namespace bprmf
