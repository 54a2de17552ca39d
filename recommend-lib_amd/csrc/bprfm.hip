// bprfm.hip — gfx950 kernels of the BPR-FM training step (include/bprfm.h), SURVEY.md §8f row 4:
// the reference's BPRFM model (BPRFMRecommender.py:28-79) trained by its loop (:203-227).
//
// Per triplet (u, i, j) of FEATURE indices each side is two features [u, x] with values 1
// (BPRFMData, util/data_loader.py:574-627: the user feature is shared by both sides):  fm = 0.5 ((e_u + e_x)^2 - (e_u^2 + e_x^2)) (Bi-Interaction),
// y = BatchNorm1d(fm) in training mode (batch statistics, a separate call per side) and Dropout(p),
// pred = sum_k y + b_u + b_x + bias_.  loss = -sum log sigmoid(pred_i - pred_j); Adagrad over
// every parameter (a row whose gradient is zero keeps its value and accumulator exactly, so only
// the batch's rows are touched).
//
// Layout: G lanes per triplet (G = next_pow2(k) <= 64), one factor per lane; TPB = 256 / G
// triplets per workgroup.  Kernels of one step (BN on):
//   k_fm_fwd    fm rows of both sides -> X; per-workgroup sums of fm and fm^2 (double; at most
//               256 workgroups striding over the batch)
//   k_fm_stats  batch mean / 1/sqrt(var + eps) per side (fixed-order sum of the partials, one
//               workgroup per 4 factors), and the running statistics (momentum 0.1, unbiased variance; i side,
//               then j side)
//   k_fm_mid    y, dropout, pred, c = sigmoid(-(pred_i - pred_j)); per-workgroup sums of gy and
//               gy * xhat per side (the BatchNorm backward's batch terms)
//   k_fm_stats2 fixed-order sums of those; dgamma, dbeta
//   k_fm_back   BatchNorm and Bi-Interaction backward, gradient rows added into G (f32 atomics)
//   k_fm_apply  Adagrad on every touched row (small tables: a sweep over the rows the backward
//               stamped; else claimed once per step by swapping its stamp), G re-zeroed;
//               gamma / beta; the step's loss (workgroup 0)
// BN off: k_fm_plain computes pred and the backward itself, then k_fm_apply.
// The user feature's bias enters pred_i and pred_j with one value, so its gradient is exactly
// zero (the reference's autograd cancels it exactly too): nothing is added to it, and Adagrad on a
// zero gradient leaves the value exactly; bias_ likewise is never touched.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "bprfm_kernels.h"
#include "device_common.h"

namespace bprmf {
namespace fm {

constexpr int kT = 256;  // threads per workgroup
constexpr uint32_t TAG_DROP = 0x44520000u;

// keep-mask of dropout for (step, triplet, side, factor): 1 / (1 - p) or 0
static __device__ __forceinline__ float drop_scale(const Args& a, int t, int side, int e) {
  if (a.p <= 0.f) return 1.f;
  uint32_t c0 = (uint32_t)t, c1 = (uint32_t)a.step, c2 = (uint32_t)(side * 1024 + e), c3 = TAG_DROP;
  philox10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  const float r = (float)(c0 >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  return r >= a.p ? 1.f / (1.f - a.p) : 0.f;
}

template <int G>
static __device__ __forceinline__ float gsum(float v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// fixed-shape LDS tree over the workgroup's TPB triplets of NV per-factor values (double)
template <int G, int NV>
static __device__ __forceinline__ void block_sums(double (&v)[NV], double* __restrict__ out,
                                                  int ld) {
  constexpr int TPB = kT / G;
  __shared__ double red[NV][TPB][G];
  const int lane = threadIdx.x & (G - 1), slot = threadIdx.x / G;
#pragma unroll
  for (int q = 0; q < NV; ++q) red[q][slot][lane] = v[q];
  __syncthreads();
#pragma unroll
  for (int half = TPB / 2; half >= 1; half >>= 1) {
    if (slot < half) {
#pragma unroll
      for (int q = 0; q < NV; ++q) red[q][slot][lane] += red[q][slot + half][lane];
    }
    __syncthreads();
  }
  if (slot == 0) {
#pragma unroll
    for (int q = 0; q < NV; ++q) out[(int64_t)q * ld + lane] = red[q][0][lane];
  }
}

// the Bi-Interaction backward: fm = 0.5 ((a + c)^2 - (a^2 + c^2)) -> d/da = gfm (s - a)
static __device__ __forceinline__ void add_row(float* __restrict__ G, int64_t row, int ld, int e,
                                               float v) {
  atomicAdd(G + row * ld + e, v);
}

// BN off: the whole step's forward and backward, one lane group per triplet
template <int G>
__global__ __launch_bounds__(kT) void k_fm_plain(Args a) {
  constexpr int TPB = kT / G;
  const int lane = threadIdx.x & (G - 1);
  const int t = blockIdx.x * TPB + threadIdx.x / G;
  const bool act = t < a.B && lane < a.k;
  int64_t u = 0, xi = 0, xj = 0;
  if (t < a.B) {
    u = a.u[t];
    xi = a.i[t];
    xj = a.j[t];
  }
  float eu = 0.f, ei = 0.f, ej = 0.f;
  if (act) {
    eu = a.E[u * a.ld + lane];
    ei = a.E[xi * a.ld + lane];
    ej = a.E[xj * a.ld + lane];
  }
  const float si = eu + ei, sj = eu + ej;
  const float fi = 0.5f * (si * si - (eu * eu + ei * ei));
  const float fj = 0.5f * (sj * sj - (eu * eu + ej * ej));
  const float mi = act ? drop_scale(a, t, 0, lane) : 0.f, mj = act ? drop_scale(a, t, 1, lane) : 0.f;
  const float yi = gsum<G>(act ? fi * mi : 0.f), yj = gsum<G>(act ? fj * mj : 0.f);
  float c = 0.f;
  if (t < a.B) {
    const float bu = a.b[u];
    const float pi = (yi + (bu + a.b[xi])) + *a.bias_;
    const float pj = (yj + (bu + a.b[xj])) + *a.bias_;
    const float d = pi - pj;
    c = 1.0f / (1.0f + expf(d));  // sigmoid(-d)
    if (lane == 0) {
      a.cbuf[t] = d;
      add_row(a.Gb, xi, 1, 0, -c);
      add_row(a.Gb, xj, 1, 0, c);
      if (a.sweep) a.stamp[u] = a.stamp[xi] = a.stamp[xj] = a.step + 1;
    }
  }
  if (act) {
    const float gi = -c * mi, gj = c * mj;  // dL/dfm per side
    add_row(a.GE, u, a.ld, lane, gi * (si - eu) + gj * (sj - eu));
    add_row(a.GE, xi, a.ld, lane, gi * (si - ei));
    add_row(a.GE, xj, a.ld, lane, gj * (sj - ej));
  }
}

// BN on, pass 1: fm rows of both sides -> X; per-workgroup sums of fm and fm^2 (double).  nb
// workgroups stride over the batch, so the statistics kernel sums few partials.
template <int G>
__global__ __launch_bounds__(kT) void k_fm_fwd(Args a, int nb) {
  constexpr int TPB = kT / G;
  const int lane = threadIdx.x & (G - 1), slot = threadIdx.x / G;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  if (lane < a.k) {
    for (int t = blockIdx.x * TPB + slot; t < a.B; t += nb * TPB) {
      const int64_t u = a.u[t], xi = a.i[t], xj = a.j[t];
      const float eu = a.E[u * a.ld + lane], ei = a.E[xi * a.ld + lane], ej = a.E[xj * a.ld + lane];
      const float si = eu + ei, sj = eu + ej;
      const float fi = 0.5f * (si * si - (eu * eu + ei * ei));
      const float fj = 0.5f * (sj * sj - (eu * eu + ej * ej));
      a.X[(int64_t)t * a.ld + lane] = fi;
      a.X[((int64_t)a.B + t) * a.ld + lane] = fj;
      v[0] += fi;
      v[1] += (double)fi * fi;
      v[2] += fj;
      v[3] += (double)fj * fj;
    }
  }
  block_sums<G, 4>(v, a.part + (int64_t)blockIdx.x * 4 * a.ld, a.ld);
}

// fixed-order sums of the 4 per-workgroup partial rows over nblk (<= kMaxParts) workgroups.
// Workgroup w of ceil(ld / 4) sums factors 4w..4w+3: thread = (pair p = (q, e) of 16, chunk c of
// 64); chunk c holds partials c, c + 64, ... (8 loads issued together), then an LDS tree over the
// chunks.  sums[q][e - 4w] for e < k on return.
constexpr int kRT = 1024;
constexpr int kMaxParts = 256;
static __device__ void reduce_parts(const Args& a, int nblk, double (*sums)[4]) {
  __shared__ double red[64][16];
  const int p = threadIdx.x & 15, c = threadIdx.x >> 4;
  const int q = p >> 2, e = blockIdx.x * 4 + (p & 3);
  double x[kMaxParts / 64];
#pragma unroll
  for (int m = 0; m < kMaxParts / 64; ++m) {
    const int b = c + 64 * m;
    x[m] = (b < nblk && e < a.ld) ? a.part[((int64_t)b * 4 + q) * a.ld + e] : 0.0;
  }
  double v = 0.0;
#pragma unroll
  for (int m = 0; m < kMaxParts / 64; ++m) v += x[m];
  red[c][p] = v;
  __syncthreads();
#pragma unroll
  for (int h = 32; h >= 1; h >>= 1) {
    if (c < h) red[c][p] += red[c + h][p];
    __syncthreads();
  }
  if (threadIdx.x < 16) sums[q][p & 3] = red[0][p];
  __syncthreads();
}

// batch statistics of both sides + running statistics
__global__ __launch_bounds__(kRT) void k_fm_stats(Args a, int nblk) {
  __shared__ double sums[4][4];
  reduce_parts(a, nblk, sums);
  const int el = threadIdx.x, e = blockIdx.x * 4 + el;
  if (el >= 4 || e >= a.k) return;
  double rm = a.run[e], rv = a.run[a.ld + e];
  for (int side = 0; side < 2; ++side) {
    const double mean = sums[2 * side][el] / a.B;
    const double var = fmax(sums[2 * side + 1][el] / a.B - mean * mean, 0.0);  // biased
    a.stats[(2 * side) * a.ld + e] = (float)mean;
    a.stats[(2 * side + 1) * a.ld + e] = (float)(1.0 / sqrt(var + 1e-5));
    // running statistics, i side then j side (the forward calls FM_layers twice, :56-57)
    const double vu = a.B > 1 ? var * a.B / (a.B - 1) : var;
    rm = 0.9 * rm + 0.1 * mean;
    rv = 0.9 * rv + 0.1 * vu;
  }
  a.run[e] = (float)rm;
  a.run[a.ld + e] = (float)rv;
}

// BN on, pass 2: y, dropout, pred, d = pred_i - pred_j -> cbuf, c = sigmoid(-d); per-workgroup
// sums of gy and gy * xhat per side (the BatchNorm backward's batch terms)
template <int G>
__global__ __launch_bounds__(kT) void k_fm_mid(Args a, int nb) {
  constexpr int TPB = kT / G;
  const int lane = threadIdx.x & (G - 1), slot = threadIdx.x / G;
  const bool act = lane < a.k;
  float ga = 0.f, be = 0.f, mu[2] = {0.f, 0.f}, inv[2] = {0.f, 0.f};
  if (act) {
    ga = a.gamma[lane];
    be = a.beta[lane];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      mu[sd] = a.stats[(2 * sd) * a.ld + lane];
      inv[sd] = a.stats[(2 * sd + 1) * a.ld + lane];
    }
  }
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  double lsum = 0.0;  // this lane group's loss terms (lane 0)
  for (int t = blockIdx.x * TPB + slot; t < a.B; t += nb * TPB) {  // uniform per lane group
    const int64_t u = a.u[t], xi = a.i[t], xj = a.j[t];
    float xh[2] = {0.f, 0.f}, m[2] = {0.f, 0.f}, yv[2] = {0.f, 0.f};
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      if (act) {
        const float x = a.X[((int64_t)sd * a.B + t) * a.ld + lane];
        xh[sd] = (x - mu[sd]) * inv[sd];
        m[sd] = drop_scale(a, t, sd, lane);
        yv[sd] = (ga * xh[sd] + be) * m[sd];
      }
    }
    const float yi = gsum<G>(yv[0]), yj = gsum<G>(yv[1]);
    const float bu = a.b[u];
    const float pi = (yi + (bu + a.b[xi])) + *a.bias_;
    const float pj = (yj + (bu + a.b[xj])) + *a.bias_;
    const float d = pi - pj;
    const float c = 1.0f / (1.0f + expf(d));
    if (lane == 0) {
      a.cbuf[t] = d;
      lsum += (double)(fmaxf(-d, 0.f) + __logf(1.0f + __expf(-fabsf(d))));  // softplus(-d), fast exp / log
    }
    // dL/dy = -c (i side), +c (j side), through the dropout mask
    const float gi = act ? -c * m[0] : 0.f, gj = act ? c * m[1] : 0.f;
    v[0] += gi;
    v[1] += (double)gi * xh[0];
    v[2] += gj;
    v[3] += (double)gj * xh[1];
  }
  block_sums<G, 4>(v, a.part + (int64_t)blockIdx.x * 4 * a.ld, a.ld);
  // the workgroup's loss, its lane groups in slot order -> lpart (k_fm_stats2 adds those)
  __shared__ double lred[TPB];
  if (lane == 0) lred[slot] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int q = 0; q < TPB; ++q) s += lred[q];
    a.lpart[blockIdx.x] = s;
  }
}

// the step's loss from k_fm_mid's per-workgroup sums, fixed order (workgroup 0 of k_fm_stats2)
static __device__ void loss_parts(const Args& a, int nblk) {
  __shared__ double lr2[kRT];
  lr2[threadIdx.x] = (int)threadIdx.x < nblk ? a.lpart[threadIdx.x] : 0.0;
  __syncthreads();
  for (int h = kRT / 2; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) lr2[threadIdx.x] += lr2[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.loss[0] += lr2[0];
}

// sums of gy and gy * xhat per side; dgamma / dbeta (the module serves both sides)
__global__ __launch_bounds__(kRT) void k_fm_stats2(Args a, int nblk) {
  __shared__ double sums[4][4];
  if (blockIdx.x == 0) loss_parts(a, nblk);  // (block-uniform)
  reduce_parts(a, nblk, sums);
  const int el = threadIdx.x, e = blockIdx.x * 4 + el;
  if (el >= 4 || e >= a.k) return;
  for (int w = 0; w < 4; ++w) a.stats2[w * a.ld + e] = (float)sums[w][el];
  a.gbeta[e] = (float)(sums[0][el] + sums[2][el]);
  a.ggamma[e] = (float)(sums[1][el] + sums[3][el]);
}


template <int G>
__global__ __launch_bounds__(kT) void k_fm_back(Args a) {
  constexpr int TPB = kT / G;
  const int lane = threadIdx.x & (G - 1);
  const int t = blockIdx.x * TPB + threadIdx.x / G;
  if (t >= a.B || lane >= a.k) return;
  const int64_t u = a.u[t], xi = a.i[t], xj = a.j[t];
  const float eu = a.E[u * a.ld + lane], ei = a.E[xi * a.ld + lane], ej = a.E[xj * a.ld + lane];
  const float d = a.cbuf[t];
  const float c = 1.0f / (1.0f + expf(d));
  const float ga = a.gamma[lane];
  float gfm[2];
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
    const float x = a.X[((int64_t)sd * a.B + t) * a.ld + lane];
    const float inv = a.stats[(2 * sd + 1) * a.ld + lane];
    const float xh = (x - a.stats[(2 * sd) * a.ld + lane]) * inv;
    const float gy = (sd == 0 ? -c : c) * drop_scale(a, t, sd, lane);
    const float dxh = gy * ga;
    const float mdx = ga * a.stats2[(2 * sd) * a.ld + lane] / a.B;      // mean of dxhat
    const float mdxx = ga * a.stats2[(2 * sd + 1) * a.ld + lane] / a.B;  // mean of dxhat * xhat
    gfm[sd] = inv * (dxh - mdx - xh * mdxx);
  }
  const float si = eu + ei, sj = eu + ej;
  add_row(a.GE, u, a.ld, lane, gfm[0] * (si - eu) + gfm[1] * (sj - eu));
  add_row(a.GE, xi, a.ld, lane, gfm[0] * (si - ei));
  add_row(a.GE, xj, a.ld, lane, gfm[1] * (sj - ej));
  if (lane == 0) {
    add_row(a.Gb, xi, 1, 0, -c);
    add_row(a.Gb, xj, 1, 0, c);
    if (a.sweep) a.stamp[u] = a.stamp[xi] = a.stamp[xj] = a.step + 1;
  }
}

// loss of the step from the stored d = pred_i - pred_j: sum of log(1 + e^-d), fixed order (one
// workgroup; each thread issues its 16 loads of a round together)
static __device__ void loss_sum(const Args& a) {
  constexpr int R = 16;
  __shared__ double red[kT];
  double s = 0.0;
  for (int t0 = 0; t0 < a.B; t0 += kT * R) {
    float d[R];
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const int t = t0 + m * kT + threadIdx.x;
      d[m] = t < a.B ? a.cbuf[t] : INFINITY;  // softplus(-inf) = 0
    }
#pragma unroll
    for (int m = 0; m < R; ++m) s += (double)softplus(-d[m]);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = kT / 2; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.loss[0] += red[0];
}

// Adagrad (torch _single_tensor_adagrad: acc += g^2; p += -lr * (g / (sqrt(acc) + 1e-10))) on one
// row and its bias, G re-zeroed
template <int G>
static __device__ __forceinline__ void adagrad_row(const Args& a, int64_t row, int lane) {
  if (lane < a.k) {
    const int64_t o = row * a.ld + lane;
    const float g = a.GE[o];
    a.GE[o] = 0.f;
    const float acc = a.acc_E[o] + g * g;
    a.acc_E[o] = acc;
    a.E[o] += -a.lr * (g / (sqrtf(acc) + 1e-10f));
  }
  if (lane == 0) {  // feature bias (a user feature's gradient is exactly zero: value kept)
    const float g = a.Gb[row];
    a.Gb[row] = 0.f;
    const float acc = a.acc_b[row] + g * g;
    a.acc_b[row] = acc;
    a.b[row] += -a.lr * (g / (sqrtf(acc) + 1e-10f));
  }
}

// every touched row once.  sweep: one lane group per feature row, applied if the backward stamped
// it this step (small tables: no atomics); otherwise one lane group per row reference (3 per
// triplet), the first to swap its stamp applies it.  Workgroup 0 also does gamma / beta and the
// loss.
template <int G>
__global__ __launch_bounds__(kT) void k_fm_apply(Args a) {
  constexpr int TPB = kT / G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x / G;
  if (blockIdx.x == 0 && !a.bn) loss_sum(a);  // (BN on: k_fm_mid / k_fm_stats2 sum it)
  if (blockIdx.x == 0 && a.bn && threadIdx.x < a.k) {  // gamma, beta
    const int e = threadIdx.x;
    const float g1 = a.ggamma[e], g2 = a.gbeta[e];
    a.acc_gamma[e] += g1 * g1;
    a.gamma[e] += -a.lr * (g1 / (sqrtf(a.acc_gamma[e]) + 1e-10f));
    a.acc_beta[e] += g2 * g2;
    a.beta[e] += -a.lr * (g2 / (sqrtf(a.acc_beta[e]) + 1e-10f));
  }
  if (a.sweep) {
    if (r >= a.F || a.stamp[r] != a.step + 1) return;
    adagrad_row<G>(a, r, lane);
    return;
  }
  if (r >= 3LL * a.B) return;
  const int64_t t = r / 3, w = r % 3;
  const int64_t row = w == 0 ? a.u[t] : w == 1 ? a.i[t] : a.j[t];
  int32_t old = 0;
  if (lane == 0) old = atomicExch(a.stamp + row, a.step + 1);
  old = __shfl(old, (threadIdx.x & 63) & ~(G - 1));
  if (old == a.step + 1) return;  // another reference of this row applies it
  adagrad_row<G>(a, row, lane);
}

// pred for n (u, x) pairs in eval mode (BatchNorm on the running statistics, no dropout)
__global__ void k_fm_predict(Args a, const int32_t* __restrict__ us, const int32_t* __restrict__ xs,
                             int64_t n, float* __restrict__ out) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = us[q], x = xs[q];
    float acc = 0.f;
    for (int e = 0; e < a.k; ++e) {
      const float eu = a.E[u * a.ld + e], ex = a.E[x * a.ld + e];
      const float s = eu + ex;
      float f = 0.5f * (s * s - (eu * eu + ex * ex));
      if (a.bn) f = a.gamma[e] * (f - a.run[e]) / sqrtf(a.run[a.ld + e] + 1e-5f) + a.beta[e];
      acc += f;
    }
    out[q] = (acc + (a.b[u] + a.b[x])) + *a.bias_;
  }
}

// nn.init.normal_(embeddings, std) on the device: Philox + Box-Muller per (row, factor); padding 0
__global__ void k_fm_init(float* __restrict__ E, int64_t F, int k, int ld, float std_,
                          uint64_t seed) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < F * ld;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = x / ld;
    const int e = (int)(x % ld);
    float v = 0.f;
    if (e < k) {
      uint32_t c0 = (uint32_t)row, c1 = (uint32_t)(row >> 32), c2 = (uint32_t)e, c3 = 0x494e4954u;
      philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
      const float r1 = ((c0 >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
      const float r2 = (c1 >> 8) * (1.0f / 16777216.0f);
      v = std_ * sqrtf(-2.f * logf(r1)) * cospif(2.f * r2);
    }
    E[x] = v;
  }
}

// the dropout keep-scales a step would draw: out [2, B, k] (tests replay them in the oracle)
__global__ void k_fm_mask(Args a, float* __restrict__ out) {
  const int64_t n = 2LL * a.B * a.k;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(x % a.k);
    const int t = (int)((x / a.k) % a.B);
    const int sd = (int)(x / ((int64_t)a.k * a.B));
    out[x] = drop_scale(a, t, sd, e);
  }
}

#define FM_G(k_, BODY)                                         \
  do {                                                         \
    const int g_ = (k_) <= 1 ? 1 : (k_) <= 2 ? 2 : (k_) <= 4 ? 4 : (k_) <= 8 ? 8 : (k_) <= 16 ? 16 : (k_) <= 32 ? 32 : 64; \
    switch (g_) {                                              \
      case 1: { constexpr int G_ = 1; BODY; } break;           \
      case 2: { constexpr int G_ = 2; BODY; } break;           \
      case 4: { constexpr int G_ = 4; BODY; } break;           \
      case 8: { constexpr int G_ = 8; BODY; } break;           \
      case 16: { constexpr int G_ = 16; BODY; } break;         \
      case 32: { constexpr int G_ = 32; BODY; } break;         \
      default: { constexpr int G_ = 64; BODY; } break;         \
    }                                                          \
  } while (0)

int lanes_for(int k) {
  int g = 1;
  while (g < k) g <<= 1;
  return g;
}

// workgroups of the BatchNorm passes: the batch's lane groups, at most kMaxParts workgroups
int64_t part_blocks(int k, int B) {
  const int64_t tpb = kT / lanes_for(k);
  return std::max<int64_t>(1, std::min<int64_t>(((int64_t)B + tpb - 1) / tpb, kMaxParts));
}

hipError_t step(const Args& a, hipStream_t s) {
  if (a.k <= 0 || a.k > 64 || a.B <= 0) return hipErrorInvalidValue;
  const int64_t tpb = kT / lanes_for(a.k);
  const unsigned nt = (unsigned)((a.B + tpb - 1) / tpb);      // one lane group per triplet
  const int64_t napply = a.sweep ? a.F : 3LL * a.B;  // feature rows, or row references
  const unsigned na = (unsigned)((napply + tpb - 1) / tpb);
  const int nb = (int)part_blocks(a.k, a.B);
  const unsigned nr = (unsigned)((a.ld + 3) / 4);  // reduce workgroups: 4 factors each
  FM_G(a.k, ({
    if (a.bn) {
      k_fm_fwd<G_><<<nb, kT, 0, s>>>(a, nb);
      k_fm_stats<<<nr, kRT, 0, s>>>(a, nb);
      k_fm_mid<G_><<<nb, kT, 0, s>>>(a, nb);
      k_fm_stats2<<<nr, kRT, 0, s>>>(a, nb);
      k_fm_back<G_><<<nt, kT, 0, s>>>(a);
    } else {
      k_fm_plain<G_><<<nt, kT, 0, s>>>(a);
    }
    k_fm_apply<G_><<<na, kT, 0, s>>>(a);
  }));
  return hipGetLastError();
}

hipError_t init_normal(float* E, int64_t F, int k, int ld, float std_, uint64_t seed,
                       hipStream_t s) {
  if (F <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((F * ld + 255) / 256, 8192);
  k_fm_init<<<(unsigned)blocks, 256, 0, s>>>(E, F, k, ld, std_, seed);
  return hipGetLastError();
}

hipError_t dropout_mask(const Args& a, float* out, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((2LL * a.B * a.k + 255) / 256, 8192);
  k_fm_mask<<<(unsigned)blocks, 256, 0, s>>>(a, out);
  return hipGetLastError();
}

hipError_t predict(const Args& a, const int32_t* us, const int32_t* xs, int64_t n, float* out,
                   hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  k_fm_predict<<<(unsigned)blocks, 256, 0, s>>>(a, us, xs, n, out);
  return hipGetLastError();
}

}  // namespace fm
}  // namespace bprmf
