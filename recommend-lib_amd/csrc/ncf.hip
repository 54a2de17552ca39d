// ncf.hip — NCF (GMF / MLP / NeuMF-end) training step on gfx950.
//
// Reference: NCFRecommender.py:27-124 (model), :255-288 (BCEWithLogitsLoss + Adam over every
// parameter with dense gradients), util/data_loader.py:931-972 (NCFData: positives, then num_ng
// negatives per positive, shuffled).
//
//   k_ncf_fwdbwd  one 1024-thread workgroup per 16 samples: embedding gathers into LDS, the MLP
//                 tower forward on f32 MFMA (v_mfma_f32_16x16x4_f32: the 16 samples are the M
//                 dimension of every layer), the prediction and dL/dz, then the tower backward:
//                 dW partial tiles per workgroup (summed in fixed order by the Adam kernel),
//                 dX = dPre . W through the transposed weight copies, and the embedding
//                 gradients as f32 atomics into dense gradient rows.
//   k_ncf_catch_up / k_ncf_adam_rows  torch's dense Adam over the embedding tables, done lazily:
//                 every row with a nonzero moment moves every step, but a step with g = 0 has a
//                 closed form, so a row is brought up to date only when something reads it (the
//                 step that gathers it, a predict, a parameter copy) and Adam proper runs on the
//                 batch's rows alone.  Equal to the dense sweep up to f32 rounding.
//   k_ncf_adam_flat  Adam over the tower + predict layer, g = sum of the workgroups' partials in
//                 workgroup order; weights also written transposed for the next backward.
#include <algorithm>

#include "device_common.h"
#include "ncf_kernels.h"

namespace bprmf {
namespace ncf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// LDS plan of k_ncf_fwdbwd (floats): sample ids / labels / z / dz, GMF rows, tower activations
struct Lds {
  int eu, ei, h[kMaxLayers + 1], misc, total;
  int ldh[kMaxLayers + 1];
};
static __host__ __device__ inline Lds lds_plan(const Dims& D) {
  Lds p{};
  int off = 0;
  p.misc = off;
  off += 4 * kSamples;  // u, i (as float bits), y, z  +  dz reuses z's slot
  p.eu = off;
  off += kSamples * (D.d + 4);
  p.ei = off;
  off += kSamples * (D.d + 4);
  for (int l = 0; l <= D.L; ++l) {
    const int n = l == 0 ? D.nin[0] : D.nout[l - 1];
    p.ldh[l] = n + 4;  // row stride: +4 floats keeps float4 reads of 16 rows conflict-free
    p.h[l] = off;
    off += kSamples * p.ldh[l];
  }
  p.total = off;
  return p;
}

size_t fwdbwd_lds_bytes(const Dims& D) { return sizeof(float) * (size_t)lds_plan(D).total; }

// y[16 x 16 tile] = X[16 x K] (LDS, stride ldx) . W[n0.., :]^T (global, W[n][k], stride K):
// 16x16x4 f32 MFMA, lane group g = l >> 4 takes k = 16t + 4g .. +3 (K % 4 == 0).  The W rows
// come from L2/HBM: eight k-steps of loads are issued before their 32 MFMAs, so one latency is
// paid per eight steps, not per step.
static __device__ __forceinline__ f32x4 tile_xwt(const float* X, int ldx, const float* W, int K,
                                                 int n0, int nmax, int lane) {
  constexpr int U = 8;
  const int r = lane & 15, g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool nok = n0 + r < nmax;
  const float* wr = W + (int64_t)(n0 + r) * K;
  for (int t0 = 0; 16 * t0 < K; t0 += U) {
    float4 a[U], b[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = 16 * (t0 + q) + 4 * g;
      b[q] = (nok && k < K) ? ld4(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = 16 * (t0 + q) + 4 * g;
      a[q] = k < K ? *reinterpret_cast<const float4*>(X + r * ldx + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].x, b[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].y, b[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].z, b[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].w, b[q].w, acc, 0, 0, 0);
    }
  }
  return acc;
}

// BPRMF_NCF_PHASES (diagnostic builds only): workgroup 0 of step 100 prints its phase times
#ifdef BPRMF_NCF_PHASES
#define NCF_PH(k)                                 \
  do {                                            \
    if (threadIdx.x == 0) s_ph[k] = wall_clock64(); \
  } while (0)
#else
#define NCF_PH(k) \
  do {            \
  } while (0)
#endif

__global__ __launch_bounds__(1024) void k_ncf_fwdbwd(Dims D, Params P, Grads G,
                                                     const int32_t* __restrict__ us,
                                                     const int32_t* __restrict__ is,
                                                     const float* __restrict__ ys, int n,
                                                     int32_t t, float* __restrict__ partial,
                                                     double* __restrict__ loss,
                                                     int32_t* __restrict__ err,
                                                     float* __restrict__ zout) {
  extern __shared__ float sm[];
#ifdef BPRMF_NCF_PHASES
  __shared__ uint64_t s_ph[24];
  if (threadIdx.x < 24) s_ph[threadIdx.x] = 0;
  NCF_PH(0);
#endif
  const Lds Lp = lds_plan(D);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = 16;
  const int s0 = blockIdx.x * kSamples;
  int32_t* su = reinterpret_cast<int32_t*>(sm + Lp.misc);
  int32_t* si = su + kSamples;
  float* sy = sm + Lp.misc + 2 * kSamples;
  float* sz = sm + Lp.misc + 3 * kSamples;
  const bool gmf = D.model != kMLP, mlp = D.model != kGMF;
  const int d = D.d, E = D.E;
  // 1. samples
  if (tid < kSamples) {
    const int s = s0 + tid;
    int32_t u = -1, i = -1;
    float y = 0.f;
    if (s < n) {
      u = us[s];
      i = is[s];
      y = ys ? ys[s] : 0.f;
      if ((uint64_t)u >= (uint64_t)D.U || (uint64_t)i >= (uint64_t)D.I) {
        atomicOr(err, 1);
        u = i = -1;
      }
    }
    su[tid] = u;
    si[tid] = i;
    sy[tid] = y;
  }
  __syncthreads();
  NCF_PH(1);
  // 2. gathers (float4): GMF rows and the tower input [Pm[u], Qm[i]]
  if (gmf) {
    const int q = d / 4;
    for (int x = tid; x < kSamples * q; x += blockDim.x) {
      const int s = x / q, c = 4 * (x % q);
      const int32_t u = su[s], i = si[s];
      const float4 a = u >= 0 ? ld4(P.Pg + (int64_t)u * d + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 b = i >= 0 ? ld4(P.Qg + (int64_t)i * d + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(sm + Lp.eu + s * (d + 4) + c) = a;
      *reinterpret_cast<float4*>(sm + Lp.ei + s * (d + 4) + c) = b;
    }
  }
  if (mlp) {
    const int q = 2 * E / 4;
    for (int x = tid; x < kSamples * q; x += blockDim.x) {
      const int s = x / q, c = 4 * (x % q);
      const int32_t u = su[s], i = si[s];
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < E) {
        if (u >= 0) v = ld4(P.Pm + (int64_t)u * E + c);
      } else if (i >= 0) {
        v = ld4(P.Qm + (int64_t)i * E + (c - E));
      }
      *reinterpret_cast<float4*>(sm + Lp.h[0] + s * Lp.ldh[0] + c) = v;
    }
  }
  __syncthreads();
  NCF_PH(2);
  // 3. tower forward: h_l = relu(h_{l-1} W_l^T + b_l)
  if (mlp) {
    for (int l = 0; l < D.L; ++l) {
      const int K = D.nin[l], N = D.nout[l];
      const float* X = sm + Lp.h[l];
      float* Y = sm + Lp.h[l + 1];
      for (int tile = wave; 16 * tile < N; tile += NW) {
        const f32x4 acc = tile_xwt(X, Lp.ldh[l], P.W[l], K, 16 * tile, N, lane);
        const int nn = 16 * tile + (lane & 15);
        if (nn < N) {
          const float bias = P.b[l][nn];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = 4 * (lane >> 4) + r;
            Y[s * Lp.ldh[l + 1] + nn] = fmaxf(acc[r] + bias, 0.f);
          }
        }
      }
      __syncthreads();
      NCF_PH(3 + l);
    }
  }
  // 4. prediction z = [gmf, h_L] . wp + bp and dL/dz of the mean BCE-with-logits loss
  const float* hL = sm + Lp.h[D.L];
  const int ldL = Lp.ldh[D.L];
  if (wave < kSamples) {
    const int s = wave;
    float acc = 0.f;
    for (int k = lane; k < D.pred; k += 64) {
      float x;
      if (gmf && k < d)
        x = sm[Lp.eu + s * (d + 4) + k] * sm[Lp.ei + s * (d + 4) + k];
      else
        x = hL[s * ldL + (k - (gmf ? d : 0))];
      acc = fmaf(x, P.wp[k], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
      const bool ok = su[s] >= 0;
      const float z = acc + P.bp[0];
      if (zout && s0 + s < n) zout[s0 + s] = z;
      const float y = sy[s];
      sz[s] = ok ? (1.0f / (1.0f + expf(-z)) - y) / (float)n : 0.f;  // dz
      if (ok && loss)  // this sample's share of the step's mean loss
        atomicAdd(&loss[blockIdx.x & (kLossSlotsNcf - 1)],
                  (double)(fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)))) / (double)n);
    }
  }
  __syncthreads();
  NCF_PH(7);
  if (zout) return;  // forward only (ncf_predict)
  // 5. predict-layer gradients (workgroup partials, samples in order) and dX of the predictor
  float* part = partial + (int64_t)blockIdx.x * D.flat_n;
  for (int k = tid; k <= D.pred; k += blockDim.x) {
    float acc = 0.f;
    if (k < D.pred) {
      for (int s = 0; s < kSamples; ++s) {
        float x;
        if (gmf && k < d)
          x = sm[Lp.eu + s * (d + 4) + k] * sm[Lp.ei + s * (d + 4) + k];
        else
          x = hL[s * ldL + (k - (gmf ? d : 0))];
        acc = fmaf(sz[s], x, acc);
      }
      part[D.off_wp + k] = acc;
    } else {
      for (int s = 0; s < kSamples; ++s) acc += sz[s];
      part[D.off_bp] = acc;
    }
  }
  __syncthreads();  // hL (read above as x) is overwritten below by dPre_L
  NCF_PH(8);
  if (gmf) {  // dPg[u] += dz wp_k Qg[i]_k ; dQg[i] += dz wp_k Pg[u]_k
    for (int x = tid; x < kSamples * d; x += blockDim.x) {
      const int s = x / d, k = x % d;
      const int32_t u = su[s], i = si[s];
      if (u < 0) continue;
      const float gk = sz[s] * P.wp[k];
      atomicAdd(G.Pg + (int64_t)u * d + k, gk * sm[Lp.ei + s * (d + 4) + k]);
      atomicAdd(G.Qg + (int64_t)i * d + k, gk * sm[Lp.eu + s * (d + 4) + k]);
    }
  }
  if (mlp) {
    // dPre_L = dz wp[tower part] * (h_L > 0), in place of h_L
    float* hw = sm + Lp.h[D.L];
    for (int x = tid; x < kSamples * d; x += blockDim.x) {
      const int s = x / d, k = x % d;
      const float h = hw[s * ldL + k];
      hw[s * ldL + k] = h > 0.f ? sz[s] * P.wp[(gmf ? d : 0) + k] : 0.f;
    }
    __syncthreads();
    NCF_PH(9);
    for (int l = D.L - 1; l >= 0; --l) {
      const int K = D.nin[l], N = D.nout[l];
      const float* dP = sm + Lp.h[l + 1];  // dPre_l [16 x N]
      const int ldp = Lp.ldh[l + 1];
      float* H = sm + Lp.h[l];  // h_{l-1} [16 x K], becomes dPre_{l-1} (or dX_0)
      const int ldx = Lp.ldh[l];
      // (a) dW_l partial [N x K] = dPre^T . H (contraction over the 16 samples), db_l
      const int tn = (N + 15) / 16, tk = (K + 15) / 16;
      for (int tile = wave; tile < tn * tk; tile += NW) {
        const int n0 = 16 * (tile / tk), k0 = 16 * (tile % tk);
        const int r = lane & 15, g = lane >> 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int s = 4 * e + g;
          const float a = n0 + r < N ? dP[s * ldp + n0 + r] : 0.f;
          const float b = k0 + r < K ? H[s * ldx + k0 + r] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        const int kk = k0 + r;
        if (kk < K) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int nn = n0 + 4 * g + q;
            if (nn < N) part[D.off_W[l] + (int64_t)nn * K + kk] = acc[q];
          }
        }
      }
      for (int nn = tid; nn < N; nn += blockDim.x) {
        float acc = 0.f;
        for (int s = 0; s < kSamples; ++s) acc += dP[s * ldp + nn];
        part[D.off_b[l] + nn] = acc;
      }
      __syncthreads();
      NCF_PH(10 + 2 * (D.L - 1 - l));
      // (b) dX [16 x K] = dPre . W_l  (B operand from the transposed copy WT_l [K x N])
      for (int tile = wave; 16 * tile < K; tile += NW) {
        const f32x4 acc = tile_xwt(dP, ldp, P.WT[l], N, 16 * tile, K, lane);
        const int kk = 16 * tile + (lane & 15);
        if (kk < K) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = 4 * (lane >> 4) + r;
            float v = acc[r];
            if (l > 0) v = H[s * ldx + kk] > 0.f ? v : 0.f;  // relu' of h_{l-1}
            H[s * ldx + kk] = v;
          }
        }
      }
      __syncthreads();
      NCF_PH(11 + 2 * (D.L - 1 - l));
    }
    // embedding gradients of the tower input: dPm[u] += dX0[:E], dQm[i] += dX0[E:]
    const float* X0 = sm + Lp.h[0];
    for (int x = tid; x < kSamples * 2 * E; x += blockDim.x) {
      const int s = x / (2 * E), k = x % (2 * E);
      const int32_t u = su[s], i = si[s];
      if (u < 0) continue;
      const float v = X0[s * Lp.ldh[0] + k];
      if (k < E)
        atomicAdd(G.Pm + (int64_t)u * E + k, v);
      else
        atomicAdd(G.Qm + (int64_t)i * E + (k - E), v);
    }
  }
#ifdef BPRMF_NCF_PHASES
  __syncthreads();
  NCF_PH(20);
  if (threadIdx.x == 0 && blockIdx.x == 0 && t == 100)
    for (int k = 1; k <= 20; ++k)
      if (s_ph[k]) printf("ncf phase %d: %.2f us\n", k, (double)(s_ph[k] - s_ph[0]) * 1e-2);
#endif
}

// torch Adam (single-tensor form): m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)
static __device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, const AdamArgs& a) {
  m = m + a.one_minus_b1 * (g - m);
  v = fmaf(a.b2, v, a.one_minus_b2 * g * g);
  p = p - a.step_size * (m / (sqrtf(v) / a.bc2_sqrt + a.eps));
}

// ---- lazy row Adam ---------------------------------------------------------------------------
// Steps s = c+1 .. e with g = 0 from a row's state (p, m, v) at step c (j = s - c):
//   m_s = b1^j m,  v_s = b2^j v,
//   p_e = p - m * sum_j a_j / (sqrt(v) w_j + eps),  a_j = step_size(s) b1^j,  w_j = b2^(j/2) / bc2_sqrt(s)
// (torch's step_size(s) = lr / (1 - b1^s), bc2_sqrt(s) = sqrt(1 - b2^s)).  A term is at most
// (b1 / sqrt(b2))^j (1 / bc2_sqrt(c+1)) times the first (0.9005^j x <= 32 at the defaults), so
// the sum stops after kCatchTerms terms: 32 x 0.9005^192 < 6e-8 of the first term.  The per-step
// and per-term factors come from tables built once on the host (in double).

// one workgroup per (sample, side): thread 0 claims the row (cur: c -> target by CAS, so a row
// repeated in the batch is caught up once); row = blockIdx.x when the sides carry no ids
static __device__ __forceinline__ int64_t side_row(const RowSides& R, int side) {
  const int64_t x = blockIdx.x;
  if (!R.ids[0]) return x < R.side[side].rows ? x : -1;
  const int32_t u = R.ids[0][x], i = R.ids[1][x];
  if ((uint64_t)u >= (uint64_t)R.U || (uint64_t)i >= (uint64_t)R.I) return -1;  // no gradient
  return side ? i : u;
}

__global__ __launch_bounds__(1024) void k_ncf_catch_up(RowSides R, CatchArgs c) {
  __shared__ float2 s_term[kCatchTerms];
  __shared__ int64_t s_row;
  __shared__ int32_t s_from;

  const int side = blockIdx.y;
  const RowSide S = side ? R.side[1] : R.side[0];  // no dynamic index into the kernel arguments
  if (threadIdx.x == 0) {
    const int64_t r = side_row(R, side);
    int32_t from = -1;
    if (r >= 0) {
      const int32_t old = S.cur[r];
      if (old >= 0 && old < c.target && atomicCAS(S.cur + r, old, c.target) == old) from = old;
    }
    s_row = r;
    s_from = from;
  }
  __syncthreads();
  const int32_t from = s_from;
  if (from < 0) return;
  const int J = min(c.target - from, kCatchTerms);
  for (int j = threadIdx.x + 1; j <= J; j += blockDim.x) {
    const int64_t s = (int64_t)from + j;
    const float2 st = s <= c.nstep ? c.step[s - 1] : make_float2(c.lr, 1.f), pw = c.pw[j - 1];
    s_term[j - 1] = make_float2(st.x * pw.x, pw.y * st.y);
  }
  __syncthreads();
  const int64_t r = s_row;
  const float k = (float)(c.target - from);
  const float dm = exp2f(k * c.log2_b1), dv = exp2f(k * c.log2_b2), eps = c.eps;
  for (int e = threadIdx.x; e < S.cols[0] + S.cols[1]; e += blockDim.x) {
    const int tb = e >= S.cols[0];
    const int64_t x = r * S.cols[tb] + (tb ? e - S.cols[0] : e);
    const float m = S.M[tb][x], v = S.V[tb][x], sv = sqrtf(v);
    float acc0 = 0.f, acc1 = 0.f;
    int j = 0;
    for (; j + 1 < J; j += 2) {
      const float2 q0 = s_term[j], q1 = s_term[j + 1];
      acc0 = fmaf(q0.x, __builtin_amdgcn_rcpf(fmaf(sv, q0.y, eps)), acc0);
      acc1 = fmaf(q1.x, __builtin_amdgcn_rcpf(fmaf(sv, q1.y, eps)), acc1);
    }
    if (j < J) acc0 = fmaf(s_term[j].x, __builtin_amdgcn_rcpf(fmaf(sv, s_term[j].y, eps)), acc0);
    S.W[tb][x] -= m * (acc0 + acc1);
    S.M[tb][x] = m * dm;
    S.V[tb][x] = v * dv;
  }
}

// Adam step t on the batch's rows (the rows are at step t - 1 or never touched): g = the
// gradient row (zeroed for the next step), cur = t; a row repeated in the batch is stepped once
__global__ __launch_bounds__(1024) void k_ncf_adam_rows(RowSides R, int32_t t, AdamArgs a) {
  __shared__ int64_t s_row;
  const int side = blockIdx.y;
  const RowSide S = side ? R.side[1] : R.side[0];  // no dynamic index into the kernel arguments
  if (threadIdx.x == 0) {
    int64_t r = side_row(R, side);
    if (r >= 0) {
      const int32_t old = S.cur[r];
      if (old == t || atomicCAS(S.cur + r, old, t) != old) r = -1;
    }
    s_row = r;
  }
  __syncthreads();
  const int64_t r = s_row;
  if (r < 0) return;
  for (int e = threadIdx.x; e < S.cols[0] + S.cols[1]; e += blockDim.x) {
    const int tb = e >= S.cols[0];
    const int64_t x = r * S.cols[tb] + (tb ? e - S.cols[0] : e);
    float p = S.W[tb][x], m = S.M[tb][x], v = S.V[tb][x];
    adam1(p, m, v, S.G[tb][x], a);
    S.G[tb][x] = 0.f;
    S.W[tb][x] = p;
    S.M[tb][x] = m;
    S.V[tb][x] = v;
  }
}

// flat region [lo, hi) of the tower+predict parameters; weights of layer l also to WT_l
__global__ __launch_bounds__(256) void k_ncf_adam_flat(Dims D, Params P, float* __restrict__ F,
                                                       float* __restrict__ M, float* __restrict__ V,
                                                       const float* __restrict__ partial, int nparts,
                                                       int lo, int hi, AdamArgs a) {
  for (int j = lo + blockIdx.x * blockDim.x + threadIdx.x; j < hi; j += gridDim.x * blockDim.x) {
    float g = 0.f;
    for (int b = 0; b < nparts; ++b) g += partial[(int64_t)b * D.flat_n + j];
    float p = F[j], m = M[j], v = V[j];
    adam1(p, m, v, g, a);
    F[j] = p;
    M[j] = m;
    V[j] = v;
    for (int l = 0; l < D.L; ++l) {
      const int w0 = D.off_W[l], K = D.nin[l], N = D.nout[l];
      if (j >= w0 && j < w0 + N * K) {
        const int nn = (j - w0) / K, kk = (j - w0) % K;
        P.WT[l][(int64_t)kk * N + nn] = p;
      }
    }
  }
}

__global__ void k_ncf_transpose(Dims D, Params P) {  // WT_l = W_l^T (after set / init)
  for (int l = 0; l < D.L; ++l) {
    const int K = D.nin[l], N = D.nout[l];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < N * K; j += gridDim.x * blockDim.x)
      P.WT[l][(int64_t)(j % K) * N + j / K] = P.W[l][j];
  }
}

// NCFData.ng_sample + shuffled DataLoader (util/data_loader.py:941-972) as a device sampler:
// slot q of the epoch's Feistel permutation over (1 + num_ng) * npos samples; q < npos is the
// positive q (label 1), else negative number (q - npos) % num_ng of positive (q - npos) / num_ng:
// the k-th item the user has no positive for, k Lemire-bounded from Philox (label 0).
__global__ __launch_bounds__(256) void k_ncf_sample(SamplerArgs a, uint32_t epoch, int64_t first,
                                                    int64_t count, int32_t* __restrict__ ou,
                                                    int32_t* __restrict__ oi, float* __restrict__ oy,
                                                    int32_t* __restrict__ err) {
  const uint64_t npos = (uint64_t)a.npos, N = npos * (uint64_t)(1 + a.num_ng);
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < count;
       s += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t q = permute((uint64_t)(first + s), N, a.feistel_a, a.feistel_c, a.k0, a.k1, epoch);
    if (q < npos) {
      ou[s] = a.pos_u[q];
      oi[s] = a.pos_i[q];
      oy[s] = 1.f;
      continue;
    }
    const int64_t p = (int64_t)((q - npos) / (uint64_t)a.num_ng);
    const int32_t u = a.pos_u[p];
    const int64_t beg = a.indptr[u], deg = a.indptr[u + 1] - beg;
    const int64_t free_items = a.item_num - deg;
    int32_t j = -1;
    if (free_items > 0) {
      const uint32_t k = bounded(q, epoch, (uint32_t)free_items, a.k0, a.k1);
      j = (int32_t)kth_nonmember(a.indices + beg, deg, (int64_t)k);
    } else {
      atomicOr(err, 2);
      j = 0;
    }
    ou[s] = u;
    oi[s] = j;
    oy[s] = 0.f;
  }
}

// init: embeddings N(0, std^2); tower weights xavier_uniform; predict kaiming_uniform(a=1,
// 'sigmoid') = U(-sqrt(3/fan_in), +); biases 0 (NCFRecommender.py:65-82).  Philox, one counter
// per element; `tag` separates the tensors.
__global__ void k_ncf_init(float* __restrict__ W, int64_t n, int kind, float param, uint32_t k0,
                           uint32_t k1, uint32_t tag) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(e >> 32), c2 = tag, c3 = TAG_INIT | 0x100u;
    philox10(c0, c1, c2, c3, k0, k1);
    float v;
    if (kind == 0) {  // normal(0, param)
      const float u1 = ((float)c0 + 1.0f) * 2.3283064365386963e-10f;
      const float u2 = (float)c1 * 2.3283064365386963e-10f;
      v = param * sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
    } else if (kind == 1) {  // uniform(-param, param)
      v = param * (2.0f * ((float)c0 * 2.3283064365386963e-10f) - 1.0f);
    } else {
      v = 0.f;
    }
    W[e] = v;
  }
}

// ---- launchers ----------------------------------------------------------------------------
static unsigned grid1(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256));
}

// dynamic LDS beyond the default 64 KB window (up to the CU's 160 KB) must be opted into
static hipError_t allow_lds(size_t bytes) {
  static size_t allowed = 64 * 1024;
  if (bytes <= allowed) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_ncf_fwdbwd),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) allowed = bytes;
  return e;
}

hipError_t fwdbwd(const Dims& D, const Params& P, const Grads& G, const int32_t* u,
                  const int32_t* i, const float* y, int n, int32_t t, float* partial,
                  double* loss, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (hipError_t e = allow_lds(fwdbwd_lds_bytes(D))) return e;
  const unsigned blocks = (unsigned)((n + kSamples - 1) / kSamples);
  k_ncf_fwdbwd<<<blocks, 1024, fwdbwd_lds_bytes(D), s>>>(D, P, G, u, i, y, n, t, partial, loss, err,
                                                         nullptr);
  return hipGetLastError();
}

hipError_t forward(const Dims& D, const Params& P, const int32_t* u, const int32_t* i, int n,
                   float* z, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (hipError_t e = allow_lds(fwdbwd_lds_bytes(D))) return e;
  const unsigned blocks = (unsigned)((n + kSamples - 1) / kSamples);
  k_ncf_fwdbwd<<<blocks, 1024, fwdbwd_lds_bytes(D), s>>>(D, P, Grads{}, u, i, nullptr, n, 0,
                                                         nullptr, nullptr, err, z);
  return hipGetLastError();
}

static dim3 rows_grid(const RowSides& R, int64_t n) {
  return dim3((unsigned)(R.ids[0] ? n : std::max(R.side[0].rows, R.side[1].rows)), 2);
}
static unsigned rows_block(const RowSides& R) {
  const int w = std::max(R.side[0].cols[0] + R.side[0].cols[1], R.side[1].cols[0] + R.side[1].cols[1]);
  return (unsigned)std::min(1024, std::max(64, (w + 63) / 64 * 64));
}

hipError_t catch_up(const RowSides& R, int64_t n, const CatchArgs& c, hipStream_t s) {
  if (c.target <= 0 || (R.ids[0] && n <= 0)) return hipSuccess;
  k_ncf_catch_up<<<rows_grid(R, n), rows_block(R), 0, s>>>(R, c);
  return hipGetLastError();
}

hipError_t adam_rows(const RowSides& R, int64_t n, int32_t t, const AdamArgs& a, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_ncf_adam_rows<<<rows_grid(R, n), rows_block(R), 0, s>>>(R, t, a);
  return hipGetLastError();
}

hipError_t adam_flat(const Dims& D, const Params& P, float* F, float* M, float* V,
                     const float* partial, int nparts, int lo, int hi, const AdamArgs& a,
                     hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  k_ncf_adam_flat<<<grid1(hi - lo), 256, 0, s>>>(D, P, F, M, V, partial, nparts, lo, hi, a);
  return hipGetLastError();
}

hipError_t transpose(const Dims& D, const Params& P, hipStream_t s) {
  k_ncf_transpose<<<256, 256, 0, s>>>(D, P);
  return hipGetLastError();
}

hipError_t sample(const SamplerArgs& a, uint32_t epoch, int64_t first, int64_t count, int32_t* u,
                  int32_t* i, float* y, int32_t* err, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  k_ncf_sample<<<grid1(count), 256, 0, s>>>(a, epoch, first, count, u, i, y, err);
  return hipGetLastError();
}

hipError_t init(float* W, int64_t n, int kind, float param, uint32_t k0, uint32_t k1, uint32_t tag,
                hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_ncf_init<<<grid1(n), 256, 0, s>>>(W, n, kind, param, k0, k1, tag);
  return hipGetLastError();
}

}  // namespace ncf
}  // namespace bprmf
