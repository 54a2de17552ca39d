// ncf.hip — NCF (GMF / MLP / NeuMF-end) training step on gfx950.
//
// Reference: NCFRecommender.py:27-124 (model), :255-288 (BCEWithLogitsLoss + Adam over every
// parameter with dense gradients), util/data_loader.py:931-972 (NCFData: positives, then num_ng
// negatives per positive, shuffled).
//
//   k_ncf_front / k_ncf_mid / k_ncf_back  the forward and backward on f32 MFMA
//                 (v_mfma_f32_16x16x4_f32; 16 samples are the M dimension of the per-sample
//                 layers), torch's Adam on the tower and predict layer fused into the weight-
//                 gradient tiles, the embedding gradients as f32 atomics into dense gradient rows
//                 (see "forward / backward" below).
//   k_ncf_catch_up / k_ncf_adam_rows  torch's dense Adam over the embedding tables, done lazily:
//                 every row with a nonzero moment moves every step, but a step with g = 0 has a
//                 closed form, so a row is brought up to date only when something reads it (the
//                 step that gathers it, a predict, a parameter copy) and Adam proper runs on the
//                 batch's rows alone.  Equal to the dense sweep up to f32 rounding.
#include <algorithm>

#include "device_common.h"
#include "ncf_kernels.h"

namespace bprmf {
namespace ncf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ---- forward / backward ----------------------------------------------------------------------
// A step's tower runs in three launches, so that no kernel streams every weight through one CU:
//   k_ncf_front  layer 0 (the widest): one workgroup per (16 samples, 16 output columns), K split
//                over its waves, reading the tower input [Pm[u], Qm[i]] straight from the rows;
//                writes h_1 (and the input itself, X0, for the weight gradient).
//   k_ncf_mid    one workgroup per 16 samples: layers 1 .. L-1, the prediction, BCE and dL/dz,
//                the GMF embedding gradients, then the tower backward down to dPre_0 (the
//                gradient of layer 0's pre-activation).  Activations and pre-activation
//                gradients go to global memory (Acts) for the next launch.
//   k_ncf_back   jobs over the whole batch: every weight-gradient tile dW_l = dPre_l^T . h_l, bias
//                and predict-layer gradient as a contraction over the batch's samples (MFMA,
//                fixed order: deterministic), each followed by torch's Adam on its elements (and
//                the transposed copy W^T); and the tower input's gradient dX_0 = dPre_0 . W_0
//                per (16 samples, 16 columns) into the MLP embedding gradient rows (f32 atomics).

// LDS plan of k_ncf_mid (floats): sample ids / labels / z / dz, GMF rows, activations h_1 .. h_L
struct Lds {
  int eu, ei, h[kMaxLayers + 1], misc, total;
  int ldh[kMaxLayers + 1];
  int hL, ldL;  // h[L], ldh[L]
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
#pragma unroll
  for (int l = 1; l <= kMaxLayers; ++l) {  // constant indices: no scratch copy of the arrays
    if (l > D.L) break;
    p.ldh[l] = D.nout[l - 1] + 4;  // row stride: +4 floats keeps float4 reads of 16 rows conflict-free
    p.h[l] = off;
    off += kSamples * p.ldh[l];
    p.hL = p.h[l];
    p.ldL = p.ldh[l];
  }
  p.total = off;
  return p;
}
size_t fwdbwd_lds_bytes(const Dims& D) { return sizeof(float) * (size_t)lds_plan(D).total; }

// y[16 x 16 tile] = X[16 x kc] . W[n0.., 0 .. kc)^T (global, W[n][k], row stride ldw): 16x16x4
// f32 MFMA, lane group g = l >> 4 takes k = 16t + 4g .. +3 (kc % 4 == 0); lane l supplies
// row l & 15 of X from xr (0 where !xok).  The W rows come from L2/HBM: eight k-steps of loads
// are issued before their 32 MFMAs, so one latency is paid per eight steps, not per step.
// xs (optional): this lane's row of X is also stored there as it is loaded
static __device__ __forceinline__ f32x4 tile_xwt(const float* xr, bool xok, const float* W, int ldw,
                                                 int kc, int n0, int nmax, int lane, float* xs = nullptr) {
  constexpr int U = 8;
  const int r = lane & 15, g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool nok = n0 + r < nmax;
  const float* wr = W + (int64_t)(n0 + r) * ldw;
  for (int t0 = 0; 16 * t0 < kc; t0 += U) {
    float4 a[U], b[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = 16 * (t0 + q) + 4 * g;
      b[q] = (nok && k < kc) ? ld4(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int k = 16 * (t0 + q) + 4 * g;
      a[q] = (xok && k < kc) ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      if (xs && k < kc) *reinterpret_cast<float4*>(xs + k) = a[q];
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

// a[i] for a run-time i without a dynamic index into the array (which would go through scratch)
template <typename T, int N>
static __device__ __forceinline__ T pick(const T (&a)[N], int i) {
  T r = a[0];
#pragma unroll
  for (int k = 1; k < N; ++k)
    if (i == k) r = a[k];
  return r;
}

// a sample's ids, or -1 / -1 past n or out of range (the error flag is raised by k_ncf_mid)
static __device__ __forceinline__ void sample_ids(const Dims& D, const int32_t* us, const int32_t* is,
                                                  int s, int n, int32_t& u, int32_t& i) {
  u = i = -1;
  if (s >= n) return;
  const int32_t a = us[s], b = is[s];
  if ((uint64_t)a < (uint64_t)D.U && (uint64_t)b < (uint64_t)D.I) {
    u = a;
    i = b;
  }
}

// one workgroup per (16 samples, 16 output columns); wave w of the ks parts of K = 2E takes
// k in [w K/ks, (w+1) K/ks) straight from the embedding rows (the first half from Pm[u], the
// second from Qm[i]), the parts summed in wave order through LDS.  The y = 0 workgroups also
// store the tower input rows (X0) for the weight gradient.
__global__ __launch_bounds__(256) void k_ncf_front(Dims D, Params P, Grads G, Acts A,
                                                   const int32_t* __restrict__ us,
                                                   const int32_t* __restrict__ is, int n, int32_t t) {
  __shared__ f32x4 s_acc[3][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15;
  const int s0 = blockIdx.x * kSamples, E = D.E, K = 2 * E, N = D.nout[0], n0 = 16 * blockIdx.y;
  if (G.touch_u && blockIdx.y == 0 && tid < kSamples) {  // the rows this step's row Adam will move
    int32_t u, i;
    sample_ids(D, us, is, s0 + tid, n, u, i);
    if (u >= 0) {
      G.touch_u[u] = t;
      G.touch_i[i] = t;
    }
  }
  const int ks = E % 8 == 0 ? 4 : 2, kq = K / ks;  // parts of K, each a multiple of 4 floats
  const int nn = n0 + r;
  const float bias = wave == 0 && nn < N ? P.b[0][nn] : 0.f;  // issued before the MFMAs
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (wave < ks) {
    int32_t u, i;
    sample_ids(D, us, is, s0 + r, n, u, i);
    const int kb = wave * kq;  // this part's first k; < E: the user's row
    const float* xr = kb < E ? P.Pm + (int64_t)max(u, 0) * E + kb : P.Qm + (int64_t)max(i, 0) * E + (kb - E);
    // the y = 0 workgroups store the rows they load as X0 (zero for a sample without ids)
    float* xs = A.X0 && blockIdx.y == 0 ? A.X0 + (int64_t)(s0 + r) * K + kb : nullptr;
    acc = tile_xwt(xr, u >= 0, P.W[0] + kb, K, kq, n0, N, lane, xs);
  }
  if (wave > 0) s_acc[wave - 1][lane] = acc;
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w) acc += s_acc[w][lane];
  if (nn >= N) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int s = 4 * (lane >> 4) + q;
    if (s0 + s < n) A.H[1][(int64_t)(s0 + s) * A.ldH[1] + nn] = fmaxf(acc[q] + bias, 0.f);
  }
}

static __device__ __forceinline__ void catch_row(const RowSides& R, int64_t x, int side, const CatchArgs& c,
                                                 int32_t skip);

// The workgroups past the batch's groups catch up the NEXT step's rows (rn samples of Rn) to this
// step t: the zero-gradient step t of a row this step does not gather (touch != t) is due anyway,
// and nothing reads such a row before the next step, so the next step's k_ncf_rows finds it
// current.  They run on the CUs the 16-workgroup middle layers leave idle.
__global__ __launch_bounds__(1024) void k_ncf_mid(Dims D, Params P, Grads G, Acts A, RowSides Rn, int rn,
                                                  CatchArgs cn,
                                                  const int32_t* __restrict__ us,
                                                  const int32_t* __restrict__ is,
                                                  const float* __restrict__ ys, int n, int32_t t,
                                                  double* __restrict__ loss,
                                                  int32_t* __restrict__ err,
                                                  float* __restrict__ zout) {
  extern __shared__ float sm[];
  const int groups = (n + kSamples - 1) / kSamples;
  if ((int)blockIdx.x >= groups) {
    const int x = (int)blockIdx.x - groups;
    if (x < 2 * rn) catch_row(Rn, x >> 1, x & 1, cn, cn.target);
    return;
  }
  const Lds Lp = lds_plan(D);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = 16;
  const int s0 = blockIdx.x * kSamples;
  int32_t* su = reinterpret_cast<int32_t*>(sm + Lp.misc);
  int32_t* si = su + kSamples;
  float* sy = sm + Lp.misc + 2 * kSamples;
  float* sz = sm + Lp.misc + 3 * kSamples;
  const bool gmf = D.model != kMLP, mlp = D.model != kGMF;
  const int d = D.d, L = D.L;
  const int rows = min(kSamples, n - s0);  // valid rows of this group in the Acts buffers
  // 1. samples
  if (tid < kSamples) {
    const int s = s0 + tid;
    int32_t u = -1, i = -1;
    float y = 0.f;
    if (s < n) {
      y = ys ? ys[s] : 0.f;
      if ((uint64_t)us[s] >= (uint64_t)D.U || (uint64_t)is[s] >= (uint64_t)D.I) atomicOr(err, 1);
      sample_ids(D, us, is, s, n, u, i);
    }
    su[tid] = u;
    si[tid] = i;
    sy[tid] = y;
  }
  __syncthreads();
  // 2. GMF rows and h_1 (k_ncf_front's output)
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
    const int q = D.nout[0] / 4;
    for (int x = tid; x < kSamples * q; x += blockDim.x) {
      const int s = x / q, c = 4 * (x % q);
      const float4 v = s < rows ? ld4(A.H[1] + (int64_t)(s0 + s) * A.ldH[1] + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(sm + Lp.h[1] + s * Lp.ldh[1] + c) = v;
    }
  }
  __syncthreads();
  // 3. tower forward, layers 1 .. L-1: h_{l+1} = relu(h_l W_l^T + b_l), also to global (not h_1)
  if (mlp) {
#pragma unroll
    for (int l = 1; l < kMaxLayers; ++l) {
      if (l >= L) break;
      const int K = D.nin[l], N = D.nout[l];
      const float* X = sm + Lp.h[l];
      float* Y = sm + Lp.h[l + 1];
      for (int tile = wave; 16 * tile < N; tile += NW) {
        const f32x4 acc = tile_xwt(X + (lane & 15) * Lp.ldh[l], true, P.W[l], K, K, 16 * tile, N, lane);
        const int nn = 16 * tile + (lane & 15);
        if (nn < N) {
          const float bias = P.b[l][nn];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = 4 * (lane >> 4) + r;
            const float h = fmaxf(acc[r] + bias, 0.f);
            Y[s * Lp.ldh[l + 1] + nn] = h;
            if (!zout && s < rows) A.H[l + 1][(int64_t)(s0 + s) * A.ldH[l + 1] + nn] = h;
          }
        }
      }
      __syncthreads();
    }
  }
  // 4. prediction z = [gmf, h_L] . wp + bp and dL/dz of the mean BCE-with-logits loss
  const float* hL = sm + Lp.hL;
  const int ldL = Lp.ldL;
  if (wave < kSamples) {
    const int s = wave;
    float acc = 0.f;
    for (int k = lane; k < D.pred; k += 64) {
      float x;
      if (gmf && k < d) {
        x = sm[Lp.eu + s * (d + 4) + k] * sm[Lp.ei + s * (d + 4) + k];
        if (!zout && s < rows) A.Xp[(int64_t)(s0 + s) * D.pred + k] = x;
      } else {
        x = hL[s * ldL + (k - (gmf ? d : 0))];
      }
      acc = fmaf(x, P.wp[k], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
      const bool ok = su[s] >= 0;
      const float z = acc + P.bp[0];
      if (zout && s0 + s < n) zout[s0 + s] = z;
      const float y = sy[s];
      const float dz = ok ? (1.0f / (1.0f + expf(-z)) - y) / (float)n : 0.f;
      sz[s] = dz;
      if (!zout && s < rows) A.dz[s0 + s] = dz;
      if (ok && loss)  // this sample's share of the step's mean loss
        atomicAdd(&loss[blockIdx.x & (kLossSlotsNcf - 1)],
                  (double)(fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)))) / (double)n);
    }
  }
  __syncthreads();
  if (zout) return;  // forward only (ncf_predict)
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
  if (!mlp && tid < kSamples && su[tid] >= 0) {  // (with a tower, k_ncf_front stamps them)
    G.touch_u[su[tid]] = t;
    G.touch_i[si[tid]] = t;
  }
  if (!mlp) return;
  // 5. dPre_{L-1} = dz wp[tower part] * (h_L > 0), in place of h_L
  float* hw = sm + Lp.hL;
  float* dPreL = pick(A.dPre, L - 1);
  for (int x = tid; x < kSamples * d; x += blockDim.x) {
    const int s = x / d, k = x % d;
    const float h = hw[s * ldL + k];
    const float g = h > 0.f ? sz[s] * P.wp[(gmf ? d : 0) + k] : 0.f;
    hw[s * ldL + k] = g;
    if (s < rows) dPreL[(int64_t)(s0 + s) * d + k] = g;
  }
  __syncthreads();
  // 6. dPre_{l-1} = (dPre_l . W_l) * (h_l > 0) for l = L-1 .. 1 (B operand: W_l^T), in place of h_l
#pragma unroll
  for (int l = kMaxLayers - 1; l >= 1; --l) {
    if (l > L - 1) continue;
    const int K = D.nin[l], N = D.nout[l];
    const float* dP = sm + Lp.h[l + 1];
    float* H = sm + Lp.h[l];
    const int ldp = Lp.ldh[l + 1], ldx = Lp.ldh[l];
    for (int tile = wave; 16 * tile < K; tile += NW) {
      const f32x4 acc = tile_xwt(dP + (lane & 15) * ldp, true, P.WT[l], N, N, 16 * tile, K, lane);
      const int kk = 16 * tile + (lane & 15);
      if (kk < K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = 4 * (lane >> 4) + r;
          const float g = H[s * ldx + kk] > 0.f ? acc[r] : 0.f;
          H[s * ldx + kk] = g;
          if (s < rows) A.dPre[l - 1][(int64_t)(s0 + s) * K + kk] = g;
        }
      }
    }
    __syncthreads();
  }
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
// repeated in the batch is caught up once); row = x when the sides carry no ids
static __device__ __forceinline__ int64_t side_row(const RowSides& R, int64_t x, int side) {
  if (!R.ids[0]) return x < R.side[side].rows ? x : -1;
  const int32_t u = R.ids[0][x], i = R.ids[1][x];
  if ((uint64_t)u >= (uint64_t)R.U || (uint64_t)i >= (uint64_t)R.I) return -1;  // no gradient
  return side ? i : u;
}

// row x of side `side` brought to c.target; a row touched at step `skip` (>= 0) is left to that
// step's Adam (k_ncf_rows: it runs in the same launch and brings the row to c.target itself)
static __device__ __forceinline__ void catch_row(const RowSides& R, int64_t x, int side, const CatchArgs& c,
                                                 int32_t skip) {
  __shared__ float2 s_term[kCatchTerms];
  __shared__ int64_t s_row;
  __shared__ int32_t s_from;
  const RowSide S = side ? R.side[1] : R.side[0];  // no dynamic index into the kernel arguments
  if (threadIdx.x == 0) {
    const int64_t r = side_row(R, x, side);
    int32_t from = -1;
    if (r >= 0 && (skip < 0 || S.touch[r] != skip)) {
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
    const int64_t o = r * S.cols[tb] + (tb ? e - S.cols[0] : e);
    const float m = S.M[tb][o], v = S.V[tb][o], sv = sqrtf(v);
    float acc0 = 0.f, acc1 = 0.f;
    int j = 0;
    for (; j + 1 < J; j += 2) {
      const float2 q0 = s_term[j], q1 = s_term[j + 1];
      acc0 = fmaf(q0.x, __builtin_amdgcn_rcpf(fmaf(sv, q0.y, eps)), acc0);
      acc1 = fmaf(q1.x, __builtin_amdgcn_rcpf(fmaf(sv, q1.y, eps)), acc1);
    }
    if (j < J) acc0 = fmaf(s_term[j].x, __builtin_amdgcn_rcpf(fmaf(sv, s_term[j].y, eps)), acc0);
    S.W[tb][o] -= m * (acc0 + acc1);
    S.M[tb][o] = m * dm;
    S.V[tb][o] = v * dv;
  }
}

// Adam step t on row x of side `side` (the row is at step t - 1 or never touched): g = the
// gradient row (zeroed for the next step), cur = t; a row repeated in the batch is stepped once
static __device__ __forceinline__ void adam_row(const RowSides& R, int64_t x, int side, int32_t t,
                                                const AdamArgs& a) {
  __shared__ int64_t s_row;
  const RowSide S = side ? R.side[1] : R.side[0];
  if (threadIdx.x == 0) {
    int64_t r = side_row(R, x, side);
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
    const int64_t o = r * S.cols[tb] + (tb ? e - S.cols[0] : e);
    float p = S.W[tb][o], m = S.M[tb][o], v = S.V[tb][o];
    adam1(p, m, v, S.G[tb][o], a);
    S.G[tb][o] = 0.f;
    S.W[tb][o] = p;
    S.M[tb][o] = m;
    S.V[tb][o] = v;
  }
}

__global__ __launch_bounds__(1024) void k_ncf_catch_up(RowSides R, CatchArgs c) {
  catch_row(R, blockIdx.x, blockIdx.y, c, -1);
}

__global__ __launch_bounds__(1024) void k_ncf_adam_rows(RowSides R, int32_t t, AdamArgs a) {
  adam_row(R, blockIdx.x, blockIdx.y, t, a);
}

// the previous step's row Adam (samples [0, np) of Rp, step c.target) and this step's catch-up
// (samples of Rc) in one launch
__global__ __launch_bounds__(1024) void k_ncf_rows(RowSides Rp, int np, AdamArgs a, RowSides Rc, CatchArgs c) {
  if ((int)blockIdx.x < np)
    adam_row(Rp, blockIdx.x, blockIdx.y, c.target, a);
  else
    catch_row(Rc, blockIdx.x - np, blockIdx.y, c, c.target);
}

// k_ncf_back: one job per wave (NcfJob, built once per handle).  Reads the step's weights at
// Fcur / P.WT and writes the Adam-updated ones to Fnext / WTnext (double-buffered: the dX_0 jobs
// of the same launch still read the old W_0).
__global__ __launch_bounds__(256) void k_ncf_back(Dims D, Params P, Grads G, const NcfJob* __restrict__ jobs,
                                                  int njobs, const int32_t* __restrict__ us,
                                                  const int32_t* __restrict__ is, int n,
                                                  const float* __restrict__ Fcur, float* __restrict__ Fnext,
                                                  float* __restrict__ WTnext, float* __restrict__ M,
                                                  float* __restrict__ V, AdamArgs a) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int jx = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (jx >= njobs) return;
  const NcfJob J = jobs[jx];
  if (J.kind == kJobDx0) {  // dX_0 [16 samples x 16 columns] = dPre_0 . W_0 -> dPm[u], dQm[i]
    if (J.m0 >= n) return;
    const f32x4 acc = tile_xwt(J.A + (int64_t)(J.m0 + (lane & 15)) * J.lda, true, P.WT[0], J.lda, J.lda,
                               J.k0, J.K, lane);
    const int kk = J.k0 + r, E = D.E;
    if (kk >= J.K) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int32_t u, i;
      sample_ids(D, us, is, J.m0 + 4 * g + q, n, u, i);
      if (u < 0) continue;
      if (kk < E)
        atomicAdd(G.Pm + (int64_t)u * E + kk, acc[q]);
      else
        atomicAdd(G.Qm + (int64_t)i * E + (kk - E), acc[q]);
    }
    return;
  }
  // C[16 x 16] = sum_s A[s][m0 + m] B[s][k0 + k] (B[s] for a vector job), the samples in order
  const bool vec = J.kind == kJobVec;
  const bool mok = J.m0 + r < J.M, kok = vec || J.k0 + r < J.K;
  const float* pa = J.A + J.m0 + r;
  const float* pb = vec ? J.B : J.B + J.k0 + r;
  const int ldb = vec ? 1 : J.ldb;
  // this lane's output elements and their Adam operands, loaded ahead of the contraction
  const int kk = J.k0 + r;
  const bool out = vec ? r == 0 : kk < J.K;  // a vector job's 16 columns are equal: lane r = 0
  int jj[4];
  float p0[4], m0[4], v0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int mm = J.m0 + 4 * g + q;
    jj[q] = out && mm < J.M ? (vec ? J.flat + mm : J.flat + mm * J.K + kk) : -1;
    p0[q] = jj[q] >= 0 ? Fcur[jj[q]] : 0.f;
    m0[q] = jj[q] >= 0 ? M[jj[q]] : 0.f;
    v0[q] = jj[q] >= 0 ? V[jj[q]] : 0.f;
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 32;  // samples 4U per round of loads
  for (int s4 = 0; s4 < n; s4 += 4 * U) {
    float av[U], bv[U];
#pragma unroll
    for (int e = 0; e < U; ++e) {
      const int s = s4 + 4 * e + g;
      av[e] = (s < n && mok) ? pa[(int64_t)s * J.lda] : 0.f;
      bv[e] = (s < n && kok) ? pb[(int64_t)s * ldb] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < U; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = jj[q];
    if (j < 0) continue;
    float p = p0[q], m = m0[q], v = v0[q];
    adam1(p, m, v, acc[q], a);
    Fnext[j] = p;
    M[j] = m;
    V[j] = v;
    if (J.layer >= 0) WTnext[J.wt + (int64_t)kk * J.M + (J.m0 + 4 * g + q)] = p;
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
template <typename K>
static hipError_t allow_lds(K* kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

static hipError_t front_mid(const Dims& D, const Params& P, const Grads& G, const Acts& A,
                            const int32_t* u, const int32_t* i, const float* y, int n, int32_t t, double* loss,
                            int32_t* err, float* z, const RowSides* Rn, int rn, const CatchArgs* cn,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned groups = (unsigned)((n + kSamples - 1) / kSamples);
  if (D.model != kGMF)
    k_ncf_front<<<dim3(groups, (unsigned)((D.nout[0] + 15) / 16)), 256, 0, s>>>(D, P, G, A, u, i, n, t);
  // the next step's catch-up beside the middle layers (needs the touch stamps k_ncf_front wrote)
  if (!Rn || !cn || D.model == kGMF || cn->target <= 0) rn = 0;
  const size_t mb = sizeof(float) * (size_t)lds_plan(D).total;
  if (hipError_t e = allow_lds(k_ncf_mid, mb)) return e;
  k_ncf_mid<<<groups + 2 * (unsigned)rn, 1024, mb, s>>>(D, P, G, A, rn ? *Rn : RowSides{}, rn,
                                                          rn ? *cn : CatchArgs{}, u, i, y, n, t, loss, err, z);
  return hipGetLastError();
}

hipError_t fwdbwd(const Dims& D, const Params& P, const Grads& G, const Acts& A, const int32_t* u,
                  const int32_t* i, const float* y, int n, int32_t t, double* loss, int32_t* err,
                  const RowSides* next, int next_n, const CatchArgs* next_c, hipStream_t s) {
  return front_mid(D, P, G, A, u, i, y, n, t, loss, err, nullptr, next, next_n, next_c, s);
}

hipError_t forward(const Dims& D, const Params& P, const Acts& A, const int32_t* u, const int32_t* i,
                   int n, float* z, int32_t* err, hipStream_t s) {
  return front_mid(D, P, Grads{}, A, u, i, nullptr, n, 0, nullptr, err, z, nullptr, 0, nullptr, s);
}

hipError_t back(const Dims& D, const Params& P, const Grads& G, const NcfJob* jobs, int njobs,
                const int32_t* u, const int32_t* i, int n, const float* Fcur, float* Fnext,
                float* WTnext, float* M, float* V, const AdamArgs& a, hipStream_t s) {
  if (n <= 0 || njobs <= 0) return hipSuccess;
  k_ncf_back<<<(unsigned)((njobs + 3) / 4), 256, 0, s>>>(D, P, G, jobs, njobs, u, i, n, Fcur, Fnext,
                                                         WTnext, M, V, a);
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

hipError_t rows(const RowSides& Rp, int np, const AdamArgs& a, const RowSides& Rc, int nc,
                const CatchArgs& c, hipStream_t s) {
  if (np <= 0) return catch_up(Rc, nc, c, s);
  k_ncf_rows<<<dim3((unsigned)(np + nc), 2), rows_block(Rc), 0, s>>>(Rp, np, a, Rc, c);
  return hipGetLastError();
}

hipError_t adam_rows(const RowSides& R, int64_t n, int32_t t, const AdamArgs& a, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_ncf_adam_rows<<<rows_grid(R, n), rows_block(R), 0, s>>>(R, t, a);
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
