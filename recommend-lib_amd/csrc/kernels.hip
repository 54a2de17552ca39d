// kernels.hip — gfx950 (MI355X / CDNA4) kernels of the BPR-MF training path.
//
// What the reference computes per step (BPRMFRecommender.py:172-176), restated for the kernels:
//   x_b  = <P_u,Q_i> - <P_u,Q_j>            (BPR.forward, :42-50)
//   c_b  = sigmoid(-x_b) = -dL/dx_b          (loss = -sum log sigmoid(x), :174)
//   G_P[u] += -c (Q_i - Q_j);  G_Q[i] += -c P_u;  G_Q[j] += c P_u   (embedding backward, duplicates summed)
//   every row: W <- W - lr (G + wd W)        (SGD weight_decay over dense grads, :154,:176)
// Rows not referenced in a step only decay; that decay is applied lazily (stamp per row, factor
// (1-lr*wd)^k computed in double) so a step touches only its 3B rows, never the whole table.
//
// Memory-bound by design (≈0.66 flop/B): no MFMA.  A group of G lanes owns one row; lane `sub`
// holds elements sub + G*k, so every global load / f32 atomic wave-instruction covers whole
// contiguous 256 B (G=64) or 128 B (G=32) row segments — the shape the memory-side atomic unit
// runs at full rate (MI355X_MICROARCH.md §Global float atomics).
#include "kernels.h"

#include <math.h>
#include <stdlib.h>

#include "device_common.h"

BPRMF_CALL_STAMPS_DEF(ker)

namespace bprmf {

// ng_sample + DataLoader shuffle of one epoch (util/data_loader.py:680-690,
// BPRMFRecommender.py:141): slot s -> triplet q = perm(s) -> positive q / num_ng -> negative j
// uniform over the user's non-positives.
__global__ __launch_bounds__(kBlock) void k_sample(SamplerArgs a, uint32_t epoch, int64_t first,
                                                   int64_t count, int32_t* __restrict__ ou,
                                                   int32_t* __restrict__ oi,
                                                   int32_t* __restrict__ oj,
                                                   int32_t* __restrict__ err) {
  CsScope cs_(1);  // diagnostic builds only (BPRMF_CALL_STAMPS)
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < count;
       s += (int64_t)gridDim.x * blockDim.x) {
    int32_t u, i, j;
    if (!sample_slot(a, epoch, (uint64_t)(first + s), u, i, j)) atomicOr(err, 2);
    ou[s] = u;
    oi[s] = i;
    oj[s] = j;
  }
}

// N(0, std^2) init (nn.init.normal_, BPRMFRecommender.py:39-40): Box-Muller on Philox output,
// one counter per element; padding columns are zero.
__global__ __launch_bounds__(kBlock) void k_init_normal(float* __restrict__ W, int64_t rows, int ld,
                                                        int D, float std, uint32_t k0, uint32_t k1,
                                                        uint32_t tag, int world, int rank) {
  const int64_t total = rows * (int64_t)ld;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / ld;
    const int c = (int)(e - r * ld);
    const int64_t rg = r * world + rank;  // global row: same init for every sharding
    float v = 0.f;
    if (c < D) {
      uint32_t c0 = (uint32_t)rg, c1 = (uint32_t)(rg >> 32), c2 = (uint32_t)c, c3 = TAG_INIT | tag;
      philox10(c0, c1, c2, c3, k0, k1);
      const float u1 = ((float)c0 + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
      const float u2 = (float)c1 * 2.3283064365386963e-10f;
      v = std * sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
    }
    W[e] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Training step kernels
// ------------------------------------------------------------------------------------------------
// Atomic path (batches larger than kMaxSegBatch): K1 — fused gather (with pending decay) + 2 dots + sigmoid + gradient scatter.
//   reads  3 rows + 3 stamps + 3 ids per triplet;  writes 3 rows of f32 atomic adds into G.
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_fwd_scatter(const int32_t* __restrict__ tu,
                                                        const int32_t* __restrict__ ti,
                                                        const int32_t* __restrict__ tj, int64_t n,
                                                        Table P, Table Q, Hyper hp, int ld,
                                                        int32_t t, double* loss,
                                                        int32_t* __restrict__ err) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  float lsum = 0.f;
  for (int64_t b = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; b < n; b += ngroups) {
    const int32_t u = tu[b], i = ti[b], j = tj[b];
    if ((uint64_t)u >= (uint64_t)P.rows || (uint64_t)i >= (uint64_t)Q.rows ||
        (uint64_t)j >= (uint64_t)Q.rows) {
      if (sub == 0) atomicOr(err, 1);
      continue;
    }
    const float fu = decay_pow(hp.log2a, t - 1 - P.stamp[u]);
    const float fi = decay_pow(hp.log2a, t - 1 - Q.stamp[i]);
    const float fj = decay_pow(hp.log2a, t - 1 - Q.stamp[j]);
    const float* pu = P.W + (int64_t)u * ld + sub;
    const float* qi = Q.W + (int64_t)i * ld + sub;
    const float* qj = Q.W + (int64_t)j * ld + sub;
    float vu[EPL], vi[EPL], vj[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      vu[k] = pu[G * k];
      vi[k] = qi[G * k];
      vj[k] = qj[G * k];
    }
    float di = 0.f, dj = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      vu[k] *= fu;
      vi[k] *= fi;
      vj[k] *= fj;
      di = fmaf(vu[k], vi[k], di);
      dj = fmaf(vu[k], vj[k], dj);
    }
    di = group_sum<G>(di);
    dj = group_sum<G>(dj);
    const float x = di - dj;
    const float c = 1.0f / (1.0f + expf(x));  // sigmoid(-x)
    if (sub == 0) lsum += softplus(-x);
    float* gu = P.G + (int64_t)u * ld + sub;
    float* gi = Q.G + (int64_t)i * ld + sub;
    float* gj = Q.G + (int64_t)j * ld + sub;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const float cu = c * vu[k];
      atomicAdd(gu + G * k, -c * (vi[k] - vj[k]));
      atomicAdd(gi + G * k, -cu);
      atomicAdd(gj + G * k, cu);
    }
  }
  wave_add_loss(loss, lsum);
}

// apply one claimed row: V = W*alpha^(t-1-old); W = V - lr*(G + wd*V); G = 0
template <int G, int EPL>
__device__ __forceinline__ void apply_row(Table T, int64_t row, int32_t old, const Hyper& hp,
                                          int ld, int32_t t, int sub) {
  const float f = decay_pow(hp.log2a, t - 1 - old);
  float* w = T.W + row * ld + sub;
  float* g = T.G + row * ld + sub;
  float wv[EPL], gv[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    wv[k] = w[G * k];
    gv[k] = g[G * k];
  }
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const float v = wv[k] * f;
    const float dp = fmaf(hp.wd, v, gv[k]);  // grad.add(param, alpha=wd)
    w[G * k] = fmaf(-hp.lr, dp, v);          // param.add_(grad, alpha=-lr)
    g[G * k] = 0.f;
  }
}

// claim row for step t: the first group to swap the stamp applies it, later duplicates skip.
template <int G>
__device__ __forceinline__ int32_t claim(int32_t* stamp, int64_t row, int32_t t, int sub) {
  int32_t old = 0;
  if (sub == 0) old = atomicExch(stamp + row, t);
  return __shfl(old, (int)(threadIdx.x & 63) - sub);
}

// K2 — every row referenced by the step's 3n ids is claimed once and updated.
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_apply_refs(const int32_t* __restrict__ tu,
                                                       const int32_t* __restrict__ ti,
                                                       const int32_t* __restrict__ tj, int64_t n,
                                                       Table P, Table Q, Hyper hp, int ld,
                                                       int32_t t) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t r = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; r < 3 * n; r += ngroups) {
    const int which = (int)(r / n);
    const int64_t b = r - (int64_t)which * n;
    const int32_t row = which == 0 ? tu[b] : (which == 1 ? ti[b] : tj[b]);
    Table T = which == 0 ? P : Q;
    if ((uint64_t)row >= (uint64_t)T.rows) continue;
    const int32_t old = claim<G>(T.stamp, row, t, sub);
    if (old == t) continue;
    apply_row<G, EPL>(T, row, old, hp, ld, t, sub);
  }
}

// rows referenced by a list (sharded path: local users of the batch, or received item ids)
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_apply_rows(const int32_t* __restrict__ rows, int64_t n,
                                                       Table T, Hyper hp, int ld, int32_t t) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t r = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; r < n; r += ngroups) {
    const int32_t row = rows[r];
    if ((uint64_t)row >= (uint64_t)T.rows) continue;
    const int32_t old = claim<G>(T.stamp, row, t, sub);
    if (old == t) continue;
    apply_row<G, EPL>(T, row, old, hp, ld, t, sub);
  }
}

// scores <P_u, Q_i> of the weights after T steps
template <int G, int EPL, typename Idx>
__global__ __launch_bounds__(kBlock) void k_score(const Idx* __restrict__ us,
                                                  const Idx* __restrict__ is,
                                                  const Idx* __restrict__ js, int64_t n, Table P,
                                                  Table Q, Hyper hp, int ld, int32_t T,
                                                  float* __restrict__ oi, float* __restrict__ oj,
                                                  int32_t* __restrict__ err) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t b = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; b < n; b += ngroups) {
    const int64_t u = (int64_t)us[b], i = (int64_t)is[b];
    const int64_t j = js ? (int64_t)js[b] : 0;
    if ((uint64_t)u >= (uint64_t)P.rows || (uint64_t)i >= (uint64_t)Q.rows ||
        (uint64_t)j >= (uint64_t)Q.rows) {
      if (sub == 0) {
        atomicOr(err, 1);
        oi[b] = NAN;
        if (oj) oj[b] = NAN;
      }
      continue;
    }
    const float fu = decay_pow(hp.log2a, T - P.stamp[u]);
    const float fi = decay_pow(hp.log2a, T - Q.stamp[i]);
    const float fj = js ? decay_pow(hp.log2a, T - Q.stamp[j]) : 0.f;
    const float* pu = P.W + u * ld + sub;
    const float* qi = Q.W + i * ld + sub;
    const float* qj = Q.W + j * ld + sub;
    float di = 0.f, dj = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const float vu = pu[G * k] * fu;
      di = fmaf(vu, qi[G * k] * fi, di);
      if (js) dj = fmaf(vu, qj[G * k] * fj, dj);
    }
    di = group_sum<G>(di);
    dj = group_sum<G>(dj);
    if (sub == 0) {
      oi[b] = di;
      if (oj) oj[b] = dj;
    }
  }
}

template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_flush(Table T, Hyper hp, int ld, int32_t Tstep) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t r = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; r < T.rows; r += ngroups) {
    const int32_t s = T.stamp[r];
    if (s == Tstep) continue;
    const float f = decay_pow(hp.log2a, Tstep - s);
    float* w = T.W + r * ld + sub;
#pragma unroll
    for (int k = 0; k < EPL; ++k) w[G * k] *= f;
    __builtin_amdgcn_wave_barrier();
    if (sub == 0) T.stamp[r] = Tstep;
  }
}

// owner side of the item exchange: rows of the shard, brought to step t-1, packed [n, ld]
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_gather_rows(Table T, const int32_t* __restrict__ rows,
                                                        int64_t n, Hyper hp, int ld, int32_t t,
                                                        float* __restrict__ out,
                                                        int32_t* __restrict__ err) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t r = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; r < n; r += ngroups) {
    const int64_t row = rows[r];
    float* o = out + r * ld + sub;
    if ((uint64_t)row >= (uint64_t)T.rows) {
      if (sub == 0) atomicOr(err, 1);
#pragma unroll
      for (int k = 0; k < EPL; ++k) o[G * k] = 0.f;
      continue;
    }
    const float f = decay_pow(hp.log2a, t - 1 - T.stamp[row]);
    const float* w = T.W + row * ld + sub;
#pragma unroll
    for (int k = 0; k < EPL; ++k) o[G * k] = w[G * k] * f;
  }
}

// owner side: received item grads summed into the shard's accumulator
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_add_rows(Table T, const int32_t* __restrict__ rows,
                                                     const float* __restrict__ grads, int64_t n,
                                                     int ld, int32_t* __restrict__ err) {
  const int sub = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  for (int64_t r = blockIdx.x * (int64_t)(kBlock / G) + threadIdx.x / G; r < n; r += ngroups) {
    const int64_t row = rows[r];
    if ((uint64_t)row >= (uint64_t)T.rows) {
      if (sub == 0) atomicOr(err, 1);
      continue;
    }
    const float* g = grads + r * ld + sub;
    float* d = T.G + row * ld + sub;
#pragma unroll
    for (int k = 0; k < EPL; ++k) atomicAdd(d + G * k, g[G * k]);
  }
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
bool make_geom(int D, Geom* g) {
  if (D <= 0 || D > 1024) return false;
  g->D = D;
  // float4 layout (segmented kernels): G4 lanes x S stripes of float4 per row
  const int q = (D + 3) / 4;
  if (q <= 64) {
    int G4 = 1;
    while (G4 < q) G4 <<= 1;
    g->G4 = G4;
    g->S = 1;
  } else {
    g->G4 = 64;
    g->S = (q + 63) / 64;
  }
  g->ld = 4 * g->G4 * g->S;
  // dword layout (atomic / sharded kernels) over the same padded stride
  if (g->ld < 64) {
    g->G = g->ld;
    g->EPL = 1;
  } else {
    g->G = 64;
    g->EPL = g->ld / 64;
  }
  return true;
}

hipError_t init_normal(const Geom& g, float* W, int64_t rows, float std, uint32_t k0, uint32_t k1,
                       uint32_t table_tag, int world, int rank, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  k_init_normal<<<grid_flat(rows * g.ld), kBlock, 0, s>>>(W, rows, g.ld, g.D, std, k0, k1, table_tag,
                                                          world, rank);
  return hipGetLastError();
}

// the step cursor {t, batch} that position-independent step graphs read (capi.cpp); the same
// launch clears the call's loss slots (one launch at the head of a call instead of two)
__global__ void k_set_cursor(int32_t* __restrict__ c, int32_t t, int32_t k, double* __restrict__ loss,
                             int nloss) {
  if (threadIdx.x == 0) {
    c[0] = t;
    c[1] = k;
  }
  for (int i = threadIdx.x; i < nloss; i += blockDim.x) loss[i] = 0.0;
}
__global__ void k_advance_cursor(int32_t* __restrict__ c, int32_t n) {
  c[0] += n;
  c[1] += n;
}
// the call's status words straight into mapped host memory (system-scope stores), so the host
// reads them without a copy command; then (seq_dst) the call's sequence number, once every lane's
// stores are acknowledged: the host spins on that word instead of synchronising the stream
__global__ void k_status_out(const uint64_t* __restrict__ src, uint64_t* dst, int n, uint64_t* seq_dst,
                             uint64_t seq) {
  CS_BEGIN(63);  // diagnostic builds only (BPRMF_CALL_STAMPS); the end: after the stores' wait
  const int i = threadIdx.x;
  if (i < n) __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (seq_dst) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (i == 0) __hip_atomic_store(seq_dst, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  CS_END(63);
}

hipError_t set_cursor(int32_t* cursor, int32_t t, int32_t k, hipStream_t s, double* loss, int nloss) {
  k_set_cursor<<<1, 256, 0, s>>>(cursor, t, k, loss, loss ? nloss : 0);
  return hipGetLastError();
}

// two int32 device words (a[0], b[0]) into mapped host memory dst[0..1], then seq (as k_status_out)
__global__ void k_pair_out(const int32_t* a, const int32_t* __restrict__ b, int32_t* dst,
                           uint64_t* seq_dst, uint64_t seq, int32_t* zero) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(dst, *a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (zero) *zero = 0;
    __hip_atomic_store(dst + 1, *b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(seq_dst, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t pair_out(const int32_t* a, const int32_t* b, void* dst_dev, void* seq_dev, uint64_t seq,
                    hipStream_t s, int32_t* zero) {
  k_pair_out<<<1, 64, 0, s>>>(a, b, static_cast<int32_t*>(dst_dev), static_cast<uint64_t*>(seq_dev), seq,
                              zero);
  return hipGetLastError();
}

hipError_t status_out(const void* d_status, void* h_status_dev, int words, hipStream_t s,
                      void* seq_dev, uint64_t seq) {
  if (words > 64) return hipErrorInvalidValue;
  k_status_out<<<1, 64, 0, s>>>(static_cast<const uint64_t*>(d_status),
                                static_cast<uint64_t*>(h_status_dev), words,
                                static_cast<uint64_t*>(seq_dev), seq);
  return hipGetLastError();
}

hipError_t advance_cursor(int32_t* cursor, int32_t n, hipStream_t s) {
  k_advance_cursor<<<1, 1, 0, s>>>(cursor, n);
  return hipGetLastError();
}

hipError_t sample(const SamplerArgs& a, uint32_t epoch, int64_t first, int64_t count, int32_t* ou,
                  int32_t* oi, int32_t* oj, int32_t* err, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  k_sample<<<grid_flat(count), kBlock, 0, s>>>(a, epoch, first, count, ou, oi, oj, err);
  return hipGetLastError();
}

hipError_t fwd_scatter(const Geom& g, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                       int64_t n, Table P, Table Q, const Hyper& hp, int32_t t, double* loss,
                       int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_fwd_scatter<G_, E_><<<grid_for(n, G_), kBlock, 0, s>>>(
                        tu, ti, tj, n, P, Q, hp, g.ld, t, loss, err)));
  return hipGetLastError();
}

hipError_t apply_refs(const Geom& g, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                      int64_t n, Table P, Table Q, const Hyper& hp, int32_t t, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_apply_refs<G_, E_><<<grid_for(3 * n, G_), kBlock, 0, s>>>(
                        tu, ti, tj, n, P, Q, hp, g.ld, t)));
  return hipGetLastError();
}

hipError_t score(const Geom& g, const int32_t* u, const int32_t* i, int64_t n, Table P, Table Q,
                 const Hyper& hp, int32_t T, float* out, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_score<G_, E_, int32_t><<<grid_for(n, G_), kBlock, 0, s>>>(
                        u, i, (const int32_t*)nullptr, n, P, Q, hp, g.ld, T, out, nullptr, err)));
  return hipGetLastError();
}

hipError_t forward64(const Geom& g, const int64_t* u, const int64_t* i, const int64_t* j,
                     int64_t n, Table P, Table Q, const Hyper& hp, int32_t T, float* oi, float* oj,
                     int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_score<G_, E_, int64_t><<<grid_for(n, G_), kBlock, 0, s>>>(
                        u, i, j, n, P, Q, hp, g.ld, T, oi, oj, err)));
  return hipGetLastError();
}

hipError_t flush(const Geom& g, Table W, const Hyper& hp, int32_t T, hipStream_t s) {
  if (W.rows <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_flush<G_, E_><<<grid_for(W.rows, G_), kBlock, 0, s>>>(W, hp, g.ld, T)));
  return hipGetLastError();
}

hipError_t gather_rows(const Geom& g, Table W, const int32_t* rows, int64_t n, const Hyper& hp,
                       int32_t t, float* out, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_gather_rows<G_, E_><<<grid_for(n, G_), kBlock, 0, s>>>(
                        W, rows, n, hp, g.ld, t, out, err)));
  return hipGetLastError();
}

hipError_t add_rows(const Geom& g, Table W, const int32_t* rows, const float* grads, int64_t n,
                    int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_add_rows<G_, E_><<<grid_for(n, G_), kBlock, 0, s>>>(W, rows, grads, n,
                                                                           g.ld, err)));
  return hipGetLastError();
}

hipError_t apply_rows(const Geom& g, Table W, const int32_t* rows, int64_t n, const Hyper& hp,
                      int32_t t, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  BPRMF_DISPATCH(g, (k_apply_rows<G_, E_><<<grid_for(n, G_), kBlock, 0, s>>>(rows, n, W, hp,
                                                                             g.ld, t)));
  return hipGetLastError();
}

}  // namespace bprmf
