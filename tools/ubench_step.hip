// ubench_step.hip — microbenchmark of the segmented step kernels and ablated variants, to locate
// where a step's time goes.  Development tool (not part of the product library).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ubench_step.hip -o tools/ubench_step
//   ./tools/ubench_step [B] [d]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#include "../recommend-lib_amd/csrc/kernels.hip"
#include "../recommend-lib_amd/csrc/segment.hip"
#include "../recommend-lib_amd/csrc/step.hip"

using namespace bprmf;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__global__ void k_empty() {}

// A1: record -> P row load -> P row store (one lane group per user segment)
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_a1(BatchView bv, Table P, int ld) {
  const int sub = threadIdx.x & (G - 1);
  const int s = blockIdx.x * (kBlock / G) + threadIdx.x / G;
  const int4 r0 = reinterpret_cast<const int4*>(bv.urec + (int64_t)s * kRec)[0];
  const int n = bv.meta[1];
  if (s >= n) return;
  float* pw = P.W + (int64_t)r0.x * ld + sub;
  float v[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) v[k] = pw[G * k];
#pragma unroll
  for (int k = 0; k < EPL; ++k) pw[G * k] = v[k] * 0.999f;
}

// A2: + Q_i, Q_j rows, dots, contrib store (no stamps, no loss, single triplet per segment)
template <int G, int EPL>
__global__ __launch_bounds__(kBlock) void k_a2(BatchView bv, Table P, Table Q, int ld,
                                               float* contrib) {
  const int sub = threadIdx.x & (G - 1);
  const int s = blockIdx.x * (kBlock / G) + threadIdx.x / G;
  const int4 r0 = reinterpret_cast<const int4*>(bv.urec + (int64_t)s * kRec)[0];
  const int r1x = bv.urec[(int64_t)s * kRec + 4];
  const int n = bv.meta[1];
  if (s >= n) return;
  float* pw = P.W + (int64_t)r0.x * ld + sub;
  const float* qi = Q.W + (int64_t)r0.w * ld + sub;
  const float* qj = Q.W + (int64_t)r1x * ld + sub;
  float pu[EPL], vi[EPL], vj[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    pu[k] = pw[G * k];
    vi[k] = qi[G * k];
    vj[k] = qj[G * k];
  }
  float di = 0.f, dj = 0.f;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    di = fmaf(pu[k], vi[k], di);
    dj = fmaf(pu[k], vj[k], dj);
  }
  di = group_sum<G>(di);
  dj = group_sum<G>(dj);
  const float c = 1.0f / (1.0f + expf(di - dj));
  float* cb = contrib + (int64_t)r0.y * ld + sub;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    cb[G * k] = c * pu[k];
    pw[G * k] = fmaf(-0.01f, -c * (vi[k] - vj[k]), pu[k]);
  }
}

// float4-layout ablations of K1 (G4 lanes per row, one stripe): STAMPS adds stamp loads + decay,
// LOSS adds the loss, the stamp store and the t load.
template <int G4, bool STAMPS, bool LOSS>
__global__ __launch_bounds__(kBlock) void k_a3(BatchView bv, Table P, Table Q, Hyper hp, int ld,
                                               const int32_t* tbase, int step, double* loss,
                                               float* contrib) {
  const int sub = threadIdx.x & (G4 - 1);
  const int s = blockIdx.x * (kBlock / G4) + threadIdx.x / G4;
  const int4 r0 = reinterpret_cast<const int4*>(bv.urec + (int64_t)s * kRec)[0];
  const int r1x = bv.urec[(int64_t)s * kRec + 4];
  const int n = bv.meta[1];
  const int32_t t = LOSS ? *tbase + step + 1 : step + 1;
  float lsum = 0.f;
  if (s < n) {
    float* pw = P.W + (int64_t)r0.x * ld + 4 * sub;
    float4 pu = ld4(pw);
    float4 vi = ld4(Q.W + (int64_t)r0.w * ld + 4 * sub);
    float4 vj = ld4(Q.W + (int64_t)r1x * ld + 4 * sub);
    if (STAMPS) {
      pu = scale4(pu, decay_pow(hp.log2a, t - 1 - P.stamp[r0.x]));
      vi = scale4(vi, decay_pow(hp.log2a, t - 1 - Q.stamp[r0.w]));
      vj = scale4(vj, decay_pow(hp.log2a, t - 1 - Q.stamp[r1x]));
    }
    float di = group_sum<G4>(dot4(pu, vi, 0.f)), dj = group_sum<G4>(dot4(pu, vj, 0.f));
    const float x = di - dj;
    const float c = 1.0f / (1.0f + expf(x));
    if (LOSS && sub == 0) lsum += softplus(-x);
    st4(contrib + (int64_t)r0.y * ld + 4 * sub, scale4(pu, c));
    st4(pw, sgd4(pu, fma4(-c, sub4(vi, vj), make_float4(0, 0, 0, 0)), hp.lr, hp.wd));
    if (LOSS && sub == 0) P.stamp[r0.x] = t;
  }
  if (LOSS) wave_add_loss(loss, lsum);
}

template <typename F>
static float time_loop(int iters, F&& f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) f(w);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int k = 0; k < iters; ++k) f(k);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096;
  const int D = argc > 2 ? atoi(argv[2]) : 128;
  const int64_t U = 138493, I = 26744;
  const int S = 256;  // steps
  Geom g;
  make_geom(D, &g);
  if (g.G != 64 || g.EPL != 2) fprintf(stderr, "note: ablations instantiated for G=64,EPL=2 only\n");
  const int ld = g.ld;
  std::mt19937_64 rng(7);
  // triplets: users uniform, positives Zipf(1), negatives uniform
  std::vector<double> cdf(I);
  double acc = 0;
  for (int64_t r = 0; r < I; ++r) cdf[r] = (acc += 1.0 / (r + 1));
  for (auto& x : cdf) x /= acc;
  std::vector<int32_t> hu(S * (int64_t)B), hi(S * (int64_t)B), hj(S * (int64_t)B);
  std::uniform_real_distribution<double> U01(0, 1);
  for (int64_t k = 0; k < (int64_t)S * B; ++k) {
    hu[k] = (int32_t)(rng() % U);
    hi[k] = (int32_t)(std::lower_bound(cdf.begin(), cdf.end(), U01(rng)) - cdf.begin());
    hj[k] = (int32_t)(rng() % I);
  }
  Table P{}, Q{};
  P.rows = U;
  Q.rows = I;
  CK(hipMalloc(&P.W, 4 * U * ld));
  CK(hipMalloc(&P.stamp, 4 * U));
  CK(hipMalloc(&Q.W, 4 * I * ld));
  CK(hipMalloc(&Q.stamp, 4 * I));
  CK(hipMemset(P.W, 0, 4 * U * ld));
  CK(hipMemset(Q.W, 0, 4 * I * ld));
  CK(hipMemset(P.stamp, 0, 4 * U));
  CK(hipMemset(Q.stamp, 0, 4 * I));
  int32_t *du, *di, *dj, *dbatch, *derr, *dt;
  float* contrib;
  double* loss;
  CK(hipMalloc(&du, 4 * hu.size()));
  CK(hipMalloc(&di, 4 * hu.size()));
  CK(hipMalloc(&dj, 4 * hu.size()));
  CK(hipMemcpy(du, hu.data(), 4 * hu.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(di, hi.data(), 4 * hu.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dj, hj.data(), 4 * hu.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&dbatch, 4 * S * BatchBuf::stride_for(B)));
  CK(hipMalloc(&derr, 4));
  CK(hipMalloc(&dt, 4));
  CK(hipMemset(derr, 0, 4));
  CK(hipMemset(dt, 0, 4));
  CK(hipMalloc(&contrib, 4 * (int64_t)B * ld));
  CK(hipMalloc(&loss, 8 * kLossSlots));
  CK(hipMemset(loss, 0, 8 * kLossSlots));
  SamplerArgs sa{};
  BatchBuf bb{dbatch, B};
  Hyper hp{0.01f, 0.001f, 1.0 - 1e-5, std::log2(1.0 - 1e-5)};
  float tb = time_loop(1, [&](int) {
    CK(build_batches(sa, 0, 0, (int64_t)S * B, B, du, di, dj, U, I, 1, false, S, bb, derr, 0));
  });
  std::vector<int32_t> meta(4);
  CK(hipMemcpy(meta.data(), bb.view(0).meta, 16, hipMemcpyDeviceToHost));
  printf("B=%d d=%d  build %d batches: %.1f us   batch0: triplets %d useg %d iseg %d long %d\n", B, D, S,
         tb, meta[0], meta[1], meta[2], meta[3]);
  const unsigned ub = (unsigned)((B + 3) / 4);
  printf("empty kernel (%u blocks):         %7.2f us\n", ub,
         time_loop(S, [&](int) { k_empty<<<ub, 256>>>(); }));
  printf("A1 record+P row r/w:              %7.2f us\n",
         time_loop(S, [&](int k) { k_a1<64, 2><<<ub, 256>>>(bb.view(k % S), P, ld); }));
  printf("A2 +Q rows, dots, contrib:        %7.2f us\n",
         time_loop(S, [&](int k) { k_a2<64, 2><<<ub, 256>>>(bb.view(k % S), P, Q, ld, contrib); }));
  const unsigned ub4 = (unsigned)((B + kBlock / 32 - 1) / (kBlock / 32));
  if (g.G4 == 32 && g.S == 1) {
    printf("A2f float4 gathers+dots+stores:   %7.2f us\n", time_loop(S, [&](int k) {
             k_a3<32, false, false><<<ub4, 256>>>(bb.view(k % S), P, Q, hp, ld, dt, k, loss, contrib);
           }));
    printf("A3  + stamps + decay:             %7.2f us\n", time_loop(S, [&](int k) {
             k_a3<32, true, false><<<ub4, 256>>>(bb.view(k % S), P, Q, hp, ld, dt, k, loss, contrib);
           }));
    printf("A4  + loss + stamp store + t:     %7.2f us\n", time_loop(S, [&](int k) {
             k_a3<32, true, true><<<ub4, 256>>>(bb.view(k % S), P, Q, hp, ld, dt, k, loss, contrib);
           }));
  }
  printf("K1 user_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, loss, contrib, nullptr, 0));
         }));
  printf("K2 item_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(item_step(g, bb.view(k % S), B, Q, hp, dt, k, contrib, nullptr, 0));
         }));
  if (g.G4 == 32 && g.S == 1) {
    const unsigned sb = (unsigned)((2 * B + 7) / 8);
    printf("K2 short segments only (timing):  %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false><<<sb, 256>>>(bb.view(k % S), Q, hp, ld, dt, k, contrib, 0, nullptr);
           }));
    const int lb = item_long_blocks(B);
    printf("K2 long segments only (timing):   %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false><<<lb, 256>>>(bb.view(k % S), Q, hp, ld, dt, k, contrib, lb, nullptr);
           }));
  }
  printf("K1+K2 step:                       %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, loss, contrib, nullptr, 0));
           CK(item_step(g, bb.view(k % S), B, Q, hp, dt, k, contrib, nullptr, 0));
         }));
  // per-kernel event pairs (every 16th step) vs the loop average: which event flavour agrees?
  for (unsigned flags : {0u, (unsigned)hipEventDisableSystemFence, (unsigned)hipEventReleaseToDevice}) {
    std::vector<hipEvent_t> ev(4 * S);
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, flags));
    CK(hipDeviceSynchronize());
    int np = 0;
    for (int k = 0; k < S; ++k) {
      const bool smp = (k % 16) == 0;
      if (smp) CK(hipEventRecord(ev[4 * np], 0));
      CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, loss, contrib, nullptr, 0));
      if (smp) CK(hipEventRecord(ev[4 * np + 1], 0));
      if (smp) CK(hipEventRecord(ev[4 * np + 2], 0));
      CK(item_step(g, bb.view(k % S), B, Q, hp, dt, k, contrib, nullptr, 0));
      if (smp) CK(hipEventRecord(ev[4 * np + 3], 0));
      np += smp;
    }
    CK(hipDeviceSynchronize());
    double a = 0, b2 = 0;
    for (int p = 0; p < np; ++p) {
      float x, y;
      CK(hipEventElapsedTime(&x, ev[4 * p], ev[4 * p + 1]));
      CK(hipEventElapsedTime(&y, ev[4 * p + 2], ev[4 * p + 3]));
      a += x;
      b2 += y;
    }
    printf("events flags=0x%08x: user_step %.2f us  item_step %.2f us (%d samples)\n", flags,
           a * 1e3 / np, b2 * 1e3 / np, np);
    for (auto& x : ev) CK(hipEventDestroy(x));
  }
  int32_t e = 0;
  CK(hipMemcpy(&e, derr, 4, hipMemcpyDeviceToHost));
  printf("err flag %d\n", e);
  return 0;
}
