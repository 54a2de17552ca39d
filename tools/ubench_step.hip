// ubench_step.hip — microbenchmark of the segmented step kernels and their parts (K2 long items,
// short items, multi-triplet users), to locate where a step's time goes.  Development tool (not part of the product library).
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
  const int ld = g.ld;
  std::mt19937_64 rng(7);
  // triplets: users ~ lognormal degree (heavy users repeat), positives Zipf(1), negatives uniform
  std::vector<double> cdf(I), ucdf(U);
  double acc = 0;
  for (int64_t r = 0; r < I; ++r) cdf[r] = (acc += 1.0 / (r + 1));
  for (auto& x : cdf) x /= acc;
  std::lognormal_distribution<double> LN(3.5, 1.2);
  acc = 0;
  for (int64_t r = 0; r < U; ++r) ucdf[r] = (acc += std::max(10.0, LN(rng)));
  for (auto& x : ucdf) x /= acc;
  std::vector<int32_t> hu(S * (int64_t)B), hi(S * (int64_t)B), hj(S * (int64_t)B);
  std::uniform_real_distribution<double> U01(0, 1);
  for (int64_t k = 0; k < (int64_t)S * B; ++k) {
    hu[k] = (int32_t)(std::lower_bound(ucdf.begin(), ucdf.end(), U01(rng)) - ucdf.begin());
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
  float *contrib, *ugrad;
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
  CK(hipMalloc(&ugrad, 4 * (int64_t)B * ld));
  CK(hipMemset(contrib, 0, 4 * (int64_t)B * ld));
  CK(hipMemset(ugrad, 0, 4 * (int64_t)B * ld));
  CK(hipMalloc(&loss, 8 * kLossSlots));
  CK(hipMemset(loss, 0, 8 * kLossSlots));
  SamplerArgs sa{};
  BatchBuf bb{dbatch, B};
  Hyper hp{0.01f, 0.001f, 1.0 - 1e-5, std::log2(1.0 - 1e-5)};
  float tb = time_loop(1, [&](int) {
    CK(build_batches(sa, 0, 0, (int64_t)S * B, B, du, di, dj, U, I, 1, false, 0, S, bb, derr, 0));
  });
  std::vector<int32_t> meta(8);
  CK(hipMemcpy(meta.data(), bb.view(0).meta, 32, hipMemcpyDeviceToHost));
  printf("B=%d d=%d  build %d batches: %.1f us   batch0: triplets %d useg %d iseg %d long %d multi-users %d\n",
         B, D, S, tb, meta[0], meta[1], meta[2], meta[3], meta[4]);
  printf("empty kernel (%u x 256):          %7.2f us\n", (unsigned)(B / 8),
         time_loop(S, [&](int) { k_empty<<<B / 8, 256>>>(); }));
  printf("empty kernel (%u x 1024):         %7.2f us\n", (unsigned)(B / 32),
         time_loop(S, [&](int) { k_empty<<<B / 32, 1024>>>(); }));
  printf("K1 user_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, loss, contrib, ugrad, nullptr, 0));
         }));
  printf("K2 item_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, 0));
         }));
  if (g.G4 == 32 && g.S == 1) {
    constexpr int KB = 1024, NG = KB / 32;
    const int lb = item_long_blocks(B);
    const int ib = (2 * B + NG - 1) / NG, ubk = (B / 2 + NG - 1) / NG;
    printf("K2 long items only:               %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<lb, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                       ugrad, lb, ib, nullptr);
           }));
    printf("K2 short items only:              %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<ib, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                       ugrad, 0, ib, nullptr);
           }));
    printf("K2 multi-triplet users only:      %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<ubk, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                        ugrad, 0, 0, nullptr);
           }));
  }
  printf("K1+K2 step:                       %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, loss, contrib, ugrad, nullptr, 0));
           CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, 0));
         }));
  int32_t e = 0;
  CK(hipMemcpy(&e, derr, 4, hipMemcpyDeviceToHost));
  printf("err flag %d\n", e);
  return 0;
}
