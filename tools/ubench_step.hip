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
__device__ int4 g_rec[4096];
__device__ int g_sink;
__global__ void k_load_noarg() {  // one dependent load, no kernel arguments
  const int4 r = g_rec[blockIdx.x * 8 + threadIdx.x / 32];
  if (r.x == -12345) g_sink = r.y;
}
// argument-free step kernels: parameters in a code-object global, the step index in counters that
// each kernel's block 0 writes for the other kernel (safe: the other kernel is not running)
struct UbParams {
  const int4* trec;
  int64_t stride;  // int4 per batch
};
__device__ UbParams g_ub;
__device__ int g_ca, g_cb;
template <int WHO>
__global__ void k_noarg_trec() {
  const int step = WHO == 0 ? g_ca : g_cb;
  const int4 r = g_ub.trec[step * g_ub.stride + blockIdx.x * 8 + threadIdx.x / 32];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (WHO == 0) g_cb = step; else g_ca = step + 1 == 256 ? 0 : step + 1;
  }
  if (r.x == -12345) g_sink = r.y;
}
template <int WHO>
__global__ void k_arg_trec(const int4* trec, int64_t stride, int step) {
  const int4 r = trec[step * stride + blockIdx.x * 8 + threadIdx.x / 32];
  if (r.x == -12345) g_sink = r.y;
}
// a copy of k_user_step (G4 = 32, S = 1) with its parts switchable (bit set = part ON):
// 1 loss, 2 decay stamps, 4 single-user update, 8 ugrad store, 16 contrib store, 32 meta/tbase loads
template <int F>
__global__ __launch_bounds__(kBlock) void k_k1x(BatchView bv, Table P, Table Q, Hyper hp, int ld,
                                                const int32_t* __restrict__ tbase, int step,
                                                double* loss, float* __restrict__ contrib,
                                                float* __restrict__ ugrad) {
  const int sub = threadIdx.x & 31;
  const int p = blockIdx.x * (kBlock / 32) + threadIdx.x / 32;
  const int4 r = reinterpret_cast<const int4*>(bv.trec)[p];
  const int n = (F & 32) ? bv.meta[0] : 4096;
  const int32_t t = (F & 32) ? *tbase + step + 1 : step + 1;
  float lsum = 0.f;
  if (p < n) {
    const int32_t i = r.x, j = r.y, u = r.z;
    float* pw = P.W + (int64_t)u * ld + 4 * sub;
    float4 pu = *reinterpret_cast<const float4*>(pw);
    float4 vi = *reinterpret_cast<const float4*>(Q.W + (int64_t)i * ld + 4 * sub);
    float4 vj = *reinterpret_cast<const float4*>(Q.W + (int64_t)j * ld + 4 * sub);
    float fi = 1.f, fj = 1.f, fu = 1.f;
    if (F & 2) {
      fi = decay_pow(hp.log2a, t - 1 - Q.stamp[i]);
      fj = decay_pow(hp.log2a, t - 1 - Q.stamp[j]);
      fu = decay_pow(hp.log2a, t - 1 - P.stamp[u]);
    }
    pu = make_float4(pu.x * fu, pu.y * fu, pu.z * fu, pu.w * fu);
    vi = make_float4(vi.x * fi, vi.y * fi, vi.z * fi, vi.w * fi);
    vj = make_float4(vj.x * fj, vj.y * fj, vj.z * fj, vj.w * fj);
    float di = pu.x * vi.x + pu.y * vi.y + pu.z * vi.z + pu.w * vi.w;
    float dj = pu.x * vj.x + pu.y * vj.y + pu.z * vj.z + pu.w * vj.w;
    di = group_sum<32>(di);
    dj = group_sum<32>(dj);
    const float x = di - dj;
    const float c = 1.0f / (1.0f + expf(x));
    if ((F & 1) && sub == 0) lsum = softplus(-x);
    if (F & 16)
      *reinterpret_cast<float4*>(contrib + (int64_t)p * ld + 4 * sub) =
          make_float4(pu.x * c, pu.y * c, pu.z * c, pu.w * c);
    const float4 gg = make_float4(-c * (vi.x - vj.x), -c * (vi.y - vj.y), -c * (vi.z - vj.z), -c * (vi.w - vj.w));
    if (r.w) {
      if (F & 4) {
        *reinterpret_cast<float4*>(pw) = make_float4(pu.x - 0.01f * gg.x, pu.y - 0.01f * gg.y,
                                                     pu.z - 0.01f * gg.z, pu.w - 0.01f * gg.w);
        if (sub == 0) P.stamp[u] = t;
      }
    } else if (F & 8) {
      *reinterpret_cast<float4*>(ugrad + (int64_t)p * ld + 4 * sub) = gg;
    }
    if (!(F & 28) && x == -12345.f) contrib[p] = x;
  }
  if (F & 1) wave_add_loss(loss, lsum);
}

template <class F>
static float graph_time(int steps, F&& body) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraph_t gr;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int k = 0; k < steps; ++k) body(k, st);
  CK(hipStreamEndCapture(st, &gr));
  CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(gr));
  CK(hipStreamDestroy(st));
  return ms * 1e3f / (10 * steps);
}

__global__ void k_arg_only(const int* a) {  // reads a kernel argument, no memory load
  if ((size_t)a == 12345) g_sink = 1;
}

// K1 decomposition (G4 = 32, S = 1: d = 128): which dependent level / store costs what
template <int LV, int ST, int LS = 0>
__global__ __launch_bounds__(kBlock) void k_v1(BatchView bv, Table P, Table Q, int ld, float* out,
                                               double* loss = nullptr, float* lpart = nullptr) {
  const int sub = threadIdx.x & 31;
  const int p = blockIdx.x * (kBlock / 32) + threadIdx.x / 32;
  const int4 r = reinterpret_cast<const int4*>(bv.trec)[p];
  float acc = (float)r.x;
  if (LV >= 2) {
    const float4 a = *reinterpret_cast<const float4*>(P.W + (int64_t)r.z * ld + 4 * sub);
    const float4 b = *reinterpret_cast<const float4*>(Q.W + (int64_t)r.x * ld + 4 * sub);
    const float4 c = *reinterpret_cast<const float4*>(Q.W + (int64_t)r.y * ld + 4 * sub);
    const int32_t su = P.stamp[r.z] + Q.stamp[r.x] + Q.stamp[r.y];
    acc = a.x * (b.x - c.x) + a.y * (b.y - c.y) + a.z * (b.z - c.z) + a.w * (b.w - c.w) + (float)su;
    acc = group_sum<32>(acc);
    if (ST == 1) {
      *reinterpret_cast<float4*>(out + (int64_t)p * ld + 4 * sub) = make_float4(a.x * acc, a.y, a.z, a.w);
      const float lv = sub == 0 ? softplus(-acc) : 0.f;
      if (LS == 1) wave_add_loss(loss, lv);
      if (LS == 2) {
        float v = lv;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0) lpart[blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)] = v;
      }
      if (LS == 3) {
        __shared__ float red[kBlock / 64];
        float v = lv;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd(&loss[blockIdx.x], (double)(red[0] + red[1] + red[2] + red[3]));
      }
      return;
    }
    if (ST == 2) {
      __builtin_nontemporal_store(a.x * acc, out + (int64_t)p * ld + 4 * sub);
      __builtin_nontemporal_store(a.y, out + (int64_t)p * ld + 4 * sub + 1);
      __builtin_nontemporal_store(a.z, out + (int64_t)p * ld + 4 * sub + 2);
      __builtin_nontemporal_store(a.w, out + (int64_t)p * ld + 4 * sub + 3);
      return;
    }
  }
  if (acc == -12345.f) out[p] = acc;
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
  float* xl;
  CK(hipMalloc(&xl, 4 * (int64_t)B));
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
  if (g.G4 == 32 && g.S == 1) {
    const unsigned nb = (unsigned)(B / (kBlock / 32));
    printf("K1 parts: trec only:              %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<1, 0><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib); }));
    printf("K1 parts: trec only, same batch:  %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<1, 0><<<nb, kBlock>>>(bb.view(0), P, Q, ld, contrib); }));
    printf("K1 parts: trec only, 2 batches:   %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<1, 0><<<nb, kBlock>>>(bb.view(k & 1), P, Q, ld, contrib); }));
    printf("K1 parts: trec->rows, no store:   %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 0><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib); }));
    printf("K1 parts: trec->rows->store:      %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 1><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib); }));
    printf("K1 parts: +loss f64 atomic/wave:  %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 1, 1><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib, loss); }));
    printf("K1 parts: +loss f32 store/wave:   %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 1, 2><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib, loss, ugrad); }));
    printf("K1 parts: +loss f64 atomic/block: %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 1, 3><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib, loss); }));
    printf("K1 parts: trec->rows->nt store:   %7.2f us\n", time_loop(S, [&](int k) {
             k_v1<2, 2><<<nb, kBlock>>>(bb.view(k % S), P, Q, ld, contrib); }));
  }
  printf("one load, no kernargs:            %7.2f us\n", time_loop(S, [&](int) { k_load_noarg<<<B / 8, 256>>>(); }));
  printf("kernarg read only:                %7.2f us\n", time_loop(S, [&](int) { k_arg_only<<<B / 8, 256>>>(dt); }));
  {
    UbParams up{reinterpret_cast<const int4*>(bb.view(0).trec),
                (int64_t)(bb.view(1).trec - bb.view(0).trec) / 4};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ub), &up, sizeof(up)));
    int zero = 0;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ca), &zero, 4));
    printf("pair of trec kernels, kernargs:   %7.2f us\n", time_loop(S, [&](int k) {
             k_arg_trec<0><<<B / 8, 256>>>(up.trec, up.stride, k % S);
             k_arg_trec<1><<<B / 8, 256>>>(up.trec, up.stride, k % S); }));
    printf("pair of trec kernels, no args:    %7.2f us\n", time_loop(S, [&](int k) {
             k_noarg_trec<0><<<B / 8, 256>>>();
             k_noarg_trec<1><<<B / 8, 256>>>(); }));
    // the same under a captured graph of 64 pairs
    for (int mode = 0; mode < 2; ++mode) {
      hipStream_t st;
      CK(hipStreamCreate(&st));
      hipGraph_t gr;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < 64; ++k) {
        if (mode == 0) {
          k_arg_trec<0><<<B / 8, 256, 0, st>>>(up.trec, up.stride, k);
          k_arg_trec<1><<<B / 8, 256, 0, st>>>(up.trec, up.stride, k);
        } else {
          k_noarg_trec<0><<<B / 8, 256, 0, st>>>();
          k_noarg_trec<1><<<B / 8, 256, 0, st>>>();
        }
      }
      CK(hipStreamEndCapture(st, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("graph pair of trec kernels, %s: %7.2f us\n", mode ? "no args " : "kernargs", ms * 1e3f / 640);
    }
  }
  printf("K1 user_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, xl, contrib, ugrad, nullptr, 0));
         }));
  printf("K1 user_step, same batch:         %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(0), B, P, Q, hp, dt, k, xl, contrib, ugrad, nullptr, 0));
         }));
  printf("K2 item_step, same batch:         %7.2f us\n", time_loop(S, [&](int k) {
           CK(item_step(g, bb.view(0), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, 0, xl, loss));
         }));
  printf("K1 user_step (no loss):           %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, nullptr, contrib, ugrad, nullptr, 0));
         }));
  printf("K2 item_step:                     %7.2f us\n", time_loop(S, [&](int k) {
           CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, 0, xl, loss));
         }));
  if (g.G4 == 32 && g.S == 1) {
    constexpr int KB = 1024, NG = KB / 32;
    const int lb = item_long_blocks(B);
    const int ib = (2 * B + NG - 1) / NG, ubk = (B / 2 + NG - 1) / NG;
    printf("K2 long items only:               %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<lb, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                       ugrad, lb, ib, nullptr, nullptr, nullptr);
           }));
    printf("K2 short items only:              %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<ib, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                       ugrad, 0, ib, nullptr, nullptr, nullptr);
           }));
    printf("K2 multi-triplet users only:      %7.2f us\n", time_loop(S, [&](int k) {
             k_item_step<32, 1, false, KB><<<ubk, KB>>>(bb.view(k % S), P, Q, hp, ld, dt, k, contrib,
                                                        ugrad, 0, 0, nullptr, nullptr, nullptr);
           }));
  }
  printf("K1+K2 step:                       %7.2f us\n", time_loop(S, [&](int k) {
           CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, xl, contrib, ugrad, nullptr, 0));
           CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, 0, xl, loss));
         }));
  if (g.G4 == 32 && g.S == 1) {
    const unsigned nb = (unsigned)(B / (kBlock / 32));
#define K1X(FL)                                                                                   \
  printf("graph K1 copy, parts %2d:          %7.2f us\n", FL, graph_time(64, [&](int k, hipStream_t st) { \
           k_k1x<FL><<<nb, kBlock, 0, st>>>(bb.view(k % S), P, Q, hp, ld, dt, k, loss, contrib, ugrad); }));
    K1X(63) K1X(62) K1X(61) K1X(59) K1X(55) K1X(47) K1X(31) K1X(16) K1X(0)
    printf("graph K1 product:                 %7.2f us\n", graph_time(64, [&](int k, hipStream_t st) {
             CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, xl, contrib, ugrad, nullptr, st)); }));
    printf("graph K2 product:                 %7.2f us\n", graph_time(64, [&](int k, hipStream_t st) {
             CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, st, xl, loss)); }));
    printf("graph empty 512x256:              %7.2f us\n", graph_time(64, [&](int k, hipStream_t st) {
             k_empty<<<nb, kBlock, 0, st>>>(); }));
  }
  for (int nbg : {64, 256}) {  // the product's form: a captured chunk of steps, replayed
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < nbg; ++k) {
      CK(user_step(g, bb.view(k % S), B, P, Q, hp, dt, k, xl, contrib, ugrad, nullptr, st));
      CK(item_step(g, bb.view(k % S), B, P, Q, hp, dt, k, contrib, ugrad, nullptr, st, xl, loss));
    }
    CK(hipStreamEndCapture(st, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("graph of %3d K1+K2 steps:         %7.2f us/step\n", nbg, ms * 1e3f / (10 * nbg));
  }
  int32_t e = 0;
  CK(hipMemcpy(&e, derr, 4, hipMemcpyDeviceToHost));
  printf("err flag %d\n", e);
  return 0;
}
