// bprfm_capi.cpp — C ABI (include/bprfm.h) of the BPR-FM training path over bprfm.hip.
//
// One handle = one GPU: the embedding table, its Adagrad accumulator and gradient rows (stride
// ld = next_pow2(num_factors) floats, zero padded), the feature biases with theirs, per-row step
// stamps, the BatchNorm parameters and running statistics, and the step scratch sized for
// max_batch.  A train call uploads its triplets once and queues every batch's kernels on the
// handle's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/bprfm.h"
#include "bprfm_kernels.h"
#include "handle.h"

using namespace bprmf;

struct bprfm_handle {
  bprfm_config cfg;
  int ld = 0;
  float *E = nullptr, *acc_E = nullptr, *GE = nullptr;
  float *b = nullptr, *acc_b = nullptr, *Gb = nullptr;
  int32_t* stamp = nullptr;
  float* bn = nullptr;  // [8, ld]: gamma, beta, acc_gamma, acc_beta, ggamma, gbeta, run mean, run var
  float* bias_ = nullptr;
  float *X = nullptr, *stats = nullptr, *stats2 = nullptr, *cbuf = nullptr, *mask = nullptr;
  double *part = nullptr, *loss = nullptr, *lpart = nullptr;
  int32_t* trip = nullptr;  // [3, cap] uploaded triplets
  int64_t cap = 0;
  int64_t steps = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {
int fset_dev(const bprfm_handle* h) {
  HIPCHK(hipSetDevice(h->cfg.device));
  return 0;
}
template <typename T>
int zalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return 0;
  HIPCHK(hipMalloc((void**)p, sizeof(T) * (size_t)count));
  HIPCHK(hipMemset(*p, 0, sizeof(T) * (size_t)count));
  return 0;
}
int fill(float* p, float v, int64_t n) {
  if (n <= 0) return 0;
  std::vector<float> host((size_t)n, v);
  HIPCHK(hipMemcpy(p, host.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
  return 0;
}
fm::Args args_of(const bprfm_handle* h, int B) {
  fm::Args a{};
  a.E = h->E;
  a.acc_E = h->acc_E;
  a.GE = h->GE;
  a.b = h->b;
  a.acc_b = h->acc_b;
  a.Gb = h->Gb;
  a.stamp = h->stamp;
  a.F = h->cfg.num_features;
  // small tables: sweeping the F row stamps beats claiming 3B references with atomics
  a.sweep = a.F <= 4LL * B ? 1 : 0;
  const int ld = h->ld;
  a.gamma = h->bn;
  a.beta = h->bn + ld;
  a.acc_gamma = h->bn + 2 * ld;
  a.acc_beta = h->bn + 3 * ld;
  a.ggamma = h->bn + 4 * ld;
  a.gbeta = h->bn + 5 * ld;
  a.run = h->bn + 6 * ld;
  a.bias_ = h->bias_;
  a.B = B;
  a.k = h->cfg.num_factors;
  a.ld = ld;
  a.bn = h->cfg.batch_norm ? 1 : 0;
  a.step = (int32_t)h->steps;
  a.lr = h->cfg.lr;
  a.p = h->cfg.drop_prob;
  a.seed = h->cfg.seed;
  a.X = h->X;
  a.part = h->part;
  a.stats = h->stats;
  a.stats2 = h->stats2;
  a.cbuf = h->cbuf;
  a.loss = h->loss;
  a.lpart = h->lpart;
  return a;
}
// a 2D copy between dense [rows, k] host rows and the padded [rows, ld] device rows
int rows_to_dev(float* dst, const float* src, int64_t rows, int k, int ld, hipStream_t s) {
  if (rows <= 0) return 0;
  HIPCHK(hipMemcpy2DAsync(dst, 4 * (size_t)ld, src, 4 * (size_t)k, 4 * (size_t)k, (size_t)rows,
                          hipMemcpyHostToDevice, s));
  return 0;
}
int rows_to_host(float* dst, const float* src, int64_t rows, int k, int ld, hipStream_t s) {
  if (rows <= 0) return 0;
  HIPCHK(hipMemcpy2DAsync(dst, 4 * (size_t)k, src, 4 * (size_t)ld, 4 * (size_t)k, (size_t)rows,
                          hipMemcpyDeviceToHost, s));
  return 0;
}
}  // namespace

extern "C" {

int bprfm_create(const bprfm_config* cfg, bprfm_handle** out) {
  if (!cfg || !out) return fail(BPRMF_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->num_features <= 0 || cfg->num_factors <= 0)
    return fail(BPRMF_E_INVALID, "need num_features > 0 and num_factors > 0");
  if (cfg->num_factors > 64) return fail(BPRMF_E_UNSUPPORTED, "num_factors must be <= 64");
  if (cfg->num_features >= INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "num_features must fit int32");
  if (!(cfg->drop_prob >= 0.f && cfg->drop_prob < 1.f))
    return fail(BPRMF_E_INVALID, "drop_prob must be in [0, 1)");
  if (!(cfg->lr > 0.f)) return fail(BPRMF_E_INVALID, "lr must be > 0");
  if (cfg->max_batch <= 0) return fail(BPRMF_E_INVALID, "max_batch must be > 0");
  auto* h = new bprfm_handle();
  h->cfg = *cfg;
  h->ld = fm::lanes_for(cfg->num_factors);
  int rc = 0;
  auto bail = [&](int r) {
    bprfm_destroy(h);
    return r;
  };
  if ((rc = fset_dev(h))) return bail(rc);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess)
    return bail(fail(BPRMF_E_HIP, "stream/event creation failed"));
  const int64_t F = cfg->num_features, ld = h->ld, B = cfg->max_batch;
  const int64_t nblk = fm::part_blocks(cfg->num_factors, (int)B);
  if ((rc = zalloc(&h->E, F * ld)) || (rc = zalloc(&h->acc_E, F * ld)) ||
      (rc = zalloc(&h->GE, F * ld)) || (rc = zalloc(&h->b, F)) || (rc = zalloc(&h->acc_b, F)) ||
      (rc = zalloc(&h->Gb, F)) || (rc = zalloc(&h->stamp, F)) || (rc = zalloc(&h->bn, 8 * ld)) ||
      (rc = zalloc(&h->bias_, 1)) || (rc = zalloc(&h->X, 2 * B * ld)) ||
      (rc = zalloc(&h->stats, 4 * ld)) || (rc = zalloc(&h->stats2, 4 * ld)) ||
      (rc = zalloc(&h->cbuf, B)) || (rc = zalloc(&h->part, nblk * 4 * ld)) ||
      (rc = zalloc(&h->loss, 1)) || (rc = zalloc(&h->lpart, nblk)))
    return bail(rc);
  // Adagrad state (initial_accumulator_value 1e-8), BatchNorm weight 1 / running var 1
  if ((rc = fill(h->acc_E, 1e-8f, F * ld)) || (rc = fill(h->acc_b, 1e-8f, F)) ||
      (rc = fill(h->bn, 1.f, ld)) || (rc = fill(h->bn + 2 * ld, 1e-8f, 2 * ld)) ||
      (rc = fill(h->bn + 7 * ld, 1.f, ld)))
    return bail(rc);
  if (hipError_t e = fm::init_normal(h->E, F, cfg->num_factors, h->ld, cfg->init_std, cfg->seed,
                                     h->stream);
      e != hipSuccess || (e = hipStreamSynchronize(h->stream)) != hipSuccess)
    return bail(fail(BPRMF_E_HIP, "embedding init: %s", hipGetErrorString(e)));
  *out = h;
  return 0;
}

int bprfm_destroy(bprfm_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  void* ptrs[] = {h->E,  h->acc_E, h->GE,     h->b,    h->acc_b, h->Gb,   h->stamp, h->bn,
                  h->bias_, h->X, h->stats, h->stats2, h->cbuf, h->mask, h->part, h->loss, h->lpart, h->trip};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int bprfm_set_weights(bprfm_handle* h, const float* embeddings, const float* biases,
                      const float* bias_, const float* bn_weight, const float* bn_bias,
                      const float* running_mean, const float* running_var) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = fset_dev(h)) return r;
  const int64_t F = h->cfg.num_features;
  const int k = h->cfg.num_factors, ld = h->ld;
  hipStream_t s = h->stream;
  if (embeddings)
    if (int r = rows_to_dev(h->E, embeddings, F, k, ld, s)) return r;
  if (biases) HIPCHK(hipMemcpyAsync(h->b, biases, 4 * F, hipMemcpyHostToDevice, s));
  if (bias_) HIPCHK(hipMemcpyAsync(h->bias_, bias_, 4, hipMemcpyHostToDevice, s));
  const float* vecs[4] = {bn_weight, bn_bias, running_mean, running_var};
  const int slot[4] = {0, 1, 6, 7};
  for (int q = 0; q < 4; ++q)
    if (vecs[q]) HIPCHK(hipMemcpyAsync(h->bn + slot[q] * ld, vecs[q], 4 * k, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int bprfm_get_weights(bprfm_handle* h, float* embeddings, float* biases, float* bias_,
                      float* bn_weight, float* bn_bias, float* running_mean, float* running_var) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = fset_dev(h)) return r;
  const int64_t F = h->cfg.num_features;
  const int k = h->cfg.num_factors, ld = h->ld;
  hipStream_t s = h->stream;
  if (embeddings)
    if (int r = rows_to_host(embeddings, h->E, F, k, ld, s)) return r;
  if (biases) HIPCHK(hipMemcpyAsync(biases, h->b, 4 * F, hipMemcpyDeviceToHost, s));
  if (bias_) HIPCHK(hipMemcpyAsync(bias_, h->bias_, 4, hipMemcpyDeviceToHost, s));
  float* vecs[4] = {bn_weight, bn_bias, running_mean, running_var};
  const int slot[4] = {0, 1, 6, 7};
  for (int q = 0; q < 4; ++q)
    if (vecs[q]) HIPCHK(hipMemcpyAsync(vecs[q], h->bn + slot[q] * ld, 4 * k, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int bprfm_train(bprfm_handle* h, const int32_t* u, const int32_t* i, const int32_t* j, int64_t n,
                int32_t batch_size, bprfm_stats* st) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !j))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (batch_size <= 0 || batch_size > h->cfg.max_batch)
    return fail(BPRMF_E_INVALID, "batch_size must be in 1..max_batch (%d)", h->cfg.max_batch);
  if (n >= INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "at most 2^31 - 1 triplets per call");
  if (int r = fset_dev(h)) return r;
  const int64_t F = h->cfg.num_features;
  for (int64_t t = 0; t < n; ++t)
    if (u[t] < 0 || u[t] >= F || i[t] < 0 || i[t] >= F || j[t] < 0 || j[t] >= F)
      return fail(BPRMF_E_RANGE, "triplet %lld = (%d, %d, %d): feature out of range [0, %lld)",
                  (long long)t, u[t], i[t], j[t], (long long)F);
  if (n > h->cap) {
    if (h->trip) HIPCHK(hipFree(h->trip));
    h->trip = nullptr;
    h->cap = 0;
    HIPCHK(hipMalloc((void**)&h->trip, 12 * (size_t)n));
    h->cap = n;
  }
  hipStream_t s = h->stream;
  if (n) {
    HIPCHK(hipMemcpyAsync(h->trip, u, 4 * n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->trip + h->cap, i, 4 * n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->trip + 2 * h->cap, j, 4 * n, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemsetAsync(h->loss, 0, 8, s));
  HIPCHK(hipEventRecord(h->ev0, s));
  int64_t nsteps = 0;
  for (int64_t beg = 0; beg < n; beg += batch_size, ++nsteps) {
    const int B = (int)std::min<int64_t>(batch_size, n - beg);
    fm::Args a = args_of(h, B);
    a.u = h->trip + beg;
    a.i = h->trip + h->cap + beg;
    a.j = h->trip + 2 * h->cap + beg;
    if (hipError_t e = fm::step(a, s); e != hipSuccess)
      return fail(BPRMF_E_HIP, "bprfm step: %s", hipGetErrorString(e));
    ++h->steps;
  }
  HIPCHK(hipEventRecord(h->ev1, s));
  double loss = 0.0;
  HIPCHK(hipMemcpyAsync(&loss, h->loss, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (st) {
    st->triplets = n;
    st->steps = nsteps;
    st->loss = loss;
    st->seconds = ms * 1e-3;
  }
  return 0;
}

int bprfm_dropout_mask(bprfm_handle* h, int32_t B, float* out) {
  if (!h || B < 0 || (B > 0 && !out)) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!B) return 0;
  if (int r = fset_dev(h)) return r;
  const int64_t n = 2LL * B * h->cfg.num_factors;
  float* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, 4 * (size_t)n));
  hipError_t e = fm::dropout_mask(args_of(h, B), d, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(BPRMF_E_HIP, "bprfm_dropout_mask: %s", hipGetErrorString(e));
  return 0;
}

int bprfm_predict(bprfm_handle* h, const int32_t* u, const int32_t* x, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!u || !x || !out))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!n) return 0;
  if (int r = fset_dev(h)) return r;
  const int64_t F = h->cfg.num_features;
  for (int64_t q = 0; q < n; ++q)
    if (u[q] < 0 || u[q] >= F || x[q] < 0 || x[q] >= F)
      return fail(BPRMF_E_RANGE, "pair %lld = (%d, %d): feature out of range", (long long)q, u[q], x[q]);
  int32_t* d = nullptr;
  float* dout = nullptr;
  HIPCHK(hipMalloc((void**)&d, 8 * (size_t)n));
  if (hipMalloc((void**)&dout, 4 * (size_t)n) != hipSuccess) {
    (void)hipFree(d);
    return fail(BPRMF_E_HIP, "hipMalloc failed");
  }
  hipStream_t s = h->stream;
  hipError_t e = hipMemcpyAsync(d, u, 4 * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d + n, x, 4 * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = fm::predict(args_of(h, 0), d, d + n, n, dout, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, 4 * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(BPRMF_E_HIP, "bprfm_predict: %s", hipGetErrorString(e));
  return 0;
}

int64_t bprfm_steps(const bprfm_handle* h) { return h ? h->steps : -1; }

}  // extern "C"
