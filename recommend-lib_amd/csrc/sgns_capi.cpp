// sgns_capi.cpp — C ABI (include/sgns.h) of the Item2Vec training path over sgns.hip, rocBLAS
// (the ovectors-gradient GEMM) and the dense Adam sweep of ncf.hip.
//
// One handle = one GPU: ivectors / ovectors [V, ld] (ld = E rounded up to 4 floats), their Adam
// moments, the ivectors gradient, the per-row touch steps, and the step scratch sized for
// max_batch: S [V, B] (the coefficient matrix of the ovectors gradient, zero between steps),
// IB [B, ld], GO [V, ld] or its split partials, per-example losses.  Per step: K1, the GEMM
// (split over B), then one elementwise launch: Adam over both tables, S cleared, the loss sum.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/sgns.h"
#include "handle.h"
#include "ncf_kernels.h"
#include "sgns_kernels.h"

using namespace bprmf;

struct sgns_handle {
  sgns_config cfg;
  int ld = 0;
  float *I = nullptr, *O = nullptr, *mI = nullptr, *vI = nullptr, *mO = nullptr, *vO = nullptr;
  float *GI = nullptr, *GO = nullptr, *GOp = nullptr, *S = nullptr, *IB = nullptr, *lbuf = nullptr, *cdf = nullptr;
  int32_t *touch_i = nullptr, *touch_o = nullptr;
  int32_t* ex = nullptr;  // uploaded examples: iwords [cap], owords [cap, C], nwords [cap, C n]
  int64_t cap = 0;
  double* loss = nullptr;
  int64_t t = 0;  // Adam steps taken
  rocblas_handle blas = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {
// the ovectors-gradient GEMM has ceil(E/128) x ceil(V/64) output tiles; with V ~ 2k that is far
// fewer workgroups than CUs, so the reduction over the batch is split into partial products
constexpr int kMaxSplit = 8;
int split_for(int B) { return std::max(1, std::min(kMaxSplit, B / 512)); }
int sset_dev(const sgns_handle* h) {
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
sgns::Args args_of(const sgns_handle* h, int B) {
  sgns::Args a{};
  a.I = h->I;
  a.O = h->O;
  a.GI = h->GI;
  a.touch_i = h->touch_i;
  a.touch_o = h->touch_o;
  a.S = h->S;
  a.IB = h->IB;
  a.lbuf = h->lbuf;
  a.cdf = h->cdf;
  a.V = h->cfg.vocab_size;
  a.E = h->cfg.embedding_size;
  a.ld = h->ld;
  a.B = B;
  a.C = h->cfg.context;
  a.n = h->cfg.n_negs;
  a.t = (int32_t)(h->t + 1);
  a.seed = h->cfg.seed;
  a.loss = h->loss;
  return a;
}
ncf::AdamArgs adam_args(const sgns_handle* h, int64_t t) {
  const double b1 = h->cfg.beta1, b2 = h->cfg.beta2;
  ncf::AdamArgs a;
  a.one_minus_b1 = (float)(1.0 - b1);
  a.b2 = (float)b2;
  a.one_minus_b2 = (float)(1.0 - b2);
  a.eps = h->cfg.eps;
  a.step_size = (float)((double)h->cfg.lr / (1.0 - std::pow(b1, (double)t)));
  a.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(b2, (double)t));
  return a;
}
int rows_in(float* dst, const float* src, int64_t rows, int E, int ld, hipStream_t s) {
  if (rows <= 0) return 0;
  HIPCHK(hipMemcpy2DAsync(dst, 4 * (size_t)ld, src, 4 * (size_t)E, 4 * (size_t)E, (size_t)rows,
                          hipMemcpyHostToDevice, s));
  return 0;
}
int rows_out(float* dst, const float* src, int64_t rows, int E, int ld, hipStream_t s) {
  if (rows <= 0) return 0;
  HIPCHK(hipMemcpy2DAsync(dst, 4 * (size_t)E, src, 4 * (size_t)ld, 4 * (size_t)E, (size_t)rows,
                          hipMemcpyDeviceToHost, s));
  return 0;
}
int check_ids(const int32_t* x, int64_t n, int64_t V, const char* what) {
  for (int64_t q = 0; q < n; ++q)
    if (x[q] < 0 || x[q] >= V)
      return fail(BPRMF_E_RANGE, "%s[%lld] = %d out of range [0, %lld)", what, (long long)q, x[q],
                  (long long)V);
  return 0;
}
}  // namespace

extern "C" {

int sgns_create(const sgns_config* cfg, sgns_handle** out) {
  if (!cfg || !out) return fail(BPRMF_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->vocab_size < 2 || cfg->embedding_size <= 0 || cfg->n_negs < 0 || cfg->context <= 0)
    return fail(BPRMF_E_INVALID, "need vocab_size >= 2, embedding_size > 0, context > 0, n_negs >= 0");
  if (cfg->embedding_size > 1024) return fail(BPRMF_E_UNSUPPORTED, "embedding_size must be <= 1024");
  if ((int64_t)cfg->context * (1 + (int64_t)cfg->n_negs) > 1024)  // sgns.hip kMaxR
    return fail(BPRMF_E_UNSUPPORTED, "context * (1 + n_negs) must be <= 1024");
  if (cfg->vocab_size >= INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "vocab_size must fit int32");
  if (cfg->max_batch <= 0) return fail(BPRMF_E_INVALID, "max_batch must be > 0");
  if (!(cfg->lr > 0.f) || !(cfg->eps > 0.f) || !(cfg->beta1 >= 0.f && cfg->beta1 < 1.f) ||
      !(cfg->beta2 >= 0.f && cfg->beta2 < 1.f))
    return fail(BPRMF_E_INVALID, "bad Adam hyper-parameters");
  auto* h = new sgns_handle();
  h->cfg = *cfg;
  h->ld = (cfg->embedding_size + 3) / 4 * 4;
  int rc = 0;
  auto bail = [&](int r) {
    sgns_destroy(h);
    return r;
  };
  if ((rc = sset_dev(h))) return bail(rc);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess)
    return bail(fail(BPRMF_E_HIP, "stream/event creation failed"));
  if (rocblas_create_handle(&h->blas) != rocblas_status_success ||
      rocblas_set_stream(h->blas, h->stream) != rocblas_status_success)
    return bail(fail(BPRMF_E_HIP, "rocblas handle creation failed"));
  const int64_t V = cfg->vocab_size, ld = h->ld, B = cfg->max_batch;
  float** tabs[] = {&h->I, &h->mI, &h->vI, &h->mO, &h->vO, &h->GI, &h->GO};
  for (float** p : tabs)
    if ((rc = zalloc(p, V * ld))) return bail(rc);
  // ovectors: one padding row of 1024 floats past the end (sgns.hip reads whole 64-lane strides)
  if ((rc = zalloc(&h->O, V * ld + 1024))) return bail(rc);
  if ((rc = zalloc(&h->GOp, (int64_t)kMaxSplit * V * ld)) || (rc = zalloc(&h->S, V * B)) || (rc = zalloc(&h->IB, B * ld)) || (rc = zalloc(&h->lbuf, B)) ||
      (rc = zalloc(&h->touch_i, V)) || (rc = zalloc(&h->touch_o, V)) || (rc = zalloc(&h->loss, 1)))
    return bail(rc);
  if (hipMemset(h->touch_i, 0xff, 4 * V) != hipSuccess || hipMemset(h->touch_o, 0xff, 4 * V) != hipSuccess)
    return bail(fail(BPRMF_E_HIP, "hipMemset failed"));
  const float lim = 0.5f / (float)cfg->embedding_size;
  hipError_t e = sgns::init_uniform(h->I, V, cfg->embedding_size, h->ld, lim, cfg->seed, 0x49564543u, h->stream);
  if (e == hipSuccess)
    e = sgns::init_uniform(h->O, V, cfg->embedding_size, h->ld, lim, cfg->seed, 0x4F564543u, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return bail(fail(BPRMF_E_HIP, "table init: %s", hipGetErrorString(e)));
  *out = h;
  return 0;
}

int sgns_destroy(sgns_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  void* ptrs[] = {h->GOp, h->I,  h->O,    h->mI,   h->vI,      h->mO,      h->vO, h->GI, h->GO, h->S,
                  h->IB, h->lbuf, h->cdf, h->touch_i, h->touch_o, h->ex, h->loss};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (h->blas) rocblas_destroy_handle(h->blas);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int sgns_set_noise(sgns_handle* h, const double* weights) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = sset_dev(h)) return r;
  if (!weights) {
    if (h->cdf) HIPCHK(hipFree(h->cdf));
    h->cdf = nullptr;
    return 0;
  }
  const int64_t V = h->cfg.vocab_size;
  // SGNS.__init__: wf = weights^0.75, wf / wf.sum() (:77-80); its CDF for inverse sampling
  std::vector<double> wf(V);
  double tot = 0.0;
  for (int64_t x = 0; x < V; ++x) {
    if (!(weights[x] >= 0.0)) return fail(BPRMF_E_INVALID, "weights must be >= 0");
    wf[x] = std::pow(weights[x], 0.75);
    tot += wf[x];
  }
  if (!(tot > 0.0)) return fail(BPRMF_E_INVALID, "weights sum to 0");
  std::vector<float> cdf(V);
  double acc = 0.0;
  for (int64_t x = 0; x < V; ++x) {
    acc += wf[x] / tot;
    cdf[x] = (float)acc;
  }
  cdf[V - 1] = 2.0f;  // every u in [0, 1) lands
  if (!h->cdf) HIPCHK(hipMalloc((void**)&h->cdf, 4 * (size_t)V));
  HIPCHK(hipMemcpy(h->cdf, cdf.data(), 4 * (size_t)V, hipMemcpyHostToDevice));
  return 0;
}

int sgns_set_weights(sgns_handle* h, const float* ivectors, const float* ovectors) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = sset_dev(h)) return r;
  const int64_t V = h->cfg.vocab_size;
  const int E = h->cfg.embedding_size;
  if (ivectors)
    if (int r = rows_in(h->I, ivectors, V, E, h->ld, h->stream)) return r;
  if (ovectors)
    if (int r = rows_in(h->O, ovectors, V, E, h->ld, h->stream)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int sgns_get_weights(sgns_handle* h, float* ivectors, float* ovectors) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = sset_dev(h)) return r;
  const int64_t V = h->cfg.vocab_size;
  const int E = h->cfg.embedding_size;
  if (ivectors)
    if (int r = rows_out(ivectors, h->I, V, E, h->ld, h->stream)) return r;
  if (ovectors)
    if (int r = rows_out(ovectors, h->O, V, E, h->ld, h->stream)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int sgns_set_adam(sgns_handle* h, int64_t step, const float* m_i, const float* v_i,
                  const float* m_o, const float* v_o) {
  if (!h || step < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = sset_dev(h)) return r;
  const int64_t V = h->cfg.vocab_size;
  const int E = h->cfg.embedding_size;
  const float* src[4] = {m_i, v_i, m_o, v_o};
  float* dst[4] = {h->mI, h->vI, h->mO, h->vO};
  std::vector<int32_t> ti(V, -1), to(V, -1);
  for (int q = 0; q < 4; ++q) {
    if (!src[q]) continue;
    if (int r = rows_in(dst[q], src[q], V, E, h->ld, h->stream)) return r;
    std::vector<int32_t>& touch = q < 2 ? ti : to;
    for (int64_t x = 0; x < V; ++x)
      for (int e = 0; e < E; ++e)
        if (src[q][x * E + e] != 0.f) {
          touch[x] = 0;  // updated in an earlier step
          break;
        }
  }
  HIPCHK(hipMemcpyAsync(h->touch_i, ti.data(), 4 * V, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->touch_o, to.data(), 4 * V, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->t = step;
  return 0;
}

int sgns_get_adam(sgns_handle* h, int64_t* step, float* m_i, float* v_i, float* m_o, float* v_o) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = sset_dev(h)) return r;
  const int64_t V = h->cfg.vocab_size;
  const int E = h->cfg.embedding_size;
  float* dst[4] = {m_i, v_i, m_o, v_o};
  const float* src[4] = {h->mI, h->vI, h->mO, h->vO};
  for (int q = 0; q < 4; ++q)
    if (dst[q])
      if (int r = rows_out(dst[q], src[q], V, E, h->ld, h->stream)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  if (step) *step = h->t;
  return 0;
}

int sgns_train(sgns_handle* h, const int32_t* iwords, const int32_t* owords, const int32_t* nwords,
               int64_t n, int32_t batch_size, sgns_stats* st) {
  if (!h || n < 0 || (n > 0 && (!iwords || !owords))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (batch_size <= 0 || batch_size > h->cfg.max_batch)
    return fail(BPRMF_E_INVALID, "batch_size must be in 1..max_batch (%d)", h->cfg.max_batch);
  if (n >= INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "at most 2^31 - 1 examples per call");
  if (int r = sset_dev(h)) return r;
  const int64_t V = h->cfg.vocab_size, C = h->cfg.context, CN = C * h->cfg.n_negs;
  if (int r = check_ids(iwords, n, V, "iwords")) return r;
  if (int r = check_ids(owords, n * C, V, "owords")) return r;
  if (nwords)
    if (int r = check_ids(nwords, n * CN, V, "nwords")) return r;
  const int64_t per = 1 + C + CN;
  if (n > h->cap) {
    if (h->ex) HIPCHK(hipFree(h->ex));
    h->ex = nullptr;
    h->cap = 0;
    HIPCHK(hipMalloc((void**)&h->ex, 4 * (size_t)(per * n)));
    h->cap = n;
  }
  int32_t *d_iw = h->ex, *d_ow = h->ex + h->cap, *d_nw = h->ex + h->cap * (1 + C);
  hipStream_t s = h->stream;
  if (n) {
    HIPCHK(hipMemcpyAsync(d_iw, iwords, 4 * n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_ow, owords, 4 * n * C, hipMemcpyHostToDevice, s));
    if (nwords && CN) HIPCHK(hipMemcpyAsync(d_nw, nwords, 4 * n * CN, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemsetAsync(h->loss, 0, 8, s));
  HIPCHK(hipEventRecord(h->ev0, s));
  const int E = h->cfg.embedding_size;
  const float one = 1.f, zero = 0.f;
  int64_t nsteps = 0;
  for (int64_t beg = 0; beg < n; beg += batch_size, ++nsteps) {
    const int B = (int)std::min<int64_t>(batch_size, n - beg);
    sgns::Args a = args_of(h, B);
    a.iw = d_iw + beg;
    a.ow = d_ow + beg * C;
    a.nw = nwords ? d_nw + beg * CN : nullptr;
    HIPCHK(sgns::forward_backward(a, s));  // S is zero: at create, then after every step
    // GO^T [E, V] = IB^T [E, B] x S^T [B, V] in rocBLAS's column-major terms, as nsp products
    // over slices of B (slice q: columns q Bs.. of IB^T, rows of S^T) summed in a fixed order
    const int nsp = split_for(B), Bs = B / nsp, tail = B - Bs * nsp;
    if (nsp == 1) {
      if (rocblas_sgemm(h->blas, rocblas_operation_none, rocblas_operation_none, E, (rocblas_int)V,
                        B, &one, h->IB, h->ld, h->S, B, &zero, h->GO, h->ld) != rocblas_status_success)
        return fail(BPRMF_E_HIP, "rocblas_sgemm failed");
    } else {
      if (rocblas_sgemm_strided_batched(h->blas, rocblas_operation_none, rocblas_operation_none, E,
                                        (rocblas_int)V, Bs, &one, h->IB, h->ld, (rocblas_stride)Bs * h->ld,
                                        h->S, B, (rocblas_stride)Bs, &zero, h->GOp, h->ld,
                                        (rocblas_stride)V * h->ld, nsp) != rocblas_status_success)
        return fail(BPRMF_E_HIP, "rocblas_sgemm_strided_batched failed");
      if (tail &&  // the last B % nsp examples into the last partial
          rocblas_sgemm(h->blas, rocblas_operation_none, rocblas_operation_none, E, (rocblas_int)V,
                        tail, &one, h->IB + (int64_t)Bs * nsp * h->ld, h->ld, h->S + Bs * nsp, B,
                        &one, h->GOp + (int64_t)(nsp - 1) * V * h->ld, h->ld) != rocblas_status_success)
        return fail(BPRMF_E_HIP, "rocblas_sgemm failed");
    }
    // Adam on both tables, S cleared, the loss: one launch
    const ncf::AdamArgs ad = adam_args(h, a.t);
    HIPCHK(sgns::post(a, nsp == 1 ? h->GO : h->GOp, nsp, ad, h->mI, h->vI, h->mO, h->vO, s));
    ++h->t;
  }
  HIPCHK(hipEventRecord(h->ev1, s));
  double loss = 0.0;
  HIPCHK(hipMemcpyAsync(&loss, h->loss, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (st) {
    st->examples = n;
    st->steps = nsteps;
    st->loss = loss;
    st->seconds = ms * 1e-3;
  }
  return 0;
}

int sgns_negatives(sgns_handle* h, int32_t B, int32_t* out) {
  if (!h || B < 0 || (B > 0 && !out)) return fail(BPRMF_E_INVALID, "bad arguments");
  const int64_t n = (int64_t)B * h->cfg.context * h->cfg.n_negs;
  if (!n) return 0;
  if (int r = sset_dev(h)) return r;
  int32_t* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, 4 * (size_t)n));
  hipError_t e = sgns::negatives(args_of(h, B), d, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(BPRMF_E_HIP, "sgns_negatives: %s", hipGetErrorString(e));
  return 0;
}

int sgns_lookup(sgns_handle* h, int32_t which, const int32_t* idx, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!idx || !out)) || (which != 0 && which != 1))
    return fail(BPRMF_E_INVALID, "bad arguments");
  if (!n) return 0;
  if (int r = sset_dev(h)) return r;
  if (int r = check_ids(idx, n, h->cfg.vocab_size, "idx")) return r;
  const int E = h->cfg.embedding_size;
  int32_t* d = nullptr;
  float* dout = nullptr;
  HIPCHK(hipMalloc((void**)&d, 4 * (size_t)n));
  if (hipMalloc((void**)&dout, 4 * (size_t)n * E) != hipSuccess) {
    (void)hipFree(d);
    return fail(BPRMF_E_HIP, "hipMalloc failed");
  }
  hipError_t e = hipMemcpyAsync(d, idx, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = sgns::lookup(which ? h->O : h->I, h->ld, E, d, n, dout, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, 4 * n * E, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(BPRMF_E_HIP, "sgns_lookup: %s", hipGetErrorString(e));
  return 0;
}

}  // extern "C"
