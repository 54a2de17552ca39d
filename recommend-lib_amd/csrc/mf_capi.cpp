// mf_capi.cpp — C ABI (include/mf.h) of the rating-SGD path over the kernels of mf.hip.
//
// One handle = one GPU: P, Q (double, row-major) and the two bias vectors in HBM, the train
// samples laid out by dependency level.  mf_set_train computes the levels on the host in one
// pass over the samples in train-set order: level(s) = 1 + max(last level of u, last level of i)
// (0-based below), then a stable counting sort by level, so samples of one level keep their
// train-set order and every sample runs after every earlier sample that shares its user or item.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/mf.h"
#include "handle.h"
#include "mf_kernels.h"

using namespace bprmf;

struct mf_handle {
  mf_config cfg;
  double *P = nullptr, *Q = nullptr, *bu = nullptr, *bi = nullptr;
  double* Y = nullptr;  // SVDpp: yj [I, k]
  int32_t *uoff = nullptr, *uitems = nullptr, *udup = nullptr, *uslot = nullptr;  // SVDpp
  int32_t *su = nullptr, *si = nullptr, *loff = nullptr;
  double* sr = nullptr;
  int64_t n = 0;
  int32_t levels = 0;
  double gm = 0.0;
  int32_t* d_err = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {
int mset_dev(mf_handle* h) {
  HIPCHK(hipSetDevice(h->cfg.device));
  return 0;
}
template <typename T>
int malloc_dev(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return 0;
  HIPCHK(hipMalloc((void**)p, sizeof(T) * (size_t)count));
  return 0;
}
mf::Args args_of(const mf_handle* h) {
  mf::Args a{};
  a.su = h->su;
  a.si = h->si;
  a.sr = h->sr;
  a.loff = h->loff;
  a.levels = h->levels;
  a.k = h->cfg.n_factors;
  a.P = h->P;
  a.Q = h->Q;
  a.bu = h->bu;
  a.bi = h->bi;
  // SVD.fit: global_mean = 0 when not biased (:121-124); RSVD keeps it for the bias decay, and
  // SVDpp always adds it (:199, :246)
  a.gm = (h->cfg.model == MF_SVD && !h->cfg.variant) ? 0.0 : h->gm;
  a.variant = h->cfg.variant;
  for (int x = 0; x < 4; ++x) {
    a.lr[x] = h->cfg.lr[x];
    a.reg[x] = h->cfg.reg[x];
  }
  a.Y = h->Y;
  a.uoff = h->uoff;
  a.uitems = h->uitems;
  a.udup = h->udup;
  a.uslot = h->uslot;
  a.lr_yj = h->cfg.lr_yj;
  a.reg_yj = h->cfg.reg_yj;
  return a;
}

// SVDpp: samples in train order (one level each) and ur[u] (:222-224) as CSR, list order = train
// order; udup[u] = 1 when u's list holds an item twice
int set_train_svdpp(mf_handle* h, const int32_t* users, const int32_t* items, const double* ratings,
                    int64_t n, double global_mean) {
  const int64_t U = h->cfg.user_num, I = h->cfg.item_num;
  std::vector<int32_t> off(U + 1, 0), list(n), dup(U, 0);
  for (int64_t s = 0; s < n; ++s) {
    const int32_t u = users[s], i = items[s];
    if (u < 0 || u >= U || i < 0 || i >= I)
      return fail(BPRMF_E_RANGE, "train row %lld = (%d, %d) out of range", (long long)s, u, i);
    off[u + 1]++;
  }
  for (int64_t u = 0; u < U; ++u) off[u + 1] += off[u];
  std::vector<int32_t> pos(off.begin(), off.end() - 1);
  for (int64_t s = 0; s < n; ++s) list[pos[users[s]]++] = items[s];
  std::vector<int32_t> seen(I, -1), first(I, 0), slot(n);
  for (int64_t u = 0; u < U; ++u)
    for (int32_t q = off[u]; q < off[u + 1]; ++q) {
      const int32_t it = list[q];
      if (seen[it] == (int32_t)u) {
        dup[u] = 1;
      } else {
        seen[it] = (int32_t)u;
        first[it] = q - off[u];
      }
      slot[q] = first[it];
    }
  void* olds[] = {h->su, h->si, h->sr, h->loff, h->uoff, h->uitems, h->udup, h->uslot};
  for (void* p : olds)
    if (p) HIPCHK(hipFree(p));
  h->su = h->si = h->loff = h->uoff = h->uitems = h->udup = h->uslot = nullptr;
  h->sr = nullptr;
  if (int r = malloc_dev(&h->su, n)) return r;
  if (int r = malloc_dev(&h->si, n)) return r;
  if (int r = malloc_dev(&h->sr, n)) return r;
  if (int r = malloc_dev(&h->uoff, U + 1)) return r;
  if (int r = malloc_dev(&h->uitems, n)) return r;
  if (int r = malloc_dev(&h->udup, U)) return r;
  if (int r = malloc_dev(&h->uslot, n)) return r;
  if (n) {
    HIPCHK(hipMemcpy(h->su, users, 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->si, items, 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->sr, ratings, 8 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->uitems, list.data(), 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->uslot, slot.data(), 4 * n, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(h->uoff, off.data(), 4 * (U + 1), hipMemcpyHostToDevice));
  if (U) HIPCHK(hipMemcpy(h->udup, dup.data(), 4 * U, hipMemcpyHostToDevice));
  h->n = n;
  h->levels = (int32_t)n;
  h->gm = global_mean;
  return 0;
}
}  // namespace

extern "C" {

int mf_create(const mf_config* cfg, mf_handle** out) {
  if (!cfg || !out) return fail(BPRMF_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->user_num < 0 || cfg->item_num < 0 || cfg->n_factors <= 0)
    return fail(BPRMF_E_INVALID, "need user_num, item_num >= 0 and n_factors > 0");
  if (cfg->n_factors > 1024) return fail(BPRMF_E_UNSUPPORTED, "n_factors must be <= 1024");
  if (cfg->model != MF_SVD && cfg->model != MF_RSVD && cfg->model != MF_SVDPP)
    return fail(BPRMF_E_INVALID, "unknown model");
  if (cfg->model == MF_RSVD && cfg->variant != 1 && cfg->variant != 2)
    return fail(BPRMF_E_INVALID, "RSVD version must be 1 or 2");
  if (cfg->user_num >= INT32_MAX || cfg->item_num >= INT32_MAX)
    return fail(BPRMF_E_UNSUPPORTED, "row counts must fit int32");
  auto* h = new mf_handle();
  h->cfg = *cfg;
  int rc = 0;
  auto bail = [&](int r) {
    mf_destroy(h);
    return r;
  };
  if ((rc = mset_dev(h))) return bail(rc);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess)
    return bail(fail(BPRMF_E_HIP, "stream/event creation failed"));
  const int64_t k = cfg->n_factors;
  if ((rc = malloc_dev(&h->P, cfg->user_num * k)) || (rc = malloc_dev(&h->Q, cfg->item_num * k)) ||
      (rc = malloc_dev(&h->bu, cfg->user_num)) || (rc = malloc_dev(&h->bi, cfg->item_num)) ||
      (rc = malloc_dev(&h->d_err, 1)) ||
      (cfg->model == MF_SVDPP && (rc = malloc_dev(&h->Y, cfg->item_num * k))))
    return bail(rc);
  auto z = [&](void* p, size_t bytes) { return p && bytes ? hipMemset(p, 0, bytes) : hipSuccess; };
  if (z(h->P, 8 * cfg->user_num * k) || z(h->Q, 8 * cfg->item_num * k) ||
      z(h->bu, 8 * cfg->user_num) || z(h->bi, 8 * cfg->item_num) || z(h->d_err, 4) ||
      z(h->Y, 8 * cfg->item_num * k))
    return bail(fail(BPRMF_E_HIP, "hipMemset failed"));
  *out = h;
  return 0;
}

int mf_destroy(mf_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  void* ptrs[] = {h->P,  h->Q,    h->bu,   h->bi,     h->su,   h->si,  h->sr,
                  h->loff, h->d_err, h->Y, h->uoff, h->uitems, h->udup, h->uslot};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int mf_set_train(mf_handle* h, const int32_t* users, const int32_t* items, const double* ratings,
                 int64_t n, double global_mean) {
  if (!h || n < 0 || (n > 0 && (!users || !items || !ratings))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (n >= INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "at most 2^31 - 1 train rows");
  if (int r = mset_dev(h)) return r;
  const int64_t U = h->cfg.user_num, I = h->cfg.item_num;
  if (h->cfg.model == MF_SVDPP) return set_train_svdpp(h, users, items, ratings, n, global_mean);
  // dependency levels, in train-set order
  std::vector<int32_t> lu(U, -1), li(I, -1), lvl(n);
  int32_t L = 0;
  for (int64_t s = 0; s < n; ++s) {
    const int32_t u = users[s], i = items[s];
    if (u < 0 || u >= U || i < 0 || i >= I)
      return fail(BPRMF_E_RANGE, "train row %lld = (%d, %d) out of range", (long long)s, u, i);
    const int32_t l = std::max(lu[u], li[i]) + 1;
    lvl[s] = lu[u] = li[i] = l;
    L = std::max(L, l + 1);
  }
  // stable counting sort by level
  std::vector<int32_t> off(L + 1, 0);
  for (int64_t s = 0; s < n; ++s) off[lvl[s] + 1]++;
  for (int32_t l = 0; l < L; ++l) off[l + 1] += off[l];
  std::vector<int32_t> pos(off.begin(), off.end() - 1), su(n), si(n);
  std::vector<double> sr(n);
  for (int64_t s = 0; s < n; ++s) {
    const int32_t d = pos[lvl[s]]++;
    su[d] = users[s];
    si[d] = items[s];
    sr[d] = ratings[s];
  }
  void* olds[] = {h->su, h->si, h->sr, h->loff};
  for (void* p : olds)
    if (p) HIPCHK(hipFree(p));
  h->su = h->si = h->loff = nullptr;
  h->sr = nullptr;
  if (int r = malloc_dev(&h->su, n)) return r;
  if (int r = malloc_dev(&h->si, n)) return r;
  if (int r = malloc_dev(&h->sr, n)) return r;
  if (int r = malloc_dev(&h->loff, (int64_t)L + 1)) return r;
  if (n) {
    HIPCHK(hipMemcpy(h->su, su.data(), 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->si, si.data(), 4 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->sr, sr.data(), 8 * n, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(h->loff, off.data(), 4 * ((size_t)L + 1), hipMemcpyHostToDevice));
  h->n = n;
  h->levels = L;
  h->gm = global_mean;
  return 0;
}

int mf_set_weights(mf_handle* h, const double* P, const double* Q, const double* bu, const double* bi) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = mset_dev(h)) return r;
  const int64_t U = h->cfg.user_num, I = h->cfg.item_num, k = h->cfg.n_factors;
  if (P && U) HIPCHK(hipMemcpy(h->P, P, 8 * U * k, hipMemcpyHostToDevice));
  if (Q && I) HIPCHK(hipMemcpy(h->Q, Q, 8 * I * k, hipMemcpyHostToDevice));
  if (U) HIPCHK(bu ? hipMemcpy(h->bu, bu, 8 * U, hipMemcpyHostToDevice) : hipMemset(h->bu, 0, 8 * U));
  if (I) HIPCHK(bi ? hipMemcpy(h->bi, bi, 8 * I, hipMemcpyHostToDevice) : hipMemset(h->bi, 0, 8 * I));
  return 0;
}

int mf_get_weights(mf_handle* h, double* P, double* Q, double* bu, double* bi) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = mset_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  const int64_t U = h->cfg.user_num, I = h->cfg.item_num, k = h->cfg.n_factors;
  if (P && U) HIPCHK(hipMemcpy(P, h->P, 8 * U * k, hipMemcpyDeviceToHost));
  if (Q && I) HIPCHK(hipMemcpy(Q, h->Q, 8 * I * k, hipMemcpyDeviceToHost));
  if (bu && U) HIPCHK(hipMemcpy(bu, h->bu, 8 * U, hipMemcpyDeviceToHost));
  if (bi && I) HIPCHK(hipMemcpy(bi, h->bi, 8 * I, hipMemcpyDeviceToHost));
  return 0;
}

int mf_set_implicit(mf_handle* h, const double* Y) {
  if (!h || !Y) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.model != MF_SVDPP) return fail(BPRMF_E_STATE, "only SVDpp has an implicit table");
  if (int r = mset_dev(h)) return r;
  const int64_t bytes = 8 * h->cfg.item_num * h->cfg.n_factors;
  if (bytes) HIPCHK(hipMemcpy(h->Y, Y, bytes, hipMemcpyHostToDevice));
  return 0;
}

int mf_get_implicit(mf_handle* h, double* Y) {
  if (!h || !Y) return fail(BPRMF_E_INVALID, "bad arguments");
  if (h->cfg.model != MF_SVDPP) return fail(BPRMF_E_STATE, "only SVDpp has an implicit table");
  if (int r = mset_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  const int64_t bytes = 8 * h->cfg.item_num * h->cfg.n_factors;
  if (bytes) HIPCHK(hipMemcpy(Y, h->Y, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int mf_fit(mf_handle* h, int32_t epochs, mf_stats* st) {
  if (!h || epochs < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = mset_dev(h)) return r;
  const mf::Args a = args_of(h);
  HIPCHK(hipEventRecord(h->ev0, h->stream));
  for (int32_t e = 0; e < epochs; ++e) HIPCHK(mf::epoch(a, h->cfg.model, h->stream));
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  HIPCHK(hipEventSynchronize(h->ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (st) {
    st->samples = (int64_t)epochs * h->n;
    st->levels = h->levels;
    st->seconds = ms * 1e-3;
  }
  return 0;
}

int mf_predict(mf_handle* h, const int32_t* users, const int32_t* items, int64_t n, double* out) {
  if (!h || n < 0 || (n > 0 && (!users || !items || !out))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!n) return 0;
  if (int r = mset_dev(h)) return r;
  if (h->cfg.model == MF_SVDPP && !h->uoff) return fail(BPRMF_E_STATE, "SVDpp predict needs the train set");
  int32_t *du = nullptr, *di = nullptr;
  double* dout = nullptr;
  int rc = 0;
  if ((rc = malloc_dev(&du, n)) || (rc = malloc_dev(&di, n)) || (rc = malloc_dev(&dout, n))) {
    (void)hipFree(du);
    (void)hipFree(di);
    return rc;
  }
  hipError_t e = hipMemcpyAsync(du, users, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(di, items, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess)
    e = mf::predict(args_of(h), h->cfg.model, du, di, n, h->cfg.user_num, h->cfg.item_num, dout,
                    h->d_err, h->stream);
  int32_t bad = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, 8 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(&bad, h->d_err, 4, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(du);
  (void)hipFree(di);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(BPRMF_E_HIP, "mf_predict: %s", hipGetErrorString(e));
  if (bad) {
    (void)hipMemset(h->d_err, 0, 4);
    return fail(BPRMF_E_RANGE, "Invalid user or item code");
  }
  return 0;
}

}  // extern "C"
