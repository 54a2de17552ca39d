// ncf_capi.cpp — C ABI (include/ncf.h) of the NCF training path over the kernels of ncf.hip.
//
// One handle = one GPU.  It owns, in HBM: the four embedding tables and the flat tower+predict
// block (the reference's parameters), their Adam moments m and v, the dense embedding gradient
// rows and per-row current-step stamps, the tower + predict block and its transposed weights
// (double-buffered: a step reads one copy and writes the other), the per-sample activations
// between the step's launches (Acts) and the backward's job list, the training positives and
// their sorted CSR (the sampler's rejection set).
// A step (NCFRecommender.py:278-285): the batch's embedding rows are brought up to step t - 1
// (k_ncf_catch_up: the zero-gradient Adam steps they missed, in closed form), the forward and
// backward (k_ncf_front, k_ncf_mid, then k_ncf_back with the tower + predict layer's Adam), then
// Adam over the batch's embedding rows, which runs with the next step's catch-up in one launch
// (k_ncf_rows; the last step of a call runs it alone, k_ncf_adam_rows).  Every read of the
// tables from outside a step (predict, get / set_param) first brings the rows it reads to the
// current step, so every observable value is torch's dense Adam.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/ncf.h"
#include "handle.h"
#include "ncf_kernels.h"

using namespace bprmf;
using namespace bprmf::ncf;

namespace {
constexpr int kChunk = 1 << 20;  // sampled samples per sampler launch
}

struct ncf_handle {
  ncf_config cfg;
  Dims D{};
  Params P{};
  Grads G{};
  float* emb[4] = {};      // Pg, Qg, Pm, Qm
  float* emb_m[4] = {};
  float* emb_v[4] = {};
  int64_t emb_rows[4] = {}, emb_cols[4] = {};
  float *F = nullptr, *Fm = nullptr, *Fv = nullptr;  // flat tower + predict block (current copy)
  float* WT = nullptr;                                // its transposed tower weights (current copy)
  float *Fo = nullptr, *WTo = nullptr;                // the other copies (the next step's)
  int wt_n = 0;                                       // floats of the W^T block
  int64_t max_blocks = 0;
  Acts A{};                                           // training activations, max_blocks * 16 rows
  float* acts = nullptr;
  NcfJob* d_jobs = nullptr;
  int njobs = 0;
  // training data
  int64_t npos = 0;
  int32_t *d_pos_u = nullptr, *d_pos_i = nullptr, *d_indices = nullptr;
  int64_t* d_indptr = nullptr;
  uint32_t feistel_a = 1, feistel_c = 1;  // permute's domain Z_a x Z_c (feistel_dims)
  uint32_t k0 = 0, k1 = 0;
  // sample chunk
  int32_t *d_u = nullptr, *d_i = nullptr;
  float* d_y = nullptr;
  int64_t chunk_cap = 0;
  double* d_loss = nullptr;
  int32_t* d_err = nullptr;
  int32_t t = 0;  // Adam steps taken
  int32_t *cur_u = nullptr, *cur_i = nullptr;  // step each row's p, m, v are current at (-1: never touched)
  int32_t flushed = 0;                         // every row is current at this step
  struct {                                     // step t's row Adam, run with step t + 1's catch-up
    const int32_t *u = nullptr, *i = nullptr;
    int n = 0;
    AdamArgs a{};
  } pend;
  float2 *d_step = nullptr, *d_pw = nullptr;   // catch-up tables (CatchArgs)
  int32_t nstep = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool prof_on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof[4];
  std::vector<hipEvent_t> pool;
};

static int ncf_dev(ncf_handle* h) {
  HIPCHK(hipSetDevice(h->cfg.device));
  return 0;
}

static hipEvent_t ncf_event(ncf_handle* h) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  h->pool.push_back(e);
  return e;
}

struct NcfProf {  // event pair around a launch while profiling
  ncf_handle* h;
  int kind;
  hipEvent_t a = nullptr;
  NcfProf(ncf_handle* hh, int k) : h(hh), kind(k) {
    if (h->prof_on && (a = ncf_event(h))) (void)hipEventRecord(a, h->stream);
  }
  ~NcfProf() {
    if (!a) return;
    hipEvent_t b = ncf_event(h);
    if (!b) return;
    (void)hipEventRecord(b, h->stream);
    h->prof[kind].push_back({a, b});
  }
};

static bool uses_table(const ncf_handle* h, int tb) {
  return tb < 2 ? h->D.model != kMLP : h->D.model != kGMF;
}

// parameter index -> (device pointer, rows, cols); state_dict order
static bool param_at(ncf_handle* h, int idx, float** p, int64_t* rows, int64_t* cols) {
  const Dims& D = h->D;
  if (idx < 4) {
    *p = h->emb[idx];
    *rows = h->emb_rows[idx];
    *cols = h->emb_cols[idx];
    return true;
  }
  idx -= 4;
  if (idx < 2 * D.L) {
    const int l = idx / 2;
    if (idx % 2 == 0) {
      *p = h->F + D.off_W[l];
      *rows = D.nout[l];
      *cols = D.nin[l];
    } else {
      *p = h->F + D.off_b[l];
      *rows = D.nout[l];
      *cols = 1;
    }
    return true;
  }
  idx -= 2 * D.L;
  if (idx == 0) {
    *p = h->F + D.off_wp;
    *rows = 1;
    *cols = D.pred;
    return true;
  }
  if (idx == 1) {
    *p = h->F + D.off_bp;
    *rows = 1;
    *cols = 1;
    return true;
  }
  return false;
}

// the embedding rows of the used tables, per side; ids: the samples' (user, item) or null (all rows)
static RowSides row_sides(const ncf_handle* h, const int32_t* u, const int32_t* i) {
  RowSides R{};
  for (int side = 0; side < 2; ++side) {
    RowSide& S = R.side[side];
    for (int k = 0; k < 2; ++k) {
      const int tb = 2 * k + side;  // Pg, Qg, Pm, Qm
      if (!uses_table(h, tb)) continue;
      S.W[k] = h->emb[tb];
      S.M[k] = h->emb_m[tb];
      S.V[k] = h->emb_v[tb];
      S.G[k] = tb == 0 ? h->G.Pg : tb == 1 ? h->G.Qg : tb == 2 ? h->G.Pm : h->G.Qm;
      S.cols[k] = (int)h->emb_cols[tb];
    }
    S.cur = side ? h->cur_i : h->cur_u;
    S.touch = side ? h->G.touch_i : h->G.touch_u;
    S.rows = side ? h->D.I : h->D.U;
  }
  R.ids[0] = u;
  R.ids[1] = i;
  R.U = h->D.U;
  R.I = h->D.I;
  return R;
}

static CatchArgs catch_args(const ncf_handle* h, int32_t target) {
  CatchArgs c;
  c.step = h->d_step;
  c.pw = h->d_pw;
  c.nstep = h->nstep;
  c.lr = h->cfg.lr;
  c.eps = h->cfg.eps;
  c.log2_b1 = (float)std::log2((double)h->cfg.beta1);
  c.log2_b2 = (float)std::log2((double)h->cfg.beta2);
  c.target = target;
  return c;
}

// the catch-up's tables, in double as the step's own AdamArgs: torch's step_size(s) and
// 1 / bc2_sqrt(s) for every step whose bias corrections f32 tells from 1 (then lr and 1), and
// b1^j, b2^(j/2) for the terms
static int catch_tables(ncf_handle* h) {
  const double b1 = h->cfg.beta1, b2 = h->cfg.beta2, lr = h->cfg.lr;
  int64_t n = 1;
  while (n < (1 << 22) && (std::pow(b1, (double)n) > 0x1p-26 || std::pow(b2, (double)n) > 0x1p-26)) n *= 2;
  std::vector<float2> st((size_t)n), pw(kCatchTerms);
  for (int64_t s = 1; s <= n; ++s)
    st[s - 1] = make_float2((float)(lr / (1.0 - std::pow(b1, (double)s))),
                            (float)(1.0 / std::sqrt(1.0 - std::pow(b2, (double)s))));
  for (int j = 1; j <= kCatchTerms; ++j)
    pw[j - 1] = make_float2((float)std::pow(b1, (double)j), (float)std::pow(b2, 0.5 * j));
  if (int r = dalloc(&h->d_step, n)) return r;
  if (int r = dalloc(&h->d_pw, kCatchTerms)) return r;
  HIPCHK(hipMemcpy(h->d_step, st.data(), sizeof(float2) * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->d_pw, pw.data(), sizeof(float2) * kCatchTerms, hipMemcpyHostToDevice));
  h->nstep = (int32_t)n;
  return 0;
}

// the last step's row Adam, when it is still pending (before anything reads the rows or the
// sample buffers it points into are refilled)
static int flush_pending(ncf_handle* h) {
  if (!h->pend.n) return 0;
  NcfProf ps(h, 2);
  HIPCHK(adam_rows(row_sides(h, h->pend.u, h->pend.i), h->pend.n, h->t, h->pend.a, h->stream));
  h->pend.n = 0;
  return 0;
}

// every embedding row brought to the current step (before the tables are read or written whole)
static int ncf_flush(ncf_handle* h) {
  if (int r = flush_pending(h)) return r;
  if (h->flushed == h->t) return 0;
  {
    NcfProf ps(h, 3);
    HIPCHK(catch_up(row_sides(h, nullptr, nullptr), 0, catch_args(h, h->t), h->stream));
  }
  h->flushed = h->t;
  return 0;
}

// Params' tower / predict pointers into the current copy of the flat block
static void point_params(ncf_handle* h) {
  const Dims& D = h->D;
  int wo = 0;
  for (int l = 0; l < D.L; ++l) {
    h->P.W[l] = h->F + D.off_W[l];
    h->P.b[l] = h->F + D.off_b[l];
    h->P.WT[l] = h->WT + wo;
    wo += D.nin[l] * D.nout[l];
  }
  h->P.wp = h->F + D.off_wp;
  h->P.bp = h->F + D.off_bp;
}

// W^T from W in the current copy, then the other copy made equal (after init / set_param)
static int sync_copies(ncf_handle* h) {
  HIPCHK(transpose(h->D, h->P, h->stream));
  HIPCHK(hipMemcpyAsync(h->Fo, h->F, 4 * (size_t)h->D.flat_n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->WTo, h->WT, 4 * (size_t)h->wt_n, hipMemcpyDeviceToDevice, h->stream));
  return 0;
}

// Acts carved from one buffer of `rows` sample rows (base null: the floats needed)
static int64_t carve_acts(const Dims& D, int64_t rows, bool train, float* base, Acts* A) {
  int64_t off = 0;
  auto take = [&](int64_t n) {
    float* p = base ? base + off : nullptr;
    off += (n + 15) & ~(int64_t)15;
    return p;
  };
  Acts a{};
  if (train) a.X0 = take(rows * 2 * D.E);
  a.Xp = take(rows * D.pred);
  for (int l = 1; l < D.L; ++l) {
    a.H[l] = take(rows * D.nin[l]);
    a.ldH[l] = D.nin[l];
  }
  a.H[D.L] = a.Xp ? a.Xp + (D.model == kNeuMF ? D.d : 0) : nullptr;
  a.ldH[D.L] = D.pred;
  a.dz = take(rows);
  if (train) {
    for (int l = 0; l < D.L; ++l) a.dPre[l] = take(rows * D.nout[l]);
    a.ones = take(rows);
  }
  if (A) *A = a;
  return off;
}

// k_ncf_back's jobs: dX_0 tiles (the longest, first), weight-gradient tiles, bias and predict
// vectors; every element of the model's tower + predict block belongs to exactly one job
static std::vector<NcfJob> make_jobs(const ncf_handle* h) {
  const Dims& D = h->D;
  const Acts& A = h->A;
  std::vector<NcfJob> v;
  auto job = [&](int kind, const float* a, int lda, const float* b, int ldb, int m0, int k0, int M, int K,
                 int flat, int layer, int wt) {
    NcfJob j;
    j.A = a;
    j.B = b;
    j.lda = lda;
    j.ldb = ldb;
    j.m0 = m0;
    j.k0 = k0;
    j.M = M;
    j.K = K;
    j.flat = flat;
    j.kind = kind;
    j.layer = layer;
    j.wt = wt;
    v.push_back(j);
  };
  if (D.model != kGMF) {
    for (int64_t s0 = 0; s0 < h->max_blocks * kSamples; s0 += kSamples)
      for (int k0 = 0; k0 < 2 * D.E; k0 += 16)
        job(kJobDx0, A.dPre[0], D.nout[0], nullptr, 0, (int)s0, k0, kSamples, 2 * D.E, 0, -1, 0);
    int wo = 0;
    for (int l = 0; l < D.L; ++l) {
      const int M = D.nout[l], K = D.nin[l];
      const float* H = l == 0 ? A.X0 : A.H[l];
      for (int m0 = 0; m0 < M; m0 += 16)
        for (int k0 = 0; k0 < K; k0 += 16) job(kJobTile, A.dPre[l], M, H, K, m0, k0, M, K, D.off_W[l], l, wo);
      for (int m0 = 0; m0 < M; m0 += 16) job(kJobVec, A.dPre[l], M, A.ones, 1, m0, 0, M, 1, D.off_b[l], -1, 0);
      wo += M * K;
    }
  }
  for (int m0 = 0; m0 < D.pred; m0 += 16) job(kJobVec, A.Xp, D.pred, A.dz, 1, m0, 0, D.pred, 1, D.off_wp, -1, 0);
  job(kJobVec, A.ones, 1, A.dz, 1, 0, 0, 1, 1, D.off_bp, -1, 0);
  return v;
}

static SamplerArgs ncf_sampler(ncf_handle* h) {
  SamplerArgs a{};
  a.pos_u = h->d_pos_u;
  a.pos_i = h->d_pos_i;
  a.indptr = h->d_indptr;
  a.indices = h->d_indices;
  a.npos = h->npos;
  a.item_num = h->cfg.item_num;
  a.num_ng = h->cfg.num_ng;
  a.world = 1;
  a.feistel_a = h->feistel_a;
  a.feistel_c = h->feistel_c;
  a.k0 = h->k0;
  a.k1 = h->k1;
  return a;
}

static int ncf_check_err(ncf_handle* h) {
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d_err, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (e) {
    HIPCHK(hipMemsetAsync(h->d_err, 0, 4, h->stream));
    if (e & 2) return fail(BPRMF_E_NO_NEGATIVE, "a user has every item as a positive: no negative to sample");
    return fail(BPRMF_E_RANGE, "user/item id out of range (device check)");
  }
  return 0;
}

// one Adam step over device samples u/i/y[0..n); nu/ni[0..nn): the next step's samples when they
// are already in device memory (their rows are then caught up beside this step's middle layers)
static int ncf_step(ncf_handle* h, const int32_t* u, const int32_t* i, const float* y, int n,
                    const int32_t* nu = nullptr, const int32_t* ni = nullptr, int nn = 0) {
  if (h->t == INT32_MAX) return fail(BPRMF_E_STATE, "step counter overflow");
  const int32_t t = ++h->t;
  const RowSides R = row_sides(h, u, i);
  {  // step t - 1's row Adam (pending) and this step's catch-up to t - 1
    NcfProf ps(h, 3);
    HIPCHK(rows(row_sides(h, h->pend.u, h->pend.i), h->pend.n, h->pend.a, R, n, catch_args(h, t - 1),
                h->stream));
    h->pend.n = 0;
  }
  const double b1 = h->cfg.beta1, b2 = h->cfg.beta2;
  AdamArgs a;
  a.one_minus_b1 = (float)(1.0 - b1);
  a.b2 = (float)b2;
  a.one_minus_b2 = (float)(1.0 - b2);
  a.eps = h->cfg.eps;
  a.step_size = (float)((double)h->cfg.lr / (1.0 - std::pow(b1, (double)t)));
  a.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(b2, (double)t));
  {
    NcfProf ps(h, 1);
    const RowSides Rn = row_sides(h, nu, ni);
    const CatchArgs cn = catch_args(h, t);
    HIPCHK(fwdbwd(h->D, h->P, h->G, h->A, u, i, y, n, t, h->d_loss, h->d_err, nu ? &Rn : nullptr, nu ? nn : 0,
                  &cn, h->stream));
    HIPCHK(back(h->D, h->P, h->G, h->d_jobs, h->njobs, u, i, n, h->F, h->Fo, h->WTo, h->Fm, h->Fv, a,
                h->stream));
  }
  std::swap(h->F, h->Fo);  // the updated tower / predict weights are the current copy
  std::swap(h->WT, h->WTo);
  point_params(h);
  h->pend.u = u;
  h->pend.i = i;
  h->pend.n = n;
  h->pend.a = a;
  return 0;
}

static int ncf_begin(ncf_handle* h) {
  if (int r = ncf_dev(h)) return r;
  if (int r = flush_pending(h)) return r;
  HIPCHK(hipMemsetAsync(h->d_loss, 0, sizeof(double) * kLossSlotsNcf, h->stream));
  HIPCHK(hipEventRecord(h->ev0, h->stream));
  return 0;
}

static int ncf_end(ncf_handle* h, bprmf_stats* st, int64_t samples, int64_t steps) {
  if (int r = flush_pending(h)) return r;
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  std::vector<double> slots(kLossSlotsNcf);
  HIPCHK(hipMemcpyAsync(slots.data(), h->d_loss, sizeof(double) * kLossSlotsNcf, hipMemcpyDeviceToHost,
                        h->stream));
  HIPCHK(hipEventSynchronize(h->ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (int r = ncf_check_err(h)) return r;
  if (st) {
    double l = 0;
    for (double v : slots) l += v;
    st->triplets = samples;
    st->steps = steps;
    st->loss = l;  // sum over the call's steps of each step's mean loss
    st->seconds = ms * 1e-3;
  }
  return 0;
}

static int ensure_chunk(ncf_handle* h, int64_t n) {
  if (n <= h->chunk_cap) return 0;
  void* ptrs[] = {h->d_u, h->d_i, h->d_y};
  for (void* p : ptrs)
    if (p) HIPCHK(hipFree(p));
  h->d_u = h->d_i = nullptr;
  h->d_y = nullptr;
  h->chunk_cap = 0;
  if (int r = dalloc(&h->d_u, n)) return r;
  if (int r = dalloc(&h->d_i, n)) return r;
  if (int r = dalloc(&h->d_y, n)) return r;
  h->chunk_cap = n;
  return 0;
}

extern "C" {

int ncf_create(const ncf_config* cfg, ncf_handle** out) {
  if (!cfg || !out) return fail(BPRMF_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->user_num <= 0 || cfg->item_num <= 0 || cfg->user_num > INT32_MAX || cfg->item_num > INT32_MAX)
    return fail(BPRMF_E_INVALID, "user_num and item_num must be in [1, 2^31)");
  if (cfg->factor_num <= 0 || cfg->factor_num % 4 || cfg->factor_num > 1024)
    return fail(BPRMF_E_UNSUPPORTED, "factor_num must be a positive multiple of 4 (<= 1024)");
  if (cfg->num_layers < 1 || cfg->num_layers > kMaxLayers)
    return fail(BPRMF_E_UNSUPPORTED, "num_layers must be in [1, %d]", kMaxLayers);
  if (cfg->model < 0 || cfg->model > 2) return fail(BPRMF_E_INVALID, "model must be NeuMF-end, GMF or MLP");
  if (cfg->batch_size <= 0 || cfg->batch_size > 8192) return fail(BPRMF_E_INVALID, "batch_size must be in [1, 8192]");
  if (cfg->num_ng < 0) return fail(BPRMF_E_INVALID, "num_ng must be >= 0");
  if (!(cfg->lr >= 0.f) || !(cfg->eps > 0.f) || !(cfg->beta1 >= 0.f && cfg->beta1 < 1.f) ||
      !(cfg->beta2 >= 0.f && cfg->beta2 < 1.f))
    return fail(BPRMF_E_INVALID, "bad Adam hyper-parameters");
  auto* h = new ncf_handle();
  h->cfg = *cfg;
  Dims& D = h->D;
  D.d = cfg->factor_num;
  D.L = cfg->num_layers;
  D.E = D.d << (D.L - 1);
  D.model = cfg->model;
  D.pred = D.model == kNeuMF ? 2 * D.d : D.d;
  D.U = cfg->user_num;
  D.I = cfg->item_num;
  int off = 0;
  for (int l = 0; l < D.L; ++l) {
    D.nin[l] = D.d << (D.L - l);
    D.nout[l] = D.nin[l] / 2;
    D.off_W[l] = off;
    off += D.nin[l] * D.nout[l];
    D.off_b[l] = off;
    off += D.nout[l];
  }
  D.off_wp = off;
  off += D.pred;
  D.off_bp = off;
  off += 1;
  D.flat_n = (off + 3) & ~3;
  h->emb_rows[0] = h->emb_rows[2] = D.U;
  h->emb_rows[1] = h->emb_rows[3] = D.I;
  h->emb_cols[0] = h->emb_cols[1] = D.d;
  h->emb_cols[2] = h->emb_cols[3] = D.E;
  h->max_blocks = (cfg->batch_size + kSamples - 1) / kSamples;
  const uint64_t seed = cfg->seed;
  h->k0 = (uint32_t)seed;
  h->k1 = (uint32_t)(seed >> 32);
  int rc = 0;
#define TRY(x)          \
  do {                  \
    if ((rc = (x))) {   \
      ncf_destroy(h);   \
      return rc;        \
    }                   \
  } while (0)
  TRY(ncf_dev(h));
  if (fwdbwd_lds_bytes(D) > 160 * 1024) {
    ncf_destroy(h);
    return fail(BPRMF_E_UNSUPPORTED, "the tower of factor_num %d x %d layers needs %zu B of LDS (> 160 KB)",
                D.d, D.L, fwdbwd_lds_bytes(D));
  }
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
    ncf_destroy(h);
    return fail(BPRMF_E_HIP, "stream/event creation failed");
  }
  auto memz = [&](void* p, size_t bytes) -> int {
    if (p && bytes) HIPCHK(hipMemsetAsync(p, 0, bytes, h->stream));
    return 0;
  };
  for (int tb = 0; tb < 4; ++tb) {
    const int64_t n = h->emb_rows[tb] * h->emb_cols[tb];
    TRY(dalloc(&h->emb[tb], n));
    TRY(dalloc(&h->emb_m[tb], n));
    TRY(dalloc(&h->emb_v[tb], n));
    TRY(memz(h->emb_m[tb], 4 * n));
    TRY(memz(h->emb_v[tb], 4 * n));
  }
  TRY(dalloc(&h->G.Pg, D.U * D.d));
  TRY(dalloc(&h->G.Qg, D.I * D.d));
  TRY(dalloc(&h->G.Pm, D.U * D.E));
  TRY(dalloc(&h->G.Qm, D.I * D.E));
  TRY(memz(h->G.Pg, 4 * D.U * D.d));
  TRY(memz(h->G.Qg, 4 * D.I * D.d));
  TRY(memz(h->G.Pm, 4 * D.U * D.E));
  TRY(memz(h->G.Qm, 4 * D.I * D.E));
  TRY(catch_tables(h));
  TRY(dalloc(&h->cur_u, D.U));
  TRY(dalloc(&h->cur_i, D.I));
  HIPCHK(hipMemsetAsync(h->cur_u, 0xFF, 4 * D.U, h->stream));  // -1: never touched
  HIPCHK(hipMemsetAsync(h->cur_i, 0xFF, 4 * D.I, h->stream));
  TRY(dalloc(&h->G.touch_u, D.U));
  TRY(dalloc(&h->G.touch_i, D.I));
  HIPCHK(hipMemsetAsync(h->G.touch_u, 0xFF, 4 * D.U, h->stream));
  HIPCHK(hipMemsetAsync(h->G.touch_i, 0xFF, 4 * D.I, h->stream));
  TRY(dalloc(&h->F, D.flat_n));
  TRY(dalloc(&h->Fo, D.flat_n));
  TRY(dalloc(&h->Fm, D.flat_n));
  TRY(dalloc(&h->Fv, D.flat_n));
  TRY(memz(h->Fm, 4 * D.flat_n));
  TRY(memz(h->Fv, 4 * D.flat_n));
  int wt = 0;
  for (int l = 0; l < D.L; ++l) wt += D.nin[l] * D.nout[l];
  h->wt_n = std::max(wt, 1);
  TRY(dalloc(&h->WT, h->wt_n));
  TRY(dalloc(&h->WTo, h->wt_n));
  {
    const int64_t rows = h->max_blocks * kSamples;
    TRY(dalloc(&h->acts, carve_acts(D, rows, true, nullptr, nullptr)));
    carve_acts(D, rows, true, h->acts, &h->A);
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h->A.ones), 0x3F800000, rows, h->stream));
    const std::vector<NcfJob> jobs = make_jobs(h);
    h->njobs = (int)jobs.size();
    TRY(dalloc(&h->d_jobs, h->njobs));
    HIPCHK(hipMemcpy(h->d_jobs, jobs.data(), sizeof(NcfJob) * jobs.size(), hipMemcpyHostToDevice));
  }
  TRY(dalloc(&h->d_loss, kLossSlotsNcf));
  TRY(dalloc(&h->d_err, 1));
  TRY(memz(h->d_err, 4));
  h->P.Pg = h->emb[0];
  h->P.Qg = h->emb[1];
  h->P.Pm = h->emb[2];
  h->P.Qm = h->emb[3];
  point_params(h);
  // NCF._init_weight_ (NCFRecommender.py:65-82): normal(0.01) embeddings, xavier_uniform tower,
  // kaiming_uniform(a=1, 'sigmoid') predictor, zero biases
  hipError_t e = hipSuccess;
  for (int tb = 0; tb < 4 && e == hipSuccess; ++tb)
    e = init(h->emb[tb], h->emb_rows[tb] * h->emb_cols[tb], 0, cfg->init_std, h->k0, h->k1, 1u + tb, h->stream);
  if (e == hipSuccess) e = hipMemsetAsync(h->F, 0, 4 * D.flat_n, h->stream);
  for (int l = 0; l < D.L && e == hipSuccess; ++l)
    e = init(h->P.W[l], (int64_t)D.nin[l] * D.nout[l], 1,
             (float)std::sqrt(6.0 / (D.nin[l] + D.nout[l])), h->k0, h->k1, 16u + l, h->stream);
  if (e == hipSuccess) e = init(h->P.wp, D.pred, 1, (float)std::sqrt(3.0 / D.pred), h->k0, h->k1, 32u, h->stream);
  if (e == hipSuccess && sync_copies(h)) e = hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    ncf_destroy(h);
    return fail(BPRMF_E_HIP, "ncf init: %s", hipGetErrorString(e));
  }
#undef TRY
  *out = h;
  return 0;
}

int ncf_destroy(ncf_handle* h) {
  if (!h) return 0;
  (void)!hipSetDevice(h->cfg.device);
  if (h->stream) (void)!hipStreamSynchronize(h->stream);
  for (int tb = 0; tb < 4; ++tb) {
    void* p[] = {h->emb[tb], h->emb_m[tb], h->emb_v[tb]};
    for (void* x : p)
      if (x) (void)!hipFree(x);
  }
  void* ptrs[] = {h->G.Pg, h->G.Qg, h->G.Pm, h->G.Qm, h->cur_u, h->cur_i, h->G.touch_u, h->G.touch_i, h->d_step, h->d_pw, h->F, h->Fm,
                  h->Fv, h->WT, h->Fo, h->WTo, h->acts, h->d_jobs, h->d_pos_u, h->d_pos_i, h->d_indices, h->d_indptr,
                  h->d_u, h->d_i, h->d_y, h->d_loss, h->d_err};
  for (void* x : ptrs)
    if (x) (void)!hipFree(x);
  for (hipEvent_t e : h->pool) (void)!hipEventDestroy(e);
  if (h->ev0) (void)!hipEventDestroy(h->ev0);
  if (h->ev1) (void)!hipEventDestroy(h->ev1);
  if (h->stream) (void)!hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int ncf_param_count(ncf_handle* h, int32_t* n) {
  if (!h || !n) return fail(BPRMF_E_INVALID, "null argument");
  *n = 4 + 2 * h->D.L + 2;
  return 0;
}

int ncf_param_shape(ncf_handle* h, int32_t index, int64_t* rows, int64_t* cols) {
  if (!h || !rows || !cols) return fail(BPRMF_E_INVALID, "null argument");
  float* p;
  if (!param_at(h, index, &p, rows, cols)) return fail(BPRMF_E_RANGE, "no parameter %d", index);
  return 0;
}

int ncf_set_param(ncf_handle* h, int32_t index, const float* data) {
  if (!h || !data) return fail(BPRMF_E_INVALID, "null argument");
  float* p;
  int64_t r, c;
  if (!param_at(h, index, &p, &r, &c)) return fail(BPRMF_E_RANGE, "no parameter %d", index);
  if (int rc = ncf_dev(h)) return rc;
  if (index < 4)  // the moments of the rows keep counting from the current step
    if (int rc = ncf_flush(h)) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(p, data, 4 * r * c, hipMemcpyHostToDevice));
  if (int rc = sync_copies(h)) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int ncf_get_param(ncf_handle* h, int32_t index, float* data) {
  if (!h || !data) return fail(BPRMF_E_INVALID, "null argument");
  float* p;
  int64_t r, c;
  if (!param_at(h, index, &p, &r, &c)) return fail(BPRMF_E_RANGE, "no parameter %d", index);
  if (int rc = ncf_dev(h)) return rc;
  if (index < 4)
    if (int rc = ncf_flush(h)) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(data, p, 4 * r * c, hipMemcpyDeviceToHost));
  return 0;
}

int ncf_set_train(ncf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz) {
  if (!h || nnz < 0 || (nnz > 0 && (!users || !items))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (int r = ncf_dev(h)) return r;
  std::vector<uint64_t> keys((size_t)nnz);
  for (int64_t k = 0; k < nnz; ++k) {
    if (users[k] < 0 || users[k] >= h->cfg.user_num || items[k] < 0 || items[k] >= h->cfg.item_num)
      return fail(BPRMF_E_RANGE, "positive %lld = (%d, %d) out of range", (long long)k, users[k], items[k]);
    keys[k] = ((uint64_t)users[k] << 32) | (uint32_t)items[k];
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  std::vector<int64_t> indptr(h->cfg.user_num + 1, 0);
  std::vector<int32_t> indices(keys.size());
  for (size_t k = 0; k < keys.size(); ++k) {
    indptr[(keys[k] >> 32) + 1]++;
    indices[k] = (int32_t)(keys[k] & 0xFFFFFFFFu);
  }
  for (int64_t u = 0; u < h->cfg.user_num; ++u) indptr[u + 1] += indptr[u];
  void* olds[] = {h->d_pos_u, h->d_pos_i, h->d_indptr, h->d_indices};
  for (void* p : olds)
    if (p) HIPCHK(hipFree(p));
  h->d_pos_u = h->d_pos_i = h->d_indices = nullptr;
  h->d_indptr = nullptr;
  if (int r = dalloc(&h->d_pos_u, nnz)) return r;
  if (int r = dalloc(&h->d_pos_i, nnz)) return r;
  if (int r = dalloc(&h->d_indptr, h->cfg.user_num + 1)) return r;
  if (int r = dalloc(&h->d_indices, (int64_t)indices.size())) return r;
  if (nnz) {
    HIPCHK(hipMemcpy(h->d_pos_u, users, 4 * nnz, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_pos_i, items, 4 * nnz, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(h->d_indptr, indptr.data(), 8 * indptr.size(), hipMemcpyHostToDevice));
  if (!indices.empty())
    HIPCHK(hipMemcpy(h->d_indices, indices.data(), 4 * indices.size(), hipMemcpyHostToDevice));
  h->npos = nnz;
  const uint64_t N = (uint64_t)nnz * (uint64_t)(1 + h->cfg.num_ng);
  feistel_dims(N, &h->feistel_a, &h->feistel_c);
  return 0;
}

int ncf_epoch_size(ncf_handle* h, int64_t* samples, int64_t* steps) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  const int64_t N = h->npos * (1 + h->cfg.num_ng);
  if (samples) *samples = N;
  if (steps) *steps = (N + h->cfg.batch_size - 1) / h->cfg.batch_size;
  return 0;
}

int ncf_train_samples(ncf_handle* h, const int32_t* u, const int32_t* i, const float* y, int64_t n,
                      bprmf_stats* st) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !y))) return fail(BPRMF_E_INVALID, "bad arguments");
  for (int64_t k = 0; k < n; ++k)
    if (u[k] < 0 || u[k] >= h->cfg.user_num || i[k] < 0 || i[k] >= h->cfg.item_num)
      return fail(BPRMF_E_RANGE, "sample %lld = (%d, %d) out of range", (long long)k, u[k], i[k]);
  if (int r = ncf_begin(h)) return r;
  const int64_t B = h->cfg.batch_size;
  const int64_t chunk = std::max<int64_t>(B, (kChunk / B) * B);
  if (int r = ensure_chunk(h, std::min(chunk, std::max<int64_t>(n, 1)))) return r;
  int64_t steps = 0;
  for (int64_t off = 0; off < n; off += chunk) {
    const int64_t m = std::min(chunk, n - off);
    if (int r = flush_pending(h)) return r;  // it points into the buffers refilled here
    HIPCHK(hipMemcpyAsync(h->d_u, u + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_i, i + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_y, y + off, 4 * m, hipMemcpyHostToDevice, h->stream));
    for (int64_t s = 0; s < m; s += B, ++steps) {
      const int64_t s2 = s + B;  // the next step's samples, when they are in this chunk
      if (int r = ncf_step(h, h->d_u + s, h->d_i + s, h->d_y + s, (int)std::min(B, m - s),
                           s2 < m ? h->d_u + s2 : nullptr, s2 < m ? h->d_i + s2 : nullptr,
                           (int)std::min(B, std::max<int64_t>(0, m - s2))))
        return r;
    }
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return ncf_end(h, st, n, steps);
}

int ncf_train_steps(ncf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps, bprmf_stats* st) {
  if (!h || first_step < 0 || n_steps < 0) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->d_pos_u || h->npos == 0) return fail(BPRMF_E_STATE, "call ncf_set_train first");
  int64_t N, S;
  ncf_epoch_size(h, &N, &S);
  if (first_step + n_steps > S) return fail(BPRMF_E_INVALID, "steps beyond the epoch's %lld", (long long)S);
  if (int r = ncf_begin(h)) return r;
  const int64_t B = h->cfg.batch_size;
  const int64_t chunk = std::max<int64_t>(B, (kChunk / B) * B);
  if (int r = ensure_chunk(h, chunk)) return r;
  const int64_t beg = first_step * B, end = std::min(N, (first_step + n_steps) * B);
  int64_t steps = 0;
  for (int64_t off = beg; off < end; off += chunk) {
    const int64_t m = std::min(chunk, end - off);
    if (int r = flush_pending(h)) return r;  // it points into the buffers refilled here
    {
      NcfProf ps(h, 0);
      HIPCHK(ncf::sample(ncf_sampler(h), epoch, off, m, h->d_u, h->d_i, h->d_y, h->d_err, h->stream));
    }
    for (int64_t s = 0; s < m; s += B, ++steps) {
      const int64_t s2 = s + B;  // the next step's samples, when they are in this chunk
      if (int r = ncf_step(h, h->d_u + s, h->d_i + s, h->d_y + s, (int)std::min(B, m - s),
                           s2 < m ? h->d_u + s2 : nullptr, s2 < m ? h->d_i + s2 : nullptr,
                           (int)std::min(B, std::max<int64_t>(0, m - s2))))
        return r;
    }
  }
  return ncf_end(h, st, end - beg, steps);
}

int ncf_train_epoch(ncf_handle* h, uint32_t epoch, bprmf_stats* st) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  int64_t N, S;
  ncf_epoch_size(h, &N, &S);
  return ncf_train_steps(h, epoch, 0, S, st);
}

int ncf_sample(ncf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u, int32_t* i, float* y) {
  if (!h || n < 0 || first < 0 || (n > 0 && (!u || !i || !y))) return fail(BPRMF_E_INVALID, "bad arguments");
  if (!h->d_pos_u || h->npos == 0) return fail(BPRMF_E_STATE, "call ncf_set_train first");
  int64_t N;
  ncf_epoch_size(h, &N, nullptr);
  if (first + n > N) return fail(BPRMF_E_INVALID, "samples outside the epoch");
  if (int r = ncf_dev(h)) return r;
  if (n == 0) return 0;
  if (int r = ensure_chunk(h, n)) return r;
  HIPCHK(ncf::sample(ncf_sampler(h), epoch, first, n, h->d_u, h->d_i, h->d_y, h->d_err, h->stream));
  HIPCHK(hipMemcpyAsync(u, h->d_u, 4 * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(i, h->d_i, 4 * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(y, h->d_y, 4 * n, hipMemcpyDeviceToHost, h->stream));
  return ncf_check_err(h);
}

int ncf_predict(ncf_handle* h, const int32_t* u, const int32_t* i, int64_t n, float* out) {
  if (!h || n < 0 || (n > 0 && (!u || !i || !out))) return fail(BPRMF_E_INVALID, "bad arguments");
  for (int64_t k = 0; k < n; ++k) {
    if (u[k] < 0 || u[k] >= h->cfg.user_num) return fail(BPRMF_E_RANGE, "Invalid user code");
    if (i[k] < 0 || i[k] >= h->cfg.item_num) return fail(BPRMF_E_RANGE, "Invalid item code");
  }
  if (n == 0) return 0;
  if (int r = ncf_dev(h)) return r;
  if (int r = flush_pending(h)) return r;
  // the rows read are brought to the current step: the requested ones, or every row for a long request
  const bool whole = 2 * n >= h->D.U + h->D.I;
  if (whole)
    if (int r = ncf_flush(h)) return r;
  // ids, logits and the forward's activations for chunks of up to 64k samples
  const int64_t chunk = std::min<int64_t>((n + kSamples - 1) / kSamples * kSamples, 1 << 16);
  const int64_t act_n = carve_acts(h->D, chunk, false, nullptr, nullptr);
  int32_t* buf = nullptr;
  const int64_t act_off = (3 * n + 15) & ~(int64_t)15;  // float4-aligned activations
  if (int r = dalloc(&buf, act_off + act_n)) return r;
  float* z = reinterpret_cast<float*>(buf + 2 * n);
  Acts A;
  carve_acts(h->D, chunk, false, reinterpret_cast<float*>(buf + act_off), &A);
  int rc = 0;
  hipError_t e = hipMemcpyAsync(buf, u, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(buf + n, i, 4 * n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && !whole && h->flushed != h->t)
    e = catch_up(row_sides(h, buf, buf + n), n, catch_args(h, h->t), h->stream);
  for (int64_t off = 0; off < n && e == hipSuccess; off += chunk)
    e = forward(h->D, h->P, A, buf + off, buf + n + off, (int)std::min(n - off, chunk), z + off, h->d_err,
                h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, z, 4 * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) rc = fail(BPRMF_E_HIP, "ncf_predict: %s", hipGetErrorString(e));
  (void)!hipFree(buf);
  if (rc) return rc;
  return ncf_check_err(h);
}

int ncf_active_rows(ncf_handle* h, int64_t* users, int64_t* items) {
  if (!h || !users || !items) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = ncf_dev(h)) return r;
  if (int r = flush_pending(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  std::vector<int32_t> tu(h->D.U), ti(h->D.I);
  HIPCHK(hipMemcpy(tu.data(), h->cur_u, 4 * h->D.U, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ti.data(), h->cur_i, 4 * h->D.I, hipMemcpyDeviceToHost));
  *users = std::count_if(tu.begin(), tu.end(), [](int32_t x) { return x >= 0; });
  *items = std::count_if(ti.begin(), ti.end(), [](int32_t x) { return x >= 0; });
  return 0;
}

int ncf_profile(ncf_handle* h, int32_t enable) {
  if (!h) return fail(BPRMF_E_INVALID, "null handle");
  if (int r = ncf_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  h->prof_on = enable != 0;
  for (auto& v : h->prof) v.clear();
  for (hipEvent_t e : h->pool) (void)!hipEventDestroy(e);
  h->pool.clear();
  return 0;
}

int ncf_profile_read(ncf_handle* h, bprmf_kprof* out) {
  if (!h || !out) return fail(BPRMF_E_INVALID, "null argument");
  if (int r = ncf_dev(h)) return r;
  HIPCHK(hipStreamSynchronize(h->stream));
  memset(out, 0, sizeof *out);
  for (int k = 0; k < 4; ++k) {
    double tot = 0;
    for (auto& pr : h->prof[k]) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
      tot += ms;
    }
    out->count[k] = (int64_t)h->prof[k].size();
    out->ms[k] = tot;
  }
  return 0;
}

}  // extern "C"
