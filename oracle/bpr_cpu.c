/*
 * ORACLE — plain-C restatement of the reference BPR-MF path.  TEST INFRASTRUCTURE ONLY:
 * linked by tests/ and timed by bench.py's cpu_baseline leg, never by the product library.
 *
 * 1. oracle_step_dense: the reference training step, literally (BPRMFRecommender.py:172-176):
 *    fresh zero dense grads (model.zero_grad / embedding_dense_backward), forward
 *    pred = <P_u,Q_i>, <P_u,Q_j> (:42-50), loss = -sum log sigmoid(pred_i - pred_j) (:174),
 *    duplicates summed, then torch SGD with weight_decay over EVERY row (:154,:176):
 *    d_p = g + wd*p ; p = p - lr*d_p.  OpenMP over rows for the dense sweeps.
 * 2. oracle_sample: the sampler specification of oracle/bpr_oracle.py (Philox4x32-10 keyed by
 *    the seed, Feistel shuffle of the epoch's triplets, negative = k-th non-positive item),
 *    restated independently in C; the HIP sampler must match it bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TAG_NEG 0x4E470000u
#define TAG_PERM 0x50520000u

static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

void oracle_philox(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox(c, k0, k1);
  memcpy(out, c, sizeof c);
}

/* domain Z_a x Z_c: c = ceil(sqrt(n)), a = ceil(n / c) */
void oracle_feistel_dims(uint64_t n, uint32_t* a, uint32_t* c) {
  if (n <= 1) {
    *a = *c = 1;
    return;
  }
  uint64_t r = (uint64_t)sqrtl((long double)n);
  while (r * r > n) --r;
  while ((r + 1) * (r + 1) <= n) ++r;
  const uint64_t cc = r * r == n ? r : r + 1;
  *c = (uint32_t)cc;
  *a = (uint32_t)((n + cc - 1) / cc);
}

/* 6-round alternating Feistel on Z_a x Z_c (x = L*c + R; even rounds L = (L + hi32(F(R)*a)) mod a,
   odd rounds R = (R + hi32(F(L)*c)) mod c), cycle-walking into [0, n) */
uint64_t oracle_permute(uint64_t x, uint64_t n, uint64_t seed, uint32_t epoch) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t fa, fc;
  oracle_feistel_dims(n, &fa, &fc);
  do {
    uint64_t L = x / fc, R = x % fc;
    for (uint32_t r = 0; r < 6; ++r) {
      uint32_t c[4] = {(uint32_t)((r & 1) ? L : R), r, epoch, TAG_PERM | r};
      philox(c, k0, k1);
      if (r & 1)
        R = (R + (((uint64_t)c[0] * fc) >> 32)) % fc;
      else
        L = (L + (((uint64_t)c[0] * fa) >> 32)) % fa;
    }
    x = L * fc + R;
  } while (x >= n);
  return x;
}

static uint32_t bounded(uint64_t q, uint32_t epoch, uint32_t n, uint32_t k0, uint32_t k1) {
  const uint32_t t = (uint32_t)((0x100000000ull - n) % n);
  for (uint32_t a = 0;; ++a) {
    uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), epoch, TAG_NEG | a};
    philox(c, k0, k1);
    uint64_t m = (uint64_t)c[0] * n;
    if ((uint32_t)m >= t) return (uint32_t)(m >> 32);
  }
}

/* positives pos_u/pos_i (features order), CSR over GLOBAL user ids (indptr [user_num+1]).
 * Writes triplet slots [first, first+count).  Returns 0, or -5 if a user has no negative. */
int oracle_sample(const int32_t* pos_u, const int32_t* pos_i, int64_t npos, const int64_t* indptr,
                  const int32_t* indices, int64_t item_num, int32_t num_ng, uint64_t seed,
                  uint32_t epoch, int64_t first, int64_t count, int32_t* ou, int32_t* oi,
                  int32_t* oj) {
  const uint64_t N = (uint64_t)npos * (uint64_t)num_ng;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t s = 0; s < count; ++s) {
    uint64_t q = oracle_permute((uint64_t)(first + s), N, seed, epoch);
    int64_t p = (int64_t)(q / (uint64_t)num_ng);
    int32_t u = pos_u[p];
    int64_t beg = indptr[u], deg = indptr[u + 1] - beg;
    int64_t nfree = item_num - deg;
    int32_t j = -1;
    if (nfree > 0) {
      int64_t k = bounded(q, epoch, (uint32_t)nfree, k0, k1);
      int64_t lo = 0, hi = deg;
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)indices[beg + mid] - mid <= k)
          lo = mid + 1;
        else
          hi = mid;
      }
      j = (int32_t)(k + lo);
    } else {
      bad = 1;
    }
    ou[s] = u;
    oi[s] = pos_i[p];
    oj[s] = j;
  }
  return bad ? -5 : 0;
}

/* One dense reference step.  gP [U,d] / gQ [I,d] are caller scratch (zeroed here, as the dense
 * embedding grads are re-created every step).  Returns the loss (sum of -log sigmoid). */
double oracle_step_dense(float* P, float* Q, int64_t U, int64_t I, int d, const int32_t* u,
                         const int32_t* i, const int32_t* j, int64_t n, float lr, float wd,
                         float* gP, float* gQ) {
  double loss = 0.0;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < U * d; ++r) gP[r] = 0.f;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < I * d; ++r) gQ[r] = 0.f;
  for (int64_t b = 0; b < n; ++b) {
    const float* pu = P + (int64_t)u[b] * d;
    const float* qi = Q + (int64_t)i[b] * d;
    const float* qj = Q + (int64_t)j[b] * d;
    float xi = 0.f, xj = 0.f;
    for (int k = 0; k < d; ++k) {
      xi += pu[k] * qi[k];
      xj += pu[k] * qj[k];
    }
    const float x = xi - xj;
    const float s = 1.0f / (1.0f + expf(-x));
    loss -= log((double)s);
    const float c = 1.0f - s;
    float* gu = gP + (int64_t)u[b] * d;
    float* gi = gQ + (int64_t)i[b] * d;
    float* gj = gQ + (int64_t)j[b] * d;
    for (int k = 0; k < d; ++k) {
      gu[k] += -c * qi[k] + c * qj[k];
      gi[k] += -c * pu[k];
      gj[k] += c * pu[k];
    }
  }
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < U * d; ++r) P[r] -= lr * (gP[r] + wd * P[r]);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < I * d; ++r) Q[r] -= lr * (gQ[r] + wd * Q[r]);
  return loss;
}

int oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
