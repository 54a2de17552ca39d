/*
 * ORACLE — plain-C restatement of the reference's Cython rating-SGD loops
 * (util/matrix_factorization.pyx).  TEST INFRASTRUCTURE ONLY: linked by tests/ and timed by
 * tools/bench_mf.py as the CPU baseline, never by the product library.
 *
 * Per-sample SGD in double, samples in train-set order, every operation in the order the
 * Cython source writes it (no fused multiply-add: -ffp-contract=off; the reference module is
 * built with the platform's -O2 and no FMA either), so results are bit-identical to the
 * reference's for the same initial tables (tests/golden/mf_cases.npz).
 *
 * oracle_svd_epochs   SVD.fit epochs (:128-151): dot = sum_f qi[i,f] * pu[u,f];
 *                     err = r - (gm + bu[u] + bi[i] + dot); biased: bu, bi updates; then per f
 *                     pu += lr_pu (err qi - reg_pu pu), qi += lr_qi (err pu - reg_qi qi) with the
 *                     values before the update.
 * oracle_rsvd_epochs  RSVD.fit epochs (:40-61): dot = sum_k ui[i,k] * vj[j,k];
 *                     err = r - (ci[i] + dj[j] + dot); version 2: both biases move by
 *                     lr (err - reg2 (ci + dj - gm)); per k ui, vj as SVD with one lr and reg.
 *                     (The reference trains only when verbose: the caller decides.)
 * oracle_svdpp_epochs SVDpp.fit epochs (:226-262): Iu = the items of u in train-set order
 *                     (uoff/uitems, ur[u] of :222-224); impl[f] = sum_j y[j,f] / sqrt|Iu| in
 *                     that order; dot = sum_f qi[i,f] * (pu[u,f] + impl[f]);
 *                     err = r - (gm + bu[u] + bi[i] + dot); bu, bi; then per f: pu, qi (qi's with
 *                     pu + impl) and, for j in Iu in order, y[j,f] += lr_yj (err qi / sqrt|Iu| -
 *                     reg_yj y[j,f]), all with the values before the update.
 */
#include <math.h>
#include <stdint.h>

void oracle_svd_epochs(int64_t n, const int32_t* us, const int32_t* is, const double* rs, int k,
                       double gm, int biased, const double* lr, const double* reg, double* P,
                       double* Q, double* bu, double* bi, int epochs) {
  const double lr_bu = lr[0], lr_bi = lr[1], lr_pu = lr[2], lr_qi = lr[3];
  const double reg_bu = reg[0], reg_bi = reg[1], reg_pu = reg[2], reg_qi = reg[3];
  for (int e = 0; e < epochs; ++e)
    for (int64_t s = 0; s < n; ++s) {
      const int64_t u = us[s], i = is[s];
      const double r = rs[s];
      double* pu = P + u * k;
      double* qi = Q + i * k;
      double dot = 0;
      for (int f = 0; f < k; ++f) dot += qi[f] * pu[f];
      const double err = r - (gm + bu[u] + bi[i] + dot);
      if (biased) {
        bu[u] += lr_bu * (err - reg_bu * bu[u]);
        bi[i] += lr_bi * (err - reg_bi * bi[i]);
      }
      for (int f = 0; f < k; ++f) {
        const double puf = pu[f], qif = qi[f];
        pu[f] += lr_pu * (err * qif - reg_pu * puf);
        qi[f] += lr_qi * (err * puf - reg_qi * qif);
      }
    }
}

void oracle_rsvd_epochs(int64_t n, const int32_t* is_, const int32_t* js, const double* rs, int k,
                        double gm, int version, double lr, double reg, double reg2, double* U,
                        double* V, double* ci, double* dj, int epochs) {
  for (int e = 0; e < epochs; ++e)
    for (int64_t s = 0; s < n; ++s) {
      const int64_t i = is_[s], j = js[s];
      const double r = rs[s];
      double* ui = U + i * k;
      double* vj = V + j * k;
      double dot = 0;
      for (int f = 0; f < k; ++f) dot += ui[f] * vj[f];
      const double err = r - (ci[i] + dj[j] + dot);
      if (version == 2) {
        const double cii = ci[i], djj = dj[j];
        ci[i] += lr * (err - reg2 * (cii + djj - gm));
        dj[j] += lr * (err - reg2 * (cii + djj - gm));
      }
      for (int f = 0; f < k; ++f) {
        const double uik = ui[f], vjk = vj[f];
        ui[f] += lr * (err * vjk - reg * uik);
        vj[f] += lr * (err * uik - reg * vjk);
      }
    }
}

void oracle_svdpp_epochs(int64_t n, const int32_t* us, const int32_t* is, const double* rs, int k,
                         double gm, const double* lr, const double* reg, double* P, double* Q,
                         double* Y, double* bu, double* bi, const int64_t* uoff,
                         const int32_t* uitems, double* impl, int epochs) {
  const double lr_bu = lr[0], lr_bi = lr[1], lr_pu = lr[2], lr_qi = lr[3], lr_yj = lr[4];
  const double reg_bu = reg[0], reg_bi = reg[1], reg_pu = reg[2], reg_qi = reg[3], reg_yj = reg[4];
  for (int e = 0; e < epochs; ++e)
    for (int64_t s = 0; s < n; ++s) {
      const int64_t u = us[s], i = is[s];
      const double r = rs[s];
      const int64_t beg = uoff[u], end = uoff[u + 1];
      const double sqrt_Iu = sqrt((double)(end - beg));
      for (int f = 0; f < k; ++f) impl[f] = 0.0;
      for (int64_t q = beg; q < end; ++q) {
        const double* yj = Y + (int64_t)uitems[q] * k;
        for (int f = 0; f < k; ++f) impl[f] += yj[f] / sqrt_Iu;
      }
      double* pu = P + u * k;
      double* qi = Q + i * k;
      double dot = 0;
      for (int f = 0; f < k; ++f) dot += qi[f] * (pu[f] + impl[f]);
      const double err = r - (gm + bu[u] + bi[i] + dot);
      bu[u] += lr_bu * (err - reg_bu * bu[u]);
      bi[i] += lr_bi * (err - reg_bi * bi[i]);
      for (int f = 0; f < k; ++f) {
        const double puf = pu[f], qif = qi[f];
        pu[f] += lr_pu * (err * qif - reg_pu * puf);
        qi[f] += lr_qi * (err * (puf + impl[f]) - reg_qi * qif);
        for (int64_t q = beg; q < end; ++q) {
          double* yj = Y + (int64_t)uitems[q] * k;
          yj[f] += lr_yj * (err * qif / sqrt_Iu - reg_yj * yj[f]);
        }
      }
    }
}
