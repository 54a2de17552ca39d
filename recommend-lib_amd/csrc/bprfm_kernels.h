// bprfm_kernels.h — launchers of the BPR-FM kernels (bprfm.hip), internal to libbprmf_amd.so;
// the public ABI is include/bprfm.h (bprfm_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bprmf {
namespace fm {

struct Args {
  // parameters, Adagrad accumulators and gradients (rows padded to ld floats)
  float *E, *acc_E, *GE;          // [F, ld] embeddings of the F features
  float *b, *acc_b, *Gb;          // [F] feature biases
  int32_t* stamp;                 // [F] step of a row's last update (apply claims a row once)
  int64_t F;                      // feature rows
  int32_t sweep;                  // apply sweeps all F rows (stamped by the backward)
  float *gamma, *beta, *acc_gamma, *acc_beta, *ggamma, *gbeta;  // [ld] BatchNorm1d affine
  float* run;                     // [2, ld] BatchNorm running mean, running variance
  const float* bias_;             // [1] global bias (its gradient is identically zero)
  // the step's batch
  const int32_t *u, *i, *j;       // [B] feature indices: user, positive item, negative item
  int32_t B, k, ld, bn, step;
  float lr, p;                    // Adagrad lr; dropout probability
  uint64_t seed;                  // dropout stream
  // scratch
  float* X;                       // [2, B, ld] fm rows of both sides
  double* part;                   // [blocks, 4, ld] per-workgroup sums
  float* stats;                   // [2 sides, (mean, 1/sqrt(var+eps)), ld]
  float* stats2;                  // [(sum gy_i, sum gy_i xhat_i, sum gy_j, sum gy_j xhat_j), ld]
  float* cbuf;                    // [B] pred_i - pred_j
  double* loss;                   // [1] accumulated loss
  double* lpart;                  // [blocks] per-workgroup loss sums of k_fm_mid
};

int lanes_for(int k);                 // lanes (and row stride) per triplet: next_pow2(k) <= 64
int64_t part_blocks(int k, int B);    // workgroups of the per-triplet kernels
hipError_t step(const Args& a, hipStream_t s);
hipError_t init_normal(float* E, int64_t F, int k, int ld, float std_, uint64_t seed, hipStream_t s);
hipError_t dropout_mask(const Args& a, float* out, hipStream_t s);  // [2, B, k] keep-scales of a.step
hipError_t predict(const Args& a, const int32_t* us, const int32_t* xs, int64_t n, float* out,
                   hipStream_t s);

}  // namespace fm
}  // namespace bprmf
