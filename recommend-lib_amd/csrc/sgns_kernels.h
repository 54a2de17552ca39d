// sgns_kernels.h — launchers of the Item2Vec / SGNS kernels (sgns.hip), internal to
// libbprmf_amd.so; the public ABI is include/sgns.h (sgns_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ncf_kernels.h"

namespace bprmf {
namespace sgns {

struct Args {
  float *I, *O;                   // [V, ld] ivectors / ovectors (row 0: padding, stays 0)
  float* GI;                      // [V, ld] ivectors gradient (f32 atomics), zero outside a step
  int32_t *touch_i, *touch_o;     // [V] step of a row's last gradient, -1: never (Adam skips it)
  float* S;                       // [V, B] d loss / d (o . i) per (ovectors row, example)
  float* IB;                      // [B, ld] the examples' centre rows (the O-gradient GEMM's A)
  float* lbuf;                    // [B] per-example loss
  const int32_t *iw, *ow, *nw;    // [B], [B, C], [B, C * n] (nw null: drawn on the device)
  const float* cdf;               // [V] noise CDF of weights^0.75 (null: uniform [0, V - 2])
  int64_t V;
  int32_t E, ld, B, C, n, t;      // t: the Adam step being taken (1-based)
  uint64_t seed;
  double* loss;                   // [1] accumulated loss (sum of the batches' losses)
};

int lanes_elems(int E);  // factors per lane of the one-wave-per-example layout (ceil(E / 64))
hipError_t init_uniform(float* W, int64_t V, int E, int ld, float lim, uint64_t seed, uint32_t tag,
                        hipStream_t s);
hipError_t forward_backward(const Args& a, hipStream_t s);  // K1: dots, coefficients, GI, S, IB
// after the GEMM: Adam on both tables (ovectors' gradient = the nsp partials summed in order),
// S zeroed for the next step, the batch's loss into loss[0]
hipError_t post(const Args& a, const float* parts, int nsp, const ncf::AdamArgs& ad, float* mI,
                float* vI, float* mO, float* vO, hipStream_t s);
hipError_t negatives(const Args& a, int32_t* out, hipStream_t s);  // [B, C * n] draws of step t
hipError_t lookup(const float* W, int ld, int E, const int32_t* idx, int64_t n, float* out,
                  hipStream_t s);

}  // namespace sgns
}  // namespace bprmf
