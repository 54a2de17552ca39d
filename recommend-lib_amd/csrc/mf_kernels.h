// mf_kernels.h — launchers of the rating-SGD kernels (mf.hip), internal to libbprmf_amd.so; the
// public ABI is include/mf.h (mf_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bprmf {
namespace mf {

struct Args {
  const int32_t* su;    // [n] user (RSVD: i) of the samples, level order
  const int32_t* si;    // [n] item (RSVD: j)
  const double* sr;     // [n] rating
  const int32_t* loff;  // [levels + 1] first sample of each level
  int32_t levels;
  int32_t k;
  double* P;            // [U, k]  pu / ui
  double* Q;            // [I, k]  qi / vj
  double* bu;           // [U]     bu / ci
  double* bi;           // [I]     bi / dj
  double gm;            // global mean (SVD: 0 when not biased, as fit() sets it, :121-124)
  int32_t variant;      // SVD: biased; RSVD: version
  double lr[4], reg[4];
  // SVDpp (model 2): samples in train order (levels = n), the implicit table and each user's
  // items in train order (ur of :222-224)
  double* Y;               // [I, k] yj
  const int32_t* uoff;     // [U + 1]
  const int32_t* uitems;   // [n]
  const int32_t* udup;     // [U] 1: the user's list holds an item twice
  const int32_t* uslot;    // [n] list position of the first occurrence of the item (within the user)
  double lr_yj, reg_yj;
};

// one epoch of SVD (model 0) or RSVD (model 1) over the level schedule, or of SVDpp (model 2)
// sample by sample
hipError_t epoch(const Args& a, int model, hipStream_t s);
// predict for n (user, item) pairs; err |= 1 on an id out of range
hipError_t predict(const Args& a, int model, const int32_t* us, const int32_t* is, int64_t n,
                   int64_t U, int64_t I, double* out, int32_t* err, hipStream_t s);

}  // namespace mf
}  // namespace bprmf
