// ncf_kernels.h — host-side view of the NCF kernels (ncf.hip).  Internal to libbprmf_amd.so; the
// public ABI is include/ncf.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace bprmf {
namespace ncf {

constexpr int kMaxLayers = 4;
constexpr int kSamples = 16;         // samples per fwd/bwd workgroup (the MFMA M dimension)
constexpr int kLossSlotsNcf = 256;   // per-workgroup loss partial slots (summed on the host)
enum { kNeuMF = 0, kGMF = 1, kMLP = 2 };

struct Dims {
  int d, E, L, model, pred;            // factor_num, tower input width per side, layers, model
  int nin[kMaxLayers], nout[kMaxLayers];
  int64_t U, I;
  // the flat (tower + predict) parameter block, in the reference's state_dict order
  int flat_n, off_W[kMaxLayers], off_b[kMaxLayers], off_wp, off_bp;
};

struct Params {
  float *Pg, *Qg, *Pm, *Qm;            // embed_{user,item}_{GMF,MLP}.weight
  float *W[kMaxLayers], *b[kMaxLayers];  // MLP_layers.{3l+1}.weight [nout x nin] / bias
  float *WT[kMaxLayers];               // W^T copies [nin x nout] for the backward
  float *wp, *bp;                      // predict_layer.weight [pred] / bias [1]
};

struct Grads {  // dense gradient rows of the embedding tables (zeroed again by the row Adam)
  float *Pg, *Qg, *Pm, *Qm;
  int32_t *touch_u, *touch_i;  // the last step that gathered each row (-1: none)
};

// The embedding rows of one side (users or items): its GMF and MLP tables (cols 0 for a table the
// model does not use) and the step through which each row's p, m, v are current (cur, -1: never
// touched, m = v = 0).
struct RowSide {
  float *W[2], *M[2], *V[2], *G[2];
  int cols[2];
  int32_t* cur;
  const int32_t* touch;
  int64_t rows;
};
struct RowSides {
  RowSide side[2];           // users, items
  const int32_t* ids[2];     // the batch's (user, item) samples; nullptr: every row of the side
  int64_t U, I;              // id bounds (a sample with an id out of range has no gradient)
};

constexpr int kCatchTerms = 192;  // terms of a catch-up's sum (k_ncf_catch_up)

struct CatchArgs {  // zero-gradient Adam steps up to step `target`
  const float2* step;  // (step_size(s), 1 / bc2_sqrt(s)) for s = 1 .. nstep; beyond, (lr, 1)
  const float2* pw;    // (b1^j, b2^(j/2)) for j = 1 .. kCatchTerms
  int32_t nstep;
  float lr, eps, log2_b1, log2_b2;
  int32_t target;
};

// Per-sample activations and gradients between the step's launches (rows = samples).
struct Acts {
  float* X0;                  // [rows x 2E] tower input [Pm[u], Qm[i]] (training only)
  float* H[kMaxLayers + 1];   // H[l], l = 1 .. L: h_l, layer l-1's output; H[L] is Xp's tower part
  int ldH[kMaxLayers + 1];
  float* Xp;                  // [rows x pred] predict-layer input [Pg[u] * Qg[i], h_L]
  float* dz;                  // [rows] dL/dz
  float* dPre[kMaxLayers];    // [rows x nout[l]] gradient of layer l's pre-activation (training only)
  float* ones;                // [rows] 1.0: bias gradients as contractions (training only)
};

// One wave of k_ncf_back: a [16 x 16] tile of sum_s A[s][m] B[s][k] (weight gradient, then Adam
// on its elements), a vector sum_s A[s][m] B[s] (bias / predict layer, then Adam), or a
// [16 samples x 16 columns] tile of dX_0 = dPre_0 . W_0 (into the MLP embedding gradients).
enum { kJobTile = 0, kJobVec = 1, kJobDx0 = 2 };
struct NcfJob {
  const float* A;
  const float* B;
  int lda, ldb, m0, k0, M, K;
  int flat;   // flat-block index of element (m, k): flat + m K + k (vector: flat + m)
  int kind;
  int layer;  // tiles: the W^T copy refreshed (its offset wt in the W^T block); else -1
  int wt;
};

struct AdamArgs {
  float one_minus_b1, b2, one_minus_b2, eps, step_size, bc2_sqrt;
};

size_t fwdbwd_lds_bytes(const Dims& D);
// k_ncf_front + k_ncf_mid (training: activations and gradients into A, loss, embedding GMF grads)
// next (optional): the next step's samples, caught up to step t beside the middle layers
hipError_t fwdbwd(const Dims& D, const Params& P, const Grads& G, const Acts& A, const int32_t* u,
                  const int32_t* i, const float* y, int n, int32_t t, double* loss, int32_t* err,
                  const RowSides* next, int next_n, const CatchArgs* next_c, hipStream_t s);
hipError_t forward(const Dims& D, const Params& P, const Acts& A, const int32_t* u, const int32_t* i,
                   int n, float* z, int32_t* err, hipStream_t s);
// k_ncf_back: the step's jobs; the tower / predict weights from Fcur (and P) to Fnext / WTnext
hipError_t back(const Dims& D, const Params& P, const Grads& G, const NcfJob* jobs, int njobs,
                const int32_t* u, const int32_t* i, int n, const float* Fcur, float* Fnext,
                float* WTnext, float* M, float* V, const AdamArgs& a, hipStream_t s);
// rows of the samples (or every row when ids are null) brought to c.target; cur = c.target
hipError_t catch_up(const RowSides& R, int64_t n, const CatchArgs& c, hipStream_t s);
// step t of Adam on the rows of the samples (g = the gradient row, then zeroed); cur = t
hipError_t adam_rows(const RowSides& R, int64_t n, int32_t t, const AdamArgs& a, hipStream_t s);
// adam_rows of the previous step (np samples of Rp, step c.target) + catch_up of this step's
// nc samples of Rc to c.target, in one launch (rows touched at c.target are left to the Adam)
hipError_t rows(const RowSides& Rp, int np, const AdamArgs& a, const RowSides& Rc, int nc,
                const CatchArgs& c, hipStream_t s);
hipError_t transpose(const Dims& D, const Params& P, hipStream_t s);
hipError_t sample(const SamplerArgs& a, uint32_t epoch, int64_t first, int64_t count, int32_t* u,
                  int32_t* i, float* y, int32_t* err, hipStream_t s);
hipError_t init(float* W, int64_t n, int kind, float param, uint32_t k0, uint32_t k1, uint32_t tag,
                hipStream_t s);

}  // namespace ncf
}  // namespace bprmf
