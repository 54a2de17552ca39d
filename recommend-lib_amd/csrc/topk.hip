// topk.hip — device scoring + per-user top-K over candidate lists.
//
// Replaces the reference's ranking loops: the final KPI (BPRMFRecommender.py:196-207: one scalar
// forward per candidate, then np.argsort(pred)[::-1][:K]) and the validation protocol
// (util/metrics.py:46-66: forward of a [gt, negatives] batch, torch.topk).  One workgroup per
// user: lane groups score the user's candidates into LDS with exactly the arithmetic of k_score
// (so scores equal BPRMF.score/forward bit for bit), then a block radix sort over 64-bit keys
// (~orderable(score) << 32 | ~position) takes the top K: score descending, ties by LATER position
// first, i.e. np.argsort(s)[::-1] on a stable sort.  Lists longer than one pass are handled in
// passes carrying the current top K.
#include <rocprim/block/block_radix_sort.hpp>

#include "device_common.h"

namespace bprmf {

constexpr int kTopkThreads = 256;
constexpr int kTopkIPT = 8;
constexpr int kTopkPass = kTopkThreads * kTopkIPT;  // keys sorted per pass (carried top K included)
constexpr int kTopkMaxK = 256;

static __device__ __forceinline__ uint32_t ord_desc(float x) {  // smaller key = larger score
  uint32_t u = __float_as_uint(x);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // monotone: larger float -> larger u
  return ~u;
}
static __device__ __forceinline__ float from_ord_desc(uint32_t k) {
  const uint32_t u = ~k;
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

template <int G, int EPL>
__global__ __launch_bounds__(kTopkThreads) void k_topk_lists(
    const int32_t* __restrict__ users, const int64_t* __restrict__ offs,
    const int32_t* __restrict__ items, int k, Table P, Table Q, Hyper hp, int ld, int32_t T,
    int32_t* __restrict__ out_pos, float* __restrict__ out_score, int32_t* __restrict__ err) {
  using Sort = rocprim::block_radix_sort<uint64_t, kTopkThreads, kTopkIPT>;
  __shared__ typename Sort::storage_type ssort;
  __shared__ uint64_t s_key[kTopkPass];
  __shared__ uint64_t s_top[kTopkMaxK];
  constexpr int NG = kTopkThreads / G;
  const int sub = threadIdx.x & (G - 1), grp = threadIdx.x / G;
  const int64_t r = blockIdx.x;
  const int64_t beg = offs[r], n = offs[r + 1] - beg;
  const int64_t u = users[r];
  const bool uok = (uint64_t)u < (uint64_t)P.rows;
  if (!uok && threadIdx.x == 0) atomicOr(err, 1);
  float pu[EPL];
  {
    const float fu = uok ? decay_pow(hp.log2a, T - P.stamp[u]) : 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) pu[e] = uok ? P.W[u * ld + sub + G * e] * fu : 0.f;
  }
  int carried = 0;  // valid entries of s_top
  const int fresh = kTopkPass - k;
  for (int64_t c0 = 0; c0 < n || (c0 == 0 && n == 0); c0 += fresh) {
    const int m = (int)min<int64_t>(fresh, n - c0);
    // scores of this pass's candidates (position c0 + x) -> keys in LDS
    for (int x = grp; x < m; x += NG) {
      const int64_t it = items[beg + c0 + x];
      float d = 0.f;
      if ((uint64_t)it < (uint64_t)Q.rows) {
        const float fi = decay_pow(hp.log2a, T - Q.stamp[it]);
        const float* qi = Q.W + it * ld + sub;
#pragma unroll
        for (int e = 0; e < EPL; ++e) d = fmaf(pu[e], qi[G * e] * fi, d);
      } else if (sub == 0) {
        atomicOr(err, 1);
      }
      d = group_sum<G>(d);
      if (sub == 0) {
        const uint32_t pos = (uint32_t)(c0 + x);
        s_key[x] = ((uint64_t)ord_desc(d) << 32) | (uint64_t)(~pos);
      }
    }
    for (int x = m + threadIdx.x; x < kTopkPass; x += kTopkThreads)
      s_key[x] = x - m < carried ? s_top[x - m] : ~0ull;
    __syncthreads();
    uint64_t key[kTopkIPT];
#pragma unroll
    for (int e = 0; e < kTopkIPT; ++e) key[e] = s_key[threadIdx.x * kTopkIPT + e];
    __syncthreads();
    Sort().sort(key, ssort);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kTopkIPT; ++e) {
      const int x = threadIdx.x * kTopkIPT + e;
      if (x < k) s_top[x] = key[e];
    }
    carried = (int)min<int64_t>(k, c0 + m);
    __syncthreads();
    if (n == 0) break;
  }
  for (int x = threadIdx.x; x < k; x += kTopkThreads) {
    const bool ok = x < carried;
    const uint64_t key = ok ? s_top[x] : 0ull;
    out_pos[r * k + x] = ok ? (int32_t)(~(uint32_t)key) : -1;
    out_score[r * k + x] = ok ? from_ord_desc((uint32_t)(key >> 32)) : -INFINITY;
  }
}

hipError_t topk_lists(const Geom& g, const int32_t* users, const int64_t* offs, const int32_t* items,
                      int64_t n_users, int k, Table P, Table Q, const Hyper& hp, int32_t T,
                      int32_t* out_pos, float* out_score, int32_t* err, hipStream_t s) {
  if (n_users <= 0) return hipSuccess;
  if (k <= 0 || k > kTopkMaxK) return hipErrorInvalidValue;
  BPRMF_DISPATCH(g, (k_topk_lists<G_, E_><<<(unsigned)n_users, kTopkThreads, 0, s>>>(
                        users, offs, items, k, P, Q, hp, g.ld, T, out_pos, out_score, err)));
  return hipGetLastError();
}

}  // namespace bprmf
