// topk.hip — device scoring + per-user top-K over candidate lists.
//
// Replaces the reference's ranking loops: the final KPI (BPRMFRecommender.py:196-207: one scalar
// forward per candidate, then np.argsort(pred)[::-1][:K]) and the validation protocol
// (util/metrics.py:46-66: forward of a [gt, negatives] batch, torch.topk).  One workgroup per
// user: lane groups score the user's candidates into LDS with exactly the arithmetic of k_score
// (so scores equal BPRMF.score/forward bit for bit), then a bitonic sort in LDS over 64-bit keys
// (~orderable(score) << 32 | ~position) takes the top K: score descending, ties by LATER position
// first, i.e. np.argsort(s)[::-1] on a stable sort.  Lists longer than one pass are handled in
// passes carrying the current top K.
#include "device_common.h"

namespace bprmf {

constexpr int kTopkThreads = 256;
constexpr int kTopkIPT = 8;
constexpr int kTopkPass = kTopkThreads * kTopkIPT;  // keys per pass (carried top K included)
static_assert((kTopkPass & (kTopkPass - 1)) == 0, "bitonic passes: a power of two");
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

// ascending bitonic sort of the first N keys in LDS (N a power of two <= kTopkPass, every valid
// key among them; the rest of s are ~0 padding): log2 N (log2 N + 1) / 2 compare-exchange stages
// (66 at N = 2048, 28 for a 100-candidate list), each thread taking N / 2 / kTopkThreads pairs
// per stage.  The keys are distinct (each carries its position), so the order is the one any
// sort gives: the same top K as the block radix sort over all kTopkPass keys it replaced (round 6).
static __device__ __forceinline__ void bitonic_sort(uint64_t* s, int N) {
  for (int k = 2; k <= N; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < N / 2; q += kTopkThreads) {
        const int i = 2 * q - (q & (j - 1));  // the pair's lower index (bit j clear)
        const uint64_t a = s[i], b = s[i + j];
        if ((a > b) == ((i & k) == 0)) {
          s[i] = b;
          s[i + j] = a;
        }
      }
      __syncthreads();
    }
}

template <int G, int EPL>
__global__ __launch_bounds__(kTopkThreads) void k_topk_lists(
    const int32_t* __restrict__ users, const int64_t* __restrict__ offs,
    const int32_t* __restrict__ items, int k, Table P, Table Q, Hyper hp, int ld, int32_t T,
    int32_t* __restrict__ out_pos, float* __restrict__ out_score, int32_t* __restrict__ err) {
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
    int npass = 64;  // the pass's valid keys (this pass's m + the carried top K), rounded up
    while (npass < m + carried) npass <<= 1;
    bitonic_sort(s_key, npass);
    for (int x = threadIdx.x; x < k; x += kTopkThreads) s_top[x] = s_key[x];
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

// ---- full-catalogue top-K: scores of every (user, item) on f32 MFMA, selection on the fly ----
// The tables are flushed to the current step first (bprmf_topk_all), so rows are read as stored.
// Workgroup = 4 waves x 16 users; all waves sweep the item catalogue in tiles of 32 items staged
// in LDS (the next tile's global loads in flight in registers during the current tile's MFMAs).
// Per wave and tile: 16 x 32 scores = two v_mfma_f32_16x16x4_f32 accumulators over ld/4
// k-steps (two independent chains cover the 40-cycle dependent latency).  Operand map (16x16x4
// f32: A[l&15][k=l>>4], B[k=l>>4][l&15]): lane group g = l>>4 holds the float4 at k = 16t + 4g
// of its row; element e of step t is one MFMA, so k runs in the order (t, e, g) and each score
// is that f32 fmaf chain (exact f32, no reduced precision).
// Selection: each lane compares its 8 scores with its rows' current k-th best (registers) and
// queues the few that beat it in its row's LDS queue; then the 16 row-owner lanes insert their
// queues into their rows' k-entry lists in parallel.  Ties: the earlier (smaller) item wins, the
// sweep is in item order.
constexpr int kAllUsersPerWave = 16;
constexpr int kAllWaves = 4;
constexpr int kAllTile = 32;
constexpr int kAllMaxK = 32;
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int LDT>  // LDT = ceil(ld / 16) k-steps of 16 (1..8: ld <= 128)
__global__ __launch_bounds__(256) void k_topk_all(
    const int32_t* __restrict__ users, int64_t n_users, int k, const float* __restrict__ PW,
    int64_t p_rows, const float* __restrict__ QW, int64_t q_rows, int ld,
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    int32_t* __restrict__ out_items, float* __restrict__ out_scores) {
  constexpr int LDP = 16 * LDT + 4;  // LDS row stride (floats): conflict-free float4 reads
  constexpr int UW = kAllUsersPerWave;
  __shared__ float4 s_tile[kAllTile][LDP / 4];
  __shared__ float s_ls[kAllWaves][UW][kAllMaxK];
  __shared__ int32_t s_li[kAllWaves][UW][kAllMaxK];
  __shared__ float s_qs[kAllWaves][UW][kAllTile];  // this tile's candidates per row
  __shared__ int32_t s_qi[kAllWaves][UW][kAllTile];
  __shared__ int32_t s_qn[kAllWaves][UW];
  __shared__ float s_tau[kAllWaves][UW];
  __shared__ uint32_t s_mask[kAllWaves][UW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = lane & 15, g = lane >> 4;
  const int64_t ub = (int64_t)blockIdx.x * (kAllWaves * UW) + w * UW;
  // A operand: user row ub + row, float4 at k = 16t + 4g
  float4 a4[LDT];
  {
    const int64_t r = ub + row;
    const bool ok = r < n_users && (uint64_t)users[r] < (uint64_t)p_rows;
    const int64_t u = ok ? users[r] : 0;
#pragma unroll
    for (int t = 0; t < LDT; ++t) {
      const int kk = 16 * t + 4 * g;
      a4[t] = (ok && kk < ld) ? *reinterpret_cast<const float4*>(PW + u * ld + kk)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // row-owner lanes (0..15): list state in registers + LDS, exclusion cursor
  int cnt = 0, worst = 0;
  int64_t pnext = 0, pend = 0;
  int32_t pval = INT32_MAX;
  if (lane < UW) {
    s_qn[w][lane] = 0;
    s_tau[w][lane] = -INFINITY;
    const int64_t r = ub + lane;
    if (indptr && r < n_users && (uint64_t)users[r] < (uint64_t)p_rows) {
      pnext = indptr[users[r]];
      pend = indptr[users[r] + 1];
      pval = pnext < pend ? indices[pnext] : INT32_MAX;
    }
  }
  float tau[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};  // rows 4g + r
  // tile loader: 32 items x ld floats as float4s
  constexpr int PER = (kAllTile * 4 * LDT + 255) / 256;  // float4s per thread
  const int q4 = ld / 4;
  float4 nxt[PER];
  auto load_tile = [&](int64_t i0) {
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const int x = threadIdx.x + 256 * m, it = x / (4 * LDT), c = x % (4 * LDT);
      const int64_t item = i0 + it;
      nxt[m] = (it < kAllTile && c < q4 && item < q_rows)
                   ? *reinterpret_cast<const float4*>(QW + item * ld + 4 * c)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const int x = threadIdx.x + 256 * m, it = x / (4 * LDT), c = x % (4 * LDT);
      if (it < kAllTile) s_tile[it][c] = nxt[m];
    }
  };
  const int64_t ntiles = (q_rows + kAllTile - 1) / kAllTile;
  load_tile(0);
  store_tile();
  __syncthreads();
  for (int64_t tile = 0; tile < ntiles; ++tile) {
    const int64_t i0 = tile * kAllTile;
    if (tile + 1 < ntiles) load_tile(i0 + kAllTile);
    if (lane < UW) {  // exclusion mask of this tile for the owner's row
      uint32_t msk = 0;
      while (pval < i0 + kAllTile) {
        if (pval >= i0) msk |= 1u << (pval - i0);
        ++pnext;
        pval = pnext < pend ? indices[pnext] : INT32_MAX;
      }
      s_mask[w][lane] = msk;
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < LDT; ++t) {
      const float4 b0 = s_tile[row][4 * t + g];
      const float4 b1 = s_tile[16 + row][4 * t + g];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].x, b0.x, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].x, b1.x, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].y, b0.y, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].y, b1.y, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].z, b0.z, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].z, b1.z, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].w, b0.w, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t].w, b1.w, acc1, 0, 0, 0);
    }
    __syncthreads();  // every wave is done reading s_tile: refill it
    if (tile + 1 < ntiles) store_tile();
    // lane holds C[row 4g + r][item (lane & 15)] (acc0) and [item 16 + (lane & 15)] (acc1)
    bool cand = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ur = 4 * g + r;
      const uint32_t msk = s_mask[w][ur];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = 16 * c + row;
        const float x = (i0 + col < q_rows && !((msk >> col) & 1u)) ? (c ? acc1[r] : acc0[r])
                                                                      : -INFINITY;
        if (x > tau[r]) {
          const int q = atomicAdd(&s_qn[w][ur], 1);
          s_qs[w][ur][q] = x;
          s_qi[w][ur][q] = (int32_t)(i0 + col);
          cand = true;
        }
      }
    }
    if (__ballot(cand)) {
      __builtin_amdgcn_wave_barrier();
      if (lane < UW) {  // the owner inserts its row's queue (rows in parallel)
        const int nq = s_qn[w][lane];
        float tl = s_tau[w][lane];
        for (int q = 0; q < nq; ++q) {
          const float v = s_qs[w][lane][q];
          if (!(v > tl)) continue;
          const int32_t item = s_qi[w][lane][q];
          int slot;
          if (cnt < k) {
            slot = cnt++;
          } else {
            slot = worst;
          }
          s_ls[w][lane][slot] = v;
          s_li[w][lane][slot] = item;
          if (cnt == k) {  // full: find the worst entry (lowest score, then largest item)
            int wi = 0;
            for (int y = 1; y < k; ++y) {
              const float a = s_ls[w][lane][y], bb = s_ls[w][lane][wi];
              if (a < bb || (a == bb && s_li[w][lane][y] > s_li[w][lane][wi])) wi = y;
            }
            worst = wi;
            tl = s_ls[w][lane][wi];
          }
        }
        s_qn[w][lane] = 0;
        s_tau[w][lane] = tl;
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 4; ++r) tau[r] = s_tau[w][4 * g + r];
    }
    __syncthreads();  // the refilled tile is complete
  }
  // results: the owner lanes sort their row's list (score desc, item asc) and write it
  if (lane < UW && ub + lane < n_users) {
    const int c = cnt;
    float* ls = s_ls[w][lane];
    int32_t* li = s_li[w][lane];
    for (int x = 1; x < c; ++x) {
      const float v = ls[x];
      const int32_t it = li[x];
      int y = x - 1;
      while (y >= 0 && (ls[y] < v || (ls[y] == v && li[y] > it))) {
        ls[y + 1] = ls[y];
        li[y + 1] = li[y];
        --y;
      }
      ls[y + 1] = v;
      li[y + 1] = it;
    }
    const int64_t o = (ub + lane) * k;
    for (int x = 0; x < k; ++x) {
      out_items[o + x] = x < c ? li[x] : -1;
      out_scores[o + x] = x < c ? ls[x] : -INFINITY;
    }
  }
}

hipError_t topk_all(const Geom& g, const int32_t* users, int64_t n_users, int k, Table P, Table Q,
                    const Hyper& hp, int32_t T, const int64_t* indptr, const int32_t* indices,
                    int32_t* out_items, float* out_scores, hipStream_t s) {
  if (n_users <= 0) return hipSuccess;
  if (k <= 0 || k > kAllMaxK || g.ld > 128) return hipErrorInvalidValue;
  // rows as stored: bring both tables to step T first (the lazy decay made explicit)
  if (hipError_t e = flush(g, P, hp, T, s)) return e;
  if (hipError_t e = flush(g, Q, hp, T, s)) return e;
  const unsigned blocks = (unsigned)((n_users + kAllWaves * kAllUsersPerWave - 1) / (kAllWaves * kAllUsersPerWave));
  const int ldt = (g.ld + 15) / 16;
#define BPRMF_TOPK_ALL(L)                                                                    \
  case L:                                                                                  \
    k_topk_all<L><<<blocks, 256, 0, s>>>(users, n_users, k, P.W, P.rows, Q.W, Q.rows, g.ld, \
                                         indptr, indices, out_items, out_scores);          \
    break;
  switch (ldt) {
    BPRMF_TOPK_ALL(1)
    BPRMF_TOPK_ALL(2)
    BPRMF_TOPK_ALL(4)
    BPRMF_TOPK_ALL(8)
    default: return hipErrorInvalidValue;
  }
#undef BPRMF_TOPK_ALL
  return hipGetLastError();
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
