// device_common.h — device helpers shared by kernels.hip and segment.hip (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kernels.h"

// Diagnostic build only (-DBPRMF_CALL_STAMPS, tools/ubench_call_stamps.py): per launch slot of a
// call, the earliest workgroup start and the latest workgroup end (s_memrealtime, 100 MHz), spread
// over 64 words per slot (blockIdx % 64) so the atomics do not serialise on one address; one table
// per translation unit (no relocatable device code), each with its reader.  The real GPU timeline
// of a call, kernel boundaries included, without a profiler in the loop.
#ifdef BPRMF_CALL_STAMPS
extern __device__ unsigned long long g_cs[64][2][64];
// and, per slot, workgroup 0's shader-clock counter (s_memtime) and 100 MHz clock
// (s_memrealtime) at its start and end: their ratio is the shader clock during the launch
extern __device__ unsigned long long g_clk[64][4];
#define BPRMF_CALL_STAMPS_DEF(tu)                                                                 \
  __device__ unsigned long long g_clk[64][4];                                                     \
  extern "C" int bprmf_debug_clk_##tu(unsigned long long* out) {                                  \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(g_clk)) == hipSuccess ? 0 : -3;    \
  }                                                                                               \
  __device__ unsigned long long g_cs[64][2][64];                                                  \
  extern "C" int bprmf_debug_call_stamps_##tu(unsigned long long* out, int reset) {              \
    if (reset) {                                                                                  \
      static unsigned long long init[64][2][64];                                                  \
      for (int a = 0; a < 64; ++a)                                                                \
        for (int b = 0; b < 64; ++b) {                                                            \
          init[a][0][b] = ~0ull;                                                                  \
          init[a][1][b] = 0;                                                                      \
        }                                                                                         \
      return hipMemcpyToSymbol(HIP_SYMBOL(g_cs), init, sizeof init) == hipSuccess ? 0 : -3;       \
    }                                                                                             \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cs), sizeof(g_cs)) == hipSuccess ? 0 : -3;      \
  }
#define CS_BEGIN(slot)                                                                            \
  do {                                                                                            \
    if (threadIdx.x == 0)                                                                         \
      atomicMin(&g_cs[(slot) & 63][0][blockIdx.x & 63], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                                    \
      g_clk[(slot) & 63][0] = __builtin_amdgcn_s_memtime();                                      \
      g_clk[(slot) & 63][1] = __builtin_amdgcn_s_memrealtime();                                  \
    }                                                                                             \
  } while (0)
#define CS_END(slot)                                                                              \
  do {                                                                                            \
    __syncthreads();                                                                              \
    if (threadIdx.x == 0)                                                                         \
      atomicMax(&g_cs[(slot) & 63][1][blockIdx.x & 63], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                                    \
      g_clk[(slot) & 63][2] = __builtin_amdgcn_s_memtime();                                      \
      g_clk[(slot) & 63][3] = __builtin_amdgcn_s_memrealtime();                                  \
    }                                                                                             \
  } while (0)
struct CsScope {  // CS_BEGIN at construction, CS_END when the kernel's threads leave its scope
  int slot;
  __device__ explicit CsScope(int s) : slot(s) { CS_BEGIN(slot); }
  __device__ ~CsScope() { CS_END(slot); }
};
#else
struct CsScope {
  __device__ explicit CsScope(int) {}
};
#define BPRMF_CALL_STAMPS_DEF(tu)
#define CS_BEGIN(slot) \
  do {                 \
  } while (0)
#define CS_END(slot) \
  do {               \
  } while (0)
#endif

namespace bprmf {

constexpr uint32_t TAG_NEG = 0x4E470000u;
constexpr uint32_t TAG_PERM = 0x50520000u;
constexpr uint32_t TAG_INIT = 0x494E0000u;
constexpr int kBlock = 256;
constexpr int kMaxBlocks = kMaxGridBlocks;  // 256 CUs x 8 resident 256-thread blocks, grid-stride beyond

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based; Salmon et al. SC'11).  Stateless: every triplet / element draws
// from its own counter, so the sampler is embarrassingly parallel and bit-reproducible.
// ------------------------------------------------------------------------------------------------
static __device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                         uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply each (v_mad_u64_u32) instead of a mul_lo + mul_hi pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// keyed bijection of [0, n): a 6-round alternating Feistel network on Z_a x Z_c (x = L*c + R,
// c = ceil(sqrt(n)), a = ceil(n/c); feistel_dims), F = Philox keyed by the seed and tagged by
// round and epoch: even rounds L = (L + hi32(F(R)*a)) mod a, odd rounds R = (R + hi32(F(L)*c))
// mod c; cycle-walking back into [0, n).  a*c - n < c, so a walk is needed with probability below
// 1/sqrt(n) (a power-of-two domain 2^b < 2n made ~86 % of 64-lane waves run a second pass at
// ml-20m, and the wave waits for its slowest lane).
static __device__ __forceinline__ uint64_t permute(uint64_t x, uint64_t n, uint32_t fa, uint32_t fc,
                                                   uint32_t k0, uint32_t k1, uint32_t epoch) {
  do {
    uint32_t L, R;
    if (x >> 32) {
      L = (uint32_t)(x / fc);
      R = (uint32_t)(x - (uint64_t)L * fc);
    } else {
      L = (uint32_t)x / fc;
      R = (uint32_t)x - L * fc;
    }
#pragma unroll
    for (uint32_t r = 0; r < 6; ++r) {
      uint32_t c0 = (r & 1) ? L : R, c1 = r, c2 = epoch, c3 = TAG_PERM | r;
      philox10(c0, c1, c2, c3, k0, k1);
      if (r & 1) {
        R += __umulhi(c0, fc);
        if (R >= fc) R -= fc;
      } else {
        L += __umulhi(c0, fa);
        if (L >= fa) L -= fa;
      }
    }
    x = (uint64_t)L * fc + R;
  } while (x >= n);
  return x;
}

// unbiased Lemire reduction into [0, n), n >= 1; retries draw fresh counters (attempt in tag).
// Split in two so a caller can draw attempt 0 (bounded_draw0: depends on q only) while the loads
// that give n are in flight, then finish with bounded_from.
static __device__ __forceinline__ uint32_t bounded_draw(uint64_t q, uint32_t epoch, uint32_t att,
                                                        uint32_t k0, uint32_t k1) {
  uint32_t c0 = (uint32_t)q, c1 = (uint32_t)(q >> 32), c2 = epoch, c3 = TAG_NEG | att;
  philox10(c0, c1, c2, c3, k0, k1);
  return c0;
}
static __device__ __forceinline__ uint32_t bounded_draw0(uint64_t q, uint32_t epoch, uint32_t k0,
                                                         uint32_t k1) {
  return bounded_draw(q, epoch, 0, k0, k1);
}
static __device__ __forceinline__ uint32_t bounded_from(uint32_t d0, uint64_t q, uint32_t epoch,
                                                        uint32_t n, uint32_t k0, uint32_t k1) {
  const uint32_t thresh = (0u - n) % n;  // (2^32 - n) mod n in 32-bit arithmetic
  uint32_t d = d0;
  for (uint32_t a = 1;; ++a) {
    const uint64_t m = (uint64_t)d * n;
    if ((uint32_t)m >= thresh) return (uint32_t)(m >> 32);
    d = bounded_draw(q, epoch, a, k0, k1);
  }
}
static __device__ __forceinline__ uint32_t bounded(uint64_t q, uint32_t epoch, uint32_t n, uint32_t k0,
                                            uint32_t k1) {
  return bounded_from(bounded_draw0(q, epoch, k0, k1), q, epoch, n, k0, k1);
}

// q / d for the sampler's triplet -> positive map: 32-bit division when q fits (the usual case)
static __device__ __forceinline__ int64_t div_small(uint64_t q, uint32_t d) {
  return q >> 32 ? (int64_t)(q / d) : (int64_t)((uint32_t)q / d);
}

// j = the k-th item id NOT in the sorted positive list a[0..n): m = #{x : a[x]-x <= k}, j = k+m.
// (A 9-ary search with 8 pivot loads per round measured no faster on the short-chunk sampler and
// slower on long chunks: the sampler's time is its Philox work, not this chain.)
static __device__ __forceinline__ int64_t kth_nonmember(const int32_t* __restrict__ a, int64_t n, int64_t k) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] - mid <= k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return k + lo;
}

// The same count through the user's 16-ary tree (host_plan.h build_search_tree): keys b[x] =
// a[x] - x, one 64-byte node (four 16-byte loads, one line) per level, m = #{x : b[x] <= k};
// equal to kth_nonmember's m for every k (same value, fewer dependent loads: ceil(log16 n)
// instead of ceil(log2 n), and ~4x fewer line requests).
static __device__ __forceinline__ int64_t kth_nonmember_tree(const int32_t* __restrict__ keys,
                                                             int64_t n, int64_t k) {
  if (n <= 0) return k;
  int L = 1;
  for (int64_t c = 16; c < n; c *= 16) ++L;
  int64_t node = 0;
  for (int l = L - 1;; --l) {
    const int4* q = reinterpret_cast<const int4*>(keys + node * 16);
    const int4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3];
    const int c = (v0.x <= k) + (v0.y <= k) + (v0.z <= k) + (v0.w <= k) + (v1.x <= k) +
                  (v1.y <= k) + (v1.z <= k) + (v1.w <= k) + (v2.x <= k) + (v2.y <= k) +
                  (v2.z <= k) + (v2.w <= k) + (v3.x <= k) + (v3.y <= k) + (v3.z <= k) + (v3.w <= k);
    if (l == 0) return k + node * 16 + c;
    if (c == 0) return k;  // k below the level's first key: no b[x] <= k
    // the next level down: past this level's nodes (ceil(n / 16^(l+1)) of them)
    const int sh = 4 * (l + 1);
    keys += 16 * ((n + (1LL << sh) - 1) >> sh);
    node = node * 16 + (c - 1);
  }
}

// One slot of the device sampler (BPRData.ng_sample + the shuffled DataLoader,
// util/data_loader.py:680-690, BPRMFRecommender.py:141): slot -> triplet q = perm(slot) ->
// positive q / num_ng -> (global user u, item i) and the negative j, uniform over u's
// non-positives.  false: u holds every item (j = -1).  k_sample and the split builder's in-launch
// sampling both call this, so their triplets are the same bits.
static __device__ __forceinline__ bool sample_slot(const SamplerArgs& a, uint32_t epoch, uint64_t slot,
                                                   int32_t& u, int32_t& i, int32_t& j) {
  const uint64_t N = (uint64_t)a.npos * (uint64_t)a.num_ng;
#if defined(BPRMF_SAMPLE_DIAG) && (BPRMF_SAMPLE_DIAG & 2)  // diagnostic: no shuffle (timing only)
  const uint64_t q = slot;
#else
  const uint64_t q = permute(slot, N, a.feistel_a, a.feistel_c, a.k0, a.k1, epoch);
#endif
  const int64_t p = div_small(q, (uint32_t)a.num_ng);
  int2 ur4 = make_int2(0, 0);
  if (a.pos4) {  // one 16-byte load: the positive and its user's record
    const int4 pr = a.pos4[p];
    u = pr.x;
    i = pr.y;
    ur4 = make_int2(pr.z, pr.w);
  } else if (a.pos2) {  // one 8-byte load: one line per positive instead of two
    const int2 pr = a.pos2[p];
    u = pr.x;
    i = pr.y;
  } else {
    u = a.pos_u[p];
    i = a.pos_i[p];
  }
  const uint32_t d0 = bounded_draw0(q, epoch, a.k0, a.k1);  // while the loads are in flight
  const int64_t ul = u / a.world;
  if (a.pos4 || a.urec) {  // {first tree key, positive count}: one line per user instead of indptr + soff
    const int2 ur = a.pos4 ? ur4 : a.urec[ul];
    const int64_t free_u = a.item_num - ur.y;
    j = -1;
    if (free_u <= 0) return false;
    const uint32_t k = bounded_from(d0, q, epoch, (uint32_t)free_u, a.k0, a.k1);
#if defined(BPRMF_SAMPLE_DIAG) && (BPRMF_SAMPLE_DIAG & 1)  // diagnostic: no search (timing only)
    j = (int32_t)k;
#else
    j = (int32_t)kth_nonmember_tree(a.skeys + ur.x, ur.y, (int64_t)k);
#endif
    return true;
  }
  const int64_t beg = a.indptr[ul], deg = a.indptr[ul + 1] - beg;
  const int64_t free_items = a.item_num - deg;
  j = -1;
  if (free_items <= 0) return false;
  const uint32_t k = bounded_from(d0, q, epoch, (uint32_t)free_items, a.k0, a.k1);
#if defined(BPRMF_SAMPLE_DIAG) && (BPRMF_SAMPLE_DIAG & 1)  // diagnostic: no search (timing only)
  j = (int32_t)k;
#else
  j = a.skeys ? (int32_t)kth_nonmember_tree(a.skeys + a.soff[ul], deg, (int64_t)k)
              : (int32_t)kth_nonmember(a.indices + beg, deg, (int64_t)k);
#endif
  return true;
}

// (1 - lr*wd)^k in double by squaring (deterministic IEEE order), rounded once to fp32.
// (1 - lr*wd)^k for a row whose last k steps were pure weight decay.  log2a = log2(1 - lr*wd) is
// formed in double on the host; k*log2a in double, one v_exp_f32 (relative error ~1e-7, far below
// the ~sqrt(k) ulp drift of the reference's own k repeated fp32 decays).  k == 0: exactly 1.
static __device__ __forceinline__ float decay_pow(double log2a, int32_t k) {
  if (k <= 0) return 1.0f;
  return exp2f((float)((double)k * log2a));
}

static __device__ __forceinline__ float softplus(float z) {  // log(1 + e^z), overflow-free
  return fmaxf(z, 0.f) + log1pf(expf(-fabsf(z)));
}

template <int G>
static __device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// sum over the wave of per-lane loss partials into this wave's own f64 slot.  Never one shared
// word: same-address atomics serialise at ~13 ns each (4096 waves = 53 us).
static __device__ __forceinline__ void wave_add_loss(double* slots, float v) {
  if (!slots) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  // no-return atomic into the wave's own slot: no contention, and the wave does not wait on it
  if ((threadIdx.x & 63) == 0) atomicAdd(&slots[blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)], (double)v);
}

// One IPC flag wait: spin until *flag >= seq.  A wait that outlives ~10 s (a peer died) raises
// err bit 4 and gives up instead of hanging the queue; once bit 4 is up (this wait's or an earlier
// one's), later waits return at once, so a dead peer costs one timeout per call, not one per wait.
// The flags and the data they guard are uncached, so relaxed polls suffice.
static __device__ __forceinline__ bool ipc_spin(const int32_t* flag, int32_t seq, int32_t* err) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4) return false;
  int64_t spins = 0;
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
    __builtin_amdgcn_s_sleep(2);
    ++spins;
    if ((spins & 4095) == 0 && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4))
      return false;
    if (spins > 150000000) {
      atomicOr(err, 4);
      return false;
    }
  }
  return true;
}

// Completion board: each producing workgroup of a grid marks its own word once its stores are
// acknowledged (sc1 store, MI355X_MICROARCH.md valid forms, table row 1); ONE finisher workgroup,
// dispatched after every producer (the grid's last block), polls all the marks with sc1 loads and
// then signals.  It replaces a same-address atomic count (memory-side and serialised, ~80 ns per
// add: a 1,168-workgroup K2 grid spent ~11 us of every step in its count).
static __device__ __forceinline__ void board_mark(int32_t* mark, int i, int32_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's (remote) stores landed
  __syncthreads();                                    // ... and every wave's of the workgroup
  if (threadIdx.x == 0) __hip_atomic_store(mark + i, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the whole workgroup: true once marks[0, n) all reached seq (false after ~10 s: err bit 4)
static __device__ __forceinline__ bool board_wait(const int32_t* mark, int n, int32_t seq,
                                                  int32_t* err) {
  for (int64_t spins = 0;; ++spins) {
    int mine = 1;
    for (int b = threadIdx.x; b < n; b += blockDim.x)
      mine &= __hip_atomic_load(mark + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= seq;
    if (__syncthreads_and(mine)) return true;
    __builtin_amdgcn_s_sleep(2);
    if (spins > 10000000) {
      if (threadIdx.x == 0) atomicOr(err, 4);
      return false;
    }
  }
}
// the finisher: every producer's mark, then each non-null flag[p] raised to seq (system scope)
static __device__ __forceinline__ void board_finish(const int32_t* mark, int n, int32_t seq,
                                                    int32_t* const* flag, int nflags,
                                                    int32_t* err) {
  if (!board_wait(mark, n, seq, err)) return;
  if (threadIdx.x == 0)
    for (int p = 0; p < nflags; ++p)
      if (flag[p]) __hip_atomic_store(flag[p], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Sharded steps over the IPC transport: the first thread of every workgroup waits until each
// peer's flag (this rank's flag array for one exchange kind, written remotely by the peers' push
// kernels) reaches the step's sequence number, then the workgroup proceeds.
static __device__ __forceinline__ void wait_peer_flags(const int32_t* flags, int world, int self,
                                                       int32_t seq, int32_t* err) {
  if (!flags) return;
  if (threadIdx.x == 0) {
    for (int p = 0; p < world; ++p) {
      if (p == self) continue;
      if (!ipc_spin(flags + p, seq, err)) break;
    }
  }
  __syncthreads();
}

static inline unsigned grid_for(int64_t units, int G) {
  const int64_t per_block = kBlock / G;
  int64_t b = (units + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > kMaxBlocks) b = kMaxBlocks;
  return (unsigned)b;
}
static inline unsigned grid_flat(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 4 * kMaxBlocks) b = 4 * kMaxBlocks;
  return (unsigned)b;
}

// Expand `BODY` for every instantiated (G, EPL) geometry.
#define BPRMF_DISPATCH(geom, BODY)                                  \
  switch ((geom).G * 100 + (geom).EPL) {                            \
    case 401: { constexpr int G_ = 4, E_ = 1; BODY; } break;        \
    case 801: { constexpr int G_ = 8, E_ = 1; BODY; } break;        \
    case 1601: { constexpr int G_ = 16, E_ = 1; BODY; } break;      \
    case 3201: { constexpr int G_ = 32, E_ = 1; BODY; } break;      \
    case 6401: { constexpr int G_ = 64, E_ = 1; BODY; } break;      \
    case 6402: { constexpr int G_ = 64, E_ = 2; BODY; } break;      \
    case 6403: { constexpr int G_ = 64, E_ = 3; BODY; } break;      \
    case 6404: { constexpr int G_ = 64, E_ = 4; BODY; } break;      \
    case 6405: { constexpr int G_ = 64, E_ = 5; BODY; } break;      \
    case 6406: { constexpr int G_ = 64, E_ = 6; BODY; } break;      \
    case 6407: { constexpr int G_ = 64, E_ = 7; BODY; } break;      \
    case 6408: { constexpr int G_ = 64, E_ = 8; BODY; } break;      \
    case 6412: { constexpr int G_ = 64, E_ = 12; BODY; } break;     \
    case 6416: { constexpr int G_ = 64, E_ = 16; BODY; } break;     \
    default: return hipErrorInvalidValue;                           \
  }

// Expand BODY for every instantiated float4 geometry (G4_, S_).
#define BPRMF_DISPATCH4(geom, BODY)                                \
  switch ((geom).G4 * 10 + (geom).S) {                             \
    case 11: { constexpr int G4_ = 1, S_ = 1; BODY; } break;       \
    case 21: { constexpr int G4_ = 2, S_ = 1; BODY; } break;       \
    case 41: { constexpr int G4_ = 4, S_ = 1; BODY; } break;       \
    case 81: { constexpr int G4_ = 8, S_ = 1; BODY; } break;       \
    case 161: { constexpr int G4_ = 16, S_ = 1; BODY; } break;     \
    case 321: { constexpr int G4_ = 32, S_ = 1; BODY; } break;     \
    case 641: { constexpr int G4_ = 64, S_ = 1; BODY; } break;     \
    case 642: { constexpr int G4_ = 64, S_ = 2; BODY; } break;     \
    case 643: { constexpr int G4_ = 64, S_ = 3; BODY; } break;     \
    case 644: { constexpr int G4_ = 64, S_ = 4; BODY; } break;     \
    default: return hipErrorInvalidValue;                          \
  }

}  // namespace bprmf
