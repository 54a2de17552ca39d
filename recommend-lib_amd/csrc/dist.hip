// dist.hip — kernels of the sharded (multi-GPU) step that run around the exchanges (dist.cpp).
//
// Users are owned by u % world and items by i % world.  A rank's batch of a step needs the rows
// of the distinct items it references (its "requests", owner-major, as the builder orders item
// segments).  Per chunk of n steps every rank exchanges its requests once:
//   ids_send [world][n][cap]  the requests of step k to owner p (local rows), -1 padded
//   ids_recv [world][n][cap]  what peer q requests from this rank (sorted ascending, -1 padded)
// and the owner derives, per step, an apply plan: for each distinct requested row its leader
// position (the lowest requesting peer) lists the positions of every peer's gradient for that
// row, in peer order, so the owner's sum over peers has a fixed order (bitwise reproducible).
// Per step: k_owner_gather (rows at step t-1, packed per requesting peer; this rank's own
// requests written straight into its slot buffer) -> exchange with the other ranks ->
// K1/K2 (step.hip, sharded instantiations) -> exchange of per-slot gradients ->
// k_owner_apply (fixed-order sum, lazy decay + SGD, one writer per row).
// Reference semantics: the same SGD step as BPRMFRecommender.py:172-176 on the union batch.
#include <algorithm>

#include <stdlib.h>

#include "device_common.h"
#include "dist_body.h"

namespace bprmf {

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// largest per-owner request count of the chunk (the exchange capacity) into *cap: ONE workgroup
// (n * world <= 256 steps x 64 owners), so no zeroing launch and no atomics
__global__ __launch_bounds__(1024) void k_own_max(BatchBuf bb, int64_t n, int world,
                                                  int32_t* __restrict__ cap) {
  __shared__ int32_t part[1024 / 64];
  int32_t m = 0;
  for (int64_t x = threadIdx.x; x < n * world; x += blockDim.x)
    m = max(m, bb.view(x / world).own[x % world]);
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x / 64); ++w) m = max(m, part[w]);
    *cap = m;
  }
}

// ids_send[p][k][idx] = request idx of step k to owner p (its local row), -1 past the count
__global__ void k_pack_ids(BatchBuf bb, int64_t n, int world, int cap,
                           int32_t* __restrict__ ids_send) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= (int64_t)world * n * cap) return;
  const int idx = (int)(x % cap);
  const int64_t k = (x / cap) % n;
  const int p = (int)(x / ((int64_t)cap * n));
  const BatchView v = bb.view(k);
  int pre = 0;
  for (int o = 0; o < p; ++o) pre += v.own[o];
  ids_send[x] = idx < v.own[p] ? v.ukey[pre + idx] : -1;
}

// first position of `row` in an ascending, -1 padded list (compared unsigned: pads sort last)
static __device__ __forceinline__ int find_row(const int32_t* __restrict__ list, int cap, uint32_t row) {
  int lo = 0, hi = cap;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((uint32_t)list[mid] < row) lo = mid + 1; else hi = mid;
  }
  return (lo < cap && (uint32_t)list[lo] == row) ? lo : -1;
}

// apply plan: aplan[k][p][idx][q] = q*cap + (position of row in peer q's list of step k), -1 if q
// does not request it; a position whose row an earlier peer also requests (or a pad) gets
// aplan[..][0] = -2 (not a leader: skipped by k_owner_apply).
// Gather plan of the fused owner step (k_owner_step: apply step k, then gather step k+lag; lag 1
// for the exact step, 2 for the stale-1 step, whose rows of step k+2 are read after step k's
// apply): gdep[k][p][idx][q] = position of the leader's row in peer q's list of step k+lag, -1 if
// q does not request it then (the leader serves those positions from the row it just wrote);
// gfree[k][p][idx] = 1 when position (p, idx) of step k holds a row that step k-lag did not apply
// (k < lag: every row), gathered on its own.
// One lane per (position, peer q): a group of G = next_pow2(world) lanes per position does its W
// searches side by side (three binary searches a lane: step k-lag, k and k+lag of peer q's list,
// one dependent chain each) instead of one thread walking ~3W searches in sequence; the group's "any
// peer" answers (the row was applied last step; a lower peer requests it too) are ballots.
__global__ void k_owner_plan(const int32_t* __restrict__ ids_recv, int64_t n, int world, int cap,
                             int gshift, int lag, int32_t* __restrict__ aplan,
                             int32_t* __restrict__ gdep, int32_t* __restrict__ gfree) {
  const int G = 1 << gshift;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t x = t >> gshift;
  const int q = (int)(t & (G - 1));
  const bool live = x < n * world * (int64_t)cap;  // the same for every lane of a group
  int idx = 0, p = 0;
  int64_t k = 0;
  int32_t row = -1;
  if (live) {
    idx = (int)(x % cap);
    p = (int)((x / cap) % world);
    k = x / ((int64_t)cap * world);
    row = ids_recv[((int64_t)p * n + k) * cap + idx];
  }
  const bool qv = live && q < world && row >= 0;
  const bool prev = qv && k >= lag && find_row(ids_recv + ((int64_t)q * n + k - lag) * cap, cap, (uint32_t)row) >= 0;
  const int cur = !qv ? -1 : q == p ? idx : find_row(ids_recv + ((int64_t)q * n + k) * cap, cap, (uint32_t)row);
  const int nxt = qv && k + lag < n ? find_row(ids_recv + ((int64_t)q * n + k + lag) * cap, cap, (uint32_t)row) : -1;
  // every lane of the wave takes part in the ballots (groups never straddle a wave: G <= 16)
  const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);
  const uint64_t gmask = (G >= 64 ? ~0ull : ((1ull << G) - 1)) << gbase;
  const uint64_t any_prev = __ballot(prev) & gmask;
  const uint64_t any_lower = __ballot(qv && q < p && cur >= 0) & gmask;
  if (!live || q >= world) return;
  int32_t* rec = aplan + x * world;
  int32_t* dep = gdep + x * world;
  if (row < 0) {
    dep[q] = -1;
    if (q == 0) {
      rec[0] = -2;
      gfree[x] = 0;
    }
    return;
  }
  if (q == 0) gfree[x] = any_prev ? 0 : 1;
  if (any_lower) {  // a lower peer leads this row
    dep[q] = -1;
    if (q == 0) rec[0] = -2;
    return;
  }
  rec[q] = cur < 0 ? -1 : q * cap + cur;
  dep[q] = nxt;
}

template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_owner_gather(Table Q, const int32_t* __restrict__ ids_recv,
                                                        int64_t n, int world, int cap, int k,
                                                        Hyper hp, int ld,
                                                        const int32_t* __restrict__ tbase,
                                                        PushArgs dst, int32_t* __restrict__ mark,
                                                        int32_t* __restrict__ err) {
  // mark set (IPC): the grid's last workgroup is the finisher
  const int nprod = mark ? (int)gridDim.x - 1 : (int)gridDim.x;
  if ((int)blockIdx.x < nprod) {
    owner_gather_body<G4, S>(blockIdx.x, nprod, Q, ids_recv, n, world, cap, k, hp, ld, tbase, dst,
                             mark);
  } else {
    board_finish(mark, nprod, *tbase + k + 1, dst.flag, world, err);
  }
}

// owner: for each distinct row of step k (its leader position) sum the peers' gradients in peer
// order and apply W = V - lr (g + wd V) with the pending decay; one writer per row.
template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_owner_apply(Table Q, const int32_t* __restrict__ ids_recv,
                                                       const int32_t* __restrict__ aplan, int64_t n,
                                                       int world, int cap, int k, Hyper hp, int ld,
                                                       const int32_t* __restrict__ tbase,
                                                       const float* __restrict__ grads_recv, int self,
                                                       const float* __restrict__ self_grads,
                                                       const int32_t* __restrict__ wait_flags,
                                                       int32_t* __restrict__ err) {
  const int sub = threadIdx.x & (G4 - 1);
  const int64_t x = blockIdx.x * (int64_t)(kBlock / G4) + threadIdx.x / G4;  // p * cap + idx
  wait_peer_flags(wait_flags, world, self, *tbase + k + 1, err);  // IPC: the peers' gradients
  if (x >= (int64_t)world * cap) return;
  const int32_t* rec = aplan + ((int64_t)k * world * cap + x) * world;
  const int32_t r0 = rec[0];
  if (r0 == -2) return;
  const int p = (int)(x / cap), idx = (int)(x % cap);
  const int32_t row = ids_recv[((int64_t)p * n + k) * cap + idx];
  const int32_t t = *tbase + k + 1;
  float* w = Q.W + (int64_t)row * ld + 4 * sub;
  float4 cur[S], g[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    cur[s] = ld4(w + 4 * G4 * s);
    g[s] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int32_t stamp = Q.stamp[row];
  for (int q0 = 0; q0 < world; q0 += 8) {  // up to 8 peers' rows in flight, summed in peer order
    int32_t pos[8];
    float4 gr[8][S];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      pos[m] = q0 + m < world ? (q0 + m == 0 ? r0 : rec[q0 + m]) : -1;
      if (pos[m] >= 0) {
        const int q = pos[m] / cap, i = pos[m] - q * cap;
        const float* gp = (q == self ? self_grads + (int64_t)i * ld : grads_recv + (int64_t)pos[m] * ld) + 4 * sub;
#pragma unroll
        for (int s = 0; s < S; ++s) gr[m][s] = ld4(gp + 4 * G4 * s);
      }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
      if (pos[m] >= 0) {
#pragma unroll
        for (int s = 0; s < S; ++s)
          g[s] = make_float4(g[s].x + gr[m][s].x, g[s].y + gr[m][s].y, g[s].z + gr[m][s].z,
                             g[s].w + gr[m][s].w);
      }
  }
  const float f = decay_pow(hp.log2a, t - 1 - stamp);
  const float lr = hp.lr, wd = hp.wd;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float4 v = make_float4(cur[s].x * f, cur[s].y * f, cur[s].z * f, cur[s].w * f);
    st4(w + 4 * G4 * s,
        make_float4(fmaf(-lr, fmaf(wd, v.x, g[s].x), v.x), fmaf(-lr, fmaf(wd, v.y, g[s].y), v.y),
                    fmaf(-lr, fmaf(wd, v.z, g[s].z), v.z), fmaf(-lr, fmaf(wd, v.w, g[s].w), v.w)));
  }
  if (sub == 0) Q.stamp[row] = t;
}

// Fused owner step (dist_body.h owner_step_body): apply step k and gather step k+1 in one launch.
template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_owner_step(Table Q, const int32_t* __restrict__ ids_recv,
                                                      const int32_t* __restrict__ aplan,
                                                      const int32_t* __restrict__ gdep,
                                                      const int32_t* __restrict__ gfree, int64_t n,
                                                      int world, int cap, int k, Hyper hp, int ld,
                                                      const int32_t* __restrict__ tbase,
                                                      const float* __restrict__ grads_recv, int self,
                                                      const float* __restrict__ self_grads,
                                                      const int32_t* __restrict__ wait_flags,
                                                      int32_t* __restrict__ err, PushArgs dst,
                                                      int32_t* __restrict__ mark) {
  const int nprod = mark ? (int)gridDim.x - 1 : (int)gridDim.x;  // IPC: the last is the finisher
  if ((int)blockIdx.x < nprod) {
    owner_step_body<G4, S>(blockIdx.x, nprod, Q, ids_recv, aplan, gdep, gfree, n, world, cap, k, hp,
                           ld, tbase, grads_recv, self, self_grads, wait_flags, err, dst, mark);
  } else {
    board_finish(mark, nprod, *tbase + k + 2, dst.flag, world, err);
  }
}

// ---- IPC transport: blocks pushed straight into the peers' buffers over xGMI ----------------
// Per-peer blocks of `bytes` (a multiple of 4) are copied into a.dst[p] (a peer's buffer mapped
// through hipIpc, or this rank's own buffer for the self block); every block fences at system
// scope (waits for its stores' acknowledgements) and marks the completion board; the grid's last
// block (the finisher) then stores the exchange's sequence number into each peer's flag for this
// rank.  seq = *tbase + k + 1 (per-step exchanges: graph-safe) or `seq`.
__global__ void k_ipc_push(PushArgs a, int world, int64_t bytes, const int32_t* __restrict__ tbase,
                           int k, int32_t seq, int32_t* __restrict__ mark, int32_t* __restrict__ err) {
  const int32_t s = tbase ? *tbase + k + 1 : seq;
  const int nprod = (int)gridDim.x - 1;
  if ((int)blockIdx.x == nprod) {
    board_finish(mark, nprod, s, a.flag, world, err);
    return;
  }
  const int64_t n16 = bytes / 16, per = n16 + (bytes % 16) / 4, total = per * world;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
       x += (int64_t)nprod * blockDim.x) {
    const int p = (int)(x / per);
    const int64_t u = x - p * per;
    if (!a.src[p]) continue;
    if (u < n16)
      reinterpret_cast<float4*>(a.dst[p])[u] = reinterpret_cast<const float4*>(a.src[p])[u];
    else
      reinterpret_cast<int32_t*>(a.dst[p])[4 * n16 + (u - n16)] =
          reinterpret_cast<const int32_t*>(a.src[p])[4 * n16 + (u - n16)];
  }
  // The destinations are uncached (peer landing buffers, or this rank's own buffer for the self
  // block, which the next kernel reads after the kernel boundary): waiting for the stores'
  // acknowledgements makes them visible; a system-scope fence would also write back the whole
  // L2 of this XCD, once per block.
  board_mark(mark, blockIdx.x, s);
}

// wait until every peer's flag for this exchange reached its sequence number (ipc_spin: a dead
// peer raises err bit 4 once, and every later wait of the call returns at once).
__global__ void k_ipc_wait(const int32_t* flags, int world, int self, const int32_t* __restrict__ tbase,
                           int k, int32_t seq, int32_t* __restrict__ err) {
  const int32_t s = tbase ? *tbase + k + 1 : seq;
  const int p = threadIdx.x;
  // relaxed polls: the flag and the data it guards live in uncached memory, so no cache needs
  // invalidating (an acquire at system scope would invalidate this XCD's L2 every poll)
  if (p < world && p != self) ipc_spin(flags + p, s, err);
  __syncthreads();
}

// receive side of a row/id exchange: per peer, wait for its flag, then copy its block from the
// uncached landing buffer into the cached working buffer the step kernels read (rows read many
// times, e.g. a hot item by every triplet that references it, must not be served uncached).
// blocks_per_peer blocks per peer; a block waits only for its own peer.
__global__ void k_ipc_recv(PushArgs a, int world, int self, int64_t bytes, int blocks_per_peer,
                           const int32_t* flags, const int32_t* __restrict__ tbase, int k,
                           int32_t seq, int32_t* __restrict__ err) {
  const int p = blockIdx.x / blocks_per_peer;
  if (p >= world || p == self || !a.src[p]) return;
  const int32_t s = tbase ? *tbase + k + 1 : seq;
  if (threadIdx.x == 0) ipc_spin(flags + p, s, err);
  __syncthreads();
  const int64_t n16 = bytes / 16, per = n16 + (bytes % 16) / 4;
  const int64_t stride = (int64_t)blocks_per_peer * blockDim.x;
  for (int64_t u = (blockIdx.x % blocks_per_peer) * (int64_t)blockDim.x + threadIdx.x; u < per;
       u += stride) {
    if (u < n16)
      reinterpret_cast<float4*>(a.dst[p])[u] = reinterpret_cast<const float4*>(a.src[p])[u];
    else
      reinterpret_cast<int32_t*>(a.dst[p])[4 * n16 + (u - n16)] =
          reinterpret_cast<const int32_t*>(a.src[p])[4 * n16 + (u - n16)];
  }
}

hipError_t ipc_recv(const PushArgs& a, int world, int self, int64_t bytes, const int32_t* flags,
                    const int32_t* tbase, int k, int32_t seq, int32_t* err, hipStream_t s) {
  const int64_t units = bytes / 16 + (bytes % 16) / 4;
  const int bpp = (int)std::max<int64_t>(1, std::min<int64_t>(256, (units + 4 * kBlock - 1) / (4 * kBlock)));
  k_ipc_recv<<<(unsigned)(bpp * world), kBlock, 0, s>>>(a, world, self, bytes, bpp, flags, tbase, k,
                                                        seq, err);
  return hipGetLastError();
}

__global__ void k_max_vals(const int32_t* __restrict__ vals, int world, int32_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    int32_t m = 0;
    for (int p = 0; p < world; ++p) m = max(m, vals[p]);
    *out = m;
  }
}

hipError_t ipc_push(const PushArgs& a, int world, int64_t bytes, const int32_t* tbase, int k,
                    int32_t seq, int32_t* mark, int32_t* err, hipStream_t s) {
  // up to 256 copying blocks (grid-stride: 256 x 256 lanes x 16 B keep the links busy) and the
  // finisher
  if (!mark) return hipErrorInvalidValue;
  const int64_t units = (bytes / 16 + (bytes % 16) / 4) * world;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(256, (units + kBlock - 1) / kBlock));
  k_ipc_push<<<blocks + 1, kBlock, 0, s>>>(a, world, bytes, tbase, k, seq, mark, err);
  return hipGetLastError();
}

hipError_t ipc_wait(const int32_t* flags, int world, int self, const int32_t* tbase, int k,
                    int32_t seq, int32_t* err, hipStream_t s) {
  k_ipc_wait<<<1, 64, 0, s>>>(flags, world, self, tbase, k, seq, err);
  return hipGetLastError();
}

hipError_t max_vals(const int32_t* vals, int world, int32_t* out, hipStream_t s) {
  k_max_vals<<<1, 64, 0, s>>>(vals, world, out);
  return hipGetLastError();
}

#define BPRMF_DISPATCH4D(geom, BODY)                               \
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

static unsigned blocks_for(int64_t threads) { return (unsigned)((threads + kBlock - 1) / kBlock); }

hipError_t dist_own_max(BatchBuf bb, int64_t n, int world, int32_t* cap, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_own_max<<<1, 1024, 0, s>>>(bb, n, world, cap);
  return hipGetLastError();
}

hipError_t dist_pack_ids(BatchBuf bb, int64_t n, int world, int cap, int32_t* ids_send,
                         hipStream_t s) {
  if (n <= 0 || cap <= 0) return hipSuccess;
  k_pack_ids<<<blocks_for((int64_t)world * n * cap), kBlock, 0, s>>>(bb, n, world, cap, ids_send);
  return hipGetLastError();
}

hipError_t dist_owner_plan(const int32_t* ids_recv, int64_t n, int world, int cap, int lag,
                           int32_t* aplan, int32_t* gdep, int32_t* gfree, hipStream_t s) {
  if (n <= 0 || cap <= 0) return hipSuccess;
  int gshift = 0;
  while ((1 << gshift) < world) ++gshift;  // world <= kMaxWorld = 16
  k_owner_plan<<<blocks_for((n * world * (int64_t)cap) << gshift), kBlock, 0, s>>>(
      ids_recv, n, world, cap, gshift, lag, aplan, gdep, gfree);
  return hipGetLastError();
}

hipError_t dist_owner_step(const Geom& g, Table Q, const int32_t* ids_recv, const int32_t* aplan,
                           const int32_t* gdep, const int32_t* gfree, int64_t n, int world, int cap,
                           int k, const Hyper& hp, const int32_t* tbase, const float* grads_recv,
                           int self, const float* self_grads, const int32_t* wait_flags,
                           int32_t* err, const PushArgs& dst, int32_t* mark, int max_blocks,
                           hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  BPRMF_DISPATCH4D(g, ({
    unsigned blocks = blocks_for(2LL * world * cap * G4_);
    if (mark) blocks = std::min<unsigned>(blocks, std::min(max_blocks, kBoardMax)) + 1;  // + finisher
    k_owner_step<G4_, S_><<<blocks, kBlock, 0, s>>>(Q, ids_recv, aplan, gdep, gfree, n, world, cap,
                                                    k, hp, g.ld, tbase, grads_recv, self,
                                                    self_grads, wait_flags, err, dst, mark);
  }));
  return hipGetLastError();
}

hipError_t dist_owner_gather(const Geom& g, Table Q, const int32_t* ids_recv, int64_t n, int world,
                             int cap, int k, const Hyper& hp, const int32_t* tbase,
                             const PushArgs& dst, int32_t* mark, int32_t* err, int max_blocks,
                             hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  BPRMF_DISPATCH4D(g, ({
    unsigned blocks = blocks_for((int64_t)world * cap * G4_);
    if (mark) blocks = std::min<unsigned>(blocks, std::min(max_blocks, kBoardMax)) + 1;  // + finisher
    k_owner_gather<G4_, S_><<<blocks, kBlock, 0, s>>>(Q, ids_recv, n, world, cap, k, hp, g.ld,
                                                      tbase, dst, mark, err);
  }));
  return hipGetLastError();
}

hipError_t dist_owner_apply(const Geom& g, Table Q, const int32_t* ids_recv, const int32_t* aplan,
                            int64_t n, int world, int cap, int k, const Hyper& hp,
                            const int32_t* tbase, const float* grads_recv, int self,
                            const float* self_grads, const int32_t* wait_flags, int32_t* err,
                            hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  BPRMF_DISPATCH4D(g, ({
    const unsigned blocks = blocks_for((int64_t)world * cap * G4_);
    k_owner_apply<G4_, S_><<<blocks, kBlock, 0, s>>>(Q, ids_recv, aplan, n, world, cap, k, hp,
                                                     g.ld, tbase, grads_recv, self, self_grads,
                                                     wait_flags, err);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
