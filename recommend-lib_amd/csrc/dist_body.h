// dist_body.h — device bodies of the owner-side phases of the sharded step (included by
// dist.hip, whose kernels run them alone, and by step.hip, whose fused front launch
// k_dist_front runs them beside K1).  Layouts and the plan: dist.hip's header comment.
#pragma once
#include "device_common.h"

namespace bprmf {

static __device__ __forceinline__ float4 dist_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void dist_st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// owner: rows requested by every peer for step k, brought to step t-1: the row of position
// (p, idx) goes to dst.to[p] + idx * ld (packed send blocks, this rank's own slots, or -- IPC
// transport -- straight into peer p's landing buffer).  With mark set (IPC), each workgroup marks
// its completion board entry once its stores are acknowledged (a finisher workgroup then raises
// the peers' row flags, device_common.h board_finish).
// (blk, nblk: this workgroup and the owner workgroups of the launch; the body is shared by
// k_owner_gather and the fused front launch of the sharded step, step.hip k_dist_front)
template <int G4, int S>
static __device__ __forceinline__ void owner_gather_body(int blk, int nblk, const Table& Q,
                                                         const int32_t* __restrict__ ids_recv,
                                                         int64_t n, int world, int cap, int k,
                                                         const Hyper& hp, int ld,
                                                         const int32_t* __restrict__ tbase,
                                                         const PushArgs& dst,
                                                         int32_t* __restrict__ mark) {
  constexpr int NG = kBlock / G4;
  const int sub = threadIdx.x & (G4 - 1);
  const int32_t t = *tbase + k + 1;
  for (int64_t x = blk * (int64_t)NG + threadIdx.x / G4; x < (int64_t)world * cap;
       x += (int64_t)nblk * NG) {
    const int p = (int)(x / cap), idx = (int)(x % cap);
    const int32_t row = ids_recv[((int64_t)p * n + k) * cap + idx];
    if ((uint32_t)row >= (uint32_t)Q.rows) continue;
    const float* w = Q.W + (int64_t)row * ld + 4 * sub;
    float4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = dist_ld4(w + 4 * G4 * s);
    const float f = decay_pow(hp.log2a, t - 1 - Q.stamp[row]);
    float* o = static_cast<float*>(dst.dst[p]) + (int64_t)idx * ld + 4 * sub;
#pragma unroll
    for (int s = 0; s < S; ++s)
      dist_st4(o + 4 * G4 * s, make_float4(v[s].x * f, v[s].y * f, v[s].z * f, v[s].w * f));
  }
  if (mark) board_mark(mark, blk, t);
}

// Fused owner step: apply step k (as k_owner_apply) and gather step k+lag (as k_owner_gather) in
// one launch (lag 1: the exact step; 2: the stale-1 step, whose rows of step k+2 are the table
// after step k brought to step t+1 by decay).  A row step k applies is served to step k+lag's
// requesters by its leader, from the value it just stored (gdep); rows step k does not apply are
// gathered by their own groups (gfree).  No row is both read by a free gather and written by an
// apply, so the groups are independent.  Past the chunk's last step there is nothing to gather.
// With mark set (IPC), each workgroup marks its completion board entry (step k+lag) once its
// stores are acknowledged; a finisher workgroup raises the peers' row flags.
template <int G4, int S>
static __device__ __forceinline__ void owner_step_body(
    int blk, int nblk, const Table& Q, const int32_t* __restrict__ ids_recv,
    const int32_t* __restrict__ aplan, const int32_t* __restrict__ gdep,
    const int32_t* __restrict__ gfree, int64_t n, int world, int cap, int k, const Hyper& hp, int ld,
    const int32_t* __restrict__ tbase, const float* __restrict__ grads_recv, int self,
    const float* __restrict__ self_grads, const int32_t* __restrict__ wait_flags,
    int32_t* __restrict__ err, const PushArgs& dst, int32_t* __restrict__ mark, int lag = 1) {
  constexpr int NG = kBlock / G4;
  const int sub = threadIdx.x & (G4 - 1);
  const int32_t t = *tbase + k + 1;
  wait_peer_flags(wait_flags, world, self, t, err);  // IPC: the peers' gradients of step k
  const int64_t WC = (int64_t)world * cap;
  const float lr = hp.lr, wd = hp.wd;
  const int64_t nx = k + lag < n ? 2 * WC : WC;  // applies, then the gathers of step k+lag
  const float f_dep = lag > 1 ? decay_pow(hp.log2a, lag - 1) : 1.f;  // served rows to step t+lag-1
  for (int64_t x = blk * (int64_t)NG + threadIdx.x / G4; x < nx; x += (int64_t)nblk * NG) {
    if (x < WC) {  // apply: the leader position of a row of step k
      const int32_t* rec = aplan + ((int64_t)k * WC + x) * world;
      const int32_t r0 = rec[0];
      if (r0 == -2) continue;
      const int p = (int)(x / cap), idx = (int)(x % cap);
      const int32_t row = ids_recv[((int64_t)p * n + k) * cap + idx];
      float* w = Q.W + (int64_t)row * ld + 4 * sub;
      float4 cur[S], g[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        cur[s] = dist_ld4(w + 4 * G4 * s);
        g[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const int32_t stamp = Q.stamp[row];
      for (int q0 = 0; q0 < world; q0 += 8) {  // peers' rows in flight, summed in peer order
        int32_t pos[8];
        float4 gr[8][S];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          pos[m] = q0 + m < world ? (q0 + m == 0 ? r0 : rec[q0 + m]) : -1;
          if (pos[m] >= 0) {
            const int q = pos[m] / cap, i = pos[m] - q * cap;
            const float* gp = (q == self ? self_grads + (int64_t)i * ld : grads_recv + (int64_t)pos[m] * ld) + 4 * sub;
#pragma unroll
            for (int s = 0; s < S; ++s) gr[m][s] = dist_ld4(gp + 4 * G4 * s);
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
      float4 nv[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float4 v = make_float4(cur[s].x * f, cur[s].y * f, cur[s].z * f, cur[s].w * f);
        nv[s] = make_float4(fmaf(-lr, fmaf(wd, v.x, g[s].x), v.x), fmaf(-lr, fmaf(wd, v.y, g[s].y), v.y),
                            fmaf(-lr, fmaf(wd, v.z, g[s].z), v.z), fmaf(-lr, fmaf(wd, v.w, g[s].w), v.w));
        dist_st4(w + 4 * G4 * s, nv[s]);
      }
      if (sub == 0) Q.stamp[row] = t;
      const int32_t* dep = gdep + ((int64_t)k * WC + x) * world;
      for (int q = 0; q < world; ++q) {  // step k+lag's requests of this row: the new value
        const int32_t i2 = dep[q];
        if (i2 < 0) continue;
        float* o = static_cast<float*>(dst.dst[q]) + (int64_t)i2 * ld + 4 * sub;
#pragma unroll
        for (int s = 0; s < S; ++s)
          dist_st4(o + 4 * G4 * s, lag > 1 ? make_float4(nv[s].x * f_dep, nv[s].y * f_dep, nv[s].z * f_dep,
                                                         nv[s].w * f_dep)
                                           : nv[s]);
      }
    } else {  // gather: a position of step k+lag whose row step k does not apply
      const int64_t y = x - WC;
      if (!gfree[(int64_t)(k + lag) * WC + y]) continue;
      const int q = (int)(y / cap), idx = (int)(y % cap);
      const int32_t row = ids_recv[((int64_t)q * n + k + lag) * cap + idx];
      const float* w = Q.W + (int64_t)row * ld + 4 * sub;
      float4 v[S];
#pragma unroll
      for (int s = 0; s < S; ++s) v[s] = dist_ld4(w + 4 * G4 * s);
      const float f = decay_pow(hp.log2a, t + lag - 1 - Q.stamp[row]);  // brought to step (t + lag) - 1
      float* o = static_cast<float*>(dst.dst[q]) + (int64_t)idx * ld + 4 * sub;
#pragma unroll
      for (int s = 0; s < S; ++s)
        dist_st4(o + 4 * G4 * s, make_float4(v[s].x * f, v[s].y * f, v[s].z * f, v[s].w * f));
    }
  }
  if (mark && k + lag < n) board_mark(mark, blk, t + lag);  // (nothing gathered: no mark)
}

}  // namespace bprmf
