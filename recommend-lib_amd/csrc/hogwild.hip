// hogwild.hip — the opt-in relaxed-synchronisation BPR step (semantics "hogwild"; the default
// stays the exact batch-synchronous step of step.hip).
//
// The reference step (BPRMFRecommender.py:172-176) is batch-synchronous SGD: every triplet of a
// batch reads the tables as the previous step left them, and duplicate rows' gradients are summed
// before one update.  That chain (K1 -> K2 -> next K1) bounds the exact path at ~16 % of the HBM
// roofline.  SURVEY.md §7 "Hard parts" asks for bounded-staleness / Hogwild modes
// as flags, with HR@10 reported for each; this is that mode:
//   - one launch per chunk of steps (up to ~1000 batches), persistent waves, no barriers;
//   - each triplet is applied on its own as soon as its rows arrive (per-sample SGD on the
//     triplet's three rows, Hogwild!-style: no locks, no atomics; concurrent updates of one row may
//     overwrite each other);
//   - weight decay keeps the reference's per-STEP schedule: a triplet of batch t brings a row it
//     touches from its stamp s to step t - 1 (factor (1 - lr wd)^(t-1-s)) and applies the wd term
//     only on the row's first touch in step t (s < t), so every row decays once per step as torch's
//     SGD does; a row already at a later step (s >= t, touched by a later batch in flight) is
//     neither decayed nor re-stamped (stamps only move forward);
//   - staleness is bounded by the launch's in-flight window: at most ~min(U, I) triplets are in
//     flight at once (the grid is capped to that), so a row sees about one other update in flight
//     whatever the table size; a wave takes `tpw` consecutive slots.
// Coherence: row and stamp stores are write-through (sc1) — the line leaves the XCD's L2 and is
// dropped there — so no XCD keeps a dirty or long-lived stale copy of a row another XCD updates;
// a reader sees another XCD's update at most one read-modify-write window late (MI355X_MICROARCH.md
// "stores of each flavour").
//
// Work layout: lane l of a wave samples slot base + l itself (the device sampler's spec,
// device_common.h: Philox + Feistel shuffle + k-th non-member; bit-exact to k_sample), so no
// triplet array makes a round trip through HBM; the wave then walks its tpw triplets G4 lanes per
// triplet (one float4 per lane and stripe), two rounds of kHwUnroll * (64 / G4) triplets' rows in
// flight at once (double-buffered: the next round's loads go out before this round's stores).
#include <stdlib.h>

#include <algorithm>

#include "device_common.h"

#if defined(__HIP_DEVICE_COMPILE__) && !(defined(__gfx950__) || defined(__gfx942__))
#error "hogwild.hip targets gfx950 (sc1 write-through stores)"
#endif

namespace bprmf {

// 16-byte row load.  NT: past this CU's L1, a non-temporal load (global_load_dwordx4 ... nt)
// served by the XCD's L2 (MI355X_MICROARCH.md: sc1 / nt loads bypass L1 only; the L2 drops every
// line the XCD stores sc1); else a plain load, which may hit a line this CU cached a little
// earlier (a relaxed read; the stamps are always sc1 loads, so a row is never decayed twice).
// Measured (round 6, tools/gpu/ab_bench.sh, profiles/r06_hogwild_nt_ab.txt): the local mode at the
// ml-20m shape (tables in the 256 MiB Infinity Cache) 2.62 us per step with plain loads, 3.16
// with nt; at a 1.5 GB shape (HBM) 2.90 plain, 2.78 nt.  So nt only when the tables exceed the
// Infinity Cache (hogwild() below).  Rounds 4-5 built one kernel with both forms behind a
// runtime flag, and the compiler merged them into plain loads: their measurements are the
// plain form.  (A compiler builtin, so the loads stay visible to its wait counting.)
template <bool NT>
static __device__ __forceinline__ float4 hw_ld4(const float* p) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  if constexpr (NT) {
    const v4f x = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(x[0], x[1], x[2], x[3]);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}
static __device__ __forceinline__ int32_t hw_ld_word(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 dword load
}

// write-through (sc1) 16-byte store: the line leaves and is dropped from the XCD's L2
static __device__ __forceinline__ void hw_st4(float* p, float4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
}
static __device__ __forceinline__ void hw_st_word(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static __device__ __forceinline__ float hw_dot4(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}

// V' = f V (the row brought to step t - 1); W = V' - lr (g + wd V') on the row's first touch in
// step t, W = V' - lr g on a later touch in the same step (the decay is taken once per step)
static __device__ __forceinline__ float4 hw_sgd(float4 v, float4 g, float lr, float wdf) {
  return make_float4(fmaf(-lr, fmaf(wdf, v.x, g.x), v.x), fmaf(-lr, fmaf(wdf, v.y, g.y), v.y),
                     fmaf(-lr, fmaf(wdf, v.z, g.z), v.z), fmaf(-lr, fmaf(wdf, v.w, g.w), v.w));
}

// One triplet's slot -> (u, i, j): the device sampler itself (device_common.h sample_slot, the
// function k_sample and the split builder call), so hogwild's triplets are the same bits.
static __device__ __forceinline__ void hw_sample(const SamplerArgs& a, uint32_t epoch, uint64_t slot,
                                                 int32_t& u, int32_t& i, int32_t& j, int32_t* err) {
  if (!sample_slot(a, epoch, slot, u, i, j)) atomicOr(err, 2);
}

#ifndef BPRMF_HW_UNROLL
#define BPRMF_HW_UNROLL 2
#endif
constexpr int kHwUnroll = BPRMF_HW_UNROLL;  // triplets per lane group per round (rows in flight
                                            // per buffer; -DBPRMF_HW_UNROLL: A/B builds)

// One round of a wave: kHwUnroll triplets per lane group, their ids, stamps and rows.
template <int S, int UNR>
struct HwRound {
  float4 pu[UNR][S], vi[UNR][S], vj[UNR][S];
  int32_t su[UNR], si[UNR], sj[UNR], uu[UNR], ii[UNR], jj[UNR];
  int32_t hi[UNR], hj[UNR];  // LOCAL: the items' replica slots (-1: cold, the shared table)
  bool ok[UNR];
};

// semantics "local" (kernels.h LocalArgs): the hot items' rows live in one replica
// per XCD, rep + (xcc * H + slot) * ld, written back (plain stores: the line stays in the XCD's L2,
// where every wave of that XCD reads it with nt loads); hot[item] = slot or -1
// this wave's XCD (0-7): which replica it trains (read, not assumed: any placement is correct)
static __device__ __forceinline__ int hw_xcc() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;  // hwreg(HW_REG_XCC_ID, 0, 4)
}

// a hot item's replica slot from la.hhash (the item is there: its bit in la.hbits is set; the
// probe count is bounded all the same)
static __device__ __forceinline__ int32_t hot_probe(const LocalArgs& la, int32_t item) {
  const uint32_t mask = (1u << la.hlog) - 1;
  uint32_t h = ((uint32_t)item * 0x9E3779B1u) >> (32 - la.hlog);
  for (uint32_t n = 0; n <= mask; ++n, h = (h + 1) & mask) {
    const int2 e = la.hhash[h];
    if (e.x == item) return e.y;
    if (e.x < 0) break;
  }
  return -1;
}

// issue the round starting at slot k0 of the wave's chunk (ids from the lanes that sampled them)
template <int G4, int S, int UNR, int GPW, bool SERIAL, bool LOCAL = false, bool NT = false>
static __device__ __forceinline__ void hw_load(HwRound<S, UNR>& R, int k0, int cnt, int32_t mu,
                                               int32_t mi, int32_t mj, const Table& P,
                                               const Table& Q, int ld, int sub, int gw,
                                               int32_t mhi = -1, int32_t mhj = -1,
                                               const float* repx = nullptr) {
#pragma unroll
  for (int r = 0; r < UNR; ++r) {
    const int src = k0 + r * GPW + gw;
    R.uu[r] = __shfl(mu, src & 63);
    R.ii[r] = __shfl(mi, src & 63);
    R.jj[r] = __shfl(mj, src & 63);
    R.hi[r] = LOCAL ? __shfl(mhi, src & 63) : -1;
    R.hj[r] = LOCAL ? __shfl(mhj, src & 63) : -1;
    R.ok[r] = (SERIAL ? gw == 0 : true) && src < cnt && R.uu[r] >= 0;
    if (R.ok[r]) {
      const float* pr = P.W + (int64_t)R.uu[r] * ld + 4 * sub;
      const float* qi = (LOCAL && R.hi[r] >= 0 ? repx + (int64_t)R.hi[r] * ld : Q.W + (int64_t)R.ii[r] * ld) + 4 * sub;
      const float* qj = (LOCAL && R.hj[r] >= 0 ? repx + (int64_t)R.hj[r] * ld : Q.W + (int64_t)R.jj[r] * ld) + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        R.pu[r][k] = hw_ld4<NT>(pr + 4 * G4 * k);
        R.vi[r][k] = hw_ld4<NT>(qi + 4 * G4 * k);
        R.vj[r][k] = hw_ld4<NT>(qj + 4 * G4 * k);
      }
      R.su[r] = hw_ld_word(P.stamp + R.uu[r]);
      // a replica row has no stamp: it is current within its period (the merge applies the
      // period's weight decay), so it reads as "already at this step"
      R.si[r] = LOCAL && R.hi[r] >= 0 ? INT32_MAX : hw_ld_word(Q.stamp + R.ii[r]);
      R.sj[r] = LOCAL && R.hj[r] >= 0 ? INT32_MAX : hw_ld_word(Q.stamp + R.jj[r]);
    } else {
      R.su[r] = R.si[r] = R.sj[r] = 0;
#pragma unroll
      for (int k = 0; k < S; ++k) R.pu[r][k] = R.vi[r][k] = R.vj[r][k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// compute and store the round at slot k0 (slot base + k0 + ... of step t0 + 1 + slot / B)
template <int G4, int S, int UNR, int GPW, bool SERIAL, bool LOCAL = false>
static __device__ __forceinline__ void hw_apply(HwRound<S, UNR>& R, int64_t base, int k0,
                                                const Table& P, const Table& Q, const Hyper& hp,
                                                int ld, int32_t t0, int B, int sub, int gw,
                                                float& lacc, float* repx = nullptr) {
  const float lr = hp.lr, wd = hp.wd;
#pragma unroll
  for (int r = 0; r < UNR; ++r) {
    const int src = k0 + r * GPW + gw;
    const int32_t t = t0 + 1 + (int32_t)((uint32_t)(base + src) / (uint32_t)B);  // chunks < 2^31 slots
    // first touch of the row in step t: decay to t - 1 and take the wd term; else neither
    const bool fu1 = R.su[r] < t, fi1 = R.si[r] < t, fj1 = R.sj[r] < t;
    const float fu = fu1 ? decay_pow(hp.log2a, t - 1 - R.su[r]) : 1.f;
    const float fi = fi1 ? decay_pow(hp.log2a, t - 1 - R.si[r]) : 1.f;
    const float fj = fj1 ? decay_pow(hp.log2a, t - 1 - R.sj[r]) : 1.f;
    float di = 0.f, dj = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      float4& pu = R.pu[r][k];
      float4& vi = R.vi[r][k];
      float4& vj = R.vj[r][k];
      pu = make_float4(pu.x * fu, pu.y * fu, pu.z * fu, pu.w * fu);
      vi = make_float4(vi.x * fi, vi.y * fi, vi.z * fi, vi.w * fi);
      vj = make_float4(vj.x * fj, vj.y * fj, vj.z * fj, vj.w * fj);
      di = hw_dot4(pu, vi, di);
      dj = hw_dot4(pu, vj, dj);
    }
    // the group's lanes are in one wave: the butterfly needs every lane of the wave, so it runs
    // whatever ok[] says (inactive groups carry zeros)
    di = group_sum<G4>(R.ok[r] ? di : 0.f);
    dj = group_sum<G4>(R.ok[r] ? dj : 0.f);
    if (!R.ok[r]) continue;
    const float x = di - dj;
    const float c = 1.0f / (1.0f + expf(x));  // sigmoid(-x) = -dL/dx
    if (sub == 0) lacc += softplus(-x);       // -log sigmoid(x)
    float* pr = P.W + (int64_t)R.uu[r] * ld + 4 * sub;
    const bool hoti = LOCAL && R.hi[r] >= 0, hotj = LOCAL && R.hj[r] >= 0;
    float* qi = (hoti ? repx + (int64_t)R.hi[r] * ld : Q.W + (int64_t)R.ii[r] * ld) + 4 * sub;
    float* qj = (hotj ? repx + (int64_t)R.hj[r] * ld : Q.W + (int64_t)R.jj[r] * ld) + 4 * sub;
    const bool same = R.ii[r] == R.jj[r];  // i == j: one row, both gradients (stored once, as i)
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const float4 pu = R.pu[r][k], vi = R.vi[r][k], vj = R.vj[r][k];
      const float4 gu = make_float4(-c * (vi.x - vj.x), -c * (vi.y - vj.y), -c * (vi.z - vj.z),
                                    -c * (vi.w - vj.w));
      const float4 gj = make_float4(c * pu.x, c * pu.y, c * pu.z, c * pu.w);
      float4 gi = make_float4(-c * pu.x, -c * pu.y, -c * pu.z, -c * pu.w);
      if (same) gi = make_float4(gi.x + gj.x, gi.y + gj.y, gi.z + gj.z, gi.w + gj.w);
      hw_st4(pr + 4 * G4 * k, hw_sgd(pu, gu, lr, fu1 ? wd : 0.f));
      // replica rows: written back into this XCD's L2 (plain stores), no weight-decay term (their
      // stamps read INT32_MAX: fi1 / fj1 false); shared rows: write-through, as hogwild
      const float4 ni = hw_sgd(vi, gi, lr, fi1 ? wd : 0.f), nj = hw_sgd(vj, gj, lr, fj1 ? wd : 0.f);
      if (hoti) *reinterpret_cast<float4*>(qi + 4 * G4 * k) = ni;
      else hw_st4(qi + 4 * G4 * k, ni);
      if (!same) {
        if (hotj) *reinterpret_cast<float4*>(qj + 4 * G4 * k) = nj;
        else hw_st4(qj + 4 * G4 * k, nj);
      }
    }
    if (sub == 0) {
      if (fu1) hw_st_word(P.stamp + R.uu[r], t);
      if (fi1) hw_st_word(Q.stamp + R.ii[r], t);
      if (fj1 && !same) hw_st_word(Q.stamp + R.jj[r], t);
    }
    if (SERIAL) {  // the next triplet reads these rows: stores done, this CU's L1 dropped
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
}

// SAMPLE: slots come from the device sampler (a, epoch, slot0 + s); else replayed ids tu/ti/tj[s].
// SERIAL (tests): one lane group, one triplet at a time, in slot order (launched as one wave).
// Rounds are double-buffered: round k+1's loads are issued BEFORE round k's stores, so waiting
// for them does not wait for round k's write-through acknowledgements (gfx9 counts stores in
// vmcnt, in order with the loads).
template <int G4, int S, bool SAMPLE, bool SERIAL, bool LOCAL = false, bool NT = false>
__global__ __launch_bounds__(kBlock) void k_hogwild(SamplerArgs a, uint32_t epoch, int64_t slot0,
                                                    const int32_t* __restrict__ tu,
                                                    const int32_t* __restrict__ ti,
                                                    const int32_t* __restrict__ tj, int64_t n,
                                                    Table P, Table Q, Hyper hp, int ld, int32_t t0,
                                                    int B, int tpw, double* __restrict__ loss,
                                                    int32_t* __restrict__ err, LocalArgs la = LocalArgs{},
                                                    int uw = 1) {
  constexpr int GPW = SERIAL ? 1 : 64 / G4;  // triplets per wave per round and unroll step
  constexpr int UNR = SERIAL ? 1 : kHwUnroll;
  constexpr int STEP = GPW * UNR;
  const int lane = threadIdx.x & 63;
  const int sub = lane & (G4 - 1);
  const int gw = lane / G4;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
  float lacc = 0.f;
  float* repx = LOCAL ? la.rep + (int64_t)hw_xcc() * la.H * ld : nullptr;  // this XCD's replica
  for (int64_t base = wave * tpw; base < n; base += nwaves * tpw) {
    const int cnt = (int)min<int64_t>(tpw, n - base);
    int32_t mu = 0, mi = 0, mj = 0, mhi = -1, mhj = -1;
    if (lane < cnt) {
      const int64_t s = base + lane;
      if (SAMPLE) {
        hw_sample(a, epoch, (uint64_t)(slot0 + s), mu, mi, mj, err);
      } else {
        mu = tu[s];
        mi = ti[s];
        mj = tj[s];
      }
      // world 1: ids are rows.  uw > 1 (semantics "local" at world uw): items are rows (every
      // rank holds the whole item table), a user's row is u / uw, and a replayed u < 0 is an
      // empty slot.  A sampler that found no negative (j = -1) has raised err bit 2; any other
      // bad id raises bit 1.  Either way: skipped.
      bool empty = false;
      if (uw > 1) {
        if (mu >= 0) mu /= uw;
        else empty = !SAMPLE;
      }
      if (empty) {
        mu = -1;
      } else if (mu < 0 || mu >= P.rows || mi < 0 || mi >= Q.rows || mj < 0 || mj >= Q.rows) {
        if (mj >= 0 || !SAMPLE) atomicOr(err, 1);
        mu = -1;
      } else if (LOCAL) {  // the items' replica slots, looked up once by the sampling lane
        if (la.hbits) {  // large catalogue: a bit per item, then the hot items' table
          const uint32_t bi = la.hbits[(uint32_t)mi >> 5], bj = la.hbits[(uint32_t)mj >> 5];
          mhi = (bi >> (mi & 31)) & 1 ? hot_probe(la, mi) : -1;
          mhj = (bj >> (mj & 31)) & 1 ? hot_probe(la, mj) : -1;
        } else {
          mhi = la.hot[mi];
          mhj = la.hot[mj];
        }
      }
    }
    HwRound<S, UNR> A, Bf;
    if (SERIAL) {  // each triplet reads what the one before it stored: no prefetch
      for (int k0 = 0; k0 < cnt; k0 += STEP) {
        hw_load<G4, S, UNR, GPW, SERIAL, LOCAL, NT>(A, k0, cnt, mu, mi, mj, P, Q, ld, sub, gw, mhi, mhj, repx);
        hw_apply<G4, S, UNR, GPW, SERIAL, LOCAL>(A, base, k0, P, Q, hp, ld, t0, B, sub, gw, lacc, repx);
      }
      continue;
    }
    hw_load<G4, S, UNR, GPW, SERIAL, LOCAL, NT>(A, 0, cnt, mu, mi, mj, P, Q, ld, sub, gw, mhi, mhj, repx);
    for (int k0 = 0; k0 < cnt; k0 += 2 * STEP) {
      const bool more1 = k0 + STEP < cnt, more2 = k0 + 2 * STEP < cnt;
      if (more1)
        hw_load<G4, S, UNR, GPW, SERIAL, LOCAL, NT>(Bf, k0 + STEP, cnt, mu, mi, mj, P, Q, ld, sub, gw, mhi,
                                                mhj, repx);
      hw_apply<G4, S, UNR, GPW, SERIAL, LOCAL>(A, base, k0, P, Q, hp, ld, t0, B, sub, gw, lacc, repx);
      if (!more1) break;
      if (more2)
        hw_load<G4, S, UNR, GPW, SERIAL, LOCAL, NT>(A, k0 + 2 * STEP, cnt, mu, mi, mj, P, Q, ld, sub, gw,
                                                mhi, mhj, repx);
      hw_apply<G4, S, UNR, GPW, SERIAL, LOCAL>(Bf, base, k0 + STEP, P, Q, hp, ld, t0, B, sub, gw, lacc,
                                               repx);
    }
  }
  // the wave's loss into one of kSegLossSlots f64 slots (no-return atomics; order is not fixed,
  // like the updates themselves)
  if (loss) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lacc += __shfl_xor(lacc, off);
    if (lane == 0 && lacc != 0.f) atomicAdd(&loss[wave & (kSegLossSlots - 1)], (double)lacc);
  }
}

// LOCAL: end of a period (steps t0+1 .. t1): each hot item's new row is its value at t0 (the
// replicas' common starting value), decayed over the period as torch's SGD decays every row every
// step, plus each XCD's change to it, added in XCD order 0..7 (a fixed order); the base row takes
// it with stamp t1 and every replica starts the next period from it.  refresh: no replica
// changes (they are reset from the base; after set_weights / a flush).  One lane group per row.
template <int G4, int S>
__global__ __launch_bounds__(kBlock) void k_local_merge(Table Q, LocalArgs la,
                                                        const int32_t* __restrict__ rows, Hyper hp,
                                                        int ld, int32_t t0, int32_t t1, int refresh) {
  const int sub = threadIdx.x & (G4 - 1);
  const int64_t h = blockIdx.x * (int64_t)(kBlock / G4) + threadIdx.x / G4;
  if (h >= la.H) return;
  const int32_t item = rows[h];
  float* w = Q.W + (int64_t)item * ld + 4 * sub;
  const int32_t st = Q.stamp[item];
  const float f0 = decay_pow(hp.log2a, t0 - st);  // the base at t0
  const float fk = decay_pow(hp.log2a, t1 - t0);  // the period's weight decay
  float4 b0[S], acc[S], rv[kLocalXcds][S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(w + 4 * G4 * k);
    b0[k] = make_float4(v.x * f0, v.y * f0, v.z * f0, v.w * f0);
    acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (!refresh) {
#pragma unroll
    for (int x = 0; x < kLocalXcds; ++x) {  // every replica's row in flight at once
      const float* r = la.rep + ((int64_t)x * la.H + h) * ld + 4 * sub;
#pragma unroll
      for (int k = 0; k < S; ++k) rv[x][k] = *reinterpret_cast<const float4*>(r + 4 * G4 * k);
    }
#pragma unroll
    for (int x = 0; x < kLocalXcds; ++x)
#pragma unroll
      for (int k = 0; k < S; ++k)
        acc[k] = make_float4(acc[k].x + (rv[x][k].x - b0[k].x), acc[k].y + (rv[x][k].y - b0[k].y),
                             acc[k].z + (rv[x][k].z - b0[k].z), acc[k].w + (rv[x][k].w - b0[k].w));
  }
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const float4 nv = make_float4(fmaf(b0[k].x, fk, acc[k].x), fmaf(b0[k].y, fk, acc[k].y),
                                  fmaf(b0[k].z, fk, acc[k].z), fmaf(b0[k].w, fk, acc[k].w));
    *reinterpret_cast<float4*>(w + 4 * G4 * k) = nv;
#pragma unroll
    for (int x = 0; x < kLocalXcds; ++x)
      *reinterpret_cast<float4*>(la.rep + ((int64_t)x * la.H + h) * ld + 4 * sub + 4 * G4 * k) = nv;
  }
  if (sub == 0) Q.stamp[item] = t1;
}

hipError_t local_merge(const Geom& g, Table Q, const LocalArgs& la, const int32_t* rows,
                       const Hyper& hp, int32_t t0, int32_t t1, bool refresh, hipStream_t s) {
  if (la.H <= 0) return hipSuccess;
  BPRMF_DISPATCH4(g, ({
    const unsigned blocks = (unsigned)((la.H + kBlock / G4_ - 1) / (kBlock / G4_));
    k_local_merge<G4_, S_><<<blocks, kBlock, 0, s>>>(Q, la, rows, hp, g.ld, t0, t1, refresh ? 1 : 0);
  }));
  return hipGetLastError();
}

// semantics "local" at world > 1: a rank's change of the item table since the
// last merge at step tm (when every row equalled `base`): delta = row brought to t1 - base decayed
// to t1.  Flat over the table's float4s (q4 per row; 32-bit index arithmetic: the launcher checks
// the table has fewer than 2^32 float4s); a row's stamp is read once per float4 (L2-resident).
// A hot item (la.H > 0) is first merged from its per-XCD replicas exactly as k_local_merge does
// over the period rep_t -> t1.  pend_sum (dp_overlap, kernels.h dp_delta): the sum started at
// step tp lands here.  keep: the row and its replicas take the result (the next period starts from
// it); otherwise k_dp_apply rewrites every row.
__global__ __launch_bounds__(kBlock) void k_dp_delta(Table Q, float* __restrict__ base,
                                                     float* __restrict__ delta,
                                                     const float* __restrict__ pend_sum, uint32_t n4,
                                                     uint32_t q4, Hyper hp, int32_t tm, int32_t tp,
                                                     int32_t t1, LocalArgs la, int32_t rep_t, int keep) {
  const float fb = decay_pow(hp.log2a, tp - tm);  // base -> tp
  const float fc = decay_pow(hp.log2a, t1 - tp);  // tp -> t1
  const float fk = decay_pow(hp.log2a, t1 - rep_t);
  float4* w = reinterpret_cast<float4*>(Q.W);
  float4* b = reinterpret_cast<float4*>(base);
  float4* d = reinterpret_cast<float4*>(delta);
  const float4* ps = reinterpret_cast<const float4*>(pend_sum);
  for (uint32_t x = blockIdx.x * kBlock + threadIdx.x; x < n4; x += gridDim.x * kBlock) {
    const uint32_t row = x / q4, col = x - row * q4;
    const int32_t st = Q.stamp[row];
    const int32_t slot = la.H > 0 ? la.hot[row] : -1;
    float4 v = w[x];
    if (slot >= 0) {  // k_local_merge's rule: fma(b0, fk, sum over XCDs of (replica - b0))
      const float f0 = decay_pow(hp.log2a, rep_t - st);
      const float4 b0 = make_float4(v.x * f0, v.y * f0, v.z * f0, v.w * f0);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < kLocalXcds; ++r) {
        const float4 rv = reinterpret_cast<const float4*>(la.rep)[((int64_t)r * la.H + slot) * q4 + col];
        acc = make_float4(acc.x + (rv.x - b0.x), acc.y + (rv.y - b0.y), acc.z + (rv.z - b0.z),
                          acc.w + (rv.w - b0.w));
      }
      v = make_float4(fmaf(b0.x, fk, acc.x), fmaf(b0.y, fk, acc.y), fmaf(b0.z, fk, acc.z),
                      fmaf(b0.w, fk, acc.w));
    } else {
      const float f = decay_pow(hp.log2a, t1 - st);
      v = make_float4(v.x * f, v.y * f, v.z * f, v.w * f);
    }
    const float4 o = b[x];
    float4 g = make_float4(o.x * fb, o.y * fb, o.z * fb, o.w * fb);
    if (ps) {  // the landed sum: the common table at tp, and the other ranks' part of it
      const float4 sm = ps[x], od = d[x];
      g = make_float4(fmaf(o.x, fb, sm.x), fmaf(o.y, fb, sm.y), fmaf(o.z, fb, sm.z), fmaf(o.w, fb, sm.w));
      v = make_float4(fmaf(sm.x - od.x, fc, v.x), fmaf(sm.y - od.y, fc, v.y), fmaf(sm.z - od.z, fc, v.z),
                      fmaf(sm.w - od.w, fc, v.w));
      b[x] = g;
    }
    d[x] = make_float4(v.x - g.x * fc, v.y - g.y * fc, v.z - g.z * fc, v.w - g.w * fc);
    if (keep) {
      w[x] = v;
      if (col == 0) Q.stamp[row] = t1;
      if (slot >= 0)
#pragma unroll
        for (int r = 0; r < kLocalXcds; ++r)
          reinterpret_cast<float4*>(la.rep)[((int64_t)r * la.H + slot) * q4 + col] = v;
    }
  }
}

// the merge: row = base = base decayed to t1 + the ranks' summed deltas, current at t1; a hot
// item's per-XCD replicas (la.H > 0) restart from it too
__global__ __launch_bounds__(kBlock) void k_dp_apply(Table Q, float* __restrict__ base,
                                                     const float* __restrict__ sum, uint32_t n4, uint32_t q4,
                                                     Hyper hp, int32_t tm, int32_t t1, LocalArgs la) {
  const float fb = decay_pow(hp.log2a, t1 - tm);
  float4* w = reinterpret_cast<float4*>(Q.W);
  float4* b = reinterpret_cast<float4*>(base);
  const float4* s = reinterpret_cast<const float4*>(sum);
  for (uint32_t x = blockIdx.x * kBlock + threadIdx.x; x < n4; x += gridDim.x * kBlock) {
    const uint32_t row = x / q4, col = x - row * q4;
    const float4 o = b[x], a = s[x];
    const float4 nv = make_float4(fmaf(o.x, fb, a.x), fmaf(o.y, fb, a.y), fmaf(o.z, fb, a.z), fmaf(o.w, fb, a.w));
    w[x] = nv;
    b[x] = nv;
    if (col == 0) Q.stamp[row] = t1;
    if (la.H > 0) {
      const int32_t slot = la.hot[row];
      if (slot >= 0)
#pragma unroll
        for (int r = 0; r < kLocalXcds; ++r)
          reinterpret_cast<float4*>(la.rep)[((int64_t)r * la.H + slot) * q4 + col] = nv;
    }
  }
}

// the in-process transport's all-reduce: the ranks' deltas summed in rank order (the same bits on
// every rank)
__global__ __launch_bounds__(kBlock) void k_dp_sum(DpSrcs src, int world, float* __restrict__ out, int64_t n4) {
  for (int64_t x = blockIdx.x * (int64_t)kBlock + threadIdx.x; x < n4; x += (int64_t)gridDim.x * kBlock) {
    float4 a = reinterpret_cast<const float4*>(src.p[0])[x];
    for (int p = 1; p < world; ++p) {
      const float4 v = reinterpret_cast<const float4*>(src.p[p])[x];
      a = make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
    }
    reinterpret_cast<float4*>(out)[x] = a;
  }
}

static unsigned dp_blocks(int64_t n4) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + kBlock - 1) / kBlock, 8192));
}

hipError_t dp_delta(Table Q, float* base, float* delta, const float* pend_sum, int ld, const Hyper& hp,
                    int32_t tm, int32_t tp, int32_t t1, const LocalArgs& la, int32_t rep_t, bool keep,
                    hipStream_t s) {
  const int64_t n4 = Q.rows * (int64_t)(ld / 4);
  if (ld % 4 || n4 >= (1LL << 32) || tp < tm || t1 < tp || (!pend_sum && tp != tm)) return hipErrorInvalidValue;
  if (n4 <= 0) return hipSuccess;
  k_dp_delta<<<dp_blocks(n4), kBlock, 0, s>>>(Q, base, delta, pend_sum, (uint32_t)n4, (uint32_t)(ld / 4), hp,
                                              tm, tp, t1, la, rep_t, keep ? 1 : 0);
  return hipGetLastError();
}

hipError_t dp_apply(Table Q, float* base, const float* sum, int ld, const Hyper& hp, int32_t tm,
                    int32_t t1, const LocalArgs& la, hipStream_t s) {
  const int64_t n4 = Q.rows * (int64_t)(ld / 4);
  if (ld % 4 || n4 >= (1LL << 32)) return hipErrorInvalidValue;
  if (n4 <= 0) return hipSuccess;
  k_dp_apply<<<dp_blocks(n4), kBlock, 0, s>>>(Q, base, sum, (uint32_t)n4, (uint32_t)(ld / 4), hp, tm, t1, la);
  return hipGetLastError();
}

hipError_t dp_sum(const DpSrcs& src, int world, float* out, int64_t n, hipStream_t s) {
  if (world < 1 || world > kMaxWorld || n % 4) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  if (n4 <= 0) return hipSuccess;
  k_dp_sum<<<dp_blocks(n4), kBlock, 0, s>>>(src, world, out, n4);
  return hipGetLastError();
}

// the geometries of the hogwild launch: by default half the rows' lanes per triplet and twice the
// stripes for 32- and 64-lane rows (d = 65..256: twice the triplets, so twice the rows, in flight
// per wave; local mode 1.56 -> 1.61e9 triplets/s at the ml-20m shape against the rows' own
// (G4, S), round 4)
#define HW_DISPATCH(geom, BODY)                                     \
  switch ((geom).G4 * 10 + (geom).S) {                             \
    case 11: { constexpr int G4_ = 1, S_ = 1; BODY; } break;       \
    case 21: { constexpr int G4_ = 2, S_ = 1; BODY; } break;       \
    case 41: { constexpr int G4_ = 4, S_ = 1; BODY; } break;       \
    case 81: { constexpr int G4_ = 8, S_ = 1; BODY; } break;       \
    case 161: { constexpr int G4_ = 16, S_ = 1; BODY; } break;     \
    case 162: { constexpr int G4_ = 16, S_ = 2; BODY; } break;     \
    case 321: { constexpr int G4_ = 32, S_ = 1; BODY; } break;     \
    case 322: { constexpr int G4_ = 32, S_ = 2; BODY; } break;     \
    case 641: { constexpr int G4_ = 64, S_ = 1; BODY; } break;     \
    case 642: { constexpr int G4_ = 64, S_ = 2; BODY; } break;     \
    case 643: { constexpr int G4_ = 64, S_ = 3; BODY; } break;     \
    case 644: { constexpr int G4_ = 64, S_ = 4; BODY; } break;     \
    default: return hipErrorInvalidValue;                          \
  }

static bool hw_serial() {
  const char* e = getenv("BPRMF_HOGWILD_SERIAL");
  return e && e[0] == '1';
}

// triplets per wave: enough waves to fill the chip for short chunks (>= ~2048 waves), 64 (one per
// lane) for long ones
static int hw_tpw(int64_t n) {
  if (n >= 64LL * 4096) return 64;
  if (n >= 32LL * 2048) return 32;
  return 16;
}

hipError_t hogwild(const Geom& g0, const SamplerArgs* sa, uint32_t epoch, int64_t slot0,
                   const int32_t* tu, const int32_t* ti, const int32_t* tj, int64_t n, Table P,
                   Table Q, const Hyper& hp, int32_t t0, int B, double* loss, int32_t* err,
                   hipStream_t s, const LocalArgs* lap, int uw) {
  if (n <= 0) return hipSuccess;
  if (uw < 1) return hipErrorInvalidValue;
  Geom g = g0;
  if ((g.G4 == 32 || g.G4 == 64) && g.S == 1) {
    g.G4 /= 2;
    g.S = 2;
  }
  const bool serial = hw_serial();
  const int tpw = serial ? 64 : hw_tpw(n);
  const int64_t waves = (n + tpw - 1) / tpw;
  const int wpb = kBlock / 64;
  int64_t blocks = serial ? 1 : (waves + wpb - 1) / wpb;
  if (blocks > kMaxGridBlocks) blocks = kMaxGridBlocks;  // grid-stride beyond
  // Staleness window: at most ~min(U, I) triplets in flight (each wave holds 64/G4 * kHwUnroll),
  // so a row sees about one other update in flight at a time whatever the table size.  Measured
  // (ml-100k, d=32: 943 x 1,682 rows): ~1k in flight trains like the exact step, ~8k (64
  // workgroups) barely trains (lost updates on every row); ml-20m (26,744 items) at the full grid
  // (~24k resident) matches the exact step's HR@10.  BPRMF_HOGWILD_WINDOW overrides (triplets:
  // the speed / quality frontier of DESIGN.md §5c is measured along it).
  {
    int64_t window = std::min<int64_t>(P.rows, Q.rows);
    if (const char* e = getenv("BPRMF_HOGWILD_WINDOW")) window = std::max<int64_t>(1, atoll(e));
    const int64_t per_block = (int64_t)wpb * (64 / g.G4) * 2 * kHwUnroll;  // two rounds in flight
    const int64_t cap = std::max<int64_t>(1, (window + per_block - 1) / per_block);
    if (blocks > cap) blocks = cap;
  }
  const unsigned threads = serial ? 64 : kBlock;
  // the row loads past L1 (nt) only for tables larger than the Infinity Cache (hw_ld4)
  const bool nt = (P.rows + Q.rows) * (int64_t)g.ld * 4 > (256LL << 20);
  SamplerArgs a{};
  if (sa) a = *sa;
  if (lap) {  // semantics "local": the hot items in per-XCD replicas
    const LocalArgs la = *lap;
    HW_DISPATCH(g, ({
      if (serial && sa)
        k_hogwild<G4_, S_, true, true, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q,
                                                                  hp, g.ld, t0, B, tpw, loss, err, la, uw);
      else if (serial)
        k_hogwild<G4_, S_, false, true, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q,
                                                                   hp, g.ld, t0, B, tpw, loss, err, la, uw);
      else if (sa && nt)
        k_hogwild<G4_, S_, true, false, true, true><<<(unsigned)blocks, threads, 0, s>>>(
            a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, la, uw);
      else if (sa)
        k_hogwild<G4_, S_, true, false, true><<<(unsigned)blocks, threads, 0, s>>>(
            a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, la, uw);
      else
        k_hogwild<G4_, S_, false, false, true><<<(unsigned)blocks, threads, 0, s>>>(
            a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, la, uw);
    }));
    return hipGetLastError();
  }
  HW_DISPATCH(g, ({
    if (serial && sa)
      k_hogwild<G4_, S_, true, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q, hp,
                                                          g.ld, t0, B, tpw, loss, err, LocalArgs{}, uw);
    else if (serial)
      k_hogwild<G4_, S_, false, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q, hp,
                                                           g.ld, t0, B, tpw, loss, err, LocalArgs{}, uw);
    else if (sa && nt)
      k_hogwild<G4_, S_, true, false, false, true><<<(unsigned)blocks, threads, 0, s>>>(
          a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, LocalArgs{}, uw);
    else if (sa)
      k_hogwild<G4_, S_, true, false><<<(unsigned)blocks, threads, 0, s>>>(
          a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, LocalArgs{}, uw);
    else
      k_hogwild<G4_, S_, false, false><<<(unsigned)blocks, threads, 0, s>>>(
          a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err, LocalArgs{}, uw);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
