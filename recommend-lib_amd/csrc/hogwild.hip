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
//   - staleness is bounded by the launch's in-flight window: a wave takes `tpw` consecutive slots,
//     all waves of the grid start together, so a triplet may run beside any triplet up to
//     grid_waves * tpw slots away (DESIGN.md §5b gives the window per shape).
// Coherence: row and stamp stores are write-through (sc1) — the line leaves the XCD's L2 and is
// dropped there — so no XCD keeps a dirty or long-lived stale copy of a row another XCD updates;
// a reader sees another XCD's update at most one read-modify-write window late (MI355X_MICROARCH.md
// "stores of each flavour").
//
// Work layout: lane l of a wave samples slot base + l itself (the device sampler's spec,
// device_common.h: Philox + Feistel shuffle + k-th non-member; bit-exact to k_sample), so no
// triplet array makes a round trip through HBM; the wave then walks its tpw triplets G4 lanes per
// triplet (one float4 per lane and stripe), kUnroll * (64 / G4) triplets' rows in flight at once.
#include <stdlib.h>

#include "device_common.h"

#if defined(__HIP_DEVICE_COMPILE__) && !(defined(__gfx950__) || defined(__gfx942__))
#error "hogwild.hip targets gfx950 (sc1 write-through stores)"
#endif

namespace bprmf {

// 16-byte row load past this CU's L1: a non-temporal load (global_load_dwordx4 ... nt) is served
// by the XCD's L2 (MI355X_MICROARCH.md: sc1 / nt loads bypass L1 only), and the L2 drops every
// line the XCD stores sc1.  A plain load may hit a line this CU cached long ago: a hot row's, or
// its stamp's, and a stale stamp then decays the row again on every touch.  (A compiler builtin,
// so the loads stay visible to its wait counting.)
static __device__ __forceinline__ float4 hw_ld4(const float* p) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f x = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(x[0], x[1], x[2], x[3]);
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

// One triplet's slot -> (u, i, j): the sampler spec of k_sample (kernels.hip), lane-parallel.
static __device__ __forceinline__ void hw_sample(const SamplerArgs& a, uint32_t epoch, uint64_t slot,
                                                 int32_t& u, int32_t& i, int32_t& j, int32_t* err) {
  const uint64_t N = (uint64_t)a.npos * (uint64_t)a.num_ng;
  const uint64_t q = permute(slot, N, a.feistel_a, a.feistel_c, a.k0, a.k1, epoch);
  const int64_t p = div_small(q, (uint32_t)a.num_ng);
  u = a.pos_u[p];
  i = a.pos_i[p];
  const uint32_t d0 = bounded_draw0(q, epoch, a.k0, a.k1);
  const int64_t ul = u / a.world;
  const int64_t beg = a.indptr[ul], deg = a.indptr[ul + 1] - beg;
  const int64_t free_items = a.item_num - deg;
  j = -1;
  if (free_items > 0) {
    const uint32_t k = bounded_from(d0, q, epoch, (uint32_t)free_items, a.k0, a.k1);
    j = (int32_t)kth_nonmember(a.indices + beg, deg, (int64_t)k);
  } else {
    atomicOr(err, 2);
  }
}

constexpr int kHwUnroll = 4;  // rounds of (64 / G4) triplets whose rows are in flight together

// SAMPLE: slots come from the device sampler (a, epoch, slot0 + s); else replayed ids tu/ti/tj[s].
// SERIAL (tests): one lane group, one triplet at a time, in slot order (launched as one wave).
template <int G4, int S, bool SAMPLE, bool SERIAL>
__global__ __launch_bounds__(kBlock) void k_hogwild(SamplerArgs a, uint32_t epoch, int64_t slot0,
                                                    const int32_t* __restrict__ tu,
                                                    const int32_t* __restrict__ ti,
                                                    const int32_t* __restrict__ tj, int64_t n,
                                                    Table P, Table Q, Hyper hp, int ld, int32_t t0,
                                                    int B, int tpw, double* __restrict__ loss,
                                                    int32_t* __restrict__ err) {
  constexpr int GPW = SERIAL ? 1 : 64 / G4;  // triplets per wave per round
  constexpr int UNR = SERIAL ? 1 : kHwUnroll;
  const int lane = threadIdx.x & 63;
  const int sub = lane & (G4 - 1);
  const int gw = lane / G4;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
  const float lr = hp.lr, wd = hp.wd;
  float lacc = 0.f;
  for (int64_t base = wave * tpw; base < n; base += nwaves * tpw) {
    const int cnt = (int)min<int64_t>(tpw, n - base);
    int32_t mu = 0, mi = 0, mj = 0;
    if (lane < cnt) {
      const int64_t s = base + lane;
      if (SAMPLE) {
        hw_sample(a, epoch, (uint64_t)(slot0 + s), mu, mi, mj, err);
      } else {
        mu = tu[s];
        mi = ti[s];
        mj = tj[s];
      }
      // single-GPU handles only (world 1): ids are rows.  A sampler that found no negative
      // (j = -1) has raised err bit 2; any other bad id raises bit 1.  Either way: skipped.
      if (mu < 0 || mu >= P.rows || mi < 0 || mi >= Q.rows || mj < 0 || mj >= Q.rows) {
        if (mj >= 0 || !SAMPLE) atomicOr(err, 1);
        mu = -1;
      }
    }
    for (int k0 = 0; k0 < cnt; k0 += GPW * UNR) {
      float4 pu[UNR][S], vi[UNR][S], vj[UNR][S];
      int32_t su[UNR], si[UNR], sj[UNR], uu[UNR], ii[UNR], jj[UNR];
      bool ok[UNR];
      // every round's ids, rows and stamps requested before any is used
#pragma unroll
      for (int r = 0; r < UNR; ++r) {
        const int src = k0 + r * GPW + gw;
        uu[r] = __shfl(mu, src & 63);
        ii[r] = __shfl(mi, src & 63);
        jj[r] = __shfl(mj, src & 63);
        ok[r] = (SERIAL ? gw == 0 : true) && src < cnt && uu[r] >= 0;
        if (ok[r]) {
          const float* pr = P.W + (int64_t)uu[r] * ld + 4 * sub;
          const float* qi = Q.W + (int64_t)ii[r] * ld + 4 * sub;
          const float* qj = Q.W + (int64_t)jj[r] * ld + 4 * sub;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            pu[r][k] = hw_ld4(pr + 4 * G4 * k);
            vi[r][k] = hw_ld4(qi + 4 * G4 * k);
            vj[r][k] = hw_ld4(qj + 4 * G4 * k);
          }
          su[r] = hw_ld_word(P.stamp + uu[r]);
          si[r] = hw_ld_word(Q.stamp + ii[r]);
          sj[r] = hw_ld_word(Q.stamp + jj[r]);
        } else {
          su[r] = si[r] = sj[r] = 0;
#pragma unroll
          for (int k = 0; k < S; ++k) pu[r][k] = vi[r][k] = vj[r][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int r = 0; r < UNR; ++r) {
        const int src = k0 + r * GPW + gw;
        const int32_t t = t0 + 1 + (int32_t)((base + src) / B);
        // first touch of the row in step t: decay to t - 1 and take the wd term; else neither
        const bool fu1 = su[r] < t, fi1 = si[r] < t, fj1 = sj[r] < t;
        const float fu = fu1 ? decay_pow(hp.log2a, t - 1 - su[r]) : 1.f;
        const float fi = fi1 ? decay_pow(hp.log2a, t - 1 - si[r]) : 1.f;
        const float fj = fj1 ? decay_pow(hp.log2a, t - 1 - sj[r]) : 1.f;
        float di = 0.f, dj = 0.f;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          pu[r][k] = make_float4(pu[r][k].x * fu, pu[r][k].y * fu, pu[r][k].z * fu, pu[r][k].w * fu);
          vi[r][k] = make_float4(vi[r][k].x * fi, vi[r][k].y * fi, vi[r][k].z * fi, vi[r][k].w * fi);
          vj[r][k] = make_float4(vj[r][k].x * fj, vj[r][k].y * fj, vj[r][k].z * fj, vj[r][k].w * fj);
          di = hw_dot4(pu[r][k], vi[r][k], di);
          dj = hw_dot4(pu[r][k], vj[r][k], dj);
        }
        // the group's lanes are in one wave: the butterfly needs every lane of the wave, so it
        // runs whatever ok[] says (inactive groups carry zeros)
        di = group_sum<G4>(ok[r] ? di : 0.f);
        dj = group_sum<G4>(ok[r] ? dj : 0.f);
        if (!ok[r]) continue;
        const float x = di - dj;
        const float c = 1.0f / (1.0f + expf(x));  // sigmoid(-x) = -dL/dx
        if (sub == 0) lacc += softplus(-x);       // -log sigmoid(x)
        float* pr = P.W + (int64_t)uu[r] * ld + 4 * sub;
        float* qi = Q.W + (int64_t)ii[r] * ld + 4 * sub;
        float* qj = Q.W + (int64_t)jj[r] * ld + 4 * sub;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const float4 gu = make_float4(-c * (vi[r][k].x - vj[r][k].x), -c * (vi[r][k].y - vj[r][k].y),
                                        -c * (vi[r][k].z - vj[r][k].z), -c * (vi[r][k].w - vj[r][k].w));
          const float4 gi = make_float4(-c * pu[r][k].x, -c * pu[r][k].y, -c * pu[r][k].z, -c * pu[r][k].w);
          const float4 gj = make_float4(c * pu[r][k].x, c * pu[r][k].y, c * pu[r][k].z, c * pu[r][k].w);
          hw_st4(pr + 4 * G4 * k, hw_sgd(pu[r][k], gu, lr, fu1 ? wd : 0.f));
          hw_st4(qi + 4 * G4 * k, hw_sgd(vi[r][k], gi, lr, fi1 ? wd : 0.f));
          hw_st4(qj + 4 * G4 * k, hw_sgd(vj[r][k], gj, lr, fj1 ? wd : 0.f));
        }
        if (sub == 0) {
          if (fu1) hw_st_word(P.stamp + uu[r], t);
          if (fi1) hw_st_word(Q.stamp + ii[r], t);
          if (fj1) hw_st_word(Q.stamp + jj[r], t);
        }
        if (SERIAL) {  // the next triplet reads these rows: stores done, this CU's L1 dropped
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
      }
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

static bool hw_serial() {
  const char* e = getenv("BPRMF_HOGWILD_SERIAL");
  return e && e[0] == '1';
}

// triplets per wave: enough waves to fill the chip for short chunks (>= ~2048 waves), 64 (one per
// lane) for long ones; BPRMF_HOGWILD_TPW overrides (A/B)
static int hw_tpw(int64_t n) {
  if (const char* e = getenv("BPRMF_HOGWILD_TPW")) {
    const int v = atoi(e);
    if (v == 8 || v == 16 || v == 32 || v == 64) return v;
  }
  if (n >= 64LL * 4096) return 64;
  if (n >= 32LL * 2048) return 32;
  return 16;
}

hipError_t hogwild(const Geom& g, const SamplerArgs* sa, uint32_t epoch, int64_t slot0,
                   const int32_t* tu, const int32_t* ti, const int32_t* tj, int64_t n, Table P,
                   Table Q, const Hyper& hp, int32_t t0, int B, double* loss, int32_t* err,
                   hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const bool serial = hw_serial();
  const int tpw = serial ? 64 : hw_tpw(n);
  const int64_t waves = (n + tpw - 1) / tpw;
  const int wpb = kBlock / 64;
  int64_t blocks = serial ? 1 : (waves + wpb - 1) / wpb;
  if (blocks > kMaxGridBlocks) blocks = kMaxGridBlocks;  // grid-stride beyond
  if (const char* e = getenv("BPRMF_HOGWILD_BLOCKS")) {  // A/B: cap the grid (smaller window)
    const int64_t cap = atoll(e);
    if (cap > 0 && blocks > cap) blocks = cap;
  }
  const unsigned threads = serial ? 64 : kBlock;
  SamplerArgs a{};
  if (sa) a = *sa;
  BPRMF_DISPATCH4(g, ({
    if (serial && sa)
      k_hogwild<G4_, S_, true, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q, hp,
                                                          g.ld, t0, B, tpw, loss, err);
    else if (serial)
      k_hogwild<G4_, S_, false, true><<<1, threads, 0, s>>>(a, epoch, slot0, tu, ti, tj, n, P, Q, hp,
                                                           g.ld, t0, B, tpw, loss, err);
    else if (sa)
      k_hogwild<G4_, S_, true, false><<<(unsigned)blocks, threads, 0, s>>>(
          a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err);
    else
      k_hogwild<G4_, S_, false, false><<<(unsigned)blocks, threads, 0, s>>>(
          a, epoch, slot0, tu, ti, tj, n, P, Q, hp, g.ld, t0, B, tpw, loss, err);
  }));
  return hipGetLastError();
}

}  // namespace bprmf
