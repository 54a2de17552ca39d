// segment.hip — batch builder of the segmented (atomic-free, deterministic) BPR-MF step.
//
// k_build_batches: one 1024-thread workgroup per batch of B <= kMaxSegBatch triplets, run once per
// chunk of steps at full-chip parallelism (off the per-step critical path):
//   1. the batch's triplets: the device sampler (bit-identical to k_sample: Feistel shuffle of the
//      epoch, negative = k-th non-positive item; util/data_loader.py:680-690 semantics) or
//      replayed ids;
//   2. sort by (local) user row in LDS (rocPRIM block radix sort) -> user segments;
//   3. sort the 2B item references (i: -, j: +) by item key = (owner, owner's row) -> item
//      segments, their references in a fixed order, hot-item records, per-owner counts;
//   4. 32-byte segment records so each step kernel needs ONE dependent load before its gathers.
// Layout: kernels.h (BatchBuf).  Step kernels: step.hip.
#include <stdlib.h>
#include <string.h>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>
#include <atomic>
#include <type_traits>

#include "device_common.h"

BPRMF_CALL_STAMPS_DEF(seg)

namespace bprmf {

constexpr int kBuildThreads = 1024;

// diagnostic build only (-DBPRMF_BUILD_STAMPS, tools/ubench_build.py): s_memrealtime at the
// builder's phase boundaries, first workgroup, first thread
#ifdef BPRMF_BUILD_STAMPS
__device__ uint64_t g_build_stamps[32];
#define BSTAMP(k)                                                                          \
  do {                                                                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_build_stamps[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define BSTAMP(k) \
  do {            \
  } while (0)
#endif
constexpr uint32_t kNone = 0xFFFFFFFFu;

static __device__ __forceinline__ void store_rec(int32_t* rec, int a, int b, int c, int d, int e,
                                                 int f, int g, int h) {
  reinterpret_cast<int4*>(rec)[0] = make_int4(a, b, c, d);
  reinterpret_cast<int4*>(rec)[1] = make_int4(e, f, g, h);
}

// ------------------------------------------------------------------------------------------------
// Bucket sort of a workgroup's (key, value) pairs in blocked arrangement (thread t holds input
// positions t*E .. t*E+E-1), replacing rocPRIM's radix passes for B <= 4096.  The result equals a
// stable sort by key (ties by input position) — the arrangement the radix sort gives, bit for bit
// — in four LDS phases instead of ceil(bits/4) radix passes:
//   1. count per bucket, bucket = key >> (bits - 12): MONOTONE in the key (4096 buckets);
//   2. exclusive scan of the counts -> bucket starts;
//   3. scatter (key << 32 | position) into the bucket's range (order inside a bucket arbitrary);
//   4. each element's rank inside its bucket = #{smaller (key, position)} -> its sorted slot.
// Phase 4 costs sum(c^2) over buckets: a batch's keys spread over ~4096 buckets (1-2 per bucket)
// except a hot item's references (<= ~80 at ml-20m shape), which share one bucket; the lanes of a
// wave scan the same bucket, so those reads are LDS broadcasts.  Invalid keys (kNone) take the
// positions after every valid key, in any order (their values are never read).
// ------------------------------------------------------------------------------------------------
constexpr int kBucketBits = 12;
constexpr int kBuckets = 1 << kBucketBits;

template <int T>
struct BucketScratch {
  uint64_t* bk;     // [n] (key << 32 | input position), bucket order
  int32_t* srt;     // [n] input position at each sorted position
  int32_t* start;   // [kBuckets + 1] bucket starts (start[kBuckets] = valid count)
  int32_t* ninv;    // invalid-key counter
  typename rocprim::block_scan<int, T>::storage_type* scan;
};

template <int T, int E, class KeyOf, class ValOf>
static __device__ __forceinline__ int bucket_sort(uint32_t (&key)[E], uint32_t (&val)[E], int bits,
                                                   const BucketScratch<T>& sc, KeyOf key_of,
                                                   ValOf val_of, int sb = -1) {
  // sb >= 0 (diagnostic build): stamps sb .. sb+4 after count, scan, scatter, rank, gather
#ifdef BPRMF_BUILD_STAMPS
#define BSTAMP_SORT(k) \
  do {                 \
    if (sb >= 0) BSTAMP(sb + (k)); \
  } while (0)
#else
#define BSTAMP_SORT(k) \
  do {                 \
  } while (0)
#endif
  using Scan = rocprim::block_scan<int, T>;
  static_assert(kBuckets % T == 0, "buckets per thread");
  constexpr int PB = kBuckets / T;
  const int tid = threadIdx.x;
  const int shift = bits > kBucketBits ? bits - kBucketBits : 0;
  for (int b = tid; b <= kBuckets; b += T) sc.start[b] = 0;
  if (tid == 0) *sc.ninv = 0;
  __syncthreads();
  int li[E];
#pragma unroll
  for (int k = 0; k < E; ++k)
    li[k] = key[k] != kNone ? atomicAdd(&sc.start[key[k] >> shift], 1) : -1;
  __syncthreads();
  BSTAMP_SORT(0);
  int c[PB], sum = 0;
#pragma unroll
  for (int m = 0; m < PB; ++m) {
    c[m] = sc.start[tid * PB + m];
    sum += c[m];
  }
  int pre = 0, total = 0;
  Scan().exclusive_scan(sum, pre, 0, total, *sc.scan, rocprim::plus<int>());
#pragma unroll
  for (int m = 0; m < PB; ++m) {
    sc.start[tid * PB + m] = pre;
    pre += c[m];
  }
  if (tid == 0) sc.start[kBuckets] = total;
  __syncthreads();
  BSTAMP_SORT(1);
#pragma unroll
  for (int k = 0; k < E; ++k) {
    const int q = tid * E + k;
    if (li[k] >= 0)
      sc.bk[sc.start[key[k] >> shift] + li[k]] = ((uint64_t)key[k] << 32) | (uint32_t)q;
    else
      sc.srt[total + atomicAdd(sc.ninv, 1)] = q;
  }
  __syncthreads();
  BSTAMP_SORT(2);
  // every element's loads issued together (E chains in flight, not one after the other): its
  // entry, its bucket's bounds, then the bucket's first two entries (nearly every bucket holds
  // at most two); only the lanes of a larger bucket loop over the rest
  {
    uint64_t me[E];
    int bs[E], be[E];
#pragma unroll
    for (int k = 0; k < E; ++k) me[k] = tid + k * T < total ? sc.bk[tid + k * T] : ~0ull;
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int b = min((int)((uint32_t)(me[k] >> 32) >> shift), kBuckets - 1);
      bs[k] = sc.start[b];
      be[k] = sc.start[b + 1];
    }
    int rank[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int last = max(total - 1, 0);
      const uint64_t a0 = sc.bk[min(bs[k], last)], a1 = sc.bk[min(bs[k] + 1, last)];
      rank[k] = (int)(be[k] > bs[k] && a0 < me[k]) + (int)(be[k] > bs[k] + 1 && a1 < me[k]);
    }
#pragma unroll
    for (int k = 0; k < E; ++k) {
      if (tid + k * T >= total) continue;
      int y = bs[k] + 2;
      for (; y + 4 <= be[k]; y += 4) {  // four reads in flight (a hot item's bucket holds ~60)
        const uint64_t a0 = sc.bk[y], a1 = sc.bk[y + 1], a2 = sc.bk[y + 2], a3 = sc.bk[y + 3];
        rank[k] += (int)(a0 < me[k]) + (int)(a1 < me[k]) + (int)(a2 < me[k]) + (int)(a3 < me[k]);
      }
      for (; y < be[k]; ++y) rank[k] += sc.bk[y] < me[k];
      sc.srt[bs[k] + rank[k]] = (int32_t)(uint32_t)me[k];
    }
  }
  __syncthreads();
  BSTAMP_SORT(3);
#pragma unroll
  for (int k = 0; k < E; ++k) {
    const int pos = tid * E + k;
    const int q = sc.srt[pos];
    if (pos < total) {
      key[k] = key_of(q);
      val[k] = val_of(q);
    } else {
      key[k] = kNone;
      val[k] = 0;
    }
  }
  __syncthreads();  // the caller reuses the scratch (its sorted keys alias bk)
  BSTAMP_SORT(4);
#undef BSTAMP_SORT
  return total;
}

// BUCKET: bucket sorts (B <= kBuildThreads * 4); else rocPRIM block radix sorts.  Both give the
// same arrangement, so the batches (and every step result) are identical either way.
// W1: one rank (world 1, item rows, no slots), so every owner / local-row division folds away
template <int IPT, bool BUCKET, bool W1>
__global__ __launch_bounds__(kBuildThreads) void k_build_batches(
    SamplerArgs a, uint32_t epoch, int64_t first_slot, int64_t n_slots, int B,
    const int32_t* __restrict__ ru, const int32_t* __restrict__ ri, const int32_t* __restrict__ rj,
    int64_t u_rows, int64_t i_rows, int world_in, int64_t iloc, int slots_in, int slot_stride,
    int user_bits, int item_bits, int tpb, int k1_items, BatchBuf bb, int32_t* __restrict__ err,
    CursorInit ci) {
  const int world = W1 ? 1 : world_in;
  const int slots = W1 ? 0 : slots_in;
  constexpr int T = kBuildThreads;
  constexpr int IPT2 = 2 * IPT;
  using SortU = rocprim::block_radix_sort<uint32_t, T, IPT, uint32_t>;
  using SortI = rocprim::block_radix_sort<uint32_t, T, IPT2, uint32_t>;
  using Scan = rocprim::block_scan<int, T>;
  using ScanL = rocprim::block_scan<uint64_t, T>;
  union RadixSmem {  // the sorted keys alias the sort storage (barrier after every sort)
    typename SortU::storage_type su;
    typename SortI::storage_type si;
    uint32_t key[T * IPT2];
  };
  // bucket layout: bk u64[T*IPT2] (sorted keys alias it; user keys by slot sit in its upper half
  // during the user sort), srt i32[T*IPT2], start i32[kBuckets + 1]
  constexpr size_t kBucketBytes = 12 * (size_t)T * IPT2 + 4 * (kBuckets + 4);
  constexpr size_t kSortBytes = BUCKET ? kBucketBytes : sizeof(RadixSmem);
  __shared__ __attribute__((aligned(16))) unsigned char s_sort[kSortBytes];
  __shared__ typename Scan::storage_type sscan;
  __shared__ typename ScanL::storage_type sscan64;
  __shared__ int32_t s_i[T * IPT];  // per sorted position: item row (world 1) or item slot
  __shared__ int32_t s_j[T * IPT];
  __shared__ int s_own[kMaxWorld];
  __shared__ int s_opre[kMaxWorld];  // first item segment of each owner (padded slots)
  __shared__ int32_t s_ninv;
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_sort);
  uint32_t* s_u = reinterpret_cast<uint32_t*>(s_sort) + 2 * T * IPT;  // bucket mode, user sort
  // bucket mode, after the item sort: LDS copies of refs and of the item segment starts, so the
  // record phases read LDS instead of their own global stores back (s_key keeps bk's first half)
  int32_t* s_refs = reinterpret_cast<int32_t*>(s_sort) + T * IPT2;
  int32_t* s_ioff = reinterpret_cast<int32_t*>(s_sort + 8 * (size_t)T * IPT2);  // srt, start
  BucketScratch<T> bs;
  bs.bk = reinterpret_cast<uint64_t*>(s_sort);
  bs.srt = reinterpret_cast<int32_t*>(s_sort + 8 * (size_t)T * IPT2);
  bs.start = reinterpret_cast<int32_t*>(s_sort + 12 * (size_t)T * IPT2);
  bs.ninv = &s_ninv;
  bs.scan = &sscan;
  const int tid = threadIdx.x;
  const int64_t batch = blockIdx.x;
  const int64_t b0 = batch * (int64_t)B;
  const int nb = (int)max<int64_t>(0, min<int64_t>(B, n_slots - b0));
  const uint64_t N = (uint64_t)a.npos * (uint64_t)a.num_ng;
  const BatchView v = bb.view(batch);
  if (tid < kMaxWorld) s_opre[tid] = -1;  // sharded: first item segment of each owner, if any
  if (batch == 0 && ci.cursor) {  // set_cursor's work (kernels.hip k_set_cursor)
    if (tid == 0) {
      ci.cursor[0] = ci.t;
      ci.cursor[1] = ci.k;
    }
    if (ci.loss && tid < ci.nloss) ci.loss[tid] = 0.0;
  }
  BSTAMP(0);

  // 1. the batch's triplets in slot order, keyed by local user row
  uint32_t key[IPT], val[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int p = tid * IPT + k;
    key[k] = kNone;
    val[k] = (uint32_t)p;
    if (p < nb && !(ru && ru[b0 + p] < 0)) {  // replay: u < 0 is an empty slot
      int32_t u, i, j;
      bool sampled_ok = true;
      if (ru) {
        u = ru[b0 + p] / world;
        i = ri[b0 + p];
        j = rj[b0 + p];
      } else {
        const uint64_t q = permute((uint64_t)(first_slot + b0 + p), N, a.feistel_a, a.feistel_c, a.k0, a.k1, epoch);
        const int64_t pp = div_small(q, (uint32_t)a.num_ng);
        const int64_t ul = a.pos_u[pp] / (W1 ? 1 : a.world);
        i = a.pos_i[pp];
        const uint32_t d0 = bounded_draw0(q, epoch, a.k0, a.k1);  // while the loads are in flight
        const int64_t beg = a.indptr[ul], deg = a.indptr[ul + 1] - beg;
        const int64_t nfree = a.item_num - deg;
        j = -1;
        if (nfree > 0) {
          const uint32_t kk = bounded_from(d0, q, epoch, (uint32_t)nfree, a.k0, a.k1);
          j = (int32_t)kth_nonmember(a.indices + beg, deg, (int64_t)kk);
        } else {
          sampled_ok = false;
        }
        u = (int32_t)ul;
      }
      if ((uint64_t)u < (uint64_t)u_rows && (uint64_t)i < (uint64_t)i_rows &&
          (uint64_t)j < (uint64_t)i_rows) {
        key[k] = (uint32_t)u;
        if (BUCKET) s_u[p] = (uint32_t)u;
        s_i[p] = i;
        s_j[p] = j;
      } else {
        atomicOr(err, sampled_ok ? 1 : 2);
      }
    }
  }
  BSTAMP(1);
  if constexpr (BUCKET) {
    bucket_sort<T, IPT>(key, val, user_bits, bs, [&](int q) { return s_u[q]; },
                        [](int q) { return (uint32_t)q; }, 16);
  } else {
    SortU().sort(key, val, reinterpret_cast<RadixSmem*>(s_sort)->su, 0, user_bits);
    __syncthreads();
  }
  BSTAMP(2);
  // blocked arrangement: sorted position p = tid*IPT + k holds key[k] (user) and val[k] (slot)
  int32_t my_i[IPT], my_j[IPT];
  int valid = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const bool ok = key[k] != kNone;
    valid += ok;
    my_i[k] = ok ? s_i[val[k]] : 0;
    my_j[k] = ok ? s_j[val[k]] : 0;
    s_key[tid * IPT + k] = key[k];
  }
  __syncthreads();  // slot-order reads of s_i/s_j done; s_key complete
  // segment heads from the neighbouring key: in this thread's registers but for its first position
  const uint32_t uprev = tid ? s_key[tid * IPT - 1] : kNone;
  bool uhead[IPT];
  int heads = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int p = tid * IPT + k;
    s_i[p] = my_i[k];  // sorted order from here on
    s_j[p] = my_j[k];
    uhead[k] = key[k] != kNone && (k ? key[k - 1] : uprev) != key[k];
    heads += uhead[k];
  }
  // one scan for both counts: segment heads in the high half, valid triplets in the low
  int pre = 0, tot = 0;
  Scan().exclusive_scan((heads << 16) | valid, pre, 0, tot, sscan, rocprim::plus<int>());
  const int seg0 = pre >> 16, n_useg = tot >> 16, nvalid = tot & 0xFFFF;
  // segment starts in LDS (the upper half of the sort scratch, free after the user sort), so each
  // position finds its segment's bounds with two reads instead of scanning its neighbours
  int32_t* s_seg = reinterpret_cast<int32_t*>(s_sort) + T * IPT;
  {
    int s = seg0;
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (uhead[k]) s_seg[s++] = tid * IPT + k;
  }
  __syncthreads();
  int uend[IPT];  // a head's segment end
  // trec.w: 1 = the user's only triplet; >= 2 = head of a segment of that length that lies in one
  // K1 workgroup (tpb consecutive positions: K1 sums it in LDS and updates the user); -1 = another
  // member of such a segment; 0 = a segment across workgroups (K2 sums its ugrad rows, mrec)
  int uw[IPT];
  {
    int s = seg0 - 1;  // segment of this thread's first position if that is not a head
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int p = tid * IPT + k;
      uend[k] = p + 1;
      uw[k] = 0;
      if (key[k] != kNone) {
        if (uhead[k]) ++s;
        const int b = s_seg[max(s, 0)], e = s + 1 < n_useg ? s_seg[s + 1] : nvalid;
        uend[k] = e;
        const int len = e - b;
        if (len == 1)
          uw[k] = 1;
        else if (b / tpb == (e - 1) / tpb)
          uw[k] = p == b ? len : -1;
      }
    }
  }
  __syncthreads();  // useg visible block-wide; s_i/s_j sorted; s_key free for the item keys
  BSTAMP(3);

  // 2. item references: r < nvalid -> i of sorted triplet r (sign -), else j of r - nvalid (sign +)
  uint32_t ik[IPT2], iv[IPT2];
#pragma unroll
  for (int k = 0; k < IPT2; ++k) {
    const int r = tid * IPT2 + k;
    ik[k] = kNone;
    iv[k] = 0;
    if (r < 2 * nvalid) {
      const int p = r < nvalid ? r : r - nvalid;
      const uint32_t item = (uint32_t)(r < nvalid ? s_i[p] : s_j[p]);
      ik[k] = (uint32_t)(item % (uint32_t)world) * (uint32_t)iloc + item / (uint32_t)world;
      iv[k] = ((uint32_t)p << 1) | (r < nvalid ? 0u : 1u);
    }
  }
  if constexpr (BUCKET) {
    const int nv = nvalid;
    bucket_sort<T, IPT2>(
        ik, iv, item_bits, bs,
        [&](int r) {
          const uint32_t item = (uint32_t)(r < nv ? s_i[r] : s_j[r - nv]);
          return (item % (uint32_t)world) * (uint32_t)iloc + item / (uint32_t)world;
        },
        [&](int r) { return r < nv ? ((uint32_t)r << 1) : (((uint32_t)(r - nv) << 1) | 1u); }, 9);
  } else {
    SortI().sort(ik, iv, reinterpret_cast<RadixSmem*>(s_sort)->si, 0, item_bits);
    __syncthreads();  // also: every read of s_i/s_j above is done
  }
  BSTAMP(4);
#pragma unroll
  for (int k = 0; k < IPT2; ++k) s_key[tid * IPT2 + k] = ik[k];
  __syncthreads();
  // k1_items (single GPU): an item with ONE reference in the batch is updated by K1 from that
  // triplet (its gradient is that one term; the same arithmetic K2 would do): no contribution row,
  // no K2 record.  Item segments K2 serves are the others, numbered compactly (`mseg`).
  // Per reference: head (first of its item), sole (only one), long (more than kLongSeg: position
  // r + kLongSeg still holds the key), from the neighbouring keys (registers but at this thread's
  // ends).  Invalid keys (kNone) sit after every valid one, so an item's last reference is
  // followed by a different key.
  const int nref = 2 * nvalid;
  const uint32_t iprev = tid ? s_key[tid * IPT2 - 1] : kNone;
  const uint32_t inext = tid + 1 < T ? s_key[(tid + 1) * IPT2] : kNone;
  uint32_t hm = 0, sm = 0, lm = 0;  // bit k: reference k of this thread is a head / sole / long
  int iheads = 0, mheads = 0, nlong = 0;
#pragma unroll
  for (int k = 0; k < IPT2; ++k) {
    const int r = tid * IPT2 + k;
    if (ik[k] == kNone) continue;
    const bool h = (k ? ik[k - 1] : iprev) != ik[k];
    const bool so = k1_items && h && (k + 1 < IPT2 ? ik[k + 1] : inext) != ik[k];
    const bool lg = h && !so && r + kLongSeg < T * IPT2 && s_key[r + kLongSeg] == ik[k];
    hm |= (uint32_t)h << k;
    sm |= (uint32_t)so << k;
    lm |= (uint32_t)lg << k;
    iheads += h;
    mheads += h && !so;
    nlong += lg;
    v.refs[r] = (int32_t)iv[k];
    if (BUCKET) s_refs[r] = (int32_t)iv[k];
  }
  // ONE scan for four counts (each <= 2B <= 16384, 16 bits apiece): item segments, K2-served item
  // segments, long item segments, and the user segments K2 finishes (w = 0 heads)
  int nmulti = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) nmulti += uhead[k] && uw[k] == 0;
  uint64_t cpre = 0, ctot = 0;
  ScanL().exclusive_scan((uint64_t)iheads | (uint64_t)mheads << 16 | (uint64_t)nlong << 32 |
                             (uint64_t)nmulti << 48,
                         cpre, 0ull, ctot, sscan64, rocprim::plus<uint64_t>());
  auto field = [](uint64_t x, int f) { return (int)((x >> (16 * f)) & 0xFFFF); };
  const int iseg0 = field(cpre, 0), n_iseg = field(ctot, 0);
  const int mseg0 = field(cpre, 1), n_mseg = field(ctot, 1);
  const int n_long = field(ctot, 2), n_multi = field(ctot, 3);
  int lpre = field(cpre, 2), mpre = field(cpre, 3);
  {
    int s = iseg0 - 1;  // segment of this thread's first ref if it is not a head
#pragma unroll
    for (int k = 0; k < IPT2; ++k) {
      const int r = tid * IPT2 + k;
      if (ik[k] == kNone) continue;
      const bool head = (hm >> k) & 1;
      const bool sole = (sm >> k) & 1;
      if (head) {
        ++s;
        if (BUCKET)
          s_ioff[s] = r;
        else
          v.ioff[s] = r;  // radix build: the segment starts go through global memory
        if (slots) {
          // segments are owner-major: an owner's first segment is the head whose previous
          // reference has another owner (no per-head atomics on a few shared counters)
          const uint32_t o = ik[k] / (uint32_t)iloc;
          const uint32_t pk = k ? ik[k - 1] : iprev;
          v.ukey[s] = (int32_t)(ik[k] % (uint32_t)iloc);
          if (pk == kNone || pk / (uint32_t)iloc != o) s_opre[o] = s;
        }
      }
      // triplet side -> its item slot (sharded); bit 31: this reference is its item's first in
      // the batch (K1 marks the item for the next step's fused K1 from that triplet only: one
      // mark per distinct item instead of one per reference on hot addresses); bit 30: it is the
      // item's only reference (K1 updates the item).  Each (triplet, side) belongs to exactly one
      // reference, so the writes need no atomics.
      int32_t& side = (iv[k] & 1 ? s_j : s_i)[iv[k] >> 1];
      if (slots)
        side = s | (head ? (int32_t)0x80000000 : 0);
      else if (head)
        side |= (int32_t)0x80000000 | (sole ? (int32_t)0x40000000 : 0);
    }
  }
  if (tid == 0) (BUCKET ? s_ioff : v.ioff)[n_iseg] = 2 * nvalid;
  auto ioff_at = [&](int seg) { return BUCKET ? s_ioff[seg] : v.ioff[seg]; };
  auto ref_at = [&](int r) { return BUCKET ? s_refs[r] : v.refs[r]; };
  __syncthreads();  // ioff, refs, slots, s_own visible block-wide
  BSTAMP(5);
  if (slots) {
    if (tid == 0) {  // owners without segments start where the next one does; counts by difference
      int next = n_iseg;
      for (int o = world - 1; o >= 0; --o) {
        if (s_opre[o] < 0) s_opre[o] = next;
        s_own[o] = next - s_opre[o];
        next = s_opre[o];
      }
    }
    __syncthreads();
  }
  // slot of item segment s as the step kernels address it: the segment index (compact), or
  // owner * slot_stride + index within the owner's range (padded: the exchange buffers of the
  // sharded runner hold slot_stride rows per owner)
  auto slot_of = [&](int s) -> int {
    if (!slot_stride) return s;
    int lo = 0, hi = world - 1;  // largest owner o with s_opre[o] <= s
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_opre[mid] <= s) lo = mid; else hi = mid - 1;
    }
    return lo * slot_stride + (s - s_opre[lo]);
  };
  BSTAMP(6);
  // item records of the K2-served segments, and the long ones' copies (the first kMaxLongItems;
  // past the cap a long segment's record drops its long bit and K2 takes the short path)
  {
    int s = iseg0, ms = mseg0;  // segment index, K2 record index
#pragma unroll
    for (int k = 0; k < IPT2; ++k) {
      const int r = tid * IPT2 + k;
      if (!((hm >> k) & 1)) continue;
      if ((sm >> k) & 1) {  // K1's: no record
        ++s;
        continue;
      }
      const int end = ioff_at(s + 1);
      const int len = end - r;
      const int lng = ((lm >> k) & 1) && lpre < kMaxLongItems;
      int pk[kInlineRefs / 2];
#pragma unroll
      for (int m = 0; m < kInlineRefs / 2; ++m) {
        const int a = ref_at(min(r + 2 * m, nref - 1)), b = ref_at(min(r + 2 * m + 1, nref - 1));
        pk[m] = (2 * m < len ? a : 0) | ((2 * m + 1 < len ? b : 0) << 16);
      }
      store_rec(v.irec + (int64_t)ms * kRec, slots ? slot_of(s) : (int)ik[k],
                r | (len << 15) | (lng << 30), pk[0], pk[1], pk[2], pk[3], pk[4], pk[5]);
      if (lng) store_rec(v.lrec + (int64_t)lpre * kRec, (int)ik[k], r, end, slot_of(s), 0, 0, 0, 1);
      lpre += (lm >> k) & 1;
      ++s;
      ++ms;
    }
  }
  BSTAMP(7);

  // 3. triplet records, now that s_i/s_j hold the final item rows (world 1) or slots, and the
  //    records of user segments with more than one triplet (K2 finishes those users)
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int p = tid * IPT + k;
    if (key[k] == kNone) continue;
    const int32_t hi = s_i[p] & (int32_t)0x80000000, hj = s_j[p] & (int32_t)0x80000000;
    const int ri_ = slots ? (slot_of(s_i[p] & 0x7FFFFFFF) | hi) : s_i[p];
    const int rj_ = slots ? (slot_of(s_j[p] & 0x7FFFFFFF) | hj) : s_j[p];
    reinterpret_cast<int4*>(v.trec)[p] = make_int4(ri_, rj_, (int)key[k], uw[k]);
    if (uhead[k] && uw[k] == 0) {  // a segment K2 finishes
      store_rec(v.mrec + (int64_t)mpre * kRec, (int)key[k], p, uend[k], 0, 0, 0, 0, 0);
      ++mpre;
    }
  }
  if (tid < world && slots) v.own[tid] = s_own[tid];
  if (tid == 0) {
    v.meta[0] = nvalid;
    v.meta[1] = n_useg;
    v.meta[2] = n_mseg;  // item segments K2 serves (= all of them unless k1_items)
    v.meta[3] = min(n_long, kMaxLongItems);
    v.meta[4] = n_multi;
  }
  BSTAMP(8);
}

// ================================================================================================
// Split builder: one rank (item rows, no slots), triplets already in memory (the grid-wide
// sampler's or replayed ids), B <= kBuildThreads * 4.  The single-workgroup builder above spends
// most of its ~32 us on the 2B item references of a batch (sort, segment heads, records) while 255
// other CUs idle.  Here each batch gets 1 + kItemParts workgroups:
//   role 0      the user side: user sort, user segments, trec {u, w} words, mrec, meta[0,1,4];
//   role 1 + q  the item references whose item lies in key range q (kItemParts equal ranges of
//               the item id space): their sort, segment heads, trec {i, j} words (item | first /
//               sole bits), refs, item and long-item records.
// Every workgroup sorts the batch's triplets by user itself (a reference's value and its place in
// the fixed summation order are the triplet's position in user order), so no workgroup waits for
// another's sort.  Item segments, K2 records and long records are numbered across the parts in key
// order, as the one-workgroup build numbers them: part q publishes its three counts (tagged with
// the launch's tag) and waits for parts 0 .. q-1's before it writes records.  The batch buffer
// comes out identical to k_build_batches's, bit for bit (refs, records, trec, meta).
// ================================================================================================
#ifndef BPRMF_ITEM_PARTS
#define BPRMF_ITEM_PARTS 8
#endif
constexpr int kItemParts = BPRMF_ITEM_PARTS;  // 2, 4 or 8 (8: 20-step calls 11.42-11.51 us/step, 4: 11.62-11.66, 2: 11.80-11.92) (-DBPRMF_ITEM_PARTS: A/B builds)
constexpr int kItemPartBits = kItemParts == 8 ? 3 : kItemParts == 4 ? 2 : 1;
static_assert(kItemParts == 1 << kItemPartBits, "item parts: a power of two <= 8");
// sorted references per thread while a part holds at most that many per thread (a part averages
// 2B / kItemParts of the batch's references), else 8
constexpr int kPartE2 = kItemParts >= 8 ? 2 : kItemParts == 4 ? 4 : 8;

// bucket_sort over the VALID elements (key != kNone) of a blocked E-per-thread input whose keys lie
// in [lo, lo + 2^bits): the same order (stable by key, ties by input position), but absent
// elements take no part (no count, no rank), and the sorted elements come out in a blocked
// E2-per-thread arrangement (positions past the count: kNone).  The caller guarantees
// count <= T * E2.  Returns the count.
// tie != nullptr: element k of this thread sorts by (key[k], tie[k]) (ties unique) instead of
// (key, input position), and key_of / val_of receive the tie as the element's identity.  The split
// builder's item parts sort their references in slot order this way with tie = (side, user, slot):
// the order of k_build_batches's references (i before j, then user order, stable by slot) without
// sorting the batch by user first.
template <int T, int E, int E2, class KeyOf, class ValOf>
static __device__ __forceinline__ int bucket_sort_sparse(const uint32_t (&key)[E], uint32_t lo,
                                                         int bits, const BucketScratch<T>& sc,
                                                         KeyOf key_of, ValOf val_of,
                                                         uint32_t (&okey)[E2], uint32_t (&oval)[E2],
                                                         const uint32_t* tie = nullptr) {
  using Scan = rocprim::block_scan<int, T>;
  constexpr int PB = kBuckets / T;
  const int tid = threadIdx.x;
  const int shift = bits > kBucketBits ? bits - kBucketBits : 0;
  for (int b = tid; b <= kBuckets; b += T) sc.start[b] = 0;
  __syncthreads();
  int li[E];
#pragma unroll
  for (int k = 0; k < E; ++k)
    li[k] = key[k] != kNone ? atomicAdd(&sc.start[(key[k] - lo) >> shift], 1) : -1;
  __syncthreads();
  int c[PB], sum = 0;
#pragma unroll
  for (int m = 0; m < PB; ++m) {
    c[m] = sc.start[tid * PB + m];
    sum += c[m];
  }
  int pre = 0, total = 0;
  Scan().exclusive_scan(sum, pre, 0, total, *sc.scan, rocprim::plus<int>());
#pragma unroll
  for (int m = 0; m < PB; ++m) {
    sc.start[tid * PB + m] = pre;
    pre += c[m];
  }
  if (tid == 0) sc.start[kBuckets] = total;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < E; ++k)
    if (li[k] >= 0)
      sc.bk[sc.start[(key[k] - lo) >> shift] + li[k]] =
          ((uint64_t)key[k] << 32) | (tie ? tie[k] : (uint32_t)(tid * E + k));
  __syncthreads();
  // rank inside the bucket (bucket_sort's phase 4), over the count's elements only
  constexpr int R = (E2 * T + T - 1) / T;  // elements per thread in the strided rank pass
  {
    uint64_t me[R];
    int bs[R], be[R];
#pragma unroll
    for (int k = 0; k < R; ++k) me[k] = tid + k * T < total ? sc.bk[tid + k * T] : ~0ull;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int b = min((int)(((uint32_t)(me[k] >> 32) - lo) >> shift), kBuckets - 1);
      bs[k] = sc.start[b];
      be[k] = sc.start[b + 1];
    }
    int rank[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int last = max(total - 1, 0);
      const uint64_t a0 = sc.bk[min(bs[k], last)], a1 = sc.bk[min(bs[k] + 1, last)];
      rank[k] = (int)(be[k] > bs[k] && a0 < me[k]) + (int)(be[k] > bs[k] + 1 && a1 < me[k]);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (tid + k * T >= total) continue;
      int y = bs[k] + 2;
      for (; y + 4 <= be[k]; y += 4) {
        const uint64_t a0 = sc.bk[y], a1 = sc.bk[y + 1], a2 = sc.bk[y + 2], a3 = sc.bk[y + 3];
        rank[k] += (int)(a0 < me[k]) + (int)(a1 < me[k]) + (int)(a2 < me[k]) + (int)(a3 < me[k]);
      }
      for (; y < be[k]; ++y) rank[k] += sc.bk[y] < me[k];
      sc.srt[bs[k] + rank[k]] = (int32_t)(uint32_t)me[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < E2; ++k) {
    const int pos = tid * E2 + k;
    if (pos < total) {
      const int q = sc.srt[pos];
      okey[k] = key_of(q);
      oval[k] = val_of(q);
    } else {
      okey[k] = kNone;
      oval[k] = 0;
    }
  }
  __syncthreads();
  return total;
}

// The parts' counts for the batch, in 64-bit words {tag, payload} (one store each, write-through),
// kXchWords per part: [0] tag << 32 | n_iseg | n_mseg << 16, [1] tag << 32 | n_long, and sharded
// [2 + o / 2] tag << 32 | cnt[o] | cnt[o + 1] << 16 with cnt[o] = the part's segments of owners
// below o.  The area is the batch's ioff range from its second int (8-byte aligned, 2B ints; the
// bucket builds never store ioff), so B >= kItemParts * kXchWords.
// A tag is never confused with what the area held before this launch: the batch buffer is zeroed
// when it is allocated (stale ints of an earlier allocation would otherwise be small numbers like
// the first tags of a process), later launches on it used other tags, and every tag has bit 31 set
// (kTagMark), which the one-workgroup radix build's ioff positions (< 2^16) never have.
constexpr int kXchWords = 2 + kMaxWorld / 2;
constexpr uint32_t kTagMark = 0x80000000u;
constexpr uint32_t kBoardMagic = 0x534D504Bu;  // "SMPK": high half of a sampling-board mark
// the user-order flag: {nvalid << 48 | kUposMagic16 << 32 | tag} (the valid count rides along)
constexpr uint32_t kUposMagic = 0x5550u;   // "UP": bits 32..47 of the user-order flag
// fast item parts' tie words: side (1 bit) | local user row | slot (kTieSlotBits): the user rows
// must fit the remaining bits (the host falls back to every part sorting by user otherwise)
constexpr int kTieSlotBits = 13;  // slots < kBuildThreads * 4 = 4096 (bucket builds)
static __device__ __forceinline__ uint64_t* xch_of(const BatchView& v) {
  return reinterpret_cast<uint64_t*>(v.ioff + 1);
}

// diagnostic build only (-DBPRMF_BUILD_STAMPS): batch 0's user workgroup stamps g_build_stamps[0..4],
// its first item part [8..15], its last item part [16..23] (absolute s_memrealtime)
#ifdef BPRMF_BUILD_STAMPS
#define SPSTAMP(k)                                                                           \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x <= kItemParts && (blockIdx.x == 0 || blockIdx.x == 1 || \
                                                         blockIdx.x == kItemParts))          \
      g_build_stamps[(blockIdx.x == 0 ? 0 : blockIdx.x == 1 ? 8 : 16) + (k)] =               \
          __builtin_amdgcn_s_memrealtime();                                                  \
  } while (0)
// and every workgroup's start and end (g_split_se[wg] = {start, end}, up to 4096 workgroups)
__device__ uint64_t g_split_se[4096][2];
struct SplitSE {
  __device__ SplitSE() {
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_split_se[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
  }
  __device__ ~SplitSE() {
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_split_se[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
  }
};
extern "C" int bprmf_debug_split_se(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_split_se), sizeof(g_split_se)) == hipSuccess ? 0 : -3;
}
#define SPLIT_SE SplitSE split_se_
#else
#define SPSTAMP(k) \
  do {             \
  } while (0)
#define SPLIT_SE \
  do {           \
  } while (0)
#endif
// x / d for 32-bit unsigned x by a multiply-high and a shift (round-up method: l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1, q = (umulhi(m, x) + x) >> l, exact for every 32-bit x); the
// sharded builder divides every reference by the world size and every head by the owner's row
// count, runtime values a plain `/` turns into a ~40-instruction sequence
struct FastDiv {
  uint32_t d = 1, m = 1, l = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t dd) : d(dd) {
    while ((1ull << l) < dd) ++l;
    m = (uint32_t)(((1ull << 32) * ((1ull << l) - dd)) / dd + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t x) const {
    return (uint32_t)(((uint64_t)__umulhi(m, x) + x) >> l);
  }
  __device__ __forceinline__ uint32_t mod(uint32_t x) const { return x - div(x) * d; }
};

// SL (the sharded runner's batches): users are global ids (local row u / world), items are keyed
// owner-major ((item % world) * iloc + item / world) and written as SLOTS: the segment index (slot
// stride 0) or owner * slot_stride + index within the owner's range; ukey and own as
// k_build_batches writes them.  !SL: one rank, item rows.
// SMP: the launch samples the batches itself (no k_sample launch before it): each of a batch's
// 1 + kItemParts workgroups draws its share of the batch's slots (sample_slot, the same bits as
// k_sample) into the staging arrays ru/ri/rj (write-through), marks the batch's sampling board
// (after the parts' exchange words in the same area) and waits for the others' marks; the loads
// below then read the staged triplets past the L2 (sc1).
template <bool SL, bool SMP>
__global__ __launch_bounds__(kBuildThreads) void k_build_split(
    int64_t n_slots, int B, const int32_t* __restrict__ ru, const int32_t* __restrict__ ri,
    const int32_t* __restrict__ rj, int64_t u_rows, int64_t i_rows, int world_in, int64_t iloc,
    int slot_stride, int user_bits, int item_bits, int tpb, int k1_items, BatchBuf bb,
    int32_t* __restrict__ err, CursorInit ci, uint32_t tag, SamplerArgs sa, uint32_t epoch,
    int64_t first_slot, FastDiv wdiv, FastDiv ldiv, int fast_parts) {
  constexpr int T = kBuildThreads;
  constexpr int IPT = 4;
  constexpr int IPT2 = 2 * IPT;
  CsScope cs_(0);  // diagnostic builds only (BPRMF_CALL_STAMPS)
  SPLIT_SE;
  using Scan = rocprim::block_scan<int, T>;
  using ScanL = rocprim::block_scan<uint64_t, T>;
  constexpr size_t kBucketBytes = 12 * (size_t)T * IPT2 + 4 * (kBuckets + 4);
  __shared__ __attribute__((aligned(16))) unsigned char s_sort[kBucketBytes];
  __shared__ typename Scan::storage_type sscan;
  __shared__ typename ScanL::storage_type sscan64;
  __shared__ int32_t s_i[T * IPT];  // per sorted position: item row
  __shared__ int32_t s_j[T * IPT];
  __shared__ int32_t s_ninv;
  __shared__ int s_base[3];  // item parts: segments, K2 records, long records of the parts before
  __shared__ int s_prev[kItemParts][3 + kMaxWorld];
  __shared__ int s_lopre[kMaxWorld];      // SL: this part's first segment of each owner (local)
  __shared__ int s_opre[kMaxWorld + 1];   // SL: the batch's first segment of each owner (global)
  const int world = SL ? world_in : 1;
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_sort);
  uint32_t* s_u = reinterpret_cast<uint32_t*>(s_sort) + 2 * T * IPT;
  int32_t* s_refs = reinterpret_cast<int32_t*>(s_sort) + T * IPT2;
  int32_t* s_ioff = reinterpret_cast<int32_t*>(s_sort + 8 * (size_t)T * IPT2);
  BucketScratch<T> bs;
  bs.bk = reinterpret_cast<uint64_t*>(s_sort);
  bs.srt = reinterpret_cast<int32_t*>(s_sort + 8 * (size_t)T * IPT2);
  bs.start = reinterpret_cast<int32_t*>(s_sort + 12 * (size_t)T * IPT2);
  bs.ninv = &s_ninv;
  bs.scan = &sscan;
  const int tid = threadIdx.x;
  const int role = (int)(blockIdx.x % (kItemParts + 1));
  const int64_t batch = blockIdx.x / (kItemParts + 1);
  const int64_t b0 = batch * (int64_t)B;
  const int nb = (int)max<int64_t>(0, min<int64_t>(B, n_slots - b0));
  const BatchView v = bb.view(batch);
  if (tid < kMaxWorld) s_lopre[tid] = -1;
  if (batch == 0 && role == 0 && ci.cursor) {  // set_cursor's work (kernels.hip k_set_cursor)
    if (tid == 0) {
      ci.cursor[0] = ci.t;
      ci.cursor[1] = ci.k;
    }
    if (ci.loss && tid < ci.nloss) ci.loss[tid] = 0.0;
  }
  SPSTAMP(0);
  if constexpr (SMP) {  // 0. this workgroup's share of the batch's slots, then everyone's
    const int share = (B + kItemParts) / (kItemParts + 1);
    const int s0 = role * share, s1 = min(nb, s0 + share);
    for (int p = s0 + tid; p < s1; p += T) {
      int32_t u, i, j;
      if (!sample_slot(sa, epoch, (uint64_t)(first_slot + b0 + p), u, i, j)) atomicOr(err, 2);
      __hip_atomic_store(const_cast<int32_t*>(ru) + b0 + p, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(const_cast<int32_t*>(ri) + b0 + p, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(const_cast<int32_t*>(rj) + b0 + p, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores are acknowledged
    __syncthreads();                                    // ... and every wave's
    // the mark is the whole 64-bit word {kBoardMagic, tag}: a stale int pair in the buffer would
    // have to equal both halves (the buffer is zeroed when allocated, capi.cpp ensure_seg)
    uint64_t* board = xch_of(v) + (int64_t)kItemParts * kXchWords;
    const uint64_t mark = (uint64_t)kBoardMagic << 32 | tag;
    if (tid == 0) __hip_atomic_store(board + role, mark, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid <= kItemParts && tid != role) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (uint32_t polls = 0;; ++polls) {
        if (__hip_atomic_load(board + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mark) break;
        __builtin_amdgcn_s_sleep(1);
        if ((polls & 255) == 255 && __builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s
          atomicOr(err, 16);
          __hip_atomic_store(v.meta + kMetaDead, kDeadMark, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
  }
  // a staged word of the batch: written in this launch by other CUs (SMP: read past the L2)
  auto staged = [](const int32_t* p) -> int32_t {
    if constexpr (SMP) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
  };

  // 1. the batch's triplets in slot order, keyed by (local) user row (as k_build_batches)
  uint32_t key[IPT], val[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int p = tid * IPT + k;
    key[k] = kNone;
    val[k] = (uint32_t)p;
    const int32_t ug = p < nb ? staged(ru + b0 + p) : -1;
    if (p < nb) s_u[p] = kNone;  // (fast item parts: an invalid or empty slot has no references)
    if (ug >= 0) {  // u < 0: an empty slot
      const int32_t u = SL ? (int32_t)wdiv.div((uint32_t)ug) : ug, i = staged(ri + b0 + p),
                    j = staged(rj + b0 + p);
      if ((uint64_t)u < (uint64_t)u_rows && (uint64_t)i < (uint64_t)i_rows &&
          (uint64_t)j < (uint64_t)i_rows) {
        key[k] = (uint32_t)u;
        s_u[p] = (uint32_t)u;
        s_i[p] = i;
        s_j[p] = j;
      } else if (role == 0) {
        atomicOr(err, 1);
      }
    }
  }
  SPSTAMP(1);
  // fast_parts: only the user workgroup sorts the batch by user; it publishes every slot's
  // position in user order (upos, in the batch's useg area, which bucket builds leave unused) for
  // the item parts, which sort their references in slot order by (item, side, user, slot) -- the
  // same order -- and read upos only to write the references' values (kernel-launch A/B:
  // BPRMF_SPLIT_UPOS=0 has every workgroup sort by user, as before)
  uint64_t* upos_flag = xch_of(v) + (int64_t)kItemParts * kXchWords + kItemParts + 1;
  const uint64_t upos_mark = (uint64_t)kUposMagic << 32 | tag;
  int nvalid = 0;
  if (role == 0 || !fast_parts) {
  nvalid = bucket_sort<T, IPT>(key, val, user_bits, bs, [&](int q) { return s_u[q]; },
                               [](int q) { return (uint32_t)q; });
  SPSTAMP(2);
  if (role == 0 && fast_parts) {
    // the permutation in sorted order (useg[p] = the slot at sorted position p, p < B): one
    // 16-byte write-through store per thread, 1 KB contiguous per wave (scattered 4-byte stores
    // of upos[slot] took ~5.7 us), then the flag with the valid count.  (fast_parts needs B % 4
    // == 0: useg is then 16-byte aligned.)
    if (tid * IPT < B) {
      uint64_t* pw = reinterpret_cast<uint64_t*>(v.useg + tid * IPT);
      __hip_atomic_store(pw, (uint64_t)val[0] | (uint64_t)val[1] << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pw + 1, (uint64_t)val[2] | (uint64_t)val[3] << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(upos_flag, upos_mark | (uint64_t)nvalid << 48, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // blocked arrangement: sorted position p = tid*IPT + k holds key[k] (user) and val[k] (slot)
  int32_t my_i[IPT], my_j[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const bool ok = key[k] != kNone;
    my_i[k] = ok ? s_i[val[k]] : 0;
    my_j[k] = ok ? s_j[val[k]] : 0;
    s_key[tid * IPT + k] = key[k];
  }
  __syncthreads();  // slot-order reads of s_i/s_j done; s_key complete
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    s_i[tid * IPT + k] = my_i[k];  // sorted order from here on
    s_j[tid * IPT + k] = my_j[k];
  }
  }  // role == 0 || !fast_parts

  if (role == 0) {
    // ---- user side: segments, w, trec {u, w}, mrec, meta (k_build_batches lines for these) ----
    const uint32_t uprev = tid ? s_key[tid * IPT - 1] : kNone;
    bool uhead[IPT];
    int heads = 0;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      uhead[k] = key[k] != kNone && (k ? key[k - 1] : uprev) != key[k];
      heads += uhead[k];
    }
    int pre = 0, tot = 0;
    Scan().exclusive_scan(heads, pre, 0, tot, sscan, rocprim::plus<int>());
    const int seg0 = pre, n_useg = tot;
    int32_t* s_seg = reinterpret_cast<int32_t*>(s_sort) + T * IPT;
    {
      int s = seg0;
#pragma unroll
      for (int k = 0; k < IPT; ++k)
        if (uhead[k]) s_seg[s++] = tid * IPT + k;
    }
    __syncthreads();
    int uend[IPT], uw[IPT], nmulti = 0;
    {
      int s = seg0 - 1;
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int p = tid * IPT + k;
        uend[k] = p + 1;
        uw[k] = 0;
        if (key[k] != kNone) {
          if (uhead[k]) ++s;
          const int b = s_seg[max(s, 0)], e = s + 1 < n_useg ? s_seg[s + 1] : nvalid;
          uend[k] = e;
          const int len = e - b;
          if (len == 1)
            uw[k] = 1;
          else if (b / tpb == (e - 1) / tpb)
            uw[k] = p == b ? len : -1;
        }
        nmulti += uhead[k] && uw[k] == 0;
      }
    }
    int mpre = 0, n_multi = 0;
    SPSTAMP(3);
    __syncthreads();  // sscan reuse
    Scan().exclusive_scan(nmulti, mpre, 0, n_multi, sscan, rocprim::plus<int>());
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int p = tid * IPT + k;
      if (key[k] == kNone) continue;
      reinterpret_cast<int2*>(v.trec + 4LL * p)[1] = make_int2((int)key[k], uw[k]);
      if (uhead[k] && uw[k] == 0) {  // a segment K2 finishes
        store_rec(v.mrec + (int64_t)mpre * kRec, (int)key[k], p, uend[k], 0, 0, 0, 0, 0);
        ++mpre;
      }
    }
    if (tid == 0) {
      v.meta[0] = nvalid;
      v.meta[1] = n_useg;
      v.meta[4] = n_multi;
    }
    SPSTAMP(4);
    return;
  }

  // ---- item part q: references whose item key lies in [lo, lo + 2^rb) ----
  const int q = role - 1;
  const int rb = max(item_bits - kItemPartBits, 0);  // parts of 2^rb keys
  const uint32_t lo = (uint32_t)q << rb;
  auto key_of_item = [&](uint32_t item) -> uint32_t {
    if constexpr (SL) {
      const uint32_t qw = wdiv.div(item);
      return (item - qw * (uint32_t)world) * (uint32_t)iloc + qw;
    } else {
      return item;
    }
  };
  __syncthreads();  // s_i/s_j in sorted order (fast_parts: slot order, s_u valid); s_key free
  uint32_t ik[IPT2], tie[IPT2];
  int below = 0, mine = 0;  // references of this thread in the parts before / in this part
  if (fast_parts) {  // references in slot order: r < nb the i side of slot r, else the j side
#pragma unroll
    for (int k = 0; k < IPT2; ++k) {
      const int r = tid * IPT2 + k;
      ik[k] = kNone;
      tie[k] = 0;
      if (r < 2 * nb) {
        const int side = r >= nb, slot = side ? r - nb : r;
        const uint32_t u = s_u[slot];
        if (u == kNone) continue;
        const uint32_t kk = key_of_item((uint32_t)(side ? s_j[slot] : s_i[slot]));
        if (kk >= lo && ((kk - lo) >> rb) == 0) ik[k] = kk;
        tie[k] = (uint32_t)side << 31 | u << kTieSlotBits | (uint32_t)slot;
        below += kk < lo;
        mine += ik[k] != kNone;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < IPT2; ++k) {
      const int r = tid * IPT2 + k;
      ik[k] = kNone;
      tie[k] = 0;
      if (r < 2 * nvalid) {
        const uint32_t kk = key_of_item((uint32_t)(r < nvalid ? s_i[r] : s_j[r - nvalid]));
        if (kk >= lo && ((kk - lo) >> rb) == 0) ik[k] = kk;
        below += kk < lo;
        mine += ik[k] != kNone;
      }
    }
  }
  int cpre0 = 0, ctot0 = 0;  // (refs before << 16 | refs here), each <= 2B <= 8192
  Scan().exclusive_scan(below << 16 | mine, cpre0, 0, ctot0, sscan, rocprim::plus<int>());
  const int rbase = ctot0 >> 16, n_mine = ctot0 & 0xFFFF;
  SPSTAMP(3);
  // the sorted references come out E2 per thread: kPartE2 while the part holds at most that many
  // per thread, else 8 (the single-workgroup builder's)
  auto part = [&](auto e2) {
  constexpr int E2 = decltype(e2)::value;
  uint32_t ok_[E2], ov[E2];
  const int nv = nvalid;
  int total;
  if (fast_parts) {
    constexpr uint32_t smask = (1u << kTieSlotBits) - 1;
    total = bucket_sort_sparse<T, IPT2, E2>(
        ik, lo, rb, bs,
        [&](int id) {
          const uint32_t t = (uint32_t)id, slot = t & smask;
          return key_of_item((uint32_t)((t >> 31) ? s_j[slot] : s_i[slot]));
        },
        [](int id) { return (uint32_t)id; }, ok_, ov, tie);
    // the user workgroup's permutation (one sc1 poll by thread 0, bounded; sc1 loads), inverted
    // in LDS (the sort's bucket starts, free now): s_upos[slot] = the slot's position in user order
    int32_t* s_upos = bs.start;
    if (tid == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t w = 0;
      for (uint32_t polls = 0;; ++polls) {
        w = __hip_atomic_load(upos_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((w & 0x0000FFFFFFFFFFFFull) == upos_mark) break;
        __builtin_amdgcn_s_sleep(1);
        if ((polls & 255) == 255 && __builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s
          atomicOr(err, 16);
          __hip_atomic_store(v.meta + kMetaDead, kDeadMark, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          w = 0;
          break;
        }
      }
      s_ninv = (int)(w >> 48);  // the batch's valid triplet count
    }
    __syncthreads();
    {
      const int nval = s_ninv;
      if (tid * IPT < nval) {
        const uint64_t* pw = reinterpret_cast<const uint64_t*>(v.useg + tid * IPT);
        const uint64_t a = __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t b = __hip_atomic_load(pw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t sl[IPT] = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          const int p = tid * IPT + k;
          if (p < nval && sl[k] < (uint32_t)nb) s_upos[sl[k]] = p;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E2; ++k) {  // (side, user, slot) -> the reference's value (pos << 1 | side)
      if (ok_[k] == kNone) continue;
      const uint32_t t = ov[k];
      ov[k] = (uint32_t)s_upos[t & smask] << 1 | (t >> 31);
    }
    __syncthreads();  // s_upos (bucket starts) free again
  } else {
    total = bucket_sort_sparse<T, IPT2, E2>(
        ik, lo, rb, bs,
        [&](int r) { return key_of_item((uint32_t)(r < nv ? s_i[r] : s_j[r - nv])); },
        [&](int r) { return r < nv ? ((uint32_t)r << 1) : (((uint32_t)(r - nv) << 1) | 1u); }, ok_, ov);
  }
  SPSTAMP(4);
#pragma unroll
  for (int k = 0; k < E2; ++k) s_key[tid * E2 + k] = ok_[k];
  __syncthreads();
  const uint32_t iprev = tid ? s_key[tid * E2 - 1] : kNone;
  const uint32_t inext = tid + 1 < T ? s_key[(tid + 1) * E2] : kNone;
  uint32_t hm = 0, sm = 0, lm = 0;
  int iheads = 0, mheads = 0, nlong = 0;
#pragma unroll
  for (int k = 0; k < E2; ++k) {
    const int r = tid * E2 + k;  // local position
    if (ok_[k] == kNone) continue;
    const bool h = (k ? ok_[k - 1] : iprev) != ok_[k];
    const bool so = !SL && k1_items && h && (k + 1 < E2 ? ok_[k + 1] : inext) != ok_[k];
    const bool lg = h && !so && r + kLongSeg < T * E2 && s_key[r + kLongSeg] == ok_[k];
    hm |= (uint32_t)h << k;
    sm |= (uint32_t)so << k;
    lm |= (uint32_t)lg << k;
    iheads += h;
    mheads += h && !so;
    nlong += lg;
    v.refs[rbase + r] = (int32_t)ov[k];
    s_refs[r] = (int32_t)ov[k];
    if (!SL) {  // the triplet's item word: row | first reference of its item | only reference
      const int32_t word = (int32_t)ok_[k] | (h ? (int32_t)0x80000000 : 0) | (so ? 0x40000000 : 0);
      v.trec[4LL * (ov[k] >> 1) + (ov[k] & 1)] = word;
    }
  }
  uint64_t cpre = 0, ctot = 0;
  ScanL().exclusive_scan((uint64_t)iheads | (uint64_t)mheads << 16 | (uint64_t)nlong << 32, cpre, 0ull,
                         ctot, sscan64, rocprim::plus<uint64_t>());
  auto field = [](uint64_t x, int f) { return (int)((x >> (16 * f)) & 0xFFFF); };
  const int iseg0 = field(cpre, 0), n_iseg = field(ctot, 0);
  const int mseg0 = field(cpre, 1), n_mseg = field(ctot, 1);
  const int n_long = field(ctot, 2);
  {
    int s = iseg0;
#pragma unroll
    for (int k = 0; k < E2; ++k) {
      if (!((hm >> k) & 1)) continue;
      if (SL) {  // an owner's first segment of this part: its head follows another owner's key
        const uint32_t o = ldiv.div(ok_[k]);
        const uint32_t pk = k ? ok_[k - 1] : iprev;
        if (pk == kNone || ldiv.div(pk) != o) s_lopre[o] = s;
      }
      s_ioff[s++] = tid * E2 + k;
    }
  }
  if (tid == 0) s_ioff[n_iseg] = total;
  __syncthreads();  // s_ioff, s_refs, s_lopre
  SPSTAMP(5);
  // publish this part's counts, then collect the parts before (the first q threads, one each)
  uint64_t* xch = xch_of(v) + (int64_t)kXchWords * q;
  if (tid == 0) {
    const uint64_t tg = (uint64_t)tag << 32;
    __hip_atomic_store(xch, tg | (uint32_t)(n_iseg | n_mseg << 16), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(xch + 1, tg | (uint32_t)n_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (SL) {  // owners without segments here start where the next owner does
      int next = n_iseg;
      for (int o = world - 1; o >= 0; --o) {
        if (s_lopre[o] < 0) s_lopre[o] = next;
        next = s_lopre[o];
      }
      for (int o = 0; o < world; o += 2) {
        const uint32_t c = (uint32_t)s_lopre[o] | (o + 1 < world ? (uint32_t)s_lopre[o + 1] << 16 : 0u);
        __hip_atomic_store(xch + 2 + o / 2, tg | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  const int nw = SL ? 2 + (world + 1) / 2 : 2;  // words per part
  if (tid < q) {
    const uint64_t* px = xch_of(v) + (int64_t)kXchWords * tid;
    uint64_t w[kXchWords];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t polls = 0;; ++polls) {
      bool all = true;
#pragma unroll
      for (int m = 0; m < kXchWords; ++m) {  // registers only (fixed indices)
        w[m] = m < nw ? __hip_atomic_load(px + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        all &= m >= nw || (uint32_t)(w[m] >> 32) == tag;
      }
      if (all) break;
      __builtin_amdgcn_s_sleep(1);
      if ((polls & 255) == 255 && __builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s
        atomicOr(err, 16);
        __hip_atomic_store(v.meta + kMetaDead, kDeadMark, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int m = 0; m < kXchWords; ++m) w[m] = 0;
        break;
      }
    }
    s_prev[tid][0] = (int)(w[0] & 0xFFFF);
    s_prev[tid][1] = (int)((w[0] >> 16) & 0xFFFF);
    s_prev[tid][2] = (int)(w[1] & 0xFFFFFFFF);
    if (SL) {
#pragma unroll
      for (int m = 2; m < kXchWords; ++m) {  // owners 2(m-2) and 2(m-2)+1 (past world: unused)
        s_prev[tid][3 + 2 * (m - 2)] = (int)(w[m] & 0xFFFF);
        s_prev[tid][4 + 2 * (m - 2)] = (int)((w[m] >> 16) & 0xFFFF);
      }
    }
  }
  __syncthreads();  // s_prev
  if (tid < 3) {
    int acc = 0;
    for (int m = 0; m < q; ++m) acc += s_prev[m][tid];
    s_base[tid] = acc;
  }
  if (SL && tid < world) {  // the batch's segments of owners below tid: the parts before + this one
    int acc = s_lopre[tid];
    for (int m = 0; m < q; ++m) acc += s_prev[m][3 + tid];
    s_opre[tid] = acc;
  }
  __syncthreads();
  const int ibase = s_base[0], mbase = s_base[1], lbase = s_base[2];
  if (SL && tid == 0) s_opre[world] = ibase + n_iseg;  // (the last part: the batch's segment count)
  __syncthreads();
  SPSTAMP(6);
  // slot of the batch's item segment sg (k_build_batches's slot_of)
  auto slot_of = [&](int sg) -> int {
    if (!SL || !slot_stride) return sg;
    int lo_o = 0, hi_o = world - 1;  // largest owner o with s_opre[o] <= sg
    while (lo_o < hi_o) {
      const int mid = (lo_o + hi_o + 1) >> 1;
      if (s_opre[mid] <= sg) lo_o = mid; else hi_o = mid - 1;
    }
    return lo_o * slot_stride + (sg - s_opre[lo_o]);
  };
  // item records of the K2-served segments, and the long ones' copies (k_build_batches's); SL:
  // the distinct items' local rows and every reference's triplet word (slot | first reference)
  {
    int s = iseg0, ms = mbase + mseg0, lpre = lbase + field(cpre, 2);
    int sr = iseg0 - 1;  // segment of this thread's first reference if it is not a head
#pragma unroll
    for (int k = 0; k < E2; ++k) {
      const int r = tid * E2 + k;
      if (SL && ok_[k] != kNone) {
        const bool h = (hm >> k) & 1;
        if (h) ++sr;
        v.trec[4LL * (ov[k] >> 1) + (ov[k] & 1)] = slot_of(ibase + sr) | (h ? (int32_t)0x80000000 : 0);
      }
      if (!((hm >> k) & 1)) continue;
      if ((sm >> k) & 1) {
        ++s;
        continue;
      }
      const int end = s_ioff[s + 1];
      const int len = end - r;
      const int lng = ((lm >> k) & 1) && lpre < kMaxLongItems;
      int pk[kInlineRefs / 2];
#pragma unroll
      for (int m = 0; m < kInlineRefs / 2; ++m) {
        const int a = s_refs[min(r + 2 * m, total - 1)], b = s_refs[min(r + 2 * m + 1, total - 1)];
        pk[m] = (2 * m < len ? a : 0) | ((2 * m + 1 < len ? b : 0) << 16);
      }
      const int sg = ibase + s;
      if (SL) v.ukey[sg] = (int32_t)ldiv.mod(ok_[k]);
      store_rec(v.irec + (int64_t)ms * kRec, SL ? slot_of(sg) : (int)ok_[k],
                (rbase + r) | (len << 15) | (lng << 30), pk[0], pk[1], pk[2], pk[3], pk[4], pk[5]);
      if (lng)
        store_rec(v.lrec + (int64_t)lpre * kRec, (int)ok_[k], rbase + r, rbase + end, slot_of(sg), 0,
                  0, 0, 1);
      lpre += (lm >> k) & 1;
      ++s;
      ++ms;
    }
  }
  if (q == kItemParts - 1) {
    if (tid == 0) {
      v.meta[2] = mbase + n_mseg;
      v.meta[3] = min(lbase + n_long, kMaxLongItems);
    }
    if (SL && tid < world) v.own[tid] = s_opre[tid + 1] - s_opre[tid];
    if (SL && ci.own_max && tid == 0) {  // dist_own_max's work, batch by batch
      int m = 0;
      for (int o = 0; o < world; ++o) m = max(m, s_opre[o + 1] - s_opre[o]);
      atomicMax(ci.own_max, m);
    }
  }
  SPSTAMP(7);
  };
  if (n_mine <= T * kPartE2)
    part(std::integral_constant<int, kPartE2>{});
  else
    part(std::integral_constant<int, 8>{});
}

#ifdef BPRMF_BUILD_STAMPS
extern "C" int bprmf_debug_build_stamps(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_build_stamps), sizeof(uint64_t) * 32) == hipSuccess ? 0 : -3;
}
#endif

// the split builder's launch tags: one counter for every handle and thread of the process, so
// each launch's tag differs from every tag written into any batch buffer before it (2^31 launches
// before a repeat); bit 31 always set (kTagMark)
static std::atomic<uint32_t> g_build_tag{0};
static uint32_t next_build_tag() { return kTagMark | (g_build_tag.fetch_add(1) + 1); }
// test hook (include/bprmf.h): the tag the next split-builder launch of this process will carry
extern "C" int bprmf_debug_next_build_tag(uint32_t* tag) {
  if (!tag) return -1;
  *tag = kTagMark | (g_build_tag.load() + 1);
  return 0;
}

static int bits_for(int64_t n) {  // radix-sort bits covering ids in [0, n)
  int b = 1;
  while (b < 32 && (1LL << b) < n) ++b;
  return b;
}

hipError_t build_batches(const SamplerArgs& a, uint32_t epoch, int64_t first_slot, int64_t n_slots,
                         int B, const int32_t* ru, const int32_t* ri, const int32_t* rj,
                         int64_t u_rows, int64_t i_rows, int world, bool slots, int slot_stride,
                         int64_t n_batches, BatchBuf bb, int32_t* err, hipStream_t s, int tpb,
                         const CursorInit& ci, bool* own_max_done, bool sample_first) {
  if (own_max_done) *own_max_done = false;
  if (n_batches <= 0) return hipSuccess;
  if (sample_first && (!ru || !ri || !rj)) return hipErrorInvalidValue;
  if (ci.cursor && ci.loss && ci.nloss > kBuildThreads) return hipErrorInvalidValue;
  if (B <= 0 || B > kMaxSegBatch || world <= 0 || world > kMaxWorld) return hipErrorInvalidValue;
  const int64_t iloc = (i_rows + world - 1) / world;
  if ((uint64_t)iloc * (uint64_t)world >= 0xFFFFFFFFull) return hipErrorInvalidValue;
  // one value above every valid key: an empty position (kNone) must sort after all of them, and
  // the sorts see only these low bits of it
  const int ub = bits_for(u_rows + 1), ib = bits_for(iloc * world + 1);
  const bool radix = getenv("BPRMF_RADIX_BUILD") != nullptr;  // A/B of the two sorts (tests)
  // single GPU: items with one reference in a batch are K1's (BPRMF_K1_ITEMS=0: all K2's, A/B);
  // the trec flag bits 30-31 need item ids below 2^30
  const char* k1e = getenv("BPRMF_K1_ITEMS");
  const int k1_items = (!slots && i_rows < (1LL << 30) && !(k1e && k1e[0] == '0')) ? 1 : 0;
  const bool w1 = world == 1 && !slots && a.world == 1;  // one rank: no owner divisions
#define BPRMF_BUILD(IPT_, BUCKET_, W1_)                                                          \
  k_build_batches<IPT_, BUCKET_, W1_><<<(unsigned)n_batches, kBuildThreads, 0, s>>>(               \
      a, epoch, first_slot, n_slots, B, ru, ri, rj, u_rows, i_rows, world, iloc, slots ? 1 : 0,  \
      slots ? slot_stride : 0, ub, ib, tpb, k1_items, bb, err, ci)
  // triplets already in memory: the split builder (1 + kItemParts workgroups per batch; one rank,
  // or the sharded runner's slots; BPRMF_SPLIT_ITEMS=0 keeps the one-workgroup build, A/B)
  const char* spe = getenv("BPRMF_SPLIT_ITEMS");
  const bool split = (w1 || slots) && ru && B >= kItemParts * kXchWords + kItemParts + 2 &&
                     B <= kBuildThreads * 4 && !radix && !(spe && spe[0] == '0');
  // the item parts skip the user sort when a (side, user, slot) tie word holds the user rows
  // (else, for very large user tables, every part sorts the batch by user itself)
  const int fast_parts = (1 + ub + kTieSlotBits <= 32 && B % 4 == 0) ? 1 : 0;
  // sample_first: ru/ri/rj are staging arrays for slots first_slot .. first_slot + n_slots; the
  // split builder samples them itself (BPRMF_SPLIT_SAMPLE=0: k_sample first, A/B), any other
  // build after a k_sample launch
  const char* sse = getenv("BPRMF_SPLIT_SAMPLE");
  const bool smp = sample_first && split && !(sse && sse[0] == '0');
  if (sample_first && !smp) {
    const hipError_t e = sample(a, epoch, first_slot, n_slots, const_cast<int32_t*>(ru),
                                const_cast<int32_t*>(ri), const_cast<int32_t*>(rj), err, s);
    if (e != hipSuccess) return e;
  }
  if (split) {
    const uint32_t tag = next_build_tag();
    const unsigned grid = (unsigned)(n_batches * (kItemParts + 1));
#define BPRMF_SPLIT(SL_, SMP_, W_, STRIDE_, K1_)                                                 \
  k_build_split<SL_, SMP_><<<grid, kBuildThreads, 0, s>>>(                                       \
      n_slots, B, ru, ri, rj, u_rows, i_rows, W_, iloc, STRIDE_, ub, ib, tpb, K1_, bb, err, ci, tag, \
      a, epoch, first_slot, FastDiv((uint32_t)W_), FastDiv((uint32_t)iloc), fast_parts)
    if (w1 && smp) BPRMF_SPLIT(false, true, 1, 0, k1_items);
    else if (w1) BPRMF_SPLIT(false, false, 1, 0, k1_items);
    else if (smp) BPRMF_SPLIT(true, true, world, slot_stride, 0);
    else BPRMF_SPLIT(true, false, world, slot_stride, 0);
#undef BPRMF_SPLIT
    if (own_max_done) *own_max_done = !w1 && ci.own_max;
    return hipGetLastError();
  }
  if (sample_first) first_slot = 0;  // the builds below replay the staged triplets
  if (B <= kBuildThreads * 4 && !radix) {
    if (w1) BPRMF_BUILD(4, true, true);
    else BPRMF_BUILD(4, true, false);
  } else if (B <= kBuildThreads * 4) {
    BPRMF_BUILD(4, false, false);
  } else {
    BPRMF_BUILD(8, false, false);
  }
#undef BPRMF_BUILD
  return hipGetLastError();
}

}  // namespace bprmf
