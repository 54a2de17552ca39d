// ingest.cpp — native ratings ingestion: the host side that replaces pandas
// and the Python loops of util/data_loader.py:load_rate (:27-146) and load_mat (:444-548) for the
// MovieLens rating files the BPR path trains on.
//
//   bprmf_dataset_load        parse a ratings file on `threads` threads (one span of whole lines
//                             each), keep rating >= min_rating (load_rate :35/:39/:43), the one-pass
//                             k-core filter of prepro='5core'/'10core' (:122-144), order rows by
//                             (user, item, timestamp) (:118) and code ids densely in ascending raw
//                             order (load_mat's pd.Categorical(...).codes, :447-448)
//   bprmf_dataset_split       per-row test labels: _split_loo(by_time=1) (:410-414) or
//                             _split_fo(by_time=1) (:422-427)
//   bprmf_dataset_candidates  the test lists: loo -> [gt, `count` items the user never rated]
//                             (_negative_sampling :430-439 + :456-469); fo -> per test user the gt
//                             items plus unseen candidates up to `count` (:471-492)
// Host-only code in the product library: no GPU is touched here.  Every ordering is a stable LSD
// radix sort (11-bit digits, per-thread histograms, stable scatter), so rows with equal keys keep
// file order on any thread count.  Where the reference draws from an unseeded RNG (shuffles before
// a time sort, random.sample) the result here is a deterministic function of the data and a seed;
// DESIGN.md §8 lists each such point.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <numeric>
#include <thread>
#include <vector>

#include "../../include/bprmf.h"
#include "status.h"

using namespace bprmf;

struct bprmf_dataset {
  std::vector<int32_t> users, items;  // dense codes, rows ordered by (user, item, timestamp)
  std::vector<float> ratings;
  std::vector<int64_t> ts;
  std::vector<int64_t> user_ids, item_ids;  // code -> raw id
  std::vector<int64_t> ustart;              // rows of user u: [ustart[u], ustart[u + 1])
  int threads = 1;
};

namespace {

// diagnostic build only (-DBPRMF_INGEST_TIMING): phase times of bprmf_dataset_load on stderr
struct PhaseClock {
#ifdef BPRMF_INGEST_TIMING
  bool on = true;
#else
  bool on = false;
#endif
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[ingest] %-10s %8.3f s\n", what, std::chrono::duration<double>(now - t).count());
    t = now;
  }
};

struct RawRow {
  int64_t u, i, t;
  float r;
};

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

const char* parse_int(const char* q, const char* eol, int64_t* v) {
  const bool neg = q < eol && *q == '-';
  if (neg) ++q;
  if (q >= eol || !is_digit(*q)) return nullptr;
  int64_t x = 0;
  while (q < eol && is_digit(*q)) x = x * 10 + (*q++ - '0');
  *v = neg ? -x : x;
  return q;
}

// decimal "[-]d*[.d*]": exact integer mantissa / 10^frac, which IEEE division rounds correctly,
// so the value equals strtod's whenever the mantissa has <= 15 digits; strtod otherwise
const char* parse_num(const char* q, const char* eol, double* v) {
  static const double p10[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7,
                                 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
  const char* s = q;
  const bool neg = q < eol && *q == '-';
  if (neg) ++q;
  uint64_t m = 0;
  int digs = 0, frac = 0;
  while (q < eol && is_digit(*q)) m = m * 10 + (uint64_t)(*q++ - '0'), ++digs;
  if (q < eol && *q == '.') {
    ++q;
    while (q < eol && is_digit(*q)) m = m * 10 + (uint64_t)(*q++ - '0'), ++digs, ++frac;
  }
  if (!digs) return nullptr;
  if (digs > 15 || (q < eol && (*q == 'e' || *q == 'E'))) {  // strtod on a bounded copy
    char tok[64];
    const size_t len = std::min<size_t>((size_t)(eol - s), sizeof(tok) - 1);
    memcpy(tok, s, len);
    tok[len] = 0;
    char* e = nullptr;
    *v = strtod(tok, &e);
    return e == tok ? nullptr : s + (e - tok);
  }
  double x = (double)m;
  if (frac) x /= p10[frac];
  *v = neg ? -x : x;
  return q;
}

inline bool num_start(char c) { return is_digit(c) || c == '-' || c == '.'; }

// "<int> sep <int> sep <number> sep <int>" per line, sep = any run of other characters ('\t', ',',
// '::'); a line that does not start with a digit (a CSV header, a blank line) is skipped
void parse_span(const char* p, const char* end, float min_rating, std::vector<RawRow>* out) {
  out->reserve((size_t)(end - p) / 20 + 16);
  while (p < end) {
    const char* eol = (const char*)memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    const char* q = p;
    while (q < eol && (*q == ' ' || *q == '\r')) ++q;
    if (q < eol && is_digit(*q)) {
      RawRow row;
      double rating = 0;
      bool ok = true;
      for (int k = 0; k < 4 && ok; ++k) {
        while (q < eol && !num_start(*q)) ++q;
        if (q >= eol) {
          ok = false;
          break;
        }
        const char* e = k == 0 ? parse_int(q, eol, &row.u)
                        : k == 1 ? parse_int(q, eol, &row.i)
                        : k == 2 ? parse_num(q, eol, &rating)
                                 : parse_int(q, eol, &row.t);
        ok = e != nullptr;
        q = e;
      }
      if (ok && rating >= min_rating) {
        row.r = (float)rating;
        out->push_back(row);
      }
    }
    p = eol + 1;
  }
}

template <class F>
void parallel_for(int nt, int64_t n, F f) {  // f(lo, hi) over nt contiguous spans
  if (nt <= 1 || n < 65536) {
    f((int64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int k = 0; k < nt; ++k) pool.emplace_back(f, n * k / nt, n * (k + 1) / nt);
  for (auto& t : pool) t.join();
}

template <class F>
void parallel_dynamic(int nt, int64_t n, int64_t chunk, F f) {  // f(thread, lo, hi) in chunks
  std::atomic<int64_t> next{0};
  auto body = [&](int tid) {
    for (;;) {
      const int64_t a = next.fetch_add(chunk);
      if (a >= n) break;
      f(tid, a, std::min(n, a + chunk));
    }
  };
  if (nt <= 1 || n <= chunk) {
    body(0);
    return;
  }
  std::vector<std::thread> pool;
  for (int k = 0; k < nt; ++k) pool.emplace_back(body, k);
  for (auto& t : pool) t.join();
}

// stable LSD radix sort of (key, idx) pairs by key (11-bit digits; keys already offset so that
// `range` is their maximum): per-thread histograms, digit-major thread-minor offsets, scatter
void radix_pairs(std::unique_ptr<uint64_t[]>& k0, std::unique_ptr<int64_t[]>& i0, int64_t n,
                 uint64_t range, int nt) {
  if (n < 2 || !range) return;
  std::unique_ptr<uint64_t[]> k1(new uint64_t[n]);
  std::unique_ptr<int64_t[]> i1(new int64_t[n]);
  const int P = n < 65536 ? 1 : std::max(1, nt);
  constexpr int D = 2048;
  std::vector<int64_t> cnt((size_t)P * D);
  auto run = [&](auto f) {
    if (P == 1) return f(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < P; ++t) pool.emplace_back(f, t);
    for (auto& th : pool) th.join();
  };
  for (int shift = 0; shift < 64 && (range >> shift); shift += 11) {
    std::fill(cnt.begin(), cnt.end(), 0);
    run([&](int t) {
      int64_t* c = &cnt[(size_t)t * D];
      for (int64_t j = n * t / P, e = n * (t + 1) / P; j < e; ++j) ++c[(k0[j] >> shift) & (D - 1)];
    });
    int64_t o = 0;
    for (int dgt = 0; dgt < D; ++dgt)
      for (int t = 0; t < P; ++t) {
        const int64_t c = cnt[(size_t)t * D + dgt];
        cnt[(size_t)t * D + dgt] = o;
        o += c;
      }
    run([&](int t) {
      int64_t* c = &cnt[(size_t)t * D];
      for (int64_t j = n * t / P, e = n * (t + 1) / P; j < e; ++j) {
        const int64_t w = c[(k0[j] >> shift) & (D - 1)]++;
        k1[w] = k0[j];
        i1[w] = i0[j];
      }
    });
    k0.swap(k1);
    i0.swap(i1);
  }
}

// stable: reorder idx so that key[idx[.]] ascends
template <class K>
void radix_stable(std::vector<int64_t>& idx, const K* key, int nt) {
  const int64_t n = (int64_t)idx.size();
  if (n < 2) return;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t v = (int64_t)key[idx[j]];
    lo = std::min(lo, v), hi = std::max(hi, v);
  }
  std::unique_ptr<uint64_t[]> k0(new uint64_t[n]);
  std::unique_ptr<int64_t[]> i0(new int64_t[n]);
  parallel_for(nt, n, [&](int64_t a, int64_t b) {
    for (int64_t j = a; j < b; ++j) k0[j] = (uint64_t)((int64_t)key[idx[j]] - lo), i0[j] = idx[j];
  });
  radix_pairs(k0, i0, n, (uint64_t)(hi - lo), nt);
  parallel_for(nt, n, [&](int64_t a, int64_t b) { std::copy(&i0[a], &i0[0] + b, idx.begin() + a); });
}

inline int bit_width(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

// dense codes of raw ids in ascending raw order (pd.Categorical over integer ids)
void encode(const std::vector<RawRow>& rows, bool item, int nt, std::vector<int32_t>* codes,
            std::vector<int64_t>* uniq) {
  const int64_t n = (int64_t)rows.size();
  codes->resize(n);
  uniq->clear();
  if (!n) return;
  auto id = [&](int64_t k) { return item ? rows[k].i : rows[k].u; };
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t k = 0; k < n; ++k) lo = std::min(lo, id(k)), hi = std::max(hi, id(k));
  const uint64_t span = (uint64_t)(hi - lo) + 1;
  if (span <= (uint64_t)(4 * n + (1 << 20))) {  // small id range (MovieLens): a direct table
    std::vector<int32_t> tab(span, 0);
    for (int64_t k = 0; k < n; ++k) tab[id(k) - lo] = 1;
    int32_t c = 0;
    for (uint64_t x = 0; x < span; ++x)
      if (tab[x]) {
        uniq->push_back(lo + (int64_t)x);
        tab[x] = c++;
      }
    parallel_for(nt, n, [&](int64_t a, int64_t b) {
      for (int64_t k = a; k < b; ++k) (*codes)[k] = tab[id(k) - lo];
    });
    return;
  }
  std::vector<int64_t> idx(n), raw(n);
  std::iota(idx.begin(), idx.end(), 0);
  for (int64_t k = 0; k < n; ++k) raw[k] = id(k);
  radix_stable(idx, raw.data(), nt);
  int32_t c = -1;
  for (int64_t k = 0; k < n; ++k) {
    if (k == 0 || raw[idx[k]] != raw[idx[k - 1]]) {
      uniq->push_back(raw[idx[k]]);
      ++c;
    }
    (*codes)[idx[k]] = c;
  }
}

// splitmix64: the per-user stream of the candidate draws
inline uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// `k` distinct values of [0, n) (Floyd's algorithm) into out, ascending; `bits` is a zeroed bitmap
// of >= n bits, returned zeroed
void floyd_sample(int64_t n, int64_t k, uint64_t seed, std::vector<uint64_t>& bits, std::vector<int64_t>* out) {
  out->clear();
  uint64_t st = seed;
  for (int64_t j = n - k; j < n; ++j) {
    st = mix64(st);
    int64_t t = (int64_t)((unsigned __int128)st * (uint64_t)(j + 1) >> 64);
    if (bits[t >> 6] >> (t & 63) & 1) t = j;
    bits[t >> 6] |= 1ull << (t & 63);
    out->push_back(t);
  }
  for (int64_t t : *out) bits[t >> 6] = 0;
  std::sort(out->begin(), out->end());
}

// ranks r (ascending) in the complement of the sorted set `ex` -> the items
void map_complement(const std::vector<int64_t>& ranks, const int32_t* ex, size_t nex, int32_t* out) {
  size_t e = 0;
  for (size_t k = 0; k < ranks.size(); ++k) {
    const int64_t r = ranks[k];  // item = r + (number of excluded items <= item)
    while (e < nex && ex[e] <= r + (int64_t)e) ++e;
    out[k] = (int32_t)(r + (int64_t)e);
  }
}

}  // namespace

extern "C" {

int bprmf_dataset_load(const char* path, float min_rating, int32_t core, int32_t threads,
                       bprmf_dataset** out) {
  if (!path || !out) return fail(BPRMF_E_INVALID, "null argument");
  if (core < 0) return fail(BPRMF_E_INVALID, "core must be >= 0");
  *out = nullptr;
  PhaseClock clk;
  FILE* fp = fopen(path, "rb");
  if (!fp) return fail(BPRMF_E_INVALID, "cannot open %s", path);
  fseek(fp, 0, SEEK_END);
  const long size = ftell(fp);
  size_t got = size > 0 ? (size_t)size : 0;
  const char* base = "";
  void* map = nullptr;
  if (got) {
    map = mmap(nullptr, got, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fileno(fp), 0);
    if (map == MAP_FAILED) {
      fclose(fp);
      return fail(BPRMF_E_INVALID, "cannot map %s", path);
    }
    madvise(map, got, MADV_SEQUENTIAL);
    base = (const char*)map;
  }
  fclose(fp);
  struct Unmap {
    void* p;
    size_t n;
    ~Unmap() {
      if (p) munmap(p, n);
    }
  } unmap{map, got};
  clk.mark("map");
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, 64));
  const int np = got < (size_t)(1 << 20) ? 1 : nt;
  std::vector<const char*> cut(np + 1);
  cut[0] = base;
  cut[np] = base + got;
  for (int k = 1; k < np; ++k) {  // spans of whole lines
    const char* c = std::max(cut[k - 1], base + got * k / np);
    const char* nl = (const char*)memchr(c, '\n', (size_t)(base + got - c));
    cut[k] = nl ? nl + 1 : base + got;
  }
  std::vector<std::vector<RawRow>> parts(np);
  {
    std::vector<std::thread> pool;
    for (int k = 0; k < np; ++k) pool.emplace_back(parse_span, cut[k], cut[k + 1], min_rating, &parts[k]);
    for (auto& t : pool) t.join();
  }
  clk.mark("parse");
  int64_t n = 0;
  std::vector<int64_t> at(np + 1, 0);
  for (int k = 0; k < np; ++k) at[k + 1] = at[k] + (int64_t)parts[k].size();
  n = at[np];
  if (n >= (int64_t)INT32_MAX) return fail(BPRMF_E_UNSUPPORTED, "more than 2^31 ratings");
  std::vector<RawRow> rows(n);
  parallel_for(np, np, [&](int64_t a, int64_t b) {
    for (int64_t k = a; k < b; ++k) {
      std::copy(parts[k].begin(), parts[k].end(), rows.begin() + at[k]);
      std::vector<RawRow>().swap(parts[k]);
    }
  });
  clk.mark("gather");
  std::vector<int32_t> uc, ic;
  std::vector<int64_t> uid, iid;
  encode(rows, false, nt, &uc, &uid);
  encode(rows, true, nt, &ic, &iid);
  if (core > 0) {  // prepro='5core'/'10core': one pass, counts over the unfiltered rows
    std::vector<int64_t> cu(uid.size(), 0), ci(iid.size(), 0);
    for (int64_t k = 0; k < n; ++k) ++cu[uc[k]], ++ci[ic[k]];
    int64_t m = 0;
    for (int64_t k = 0; k < n; ++k)
      if (cu[uc[k]] >= core && ci[ic[k]] >= core) rows[m++] = rows[k];
    n = m;
    rows.resize(n);
    encode(rows, false, nt, &uc, &uid);
    encode(rows, true, nt, &ic, &iid);
  }
  clk.mark("encode");
  // sort_values(['user', 'item', 'timestamp']) with full ties in file order: stable passes by
  // timestamp, then item, then user
  std::vector<int64_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  int64_t tlo = INT64_MAX, thi = INT64_MIN;
  for (int64_t k = 0; k < n; ++k) tlo = std::min(tlo, rows[k].t), thi = std::max(thi, rows[k].t);
  const int bu = bit_width(uid.size()), bi = bit_width(iid.size()), bt = n ? bit_width((uint64_t)(thi - tlo)) : 0;
  if (bu + bi + bt <= 64) {  // one pass over a (user | item | timestamp) key
    std::unique_ptr<uint64_t[]> k0(new uint64_t[n]);
    std::unique_ptr<int64_t[]> i0(new int64_t[n]);
    parallel_for(nt, n, [&](int64_t a, int64_t b) {
      for (int64_t k = a; k < b; ++k) {
        k0[k] = (uint64_t)uc[k] << (bi + bt) | (uint64_t)ic[k] << bt | (uint64_t)(rows[k].t - tlo);
        i0[k] = k;
      }
    });
    const uint64_t range = bu + bi + bt == 64 ? ~0ull : (1ull << (bu + bi + bt)) - 1;
    radix_pairs(k0, i0, n, range, nt);
    parallel_for(nt, n, [&](int64_t a, int64_t b) { std::copy(&i0[a], &i0[0] + b, ord.begin() + a); });
  } else {
    std::vector<int64_t> tsv(n);
    for (int64_t k = 0; k < n; ++k) tsv[k] = rows[k].t;
    radix_stable(ord, tsv.data(), nt);
    radix_stable(ord, ic.data(), nt);
    radix_stable(ord, uc.data(), nt);
  }
  clk.mark("sort");
  auto* d = new bprmf_dataset();
  d->threads = nt;
  d->users.resize(n), d->items.resize(n), d->ts.resize(n), d->ratings.resize(n);
  parallel_for(nt, n, [&](int64_t a, int64_t b) {
    for (int64_t k = a; k < b; ++k) {
      const int64_t s = ord[k];
      d->users[k] = uc[s];
      d->items[k] = ic[s];
      d->ts[k] = rows[s].t;
      d->ratings[k] = rows[s].r;
    }
  });
  d->user_ids.swap(uid);
  d->item_ids.swap(iid);
  d->ustart.assign(d->user_ids.size() + 1, 0);
  for (int64_t k = 0; k < n; ++k) ++d->ustart[d->users[k] + 1];
  for (size_t u = 0; u + 1 < d->ustart.size(); ++u) d->ustart[u + 1] += d->ustart[u];
  clk.mark("emit");
  *out = d;
  return 0;
}

int bprmf_dataset_info(bprmf_dataset* d, int64_t* n, int64_t* user_num, int64_t* item_num) {
  if (!d) return fail(BPRMF_E_INVALID, "null dataset");
  if (n) *n = (int64_t)d->users.size();
  if (user_num) *user_num = (int64_t)d->user_ids.size();
  if (item_num) *item_num = (int64_t)d->item_ids.size();
  return 0;
}

int bprmf_dataset_copy(bprmf_dataset* d, int32_t* users, int32_t* items, float* ratings,
                       int64_t* timestamps, int64_t* user_ids, int64_t* item_ids) {
  if (!d) return fail(BPRMF_E_INVALID, "null dataset");
  const size_t n = d->users.size();
  // an empty dataset's vectors have no storage (data() may be null: memcpy's source must not be)
  if (n) {
    if (users) memcpy(users, d->users.data(), 4 * n);
    if (items) memcpy(items, d->items.data(), 4 * n);
    if (ratings) memcpy(ratings, d->ratings.data(), 4 * n);
    if (timestamps) memcpy(timestamps, d->ts.data(), 8 * n);
  }
  if (user_ids && !d->user_ids.empty()) memcpy(user_ids, d->user_ids.data(), 8 * d->user_ids.size());
  if (item_ids && !d->item_ids.empty()) memcpy(item_ids, d->item_ids.data(), 8 * d->item_ids.size());
  return 0;
}

int bprmf_dataset_split(bprmf_dataset* d, int32_t method, double test_frac, uint8_t* is_test) {
  if (!d || !is_test) return fail(BPRMF_E_INVALID, "null argument");
  const int64_t n = (int64_t)d->users.size();
  if (method == BPRMF_SPLIT_LOO_TIME) {
    // rank(method='first', ascending=False) == 1: the first row (in (user, item, timestamp)
    // order) holding the user's latest timestamp
    memset(is_test, 0, (size_t)n);
    const int64_t U = (int64_t)d->user_ids.size();
    parallel_for(d->threads, U, [&](int64_t a, int64_t b) {
      for (int64_t u = a; u < b; ++u) {
        int64_t best = d->ustart[u];
        for (int64_t k = d->ustart[u] + 1; k < d->ustart[u + 1]; ++k)
          if (d->ts[k] > d->ts[best]) best = k;
        if (best < d->ustart[u + 1]) is_test[best] = 1;
      }
    });
    return 0;
  }
  if (method == BPRMF_SPLIT_FO_TIME) {
    // the first ceil(n (1 - test_frac)) rows in time order train; equal timestamps keep
    // (user, item) order where the reference shuffles them
    if (!(test_frac >= 0.0 && test_frac <= 1.0)) return fail(BPRMF_E_INVALID, "test_frac must be in [0, 1]");
    memset(is_test, 0, (size_t)n);
    std::vector<int64_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    radix_stable(ord, d->ts.data(), d->threads);
    const int64_t split = (int64_t)ceil((double)n * (1.0 - test_frac));
    for (int64_t k = std::max<int64_t>(split, 0); k < n; ++k) is_test[ord[k]] = 1;
    return 0;
  }
  return fail(BPRMF_E_UNSUPPORTED, "unknown split method %d", method);
}

int bprmf_dataset_candidates(bprmf_dataset* d, const uint8_t* is_test, int32_t method, int32_t count,
                             uint64_t seed, int64_t* n_out, int32_t* users, int32_t* items) {
  if (!d || !is_test || !n_out) return fail(BPRMF_E_INVALID, "null argument");
  if (count < 1) return fail(BPRMF_E_INVALID, "count must be >= 1");
  if (method != BPRMF_SPLIT_LOO_TIME && method != BPRMF_SPLIT_FO_TIME)
    return fail(BPRMF_E_UNSUPPORTED, "unknown split method %d", method);
  const bool loo = method == BPRMF_SPLIT_LOO_TIME;
  const int64_t n = (int64_t)d->users.size();
  const int64_t U = (int64_t)d->user_ids.size(), I = (int64_t)d->item_ids.size();
  // the emitting users and their order: loo -> users with a test row, ascending (one list each,
  // led by the last test row); fo -> users in order of their first test row in time order
  std::vector<int32_t> order;
  if (loo) {
    for (int64_t u = 0; u < U; ++u)
      for (int64_t k = d->ustart[u]; k < d->ustart[u + 1]; ++k)
        if (is_test[k]) {
          order.push_back((int32_t)u);
          break;
        }
  } else {
    std::vector<int64_t> trows;
    for (int64_t k = 0; k < n; ++k)
      if (is_test[k]) trows.push_back(k);
    radix_stable(trows, d->ts.data(), d->threads);
    std::vector<uint8_t> seen(U, 0);
    for (int64_t k : trows) {
      const int32_t u = d->users[k];
      if (!seen[u]) seen[u] = 1, order.push_back(u);
    }
  }
  const int64_t per = loo ? (int64_t)count + 1 : (int64_t)count;
  const int64_t total = (int64_t)order.size() * per;
  if (!users || !items) {
    *n_out = total;
    return 0;
  }
  if (*n_out < total) return fail(BPRMF_E_INVALID, "output holds %lld rows, %lld needed", (long long)*n_out, (long long)total);
  const int nt = d->threads;
  std::atomic<int64_t> bad{-1};
  std::atomic<int64_t> bad_free{0};
  std::vector<std::vector<uint64_t>> bits(nt, std::vector<uint64_t>((size_t)(I + 64) / 64, 0));
  parallel_dynamic(nt, (int64_t)order.size(), 64, [&](int tid, int64_t a, int64_t b) {
    std::vector<int64_t> ranks;
    std::vector<int32_t> ex, gt, picked;
    for (int64_t o = a; o < b; ++o) {
      const int32_t u = order[o];
      ex.clear(), gt.clear();
      for (int64_t k = d->ustart[u]; k < d->ustart[u + 1]; ++k) {
        if (ex.empty() || ex.back() != d->items[k]) ex.push_back(d->items[k]);
        if (is_test[k] && (gt.empty() || gt.back() != d->items[k])) gt.push_back(d->items[k]);
      }
      int32_t* ou = users + o * per;
      int32_t* oi = items + o * per;
      const uint64_t us = mix64(seed ^ mix64((uint64_t)u));
      const int64_t want = loo ? count : count - (int64_t)gt.size();
      if (want > 0) {
        const int64_t free = I - (int64_t)ex.size();
        if (free < want) {
          int64_t exp = -1;
          if (bad.compare_exchange_strong(exp, u)) bad_free = free;
          continue;
        }
        floyd_sample(free, want, us, bits[tid], &ranks);
        picked.resize(want);
        map_complement(ranks, ex.data(), ex.size(), picked.data());
      } else {
        picked.clear();
      }
      if (loo) {  // [the last test item, count negatives ascending]
        int32_t gi = 0;
        for (int64_t k = d->ustart[u]; k < d->ustart[u + 1]; ++k)
          if (is_test[k]) gi = d->items[k];
        ou[0] = u, oi[0] = gi;
        for (int64_t k = 0; k < count; ++k) ou[1 + k] = u, oi[1 + k] = picked[k];
      } else {  // gt plus candidates, ascending; or `count` of the gt items
        if (want > 0) {
          picked.insert(picked.end(), gt.begin(), gt.end());
        } else {
          floyd_sample((int64_t)gt.size(), count, us, bits[tid], &ranks);
          picked.clear();
          for (int64_t x : ranks) picked.push_back(gt[x]);
        }
        std::sort(picked.begin(), picked.end());
        for (int64_t k = 0; k < count; ++k) ou[k] = u, oi[k] = picked[k];
      }
    }
  });
  if (bad >= 0)
    return fail(BPRMF_E_NO_NEGATIVE, "user %lld has %lld unrated items, fewer than the %d asked (Sample larger than population)",
                (long long)bad.load(), (long long)bad_free.load(), count);
  *n_out = total;
  return 0;
}

int bprmf_dataset_free(bprmf_dataset* d) {
  delete d;
  return 0;
}

}  // extern "C"
