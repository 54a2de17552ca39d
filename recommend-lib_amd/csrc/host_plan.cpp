// host_plan.cpp — host-only planning logic (host_plan.h).  No HIP: linked into libbprmf_amd.so and,
// alone with status.cpp, into the ASan + UBSan checker of tests/sanitize.
#include "host_plan.h"

#include <string.h>

#include <algorithm>

#include "../../include/bprmf.h"
#include "status.h"

namespace bprmf {

int build_shard_csr(const int32_t* users, const int32_t* items, int64_t nnz, const int32_t* ex_users,
                    const int32_t* ex_items, int64_t n_ex, int64_t user_num, int64_t item_num,
                    int world, int rank, int64_t local_users, ShardCsr* out) {
  if (!out || nnz < 0 || n_ex < 0 || (nnz > 0 && (!users || !items)) ||
      (n_ex > 0 && (!ex_users || !ex_items)))
    return fail(BPRMF_E_INVALID, "bad arguments");
  if (world <= 0 || rank < 0 || rank >= world || local_users != shard_rows(user_num, world, rank))
    return fail(BPRMF_E_INVALID, "bad shard geometry");
  const int64_t W = world, R = rank;
  ShardCsr c;
  c.pos_u.reserve(nnz / W + 16);
  c.pos_i.reserve(nnz / W + 16);
  for (int64_t k = 0; k < nnz; ++k) {
    const int32_t u = users[k], i = items[k];
    if (u < 0 || u >= user_num || i < 0 || i >= item_num)
      return fail(BPRMF_E_RANGE, "positive %lld = (%d, %d) out of range", (long long)k, u, i);
    if (u % W == R) {
      c.pos_u.push_back(u);
      c.pos_i.push_back(i);
    }
  }
  // the dok train_mat's keys of this shard: (local user << 32 | item), sorted, de-duplicated
  std::vector<uint64_t> keys(c.pos_u.size());
  for (size_t k = 0; k < c.pos_u.size(); ++k)
    keys[k] = ((uint64_t)(c.pos_u[k] / W) << 32) | (uint32_t)c.pos_i[k];
  for (int64_t k = 0; k < n_ex; ++k) {
    const int32_t u = ex_users[k], i = ex_items[k];
    if (u < 0 || u >= user_num || i < 0 || i >= item_num)
      return fail(BPRMF_E_RANGE, "train_mat entry (%d, %d) out of range", u, i);
    if (u % W == R) keys.push_back(((uint64_t)(u / W) << 32) | (uint32_t)i);
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  c.indptr.assign(local_users + 1, 0);
  c.indices.resize(keys.size());
  for (size_t k = 0; k < keys.size(); ++k) {
    c.indptr[(keys[k] >> 32) + 1]++;
    c.indices[k] = (int32_t)(keys[k] & 0xFFFFFFFFu);
  }
  for (int64_t u = 0; u < local_users; ++u) c.indptr[u + 1] += c.indptr[u];
  *out = std::move(c);
  return 0;
}

void build_search_tree(const std::vector<int64_t>& indptr, const std::vector<int32_t>& indices,
                       SearchTree* out) {
  const int64_t U = (int64_t)indptr.size() - 1;
  SearchTree t;
  t.soff.assign(U + 1, 0);
  // sizes first: level l (0 = leaves) has ceil(n / 16^(l+1)) nodes of 16 keys
  for (int64_t u = 0; u < U; ++u) {
    const int64_t n = indptr[u + 1] - indptr[u];
    int64_t keys = 0;
    for (int64_t m = n, l = 0; l < search_levels(n); ++l) {
      m = (m + 15) / 16;  // nodes at this level
      keys += 16 * m;
    }
    t.soff[u + 1] = t.soff[u] + keys;
  }
  t.keys.assign(t.soff[U], INT32_MAX);
  std::vector<int32_t> cur, up;
  for (int64_t u = 0; u < U; ++u) {
    const int64_t n = indptr[u + 1] - indptr[u];
    const int L = search_levels(n);
    if (!L) continue;
    cur.resize(n);
    for (int64_t x = 0; x < n; ++x) cur[x] = indices[indptr[u] + x] - (int32_t)x;  // b, non-decreasing
    // level sizes bottom-up, then write top-down: the root level first
    std::vector<std::vector<int32_t>> lv;
    lv.push_back(cur);
    for (int l = 1; l < L; ++l) {
      const std::vector<int32_t>& below = lv.back();
      up.clear();
      for (size_t q = 0; q < below.size(); q += 16) up.push_back(below[q]);
      lv.push_back(up);
    }
    int64_t o = t.soff[u];
    for (int l = L - 1; l >= 0; --l) {
      const std::vector<int32_t>& v = lv[l];
      std::copy(v.begin(), v.end(), t.keys.begin() + o);
      o += 16 * (((int64_t)v.size() + 15) / 16);
    }
  }
  *out = std::move(t);
}

int runner_geom(int64_t batch, int64_t item_num, int world, int ld, int64_t chunk_steps,
                RunnerGeom* g) {
  if (!g || batch <= 0 || item_num <= 0 || world <= 0 || ld <= 0 || chunk_steps <= 0)
    return fail(BPRMF_E_INVALID, "bad runner geometry");
  const int64_t iloc = (item_num + world - 1) / world;
  const int64_t S = std::min<int64_t>(2 * batch, iloc);
  if (S > INT32_MAX / 2) return fail(BPRMF_E_UNSUPPORTED, "slot stride %lld too large", (long long)S);
  g->S = (int)S;
  g->nmax = chunk_steps;
  g->row_elems = (int64_t)world * S * ld;
  g->id_elems = (int64_t)world * chunk_steps * S;
  return 0;
}

int64_t aplan_words(int64_t n, int world, int cap) {
  return n * world * (int64_t)std::max(cap, 1) * (2LL * world + 1);
}

int exchange_capacity(int raw, int S, bool graph) {
  if (raw < 0 || raw > S) return -1;
  if (graph && raw > 0) return std::min(S, (raw + 63) / 64 * 64);
  return raw;
}

bool ipc_shares_device(const uint8_t* blobs, int world, int rank, size_t blob_bytes, size_t bus_off,
                       size_t bus_bytes) {
  if (!blobs || world <= 1 || rank < 0 || rank >= world || bus_off + bus_bytes > blob_bytes)
    return false;
  const char* mine = reinterpret_cast<const char*>(blobs) + (size_t)rank * blob_bytes + bus_off;
  for (int p = 0; p < world; ++p) {
    if (p == rank) continue;
    const char* theirs = reinterpret_cast<const char*>(blobs) + (size_t)p * blob_bytes + bus_off;
    if (strncmp(mine, theirs, bus_bytes) == 0) return true;
  }
  return false;
}

}  // namespace bprmf
