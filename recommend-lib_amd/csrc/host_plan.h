// host_plan.h — the host-only (no HIP) planning logic of the BPR-MF handle and its sharded runner:
// the shard's positive lists (capi.cpp bprmf_set_train_ex), the runner's buffer geometry and
// exchange capacity (dist.cpp), and the IPC handle blobs' device comparison (dist.cpp
// bprmf_dist_init_ipc).  Kept out of the HIP translation units so tests/sanitize can build it
// under AddressSanitizer + UndefinedBehaviorSanitizer and drive it from a plain C++ checker.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace bprmf {

// One shard's training data (BPRData.features + train_mat, util/data_loader.py:667-678):
// positives of the shard's users (u % world == rank) in features order, and per local user
// (u / world) the sorted, de-duplicated items never drawn as negatives (features + exclusions).
struct ShardCsr {
  std::vector<int32_t> pos_u, pos_i;  // global ids, features order
  std::vector<int64_t> indptr;        // [local users + 1]
  std::vector<int32_t> indices;
};
// 0 or a bprmf_status (ids out of range, bad sizes); `out` is complete only on success
int build_shard_csr(const int32_t* users, const int32_t* items, int64_t nnz, const int32_t* ex_users,
                    const int32_t* ex_items, int64_t n_ex, int64_t user_num, int64_t item_num,
                    int world, int rank, int64_t local_users, ShardCsr* out);

// The sampler's search structure (device_common.h sample_slot): per user with sorted positives
// a[0..n), b[x] = a[x] - x is non-decreasing and the k-th non-member is k + #{x : b[x] <= k}.
// Per user a 16-ary tree of 64-byte nodes (16 int32 keys, padded with INT32_MAX), levels stored
// top-down: the leaves are b itself in 16-key nodes, a level above holds the first key of each
// node below.  soff[u] = the user's first key (a multiple of 16), levels = ceil(log16(n)) (n >= 1;
// n = 0: no keys).  One 64-byte load per level instead of one dependent load per halving.
struct SearchTree {
  std::vector<int64_t> soff;  // [users + 1]
  std::vector<int32_t> keys;
};
void build_search_tree(const std::vector<int64_t>& indptr, const std::vector<int32_t>& indices,
                       SearchTree* out);
// levels of a user's tree with n positives (0 for n = 0)
inline int search_levels(int64_t n) {
  int L = 0;
  for (int64_t c = 1; c < n; c *= 16) ++L;
  return n > 0 ? (L > 0 ? L : 1) : 0;
}

// rows of a rank's shard of `total` rows under strided sharding (row r lives on r % world)
inline int64_t shard_rows(int64_t total, int world, int rank) {
  return (total - rank + world - 1) / world;
}

// The sharded runner's fixed geometry (dist.cpp dist_attach): S = slot rows per owner in a
// requester's buffers (a batch references at most 2B distinct items, an owner holds at most
// ceil(I / W)); buffer sizes in elements.
struct RunnerGeom {
  int S = 0;
  int64_t nmax = 0;         // steps per chunk
  int64_t row_elems = 0;    // [W][S][ld] floats (landing rows, gradients)
  int64_t id_elems = 0;     // [W][nmax][S] int32 per request-list parity
};
int runner_geom(int64_t batch, int64_t item_num, int world, int ld, int64_t chunk_steps,
                RunnerGeom* g);
// int32 words of one parity's apply plan: aplan + gdep [n][W][cap][W] each, gfree [n][W][cap]
int64_t aplan_words(int64_t n, int world, int cap);
// The exchange capacity a chunk runs with: the agreed maximum request count `raw`, checked
// against the slot stride S, and (graph-captured chunks) rounded up to 64 rows so few distinct
// plans exist.  -1: raw is outside [0, S] (a corrupt agreement).
int exchange_capacity(int raw, int S, bool graph);

// IPC handle blobs (BPRMF_IPC_BLOB_BYTES each, rank order) carry the exporting device's PCI bus
// id at `bus_off`: true when some other rank's bus id equals this rank's (ranks sharing a GPU)
bool ipc_shares_device(const uint8_t* blobs, int world, int rank, size_t blob_bytes,
                       size_t bus_off, size_t bus_bytes);

}  // namespace bprmf
