// host_plan_check.cpp — drives the host-only planning logic of libbprmf_amd (csrc/host_plan.cpp:
// the shard's positive lists behind bprmf_set_train_ex, the sharded runner's geometry, exchange
// capacity and apply-plan sizes, the IPC blobs' device comparison) under AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/sanitize/Makefile; run by tests/test_sanitizers.py).
// Every result is checked against a direct restatement; any sanitizer report aborts the run.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/wait.h>
#include <unistd.h>

#include <map>
#include <random>
#include <set>
#include <vector>

#include "../../include/bprmf.h"
#include "../../recommend-lib_amd/csrc/host_plan.h"

using namespace bprmf;

static int g_fail = 0, g_cases = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    ++g_cases;                                                        \
    if (!(c)) {                                                       \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

// the shard CSR, restated with ordered sets (train_mat as a dok of this shard's users)
static void check_csr(std::mt19937_64& g, int64_t U, int64_t I, int64_t nnz, int64_t n_ex, int W) {
  std::vector<int32_t> u(nnz), it(nnz), eu(n_ex), ei(n_ex);
  for (int64_t k = 0; k < nnz; ++k) {
    u[k] = (int32_t)(g() % U);
    it[k] = (int32_t)(g() % I);
    if (k && g() % 5 == 0) {  // duplicates of an earlier pair
      u[k] = u[k - 1];
      it[k] = it[k - 1];
    }
  }
  for (int64_t k = 0; k < n_ex; ++k) {
    eu[k] = (int32_t)(g() % U);
    ei[k] = (int32_t)(g() % I);
  }
  for (int R = 0; R < W; ++R) {
    const int64_t L = shard_rows(U, W, R);
    ShardCsr c;
    const int rc = build_shard_csr(nnz ? u.data() : nullptr, nnz ? it.data() : nullptr, nnz,
                                   n_ex ? eu.data() : nullptr, n_ex ? ei.data() : nullptr, n_ex, U, I,
                                   W, R, L, &c);
    CHECK(rc == 0);
    if (rc) continue;
    std::vector<int32_t> wu, wi;
    std::map<int64_t, std::set<int32_t>> dok;
    for (int64_t k = 0; k < nnz; ++k)
      if (u[k] % W == R) {
        wu.push_back(u[k]);
        wi.push_back(it[k]);
        dok[u[k] / W].insert(it[k]);
      }
    for (int64_t k = 0; k < n_ex; ++k)
      if (eu[k] % W == R) dok[eu[k] / W].insert(ei[k]);
    CHECK(c.pos_u == wu && c.pos_i == wi);
    CHECK((int64_t)c.indptr.size() == L + 1 && c.indptr[0] == 0);
    bool ok = true;
    for (int64_t lu = 0; lu < L && ok; ++lu) {
      const auto f = dok.find(lu);
      const size_t want = f == dok.end() ? 0 : f->second.size();
      ok = (size_t)(c.indptr[lu + 1] - c.indptr[lu]) == want;
      if (ok && want) ok = std::equal(f->second.begin(), f->second.end(), c.indices.begin() + c.indptr[lu]);
    }
    CHECK(ok);
    CHECK(c.indptr[L] == (int64_t)c.indices.size());
  }
}

// the device search (device_common.h kth_nonmember_tree), restated on the host
static int64_t tree_count(const int32_t* keys, int64_t n, int64_t k) {
  if (n <= 0) return 0;
  int L = 1;
  for (int64_t c = 16; c < n; c *= 16) ++L;
  int64_t node = 0;
  for (int l = L - 1;; --l) {
    int c = 0;
    for (int x = 0; x < 16; ++x) c += keys[node * 16 + x] <= k;
    if (l == 0) return node * 16 + c;
    if (c == 0) return 0;
    const int sh = 4 * (l + 1);
    keys += 16 * ((n + (1LL << sh) - 1) >> sh);
    node = node * 16 + (c - 1);
  }
}

static void check_tree(std::mt19937_64& g, int64_t U, int64_t I, int64_t maxdeg) {
  std::vector<int64_t> indptr(U + 1, 0);
  std::vector<int32_t> indices;
  for (int64_t u = 0; u < U; ++u) {
    const int64_t want = g() % 7 == 0 ? 0 : (int64_t)(g() % (maxdeg + 1));
    std::set<int32_t> s;
    while ((int64_t)s.size() < std::min(want, I)) s.insert((int32_t)(g() % I));
    indices.insert(indices.end(), s.begin(), s.end());
    indptr[u + 1] = (int64_t)indices.size();
  }
  SearchTree t;
  build_search_tree(indptr, indices, &t);
  CHECK((int64_t)t.soff.size() == U + 1 && t.soff[U] == (int64_t)t.keys.size());
  bool ok = true;
  for (int64_t u = 0; u < U && ok; ++u) {
    const int64_t n = indptr[u + 1] - indptr[u];
    ok = t.soff[u] % 16 == 0;
    const int32_t* a = indices.data() + indptr[u];
    for (int rep = 0; rep < 40 && ok; ++rep) {
      const int64_t k = rep < 4 ? rep : (int64_t)(g() % (uint64_t)std::max<int64_t>(1, I - n));
      int64_t m = 0;  // brute force: #{x : a[x] - x <= k}
      for (int64_t x = 0; x < n; ++x) m += a[x] - x <= k;
      ok = tree_count(t.keys.data() + t.soff[u], n, k) == m;
    }
  }
  CHECK(ok);
}

int main() {
  std::mt19937_64 g(20261017);
  // the sampler's search trees: empty users, one node, 2-4 levels (up to 16^3 + positives)
  check_tree(g, 50, 40, 16);
  check_tree(g, 200, 3000, 300);
  check_tree(g, 12, 100000, 70000);
  // shard CSR: empty input, small and skewed shapes, every world size up to one node's 16 ranks
  check_csr(g, 1, 1, 0, 0, 1);
  check_csr(g, 5, 3, 0, 4, 2);
  for (int W : {1, 2, 3, 4, 7, 8, 16})
    for (int rep = 0; rep < 3; ++rep)
      check_csr(g, 1 + (int64_t)(g() % 300), 1 + (int64_t)(g() % 200), (int64_t)(g() % 5000),
                (int64_t)(g() % 300), W);
  {  // out-of-range ids and bad geometry are refused, with nothing half-built
    const int32_t u[2] = {0, 7}, it[2] = {1, 1};
    ShardCsr c;
    CHECK(build_shard_csr(u, it, 2, nullptr, nullptr, 0, 5, 4, 1, 0, 5, &c) == BPRMF_E_RANGE);
    const int32_t eu[1] = {1}, ei[1] = {9};
    CHECK(build_shard_csr(u, it, 1, eu, ei, 1, 5, 4, 1, 0, 5, &c) == BPRMF_E_RANGE);
    CHECK(build_shard_csr(u, it, 1, nullptr, nullptr, 0, 5, 4, 2, 0, 5, &c) == BPRMF_E_INVALID);
    CHECK(build_shard_csr(u, it, 1, nullptr, nullptr, 0, 5, 4, 2, 2, 2, &c) == BPRMF_E_INVALID);
    CHECK(build_shard_csr(nullptr, nullptr, 3, nullptr, nullptr, 0, 5, 4, 1, 0, 5, &c) == BPRMF_E_INVALID);
    CHECK(c.indptr.empty());
  }
  // shard rows partition every table
  for (int W = 1; W <= 16; ++W)
    for (int64_t T : {1LL, 2LL, 15LL, 16LL, 17LL, 26744LL, 100000000LL}) {
      int64_t s = 0;
      for (int R = 0; R < W; ++R) s += shard_rows(T, W, R);
      CHECK(s == T);
    }
  // runner geometry: ml-20m and C5 shapes at every world size, sizes without overflow
  for (int W = 1; W <= 16; ++W)
    for (int64_t I : {1LL, 7LL, 26744LL, 100000000LL})
      for (int64_t B : {1LL, 512LL, 4096LL, 8192LL}) {
        RunnerGeom rg;
        CHECK(runner_geom(B, I, W, 256, 256, &rg) == 0);
        const int64_t iloc = (I + W - 1) / W;
        CHECK(rg.S == (int)std::min<int64_t>(2 * B, iloc) && rg.S >= 1);
        CHECK((__int128)rg.row_elems == (__int128)W * rg.S * 256);
        CHECK((__int128)rg.id_elems == (__int128)W * 256 * rg.S);
        for (int cap : {0, 1, 63, 64, 65, rg.S})
          CHECK((__int128)aplan_words(256, W, cap) == (__int128)256 * W * (cap > 0 ? cap : 1) * (2 * W + 1));
      }
  {
    RunnerGeom rg;
    CHECK(runner_geom(0, 5, 1, 32, 1, &rg) == BPRMF_E_INVALID);
    CHECK(runner_geom(4, 5, 0, 32, 1, &rg) == BPRMF_E_INVALID);
  }
  // exchange capacity: in range it is raw (eager) or raw rounded up to 64, capped at S (graph)
  for (int S : {1, 63, 64, 65, 1000, 8192})
    for (int raw = -2; raw <= S + 2; ++raw) {
      const int e = exchange_capacity(raw, S, false), q = exchange_capacity(raw, S, true);
      if (raw < 0 || raw > S) {
        CHECK(e == -1 && q == -1);
      } else {
        CHECK(e == raw);
        CHECK(q >= raw && q <= S && (q == S || q % 64 == 0) && (raw > 0 || q == 0));
      }
    }
  // IPC blobs: ranks on one device are seen, ranks on distinct devices are not
  {
    const size_t bb = 512, off = 5 * 64, bus = 64;
    std::vector<uint8_t> blobs(8 * bb, 0);
    auto put = [&](int r, const char* id) { strncpy((char*)blobs.data() + r * bb + off, id, bus - 1); };
    for (int r = 0; r < 8; ++r) {
      char id[32];
      snprintf(id, sizeof id, "0000:%02x:00.0", 0x11 + r);
      put(r, id);
    }
    for (int r = 0; r < 8; ++r) CHECK(!ipc_shares_device(blobs.data(), 8, r, bb, off, bus));
    put(5, "0000:13:00.0");  // rank 5 on rank 2's GPU
    CHECK(ipc_shares_device(blobs.data(), 8, 2, bb, off, bus));
    CHECK(ipc_shares_device(blobs.data(), 8, 5, bb, off, bus));
    CHECK(!ipc_shares_device(blobs.data(), 8, 0, bb, off, bus));
    CHECK(!ipc_shares_device(blobs.data(), 1, 0, bb, off, bus));
    CHECK(!ipc_shares_device(blobs.data(), 8, 0, bb, bb - 8, bus));  // field past the blob
  }
  {  // the node barrier (node_barrier.cpp): one rank, a wrong world, then forked ranks
    char path[64];
    snprintf(path, sizeof path, "/tmp/bprmf_nb_check_%d", (int)getpid());
    void* b = nullptr;
    CHECK(bprmf_node_barrier_open(path, 1, 0, 1, &b) == 0);
    for (int k = 0; k < 1000; ++k) CHECK(bprmf_node_barrier_wait(b, 5.0) == 0);
    void* w = nullptr;
    CHECK(bprmf_node_barrier_open(path, 3, 1, 0, &w) == BPRMF_E_STATE && w == nullptr);
    CHECK(bprmf_node_barrier_close(b) == 0);
    const int W = 3, iters = 300;
    CHECK(bprmf_node_barrier_open(path, W, 0, 1, &b) == 0);
    for (int r = 1; r < W; ++r) {
      if (fork() == 0) {  // a rank: meets the others iters times, then exits with its status
        void* c = nullptr;
        int bad = bprmf_node_barrier_open(path, W, r, 0, &c) != 0;
        for (int k = 0; k < iters && !bad; ++k) bad = bprmf_node_barrier_wait(c, 30.0) != 0;
        bprmf_node_barrier_close(c);
        _exit(bad);
      }
    }
    bool ok = true;
    for (int k = 0; k < iters && ok; ++k) ok = bprmf_node_barrier_wait(b, 30.0) == 0;
    CHECK(ok);
    for (int r = 1; r < W; ++r) {
      int st = 0;
      wait(&st);
      CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    }
    CHECK(bprmf_node_barrier_close(b) == 0);
    unlink(path);
  }
  printf("host_plan_check: %s, %d cases\n", g_fail ? "FAILED" : "ok", g_cases);
  return g_fail ? 1 : 0;
}
