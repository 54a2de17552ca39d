// node_barrier.cpp — a barrier for the ranks of one node (include/bprmf.h bprmf_node_barrier_*).
// Host only.  bench.py brackets its timed region with a barrier on every rank; a process group's
// barrier (gloo sockets, or an RCCL all-reduce plus a device synchronisation) costs ~0.1 ms, which
// lands inside the timed region of every multi-GPU line.  The ranks of one node instead meet on
// two words of a shared file mapping (/dev/shm): a sense-reversing counter barrier, ~1 us.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <new>

#include "../../include/bprmf.h"
#include "status.h"

using bprmf::fail;

namespace {

constexpr size_t kBarrierBytes = 4096;

struct Shared {
  std::atomic<int32_t> count;  // ranks arrived in the current generation
  std::atomic<int32_t> gen;    // generation: bumped by the last rank to arrive
  int32_t world;
  std::atomic<int32_t> broken;  // a rank timed out: its arrival stays counted, so the barrier is
                                // poisoned and every later wait fails at once (close and reopen)
};
static_assert(std::atomic<int32_t>::is_always_lock_free, "lock-free int32 atomics");

struct NodeBarrier {
  Shared* s = nullptr;
  int world = 0, rank = 0;
};

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

}  // namespace

extern "C" {

int bprmf_node_barrier_open(const char* path, int32_t world, int32_t rank, int32_t create, void** out) {
  if (!path || !out || world <= 0 || rank < 0 || rank >= world) return fail(BPRMF_E_INVALID, "bad arguments");
  *out = nullptr;
  const int fd = open(path, O_RDWR | (create ? O_CREAT | O_TRUNC : 0), 0600);
  if (fd < 0) return fail(BPRMF_E_STATE, "node barrier: cannot open %s", path);
  if (create && ftruncate(fd, (off_t)kBarrierBytes) != 0) {
    close(fd);
    return fail(BPRMF_E_STATE, "node barrier: cannot size %s", path);
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < kBarrierBytes) {
    close(fd);
    return fail(BPRMF_E_STATE, "node barrier: %s is not initialised", path);
  }
  void* p = mmap(nullptr, kBarrierBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return fail(BPRMF_E_STATE, "node barrier: cannot map %s", path);
  Shared* s = static_cast<Shared*>(p);
  if (create) {
    new (&s->count) std::atomic<int32_t>(0);
    new (&s->gen) std::atomic<int32_t>(0);
    new (&s->broken) std::atomic<int32_t>(0);
    s->world = world;
  } else if (s->world != world) {
    const int made = s->world;  // read before the unmap
    munmap(p, kBarrierBytes);
    return fail(BPRMF_E_STATE, "node barrier: %s was made for %d ranks, not %d", path, made, world);
  }
  auto* b = new NodeBarrier();
  b->s = s;
  b->world = world;
  b->rank = rank;
  *out = b;
  return 0;
}

// Every rank returns once all `world` ranks have called it (for this generation); a rank that
// waits longer than timeout_s seconds (a peer died) gets BPRMF_E_STATE and poisons the barrier:
// its arrival is still in `count`, so a later generation could release one rank early.  Every
// wait on a poisoned barrier (this rank's or a peer's, also one already spinning) fails at once;
// recreate the mapping to go on.
int bprmf_node_barrier_wait(void* h, double timeout_s) {
  auto* b = static_cast<NodeBarrier*>(h);
  if (!b || !b->s) return fail(BPRMF_E_INVALID, "null barrier");
  Shared* s = b->s;
  if (s->broken.load(std::memory_order_acquire))
    return fail(BPRMF_E_STATE, "node barrier: poisoned by an earlier timeout (recreate it)");
  const int32_t g = s->gen.load(std::memory_order_acquire);
  if (s->count.fetch_add(1, std::memory_order_acq_rel) + 1 == b->world) {
    s->count.store(0, std::memory_order_relaxed);  // before the release below: the next
    s->gen.fetch_add(1, std::memory_order_release);  // generation starts from zero
    return 0;
  }
  const double t0 = now_s();
  for (uint32_t spin = 1; s->gen.load(std::memory_order_acquire) == g; ++spin) {
    __builtin_ia32_pause();
    if ((spin & 4095) == 0) {
      if (s->broken.load(std::memory_order_acquire))
        return fail(BPRMF_E_STATE, "node barrier: poisoned by a peer's timeout");
      if (timeout_s > 0 && now_s() - t0 > timeout_s) {
        s->broken.store(1, std::memory_order_release);
        return fail(BPRMF_E_STATE, "node barrier: a rank did not arrive within %g s", timeout_s);
      }
    }
  }
  return 0;
}

int bprmf_node_barrier_close(void* h) {
  auto* b = static_cast<NodeBarrier*>(h);
  if (!b) return 0;
  if (b->s) munmap(b->s, kBarrierBytes);
  delete b;
  return 0;
}

}  // extern "C"
