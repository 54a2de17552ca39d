// handle.h — the bprmf_handle behind include/bprmf.h and the host helpers shared by capi.cpp
// (single-GPU training, weights, scoring) and dist.cpp (the sharded multi-GPU runner).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <string>
#include <utility>
#include <vector>

#include "../../include/bprmf.h"
#include "kernels.h"
#include "status.h"

namespace bprmf {

#define HIPCHK(x)                                                                           \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return bprmf::fail(BPRMF_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// position-independent step graphs (launch_step_graph): a graph of n steps runs the batches and
// optimizer steps the device cursor d_tbase = {t, k} names, then (advancing variant) advances it
// by n; a chunk is whole 64- and 16-step graphs plus fewer than 16 eagerly launched steps, so no
// chunk length or offset ever triggers a capture after the first
constexpr int64_t kGraphSizes[] = {64, 16};
constexpr int kGraphSizeKinds = 2;
constexpr int kGraphKinds = 2 * kGraphSizeKinds;  // each size with and without the advance
struct StepGraph {
  int64_t n = 0;         // steps per replay
  bool advance = false;  // ends by advancing the cursor (a later graph of the chunk follows)
  hipGraphExec_t exec = nullptr;
};
constexpr int kProfStride = 16;  // profiling: time the kernels of every 16th step

struct DistState;  // dist.cpp: the sharded runner's transport, plan and exchange buffers
void dist_free(DistState* d);
// semantics LOCAL at world > 1 (dist.cpp): the item table on every rank (not sharded)
// (BPRMF_DP_ONE_RANK=1, a test hook: a one-rank world of LOCAL handles also merges through the
// transport, so the one-GPU test box runs the RCCL all-reduce path: tests/test_gpu_local_dp.py)
inline bool dp_items(const bprmf_config& c) {
  if (c.semantics != BPRMF_SEM_LOCAL) return false;
  if (c.world > 1) return true;
  const char* e = getenv("BPRMF_DP_ONE_RANK");
  return e && e[0] == '1';
}
// an all-reduce a failed call left in flight (dp_overlap) is waited for and dropped
int dp_quiesce(bprmf_handle* h);

}  // namespace bprmf

struct bprmf_handle {
  bprmf_config cfg;
  bprmf::Geom geom;
  bprmf::Hyper hp;
  int64_t U = 0, I = 0;  // local rows
  bprmf::Table P{}, Q{};
  // training data
  int64_t npos = 0;
  int32_t* d_pos_u = nullptr;
  int32_t* d_pos_i = nullptr;
  int64_t* d_indptr = nullptr;
  int32_t* d_indices = nullptr;
  int64_t* d_soff = nullptr;    // the sampler's search trees (host_plan.h SearchTree)
  int32_t* d_skeys = nullptr;
  int2* d_pos2 = nullptr;       // {pos_u, pos_i} interleaved (the sampler's packed reads)
  int2* d_urec = nullptr;       // per local user {first tree key, positive count}
  int4* d_pos4 = nullptr;       // large positive sets: {pos_u, pos_i, urec of the user} per positive
  uint32_t feistel_a = 1, feistel_c = 1;  // permute's domain Z_a x Z_c (feistel_dims)
  uint32_t k0 = 0, k1 = 0;  // shard sampler key
  // triplet chunk
  int32_t* d_trip = nullptr;  // [3, cap]
  // segmented step (batch_size <= kMaxSegBatch): per-batch sorted layouts + per-triplet c*P_u
  int32_t* d_batch = nullptr;  // batch_cap * BatchBuf::stride_for(B) int32
  int64_t batch_cap = 0;
  float* d_contrib = nullptr;  // [2][B, ld] c*P_u per triplet (K1 -> K2), halves by step parity
  float* d_ugrad = nullptr;    // [2][B, ld] user gradient per triplet of multi-triplet users
  float* d_xloss = nullptr;    // [2][B] x per triplet (K1 -> K2's loss workgroups)
  int32_t* d_pend_q = nullptr;  // [2][I] step that last marked an item row (fused step)
  int32_t* d_pend_p = nullptr;  // [2][U] the same for user rows K2 finishes
  int32_t semantics = BPRMF_SEM_EXACT;  // cfg.semantics (BPRMF_SEM_HOGWILD / LOCAL: hogwild.hip)
  // BPRMF_SEM_LOCAL: the hot items' per-XCD replicas (hogwild.hip k_local_merge)
  int32_t* d_hot = nullptr;       // [I] replica slot of an item, -1 = cold
  uint32_t* d_hbits = nullptr;    // large catalogues: [I / 32] hot bit per item ...
  int2* d_hhash = nullptr;        // ... and [2^hot_hlog] {item, slot} of the hot items
  int hot_hlog = 0;
  int32_t* d_hot_rows = nullptr;  // [H] item of each slot
  float* d_qrep = nullptr;        // [kLocalXcds][H][ld]
  int64_t hot_H = 0;
  int32_t rep_t = 0;              // the step every replica row is current at (the last merge)
  int32_t local_steps = 128;      // steps per period (cfg.local_steps)
  // BPRMF_SEM_LOCAL at world > 1 (dist.cpp dp_merge): the whole item table on every rank, merged
  // across ranks every dp_steps steps and at the end of every call
  float* d_qbase = nullptr;  // [I][ld] the table at the last merge (current at dp_t)
  float* d_qdelta = nullptr; // [I][ld] this rank's change since then (the all-reduce's buffer)
  int32_t dp_t = 0;             // the step qbase is current at
  int32_t dp_steps = 256;
  // cfg.dp_overlap: a merge's all-reduce runs beside the next period; its sum (dp_sum, in d_qsum
  // or the transport's scratch) is added at the next merge, and d_qdelta keeps this rank's part
  bool dp_overlap = false;
  bool dp_mode = false;         // dp_items(cfg) at create: the item merges run (dist.cpp)
  bool dp_pending = false;      // an all-reduce was started at step dp_tp and not applied yet
  int32_t dp_tp = 0;
  const float* dp_sum = nullptr;
  float* d_qsum = nullptr;      // [I][ld] the overlapped all-reduce's result (RCCL, out of place)
  bool fused = true;           // chunks run K1, fused K2+K1 launches, K2 (BPRMF_FUSED=0: K1+K2 pairs)
  int32_t* d_tbase = nullptr;  // step cursor {t, batch}: t before the chunk (kernels read it here)
  int64_t plan_steps = 0;      // batches of the current sharded plan
  int64_t trip_cap = 0;
  // misc device scalars
  // device status block: {int32 err, pad, double loss[kLossSlots]} (one copy back per call)
  unsigned char* d_status = nullptr;
  unsigned char* h_status = nullptr;      // pinned, mapped host mirror
  unsigned char* h_status_dev = nullptr;  // its device address (k_status_out writes there)
  uint64_t status_seq = 0;                // sequence number of the last call's status block
  double* d_loss = nullptr;               // = d_status + 16
  int32_t* d_err = nullptr;               // = d_status
  bool loss_pending = false;    // a call began: the loss slots are zeroed before the first step
  bool slots_dirty = true;      // slots past 0 may hold values (the f32-atomic path uses them)
  bool call_slots = false;      // this call's loss is spread over every slot (atomic path)
  double call_t0 = 0;           // host clock at begin_call (stats.seconds)
  int32_t t = 0;  // optimizer steps taken
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // live per-kernel timing (bprmf_profile): event pairs around each launch of each kind
  bool prof_on = false;
  std::vector<hipEvent_t> prof_pool;
  size_t prof_used = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_rec[BPRMF_KPROF_KINDS];
  int64_t prof_weight[BPRMF_KPROF_KINDS] = {};  // extra units per pair (a step-graph pair = nb steps)
  // captured step sequences (BPRMF_NO_GRAPH=1 disables: eager launches)
  bool use_graphs = true;
  std::vector<bprmf::StepGraph> graphs;
  // sharded runner (bprmf_dist_init*), null until a transport is attached
  bprmf::DistState* dist = nullptr;
};

namespace bprmf {

int set_dev(bprmf_handle* h);
template <typename T>
int dalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return 0;
  HIPCHK(hipMalloc((void**)p, sizeof(T) * (size_t)count));
  return 0;
}
hipEvent_t prof_event(bprmf_handle* h);
// record an event before (begin) / after a launch of `kind` when profiling is on
struct ProfScope {
  bprmf_handle* h;
  int kind;
  hipEvent_t a = nullptr;
  ProfScope(bprmf_handle* hh, int k, bool sampled = true) : h(hh), kind(k) {
    if (h->prof_on && sampled && (a = prof_event(h))) (void)hipEventRecord(a, h->stream);
  }
  ~ProfScope() {
    if (!a) return;
    hipEvent_t b = prof_event(h);
    if (!b) return;
    (void)hipEventRecord(b, h->stream);
    h->prof_rec[kind].push_back({a, b});
  }
};
int ensure_trip(bprmf_handle* h, int64_t n);
int ensure_seg(bprmf_handle* h, int64_t n_batches);
StepBufs step_bufs(const bprmf_handle* h);    // the single-GPU step buffers (both halves, pend)
LocalArgs local_args(const bprmf_handle* h);  // semantics LOCAL: hot items, replicas, lookups
int ensure_grad(bprmf_handle* h);
bool seg_mode(const bprmf_handle* h);
// a sampled chunk of nb batches draws its triplets with the grid-wide sampler before the builder
bool split_build(int64_t nb);
int64_t dist_chunk_steps(const bprmf_handle* h);  // steps per chunk of the sharded runner
int check_err_flag(bprmf_handle* h);
SamplerArgs sampler_args(bprmf_handle* h);
int read_loss(bprmf_handle* h, double* loss);
// loss slots the first launch of a call must zero (0 once done for this call)
int loss_zero_slots(bprmf_handle* h);
int begin_call(bprmf_handle* h);
int end_call(bprmf_handle* h, bprmf_stats* st, int64_t triplets, int64_t steps);
// mapped status block: byte offsets of the two call sequence words (end_call, the sharded
// runner's capacity read-back)
constexpr size_t kSeqEndOff = 16 + sizeof(double) * kLossSlots;
constexpr size_t kSeqCapOff = kSeqEndOff + 8;
// spin until a kernel has stored seq into the mapped word at byte offset `off` of h_status (a
// blocking stream sync wakes up tens of microseconds later); synchronise the stream instead if
// it ends or fails without that store
int wait_mapped_seq(bprmf_handle* h, size_t off, uint64_t seq);

}  // namespace bprmf
