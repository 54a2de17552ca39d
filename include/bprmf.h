/*
 * bprmf.h — C ABI of the MI355X-native BPR-MF training path (libbprmf_amd.so).
 *
 * Drop-in boundary for the reference's BPR-MF path (NotFoundGG/recommend-lib):
 *   model      BPRMFRecommender.py:28-50   class BPR(nn.Module): two nn.Embedding tables, forward()
 *   step       BPRMFRecommender.py:172-176 zero_grad / forward / -(x).sigmoid().log().sum() / SGD(wd)
 *   sampler    util/data_loader.py:667-700 BPRData.ng_sample / __getitem__ -> (u, i, j)
 *   surface    util/matrix_factorization.pyx:81-167 fit()/predict() convention (ValueError on bad ids)
 * The reference has no FFI; a maintainer binds these symbols with ctypes.
 *
 * Conventions
 *   - every function returns 0 (BPRMF_OK) or a negative bprmf_status; bprmf_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - host buffers are caller-owned; the library owns device memory.  `_dev` functions take device
 *     pointers (e.g. torch tensors' data_ptr()) and run on the handle's stream (bprmf_set_stream).
 *   - a handle is not thread-safe: one host thread per handle.  One handle per GPU / process.
 *   - tables are row-major fp32 [rows, factor_num] at the ABI (device rows are padded internally).
 *   - weight decay is applied lazily: get_weights/score see the exact dense-decay values.
 */
#ifndef BPRMF_H
#define BPRMF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  BPRMF_OK = 0,
  BPRMF_E_INVALID = -1,     /* bad argument (ValueError in the reference surface) */
  BPRMF_E_RANGE = -2,       /* user/item id out of range (IndexError / 'Invalid user code') */
  BPRMF_E_HIP = -3,         /* HIP runtime error */
  BPRMF_E_STATE = -4,       /* call order (e.g. train before set_train) */
  BPRMF_E_NO_NEGATIVE = -5, /* a user has every item as positive: ng_sample would never end */
  BPRMF_E_UNSUPPORTED = -6
} bprmf_status;

/* Step semantics.  EXACT: every step reads the tables as the previous step left them, duplicate
 * rows' gradients are summed (BPRMFRecommender.py:172-176), bitwise reproducible.  HOGWILD:
 * each triplet is applied on its own as soon as its rows arrive, lock-free (concurrent updates
 * of a row may overwrite each other), weight decay still once per row per step; staleness is
 * bounded by the launch's in-flight window.  Single-GPU handles only. */
enum { BPRMF_SEM_EXACT = 0, BPRMF_SEM_HOGWILD = 1, BPRMF_SEM_LOCAL = 2, BPRMF_SEM_STALE1 = 3 };
/* STALE1 (opt-in, the sharded runner only: bprmf_dist_train_*): the exact sharded step with the
 * item rows one step stale.  Step k's gradient exchange and the owners' apply run beside step
 * k+1's compute (transports rccl / loopback: on a second stream; ipc, one rank per GPU or
 * BPRMF_DIST_FUSE=1: inside the next step's launch, ordered by device flags), so the rows step t
 * reads are the table after step t-2 brought to step t-1 by weight decay alone (they miss step
 * t-1's gradients); users stay exact; the first step of every runner chunk reads the current
 * table.  Spec: oracle/bpr_oracle.py sharded_stale1_serial. */
/* LOCAL (bounded staleness, opt-in): HOGWILD for users and for all but the most popular items;
 * the hot items (the top min(I, 4096) by positive count) are trained in one replica per XCD of the
 * GPU (each XCD's waves see their own XCD's updates at once, the other XCDs' only at the next
 * merge), and every `local_steps` steps (default 128) the replicas are merged: new = decayed base +
 * sum over XCDs of each replica's change.  Staleness across XCDs is bounded by `local_steps`
 * steps.
 * LOCAL at world > 1 (data-parallel items): users stay sharded (u % world == rank, each rank
 * samples only its own users' positives) but every rank holds the WHOLE item table and trains it
 * as above; every `dp_steps` steps (default 256) and at the end of every call the ranks' item
 * tables are merged: new = decayed base + sum over ranks of each rank's change since the last
 * merge (one all-reduce of the table: RCCL's, the IPC transport's reduce-scatter + all-gather
 * pushes, or the loopback's).  Staleness across GPUs is bounded by `dp_steps` steps (§5d).
 * dp_overlap = 1: the all-reduce of a merge runs on a side stream while the next period trains;
 * its sum is added one period later (the other ranks' changes arrive up to 2 dp_steps late);
 * the last merge of every call is blocking, so every rank ends a call with the same table.
 * Footprint per rank at world > 1: the item table 5-6 times (Q, merge base, delta, the overlap's
 * sum, the IPC transport's two exported buffers) plus the hot items' XCD replicas; bprmf_create
 * refuses with BPRMF_E_UNSUPPORTED when that exceeds the device's free memory.  The per-step
 * sharded calls (bprmf_dist_plan*, _gather_items, _apply_items, _user_step, _item_grads) address
 * items by owner and refuse this mode; the runner (bprmf_dist_train_*) runs it. */

/* How an EXACT step sums duplicate rows' gradients ("ship both").  SEGMENTED: the
 * batch is sorted by user and by item and every row is summed by one writer in a fixed order,
 * bitwise reproducible (batch_size <= 8192; the sharded runner needs it).  ATOMIC: f32 atomics
 * into per-row gradient accumulators, then one pass applies every touched row; any batch size,
 * the same step up to the order of the fp32 sums (not bitwise reproducible).  Larger batches
 * than 8192 always take ATOMIC. */
enum { BPRMF_STEP_SEGMENTED = 0, BPRMF_STEP_ATOMIC = 1 };

typedef struct {
  int64_t user_num;     /* rows of embed_user  (BPRMFRecommender.py:36) — global count */
  int64_t item_num;     /* rows of embed_item  (BPRMFRecommender.py:37) — global count */
  int32_t factor_num;   /* --factor_num        (BPRMFRecommender.py:78-81) */
  float lr;             /* --lr                (BPRMFRecommender.py:58-61) */
  float weight_decay;   /* --wd                (BPRMFRecommender.py:62-65, SGD weight_decay :154) */
  int32_t batch_size;   /* --batch_size        (BPRMFRecommender.py:66-69), per process */
  int32_t num_ng;       /* --num_ng            (BPRMFRecommender.py:82-85) */
  float init_std;       /* nn.init.normal_(std=0.01) (BPRMFRecommender.py:39-40) */
  uint64_t seed;        /* seeds init, sampler and shuffle (the reference is unseeded) */
  int32_t device;       /* HIP device ordinal */
  int32_t rank;         /* shard of this handle: owns users u%world==rank, items i%world==rank
                           (BPRMF_SEM_LOCAL: every item, see above) */
  int32_t world;        /* 1 for a single GPU */
  int32_t semantics;    /* BPRMF_SEM_EXACT (0, default): the reference's batch-synchronous step;
                           BPRMF_SEM_HOGWILD (1): opt-in relaxed synchronisation, see below */
  int32_t step_mode;    /* BPRMF_STEP_SEGMENTED (0, default) or BPRMF_STEP_ATOMIC (1), single GPU */
  int32_t local_steps;  /* BPRMF_SEM_LOCAL: steps between replica merges (0: 128) */
  int32_t dp_steps;     /* BPRMF_SEM_LOCAL, world > 1: steps between the ranks' item merges (0: 256) */
  int32_t dp_overlap;   /* BPRMF_SEM_LOCAL, world > 1: 1 = each merge's all-reduce runs beside the
                           next period (its result lands one period later), 0 = blocking merges */
} bprmf_config;

typedef struct {
  int64_t triplets;     /* triplets processed by the call */
  int64_t steps;        /* optimizer steps taken by the call */
  double loss;          /* sum over the call of -log(sigmoid(pred_i - pred_j)) (BPRMFRecommender.py:174) */
  double seconds;       /* HOST wall-clock time of the call, from entry to the status read that
                           ends it: host launch and capture time, the final wait, and any work
                           already queued on a shared caller stream are included.  Device time
                           per kernel kind: bprmf_profile / bprmf_profile_read (HIP events). */
} bprmf_stats;

/* live kernel timing (HIP events around every launch of each kind while enabled) */
/* kinds: sample/build, step kernel 1 (users), step kernel 2 (items), owner-side item update,
 * whole steps replayed from a captured graph (count = steps, ms = their summed device time), and
 * full-catalogue top-k launches */
enum {
  BPRMF_KPROF_SAMPLE = 0,
  BPRMF_KPROF_FWD_SCATTER = 1,
  BPRMF_KPROF_APPLY = 2,
  BPRMF_KPROF_OWNER = 3,
  BPRMF_KPROF_STEPS = 4,
  BPRMF_KPROF_TOPK = 5,
  BPRMF_KPROF_KINDS = 6
};
typedef struct {
  int64_t count[8];     /* launches (steps for BPRMF_KPROF_STEPS) recorded per kind */
  double ms[8];         /* summed device time per kind (ms) */
} bprmf_kprof;

typedef struct bprmf_handle bprmf_handle;

/* ---- lifecycle ---------------------------------------------------------------------------- */
/* replaces BPR.__init__ + optim.SGD(...) (BPRMFRecommender.py:29-40,148-154) */
int bprmf_create(const bprmf_config* cfg, bprmf_handle** out);
int bprmf_destroy(bprmf_handle* h);
const char* bprmf_last_error(void);
int bprmf_version(void);
/* Run on this hipStream_t (NULL = the handle's own stream). */
int bprmf_set_stream(bprmf_handle* h, void* hip_stream);
int bprmf_synchronize(bprmf_handle* h);

/* ---- input -------------------------------------------------------------------------------- */
/* Train positives in features order (load_mat train list + dok train_mat, util/data_loader.py:
 * 538-545; BPRData.__init__ :668-678).  Global ids; a sharded handle keeps its own users' rows. */
int bprmf_set_train(bprmf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz);
/* Same, with extra (user, item) pairs that are never drawn as negatives: the keys of a train_mat
 * that holds more than `features` (BPRData(features, num_item, train_mat), data_loader.py:668). */
int bprmf_set_train_ex(bprmf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz,
                       const int32_t* ex_users, const int32_t* ex_items, int64_t n_ex);
/* Triplets and steps of one epoch of this handle (BPRData.__len__ :692-693, DataLoader len). */
int bprmf_epoch_size(bprmf_handle* h, int64_t* n_triplets, int64_t* n_steps);

/* ---- weights (checkpoint / parity) -------------------------------------------------------- */
/* embed_user.weight / embed_item.weight (BPRMFRecommender.py:36-37); [rows, factor_num] fp32.
 * Sharded handles: P holds local users (global id = local*world + rank), Q local items likewise. */
int bprmf_set_weights(bprmf_handle* h, const float* P, const float* Q);
int bprmf_get_weights(bprmf_handle* h, float* P, float* Q);
int bprmf_local_rows(bprmf_handle* h, int64_t* users, int64_t* items);
/* Rows of one table as of the current step (the pending weight decay applied on the way out; the
 * table itself is not flushed): table 0 = embed_user, 1 = embed_item; rows are local row ids
 * (global id / world); out [n, factor_num] fp32.  The embedding lookup of BPR.forward
 * (BPRMFRecommender.py:45-47) for callers that need the vectors, not the scores, and the way to
 * read a table too large to copy whole (C5: 112.6 GB). */
int bprmf_get_rows(bprmf_handle* h, int32_t table, const int32_t* rows, int64_t n, float* out);
int bprmf_step_count(bprmf_handle* h, int64_t* steps);

/* ---- training ----------------------------------------------------------------------------- */
/* One epoch: ng_sample() on device + the shuffled DataLoader + steps
 * (BPRMFRecommender.py:157-178, util/data_loader.py:680-690). */
int bprmf_train_epoch(bprmf_handle* h, uint32_t epoch, bprmf_stats* stats);
/* Steps [first_step, first_step+n_steps) of an epoch (bench / resumable training). */
int bprmf_train_steps(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                      bprmf_stats* stats);
/* Replay reference-format triplets in order, batch_size per step (last batch partial):
 * the `for user, item_i, item_j in train_loader` body, BPRMFRecommender.py:162-176. */
int bprmf_train_triplets(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                         int64_t n, bprmf_stats* stats);
int bprmf_train_triplets_dev(bprmf_handle* h, const int32_t* u, const int32_t* i,
                             const int32_t* j, int64_t n, bprmf_stats* stats);

/* ---- sampler (exposed for bit-exact tests) ------------------------------------------------ */
/* Triplet slots [first, first+n) of `epoch` in shuffled order -> (u, i, j), global ids. */
int bprmf_sample(bprmf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u,
                 int32_t* i, int32_t* j);

/* ---- scoring ------------------------------------------------------------------------------ */
/* pred = <P_u, Q_i> (BPR.forward, BPRMFRecommender.py:42-50; predict() convention
 * util/matrix_factorization.pyx:157-167).  Single-GPU handles only. */
int bprmf_score(bprmf_handle* h, const int32_t* u, const int32_t* i, int64_t n, float* out);
/* forward(user, item_i, item_j) on device int64 ids -> pred_i, pred_j (device fp32). */
int bprmf_forward_dev(bprmf_handle* h, const int64_t* u, const int64_t* i, const int64_t* j,
                      int64_t n, float* pred_i, float* pred_j);

/* ---- ranking ------------------------------------------------------- */
/* Per user r: score its candidates items[offsets[r] .. offsets[r+1]) as bprmf_score does and
 * return the positions (within the list) of the k best, score descending, ties by the later
 * position first (np.argsort(pred)[::-1][:k], BPRMFRecommender.py:196-207; torch.topk of
 * util/metrics.py:53-54); -1 / -inf past the list's end.  out_pos, out_score: [n_users, k]. */
int bprmf_topk_lists(bprmf_handle* h, const int32_t* users, const int64_t* offsets,
                     const int32_t* items, int64_t n_users, int32_t k, int32_t* out_pos,
                     float* out_score);

/* Per user: the k best items of the WHOLE catalogue (the serving form of predict): scores on f32
 * MFMA (exact f32 products and sums, k-ordered fmaf chain), exclude_train != 0 skips the user's
 * training positives; score descending, ties by the smaller item; -1 / -inf when fewer remain.
 * factor_num <= 128, k <= 32.  out_items, out_scores: [n_users, k].  Like bprmf_get_weights,
 * it first brings both tables to the current step (applies the pending weight decay). */
int bprmf_topk_all(bprmf_handle* h, const int32_t* users, int64_t n_users, int32_t k,
                   int32_t exclude_train, int32_t* out_items, float* out_scores);

/* ---- measurement -------------------------------------------------------------------------- */
/* Enable (1) / disable (0) and reset per-kernel event timing; read the sums since enabling. */
int bprmf_profile(bprmf_handle* h, int32_t enable);
int bprmf_profile_read(bprmf_handle* h, bprmf_kprof* out);

/* ---- sharded steps (one process per GPU; the caller moves the buffers over RCCL) ---------- */
/* Users u live on rank u % world, items i on rank i % world (strided row sharding).  A step:
 *   request_ids -> [all-to-all ids] -> gather_items (owner) -> [all-to-all rows back]
 *   -> user_step (local users vs the received rows) -> item_grads (one row per requested item)
 *   -> [all-to-all grads to the owners] -> apply_items (owner) -> end_step.
 * Requests are owner-major: the first owner_counts[k][0] ids go to rank 0, and so on; ids are the
 * owner's LOCAL rows (item / world).  Device buffers have row stride bprmf_row_stride floats. */
/* Build steps [first_step, first_step+n_steps) of `epoch` for this shard (device sampler over its
 * own users; steps past the shard's epoch are empty) and copy the per-owner request counts
 * owner_counts[n_steps][world] to the host (the exchange sizes).  Replaces the previous plan. */
int bprmf_dist_plan(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                    int32_t* owner_counts);
/* Same from host triplets u/i/j[n_steps * batch_size] (global ids, this shard's users only;
 * u < 0 marks an empty slot): the replay form of BPRData batches. */
int bprmf_dist_plan_replay(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                           int64_t n_steps, int32_t* owner_counts);
int bprmf_dist_request_ids(bprmf_handle* h, int64_t step, int32_t* ids, int64_t n);
int bprmf_dist_gather_items(bprmf_handle* h, const int32_t* rows, int64_t n, float* out);
int bprmf_dist_user_step(bprmf_handle* h, int64_t step, const float* item_rows);
int bprmf_dist_item_grads(bprmf_handle* h, int64_t step, float* grads);
int bprmf_dist_apply_items(bprmf_handle* h, const int32_t* rows, const float* grads, int64_t n);
/* Advance the step counter; loss != NULL: loss since the last read (synchronises). */
int bprmf_dist_end_step(bprmf_handle* h, double* loss);
/* Device triplets (global ids) of slots [first, first+n) of the shard's epoch order. */
int bprmf_dist_sample_dev(bprmf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u,
                          int32_t* i, int32_t* j);
/* row stride (floats) of device row buffers used by the dist_* exchange functions */
int bprmf_row_stride(bprmf_handle* h, int32_t* ld);

/* ---- sharded runner: whole chunks of sharded steps driven by the library ------------------ */
/* The same step as the phases above, with the exchanges issued by the library: no host round
 * trip per step.  Transport: an RCCL communicator the handle owns (rank 0 makes the 128-byte
 * unique id, the caller broadcasts it, every rank calls bprmf_dist_init_rccl), or `loopback`:
 * handles of ONE process with the same group key exchange through device copies (tests; one host
 * thread per handle).  Steps are global: every rank runs the same (epoch, first_step, n_steps),
 * steps past a shard's own epoch are empty for it. */
int bprmf_dist_unique_id(uint8_t* id128);
int bprmf_dist_init_rccl(bprmf_handle* h, const uint8_t* id128);
/* IPC transport (one process per GPU, same node): phase 1 allocates the buffers peers write into
 * and returns their hipIpc handles in blob[BPRMF_IPC_BLOB_BYTES]; the caller all-gathers the
 * blobs (rank order); phase 2 maps every peer's buffers.  Exchanges are kernels writing straight
 * into the peers' memory over xGMI, completion by per-source flags (no host round trip). */
#define BPRMF_IPC_BLOB_BYTES 512
int bprmf_dist_ipc_export(bprmf_handle* h, uint8_t* blob);
int bprmf_dist_init_ipc(bprmf_handle* h, const uint8_t* blobs);
int bprmf_dist_init_loopback(bprmf_handle* h, int64_t group);
/* Steps [first_step, first_step+n_steps) of `epoch` from the device sampler (BPRMFRecommender.py:
 * 157-178 over this shard's users); stats: this shard's triplets and loss. */
int bprmf_dist_train_steps(bprmf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                           bprmf_stats* stats);
/* Bytes this rank sent to its peers since the transport was attached, as the transport moved
 * them (padded to each chunk's exchange capacity): item rows (owner -> requesters), gradients
 * (requester -> owners), request lists (once per chunk), and the steps they cover.  World 1
 * sends nothing (bprmf_dist_train_steps then runs the single-GPU step). */
int bprmf_dist_exchange_stats(bprmf_handle* h, int64_t* steps, int64_t* row_bytes,
                              int64_t* grad_bytes, int64_t* id_bytes);
/* Replay: u/i/j[n_steps * batch_size] host triplets (global ids, this shard's users; u < 0 marks
 * an empty slot), batch_size slots per step. */
int bprmf_dist_train_replay(bprmf_handle* h, const int32_t* u, const int32_t* i, const int32_t* j,
                            int64_t n_steps, bprmf_stats* stats);

/* ---- a barrier for the ranks of one node (host only; no reference counterpart) -------------
 * bench.py brackets its timed region with a barrier on every rank (the measurement contract); a
 * process group's barrier costs ~0.1 ms, the ranks of one node meet on two shared words of a
 * /dev/shm file instead (~1 us).  One rank opens it with create = 1, the others after it with 0
 * (same path and world); wait returns once every rank has called it, or BPRMF_E_STATE after
 * timeout_s seconds (<= 0: no limit). */
int bprmf_node_barrier_open(const char* path, int32_t world, int32_t rank, int32_t create, void** out);
int bprmf_node_barrier_wait(void* barrier, double timeout_s);
int bprmf_node_barrier_close(void* barrier);

/* ---- test hooks (no reference counterpart) ------------------------------------------------ */
/* The launch tag the next split batch build of this process will carry (segment.hip): the tests
 * use it to plant stale words that an unsafe tag scheme would mistake for this launch's. */
int bprmf_debug_next_build_tag(uint32_t* tag);
/* Fill every int32 of the handle's batch buffer with `value` (stale memory, deliberately). */
int bprmf_debug_fill_batches(bprmf_handle* h, int32_t value);
/* Leave the batch buffer as a timed-out split build would (every batch marked dead, err bit 16):
 * the next call's steps must skip every batch, leave the tables untouched and fail. */
int bprmf_debug_fail_build(bprmf_handle* h);

/* ---- ingestion: ratings files -> dense-coded rows (util/data_loader.py:27-146, :410-548) ---- */
/* Host-only (no GPU).  Lines "<user> <sep> <item> <sep> <rating> <sep> <timestamp>" with any
 * separator run ('\t' ml-100k u.data, '::' ml-1m/ml-10m ratings.dat, ',' ml-20m ratings.csv; a
 * header line is skipped).  Rows with rating >= min_rating are kept (load_rate :35/:39/:43: 4 for
 * ml-1m/10m/20m, 0 for ml-100k); core > 0 applies prepro='5core'/'10core' (:122-144, one pass:
 * rows whose user and item both have >= core ratings); rows are ordered by (user, item, timestamp)
 * (:118) and ids coded densely in ascending raw order (load_mat :447-448, pd.Categorical codes).
 * threads <= 0: all hardware threads. */
typedef struct bprmf_dataset bprmf_dataset;
enum { BPRMF_SPLIT_LOO_TIME = 0, BPRMF_SPLIT_FO_TIME = 1 };
int bprmf_dataset_load(const char* path, float min_rating, int32_t core, int32_t threads,
                       bprmf_dataset** out);
int bprmf_dataset_info(bprmf_dataset* d, int64_t* n, int64_t* user_num, int64_t* item_num);
/* any pointer may be NULL; users/items/ratings/timestamps [n], user_ids [user_num], item_ids
 * [item_num] (code -> raw id) */
int bprmf_dataset_copy(bprmf_dataset* d, int32_t* users, int32_t* items, float* ratings,
                       int64_t* timestamps, int64_t* user_ids, int64_t* item_ids);
/* is_test[n] per row: LOO_TIME = _split_loo(by_time=1) (:410-414, each user's latest row, ties to
 * the first in row order); FO_TIME = _split_fo(by_time=1) (:422-427, rows past the first
 * ceil(n (1 - test_frac)) in time order; equal timestamps in row order, where the reference
 * shuffles) */
int bprmf_dataset_split(bprmf_dataset* d, int32_t method, double test_frac, uint8_t* is_test);
/* Test lists (load_mat's test_data, :453-492) as (user, item) rows.  LOO_TIME: per user
 * ascending, the test item then `count` distinct items the user never rated, ascending
 * (_negative_sampling :430-439, count = 999; BPRMF_E_NO_NEGATIVE when fewer exist, as
 * random.sample raises).  FO_TIME: per test user in order of first test timestamp, the test items
 * plus never-rated candidates up to `count` in all (or `count` of the test items), ascending.
 * Draws are a function of (seed, user).  Call with users == NULL to get the row count in *n_out;
 * otherwise *n_out is the capacity in and the count out. */
int bprmf_dataset_candidates(bprmf_dataset* d, const uint8_t* is_test, int32_t method,
                             int32_t count, uint64_t seed, int64_t* n_out, int32_t* users,
                             int32_t* items);
int bprmf_dataset_free(bprmf_dataset* d);

#ifdef __cplusplus
}
#endif
#endif /* BPRMF_H */
