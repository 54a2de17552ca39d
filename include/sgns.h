/*
 * sgns.h — C ABI of the MI355X Item2Vec training path (libbprmf_amd.so), SURVEY.md §8f row 4:
 * skip-gram with negative sampling over the users' item sequences.
 *
 * Drop-in boundary (NotFoundGG/recommend-lib):
 *   Item2Vec(vocab_size, embedding_size, padding_idx=0)      Item2VecRecommender.py:39-68
 *   SGNS(embedding, vocab_size, n_negs, weights).forward     Item2VecRecommender.py:70-97
 *   optim.Adam(sgns.parameters()) and the training loop       Item2VecRecommender.py:272-291
 *   the corpus: BuildCorpus / PermutedSubsampledCorpus        util/data_loader.py:1118-1189
 *
 * One sgns_train call runs the loop's inner body over caller-ordered examples (the DataLoader's
 * shuffle is the caller's) in batches of batch_size, the last one smaller: the reference's loss
 * (mean over the batch of the context and negative log-sigmoid terms), its gradients and one
 * Adam step over both tables — dense, as torch does it: every row that has ever had a gradient
 * moves with its moments each step.  Negatives are drawn on the device like the reference's
 * (uniform integers in [0, V - 2], or with probability weights^0.75 / sum after sgns_set_noise)
 * from a counter-based stream; a caller may pass its own negatives instead, e.g. to replay the
 * reference's draws.  float32.  Row 0 is the embeddings' padding_idx and gets no gradient.
 * Conventions are those of bprmf.h: 0 = OK, negative bprmf_status, bprmf_last_error() for the
 * message; host buffers caller-owned, row-major; one host thread per handle.
 */
#ifndef SGNS_H
#define SGNS_H

#include <stdint.h>

#include "bprmf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sgns_handle sgns_handle;

typedef struct {
  int64_t vocab_size;     /* rows of ivectors / ovectors (len(idx2item)) */
  int32_t embedding_size; /* --e_dim (default 300), 1..1024 */
  int32_t n_negs;         /* --n_negs (default 20) */
  int32_t context;        /* context words per example: 2 x --window (default 10);
                             context x (1 + n_negs) <= 1024 */
  int32_t max_batch;      /* largest batch a train call may use (--mb, default 4096) */
  float lr, beta1, beta2, eps; /* optim.Adam defaults: 1e-3, 0.9, 0.999, 1e-8 */
  uint64_t seed;          /* table init and negative draws */
  int32_t device;
  int32_t reserved[3];
} sgns_config;

typedef struct {
  int64_t examples; /* examples trained by the call */
  int64_t steps;    /* optimizer steps of the call */
  double loss;      /* sum over the call's batches of the reference's loss (:97) */
  double seconds;   /* device time of the call */
} sgns_stats;

/* Item2Vec(...) + Adam(...): row 0 zeros, the rest uniform(-0.5/E, 0.5/E) (:46-53); Adam step 0 */
int sgns_create(const sgns_config* cfg, sgns_handle** out);
int sgns_destroy(sgns_handle* h);
/* SGNS(weights=...): negatives with probability weights^0.75 / sum (:77-80); null: uniform */
int sgns_set_noise(sgns_handle* h, const double* weights);
/* ivectors.weight / ovectors.weight [V, E] (null: keep) */
int sgns_set_weights(sgns_handle* h, const float* ivectors, const float* ovectors);
int sgns_get_weights(sgns_handle* h, float* ivectors, float* ovectors);
/* Adam state (optimizer.state_dict(): step, exp_avg, exp_avg_sq per table; the --conti resume,
 * :266-275).  Rows whose moments are all zero count as never updated. */
int sgns_set_adam(sgns_handle* h, int64_t step, const float* m_i, const float* v_i,
                  const float* m_o, const float* v_o);
int sgns_get_adam(sgns_handle* h, int64_t* step, float* m_i, float* v_i, float* m_o, float* v_o);
/* the loop body (:282-286) over n examples: iwords [n], owords [n, context], nwords
 * [n, context * n_negs] or null (drawn on the device); ids out of range fail with
 * BPRMF_E_RANGE before anything runs */
int sgns_train(sgns_handle* h, const int32_t* iwords, const int32_t* owords, const int32_t* nwords,
               int64_t n, int32_t batch_size, sgns_stats* st);
/* the negatives the NEXT optimizer step draws for a batch of B: out [B, context * n_negs] */
int sgns_negatives(sgns_handle* h, int32_t B, int32_t* out);
/* forward_i / forward_o (:60-68): rows of ivectors (which 0) or ovectors (1) for n ids,
 * out [n, E] */
int sgns_lookup(sgns_handle* h, int32_t which, const int32_t* idx, int64_t n, float* out);

#ifdef __cplusplus
}
#endif

#endif /* SGNS_H */
