/*
 * bprfm.h — C ABI of the MI355X BPR-FM training path (libbprmf_amd.so), SURVEY.md §8f row 4: the
 * reference's factorization-machine variant of BPR.
 *
 * Drop-in boundary (NotFoundGG/recommend-lib):
 *   BPRFM(num_features, num_factors, batch_norm, drop_prob)   BPRFMRecommender.py:28-53
 *   forward(features_i, values_i, features_j, values_j)        BPRFMRecommender.py:55-79
 *   the training loop: zero_grad / forward / -log sigmoid(pred_i - pred_j).sum() / backward /
 *   Adagrad(lr, initial_accumulator_value=1e-8).step()          BPRFMRecommender.py:196-227
 *   the triplets: BPRFMData.ng_sample / __getitem__              util/data_loader.py:574-627
 *
 * A triplet is three FEATURE indices (u, i, j): side i is the feature pair [u, i], side j is
 * [u, j], every feature value 1 — the only shape BPRFMData produces.  One bprfm_train call runs
 * the reference's inner loop over caller-ordered triplets (the DataLoader's shuffle is the
 * caller's) in batches of batch_size (the last one smaller, as drop_last=False): per batch one
 * forward of both sides (BatchNorm1d in training mode per side, Dropout(drop_prob)), the BPR loss,
 * its gradients and one Adagrad step over every parameter.  Dropout draws come from a
 * counter-based stream (seed, step, triplet, side, factor) instead of torch's generator;
 * bprfm_dropout_mask returns them so a checker can replay a step exactly.
 * Arithmetic is float32 like the reference; reductions over the batch are fixed-order (BatchNorm
 * statistics, dgamma/dbeta, the loss), the embedding-gradient scatter uses float atomics.
 * Conventions are those of bprmf.h: 0 = OK, negative bprmf_status, bprmf_last_error() for the
 * message; host buffers caller-owned, row-major; one host thread per handle.
 */
#ifndef BPRFM_H
#define BPRFM_H

#include <stdint.h>

#include "bprmf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bprfm_handle bprfm_handle;

typedef struct {
  int64_t num_features; /* rows of embeddings / biases (:42-43) */
  int32_t num_factors;  /* embedding width (:42; --hidden_factor, default 64), 1..64 */
  int32_t batch_norm;   /* FM_layers starts with BatchNorm1d(num_factors) (:47-48) */
  float drop_prob;      /* Dropout(drop_prob[0]) (:49; default 0.5), 0 <= p < 1 */
  float lr;             /* Adagrad learning rate (:146-149, :196-198; default 0.05) */
  float init_std;       /* nn.init.normal_(embeddings, std=0.01) (:52) */
  int32_t max_batch;    /* largest batch a train call may use (--batch_size, default 4096) */
  uint64_t seed;        /* embedding init and dropout stream */
  int32_t device;
  int32_t reserved[3];
} bprfm_config;

typedef struct {
  int64_t triplets; /* triplets trained by the call */
  int64_t steps;    /* optimizer steps of the call */
  double loss;      /* sum over the call's batches of the reference's loss (:225) */
  double seconds;   /* device time of the call */
} bprfm_stats;

/* BPRFM(...) + Adagrad(...): embeddings ~ N(0, init_std^2), biases 0, bias_ 0, BatchNorm weight 1,
 * bias 0, running mean 0, running var 1; Adagrad accumulators 1e-8 */
int bprfm_create(const bprfm_config* cfg, bprfm_handle** out);
int bprfm_destroy(bprfm_handle* h);
/* load_state_dict: embeddings [F, k], biases [F], bias_ [1], BatchNorm weight / bias / running
 * mean / running var [k] (null: keep) */
int bprfm_set_weights(bprfm_handle* h, const float* embeddings, const float* biases,
                      const float* bias_, const float* bn_weight, const float* bn_bias,
                      const float* running_mean, const float* running_var);
int bprfm_get_weights(bprfm_handle* h, float* embeddings, float* biases, float* bias_,
                      float* bn_weight, float* bn_bias, float* running_mean, float* running_var);
/* one pass of the training loop (:211-227) over n triplets (feature indices) in the given order,
 * batch_size (<= max_batch) per optimizer step; feature ids out of range fail with
 * BPRMF_E_RANGE before anything runs */
int bprfm_train(bprfm_handle* h, const int32_t* u, const int32_t* i, const int32_t* j, int64_t n,
                int32_t batch_size, bprfm_stats* st);
/* the dropout keep-scales (0 or 1/(1-p)) the NEXT optimizer step draws for a batch of B:
 * out [2 sides, B, k] */
int bprfm_dropout_mask(bprfm_handle* h, int32_t B, float* out);
/* model.eval() forward of one side (:61-79): pred for n feature pairs [u, x] (running statistics,
 * no dropout) */
int bprfm_predict(bprfm_handle* h, const int32_t* u, const int32_t* x, int64_t n, float* out);
/* optimizer steps taken so far (BatchNorm num_batches_tracked = 2 x this when batch_norm) */
int64_t bprfm_steps(const bprfm_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* BPRFM_H */
