/*
 * ncf.h — C ABI of the MI355X-native NCF training path (libbprmf_amd.so), SURVEY.md §8f row 2.
 *
 * Drop-in boundary for the reference's NCF path (NotFoundGG/recommend-lib):
 *   model      NCFRecommender.py:27-124   class NCF(nn.Module): GMF / MLP / NeuMF-end, forward()
 *   step       NCFRecommender.py:278-285  zero_grad / forward / BCEWithLogitsLoss / backward /
 *                                         Adam(lr).step() (every parameter, dense gradients)
 *   sampler    util/data_loader.py:931-972 NCFData.ng_sample / __getitem__ -> (user, item, label)
 * Conventions are those of bprmf.h (0 = OK, negative bprmf_status; bprmf_last_error() for the
 * message; host buffers caller-owned; one host thread per handle).  Parameters are addressed in
 * the reference's state_dict order (ncf_param_shape): embed_user_GMF.weight,
 * embed_item_GMF.weight, embed_user_MLP.weight, embed_item_MLP.weight, then per tower layer
 * MLP_layers.{3l+1}.weight [out, in] and .bias, then predict_layer.weight [1, pred] and .bias.
 */
#ifndef NCF_H
#define NCF_H

#include <stdint.h>

#include "bprmf.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { NCF_NEUMF_END = 0, NCF_GMF = 1, NCF_MLP = 2 }; /* --model_name (NCFRecommender.py:182) */

typedef struct {
  int64_t user_num;   /* rows of the user embeddings (load_mat user_num) */
  int64_t item_num;   /* rows of the item embeddings */
  int32_t factor_num; /* --factor_num (NCFRecommender.py:155), a multiple of 4 */
  int32_t num_layers; /* --num_layers (:159), 1..4: tower widths 2E -> E -> ... -> factor_num */
  int32_t model;      /* NCF_NEUMF_END / NCF_GMF / NCF_MLP (NeuMF-pre: set trained weights) */
  int32_t batch_size; /* --batch_size (:143), <= 8192 */
  int32_t num_ng;     /* --num_ng (:163) negatives per positive */
  float lr;           /* --lr (:135), Adam */
  float beta1, beta2, eps; /* torch Adam defaults 0.9, 0.999, 1e-8 */
  float init_std;     /* nn.init.normal_(std=0.01) of the embeddings (:71-74) */
  uint64_t seed;      /* init, sampler and shuffle */
  int32_t device;
  int32_t reserved[4];
} ncf_config;

typedef struct ncf_handle ncf_handle;

/* replaces NCF.__init__ + optim.Adam (NCFRecommender.py:249-260) */
int ncf_create(const ncf_config* cfg, ncf_handle** out);
int ncf_destroy(ncf_handle* h);
/* parameters in state_dict order: count, shape, host copies in / out ([rows, cols] row-major) */
int ncf_param_count(ncf_handle* h, int32_t* n);
int ncf_param_shape(ncf_handle* h, int32_t index, int64_t* rows, int64_t* cols);
int ncf_set_param(ncf_handle* h, int32_t index, const float* data);
int ncf_get_param(ncf_handle* h, int32_t index, float* data);
/* train positives (NCFData features; train_mat keys are the rejection set, data_loader.py:945) */
int ncf_set_train(ncf_handle* h, const int32_t* users, const int32_t* items, int64_t nnz);
int ncf_epoch_size(ncf_handle* h, int64_t* samples, int64_t* steps);
/* one Adam step per batch_size samples of reference-format (user, item, label) in order
 * (the `for user, item, label in train_loader` body, NCFRecommender.py:271-285) */
int ncf_train_samples(ncf_handle* h, const int32_t* u, const int32_t* i, const float* y,
                      int64_t n, bprmf_stats* stats);
/* steps [first_step, first_step + n_steps) of `epoch` from the device sampler */
int ncf_train_steps(ncf_handle* h, uint32_t epoch, int64_t first_step, int64_t n_steps,
                    bprmf_stats* stats);
int ncf_train_epoch(ncf_handle* h, uint32_t epoch, bprmf_stats* stats);
/* the sampler's samples [first, first + n) of `epoch` (bit-exact tests) */
int ncf_sample(ncf_handle* h, uint32_t epoch, int64_t first, int64_t n, int32_t* u, int32_t* i,
               float* y);
/* NCF.forward(user, item) -> prediction logits (NCFRecommender.py:103-124) */
int ncf_predict(ncf_handle* h, const int32_t* u, const int32_t* i, int64_t n, float* out);
/* embedding rows Adam steps every step from now on: rows with a nonzero moment (ever touched).
 * (Their zero-gradient steps are applied lazily, in closed form, before anything reads them.) */
int ncf_active_rows(ncf_handle* h, int64_t* users, int64_t* items);
/* live timing (bprmf_kprof): kinds 0 sample, 1 forward/backward with the tower's Adam, 2 a call's
 * last row Adam, 3 the row launch (the previous step's row Adam + this step's catch-up) */
int ncf_profile(ncf_handle* h, int32_t enable);
int ncf_profile_read(ncf_handle* h, bprmf_kprof* out);

#ifdef __cplusplus
}
#endif
#endif /* NCF_H */
