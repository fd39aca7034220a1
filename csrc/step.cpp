// Host-side launcher of the fused local step.
//
// The Python engine passes one GfkModel (dims + raw device pointers) and one
// GfkAdam descriptor, and a list of phase ids; every kernel of the step is
// launched from here on the caller's HIP stream, so a whole minibatch step is
// a single ctypes call (eager mode) or a single hipGraph replay (graph mode,
// captured around this call).  No allocation, no synchronisation: the call is
// capture-safe.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gfk_common.h"

extern "C" {
int gfk_launch_enc_in(const GfkModel*, hipStream_t);
int gfk_launch_post_fwd(const GfkModel*, hipStream_t);
int gfk_launch_post_bwd(const GfkModel*, hipStream_t);
int gfk_launch_win_update(const GfkModel*, const GfkUpdate*, hipStream_t);
int gfk_launch_batch_docs(const GfkModel*, hipStream_t);
int gfk_launch_batch_prep(const GfkModel*, hipStream_t);
int gfk_launch_prodlda_fwd(const GfkModel*, hipStream_t);
int gfk_launch_prodlda_bwd(const GfkModel*, hipStream_t);
int gfk_launch_prodlda_row_loss(const GfkModel*, hipStream_t);
int gfk_launch_lda_beta_fwd(const GfkModel*, hipStream_t);
int gfk_launch_lda_row(const GfkModel*, hipStream_t);
int gfk_launch_lda_beta_bwd(const GfkModel*, hipStream_t);
int gfk_launch_adam(const GfkAdam*, int, hipStream_t);
int gfk_launch_scale(float*, int64_t, float, hipStream_t);
int gfk_launch_ctx_fwd(const GfkModel*, hipStream_t);
int gfk_launch_ctx_bwd(const GfkModel*, hipStream_t);
size_t gfk_ctx_smem(const GfkModel*);
int gfk_ctx_set_smem(size_t);
size_t gfk_prodlda_fwd_smem(const GfkModel*);
size_t gfk_prodlda_bwd_smem(const GfkModel*);
size_t gfk_lda_fwd_smem(int);
size_t gfk_lda_bwd_smem(const GfkModel*);
size_t gfk_post_smem(const GfkModel*);
size_t gfk_win_update_smem(const GfkModel*);
size_t gfk_enc_in_smem(const GfkModel*);
int gfk_enc_in_set_smem(size_t);
int gfk_post_set_smem(size_t);
int gfk_win_update_set_smem(size_t);
int gfk_prodlda_set_smem(size_t);
int gfk_lda_set_smem(size_t);

// Phase ids (mirrored in gfedntm_amd/ops/kernel_abi.py).
enum GfkPhase {
  GFK_PH_BATCH_DOCS = 0,
  GFK_PH_ENC_FWD = 1,
  GFK_PH_POST_FWD = 2,
  GFK_PH_PRODLDA_FWD = 3,
  GFK_PH_PRODLDA_LOSS = 4,
  GFK_PH_PRODLDA_BWD = 5,
  GFK_PH_LDA_BETA_FWD = 6,
  GFK_PH_LDA_ROW = 7,
  GFK_PH_POST_BWD = 8,
  GFK_PH_LDA_BETA_BWD = 9,
  GFK_PH_ENC_BWD = 10,
  GFK_PH_ADAM = 11,
  GFK_PH_BATCH_PREP = 12,
  GFK_PH_CTXF_FWD = 13,
  GFK_PH_CTXF_BWD = 14,
  // (15: the split W_in update's dense half, removed in round 6)
};



// LDS each kernel family needs for this model.
size_t gfk_smem_required(const GfkModel* m, int which) {
  switch (which) {
    case 0: return gfk_prodlda_fwd_smem(m);
    case 1: return gfk_prodlda_bwd_smem(m);
    case 2: return gfk_lda_fwd_smem(m->K);
    case 3: return gfk_lda_bwd_smem(m);
    case 4: return gfk_post_smem(m);
    case 5: return gfk_win_update_smem(m);
    case 7: return gfk_enc_in_smem(m);
    case 8: return m->ctx_fused == 1 ? gfk_ctx_smem(m) : 0;
    default: return 0;
  }
}

// One-time per model shape: raise the dynamic-LDS limit of the kernels that use
// more than the 64 KiB default (MI355X has 160 KiB per CU).
int gfk_setup(const GfkModel* m) {
  int e = 0;
  // (only the model's own decoder family: the other's plan for this shape may not even fit
  // the LDS -- NeuralLDA's beta backward at K > 256)
  if (m->kind == GFK_PRODLDA) {
    const size_t p = gfk_prodlda_fwd_smem(m), q = gfk_prodlda_bwd_smem(m);
    if ((e = gfk_prodlda_set_smem(p > q ? p : q))) return e;
  } else {
    const size_t p = gfk_lda_fwd_smem(m->K), q = gfk_lda_bwd_smem(m);
    if ((e = gfk_lda_set_smem(p > q ? p : q))) return e;
  }
  if ((e = gfk_enc_in_set_smem(gfk_enc_in_smem(m)))) return e;
  if ((e = gfk_post_set_smem(gfk_post_smem(m)))) return e;
  if (m->ctx_fused == 1 && (e = gfk_ctx_set_smem(gfk_ctx_smem(m)))) return e;
  return gfk_win_update_set_smem(gfk_win_update_smem(m));
}

// a / adam_grid: the generic Adam (PH_ADAM, gradient mode); u: the small-tensor
// gradient / update jobs of win_update.
int gfk_run(const GfkModel* m, const GfkAdam* a, int adam_grid, const GfkUpdate* u, hipStream_t s,
            const int32_t* phases, int n_phases) {
  for (int i = 0; i < n_phases; ++i) {
    int e = 0;
    switch (phases[i]) {
      case GFK_PH_BATCH_DOCS: e = gfk_launch_batch_docs(m, s); break;
      case GFK_PH_ENC_FWD: e = gfk_launch_enc_in(m, s); break;
      // (folded into the strip forward: running it as well would advance the step twice)
      case GFK_PH_POST_FWD: e = gfk_postfold(*m) ? 0 : gfk_launch_post_fwd(m, s); break;
      case GFK_PH_PRODLDA_FWD: e = gfk_launch_prodlda_fwd(m, s); break;
      case GFK_PH_PRODLDA_LOSS: e = gfk_launch_prodlda_row_loss(m, s); break;
      case GFK_PH_PRODLDA_BWD: e = gfk_launch_prodlda_bwd(m, s); break;
      case GFK_PH_LDA_BETA_FWD: e = gfk_launch_lda_beta_fwd(m, s); break;
      case GFK_PH_LDA_ROW: e = gfk_launch_lda_row(m, s); break;
      case GFK_PH_POST_BWD: e = gfk_launch_post_bwd(m, s); break;
      case GFK_PH_LDA_BETA_BWD: e = gfk_launch_lda_beta_bwd(m, s); break;
      case GFK_PH_ENC_BWD: e = gfk_launch_win_update(m, u, s); break;
      case GFK_PH_ADAM: e = gfk_launch_adam(a, adam_grid, s); break;
      case GFK_PH_BATCH_PREP: e = gfk_launch_batch_prep(m, s); break;
      case GFK_PH_CTXF_FWD: e = gfk_launch_ctx_fwd(m, s); break;
      case GFK_PH_CTXF_BWD: e = gfk_launch_ctx_bwd(m, s); break;
      default: e = -2;
    }
    if (e) return e * 100 + phases[i];
  }
  return 0;
}

int gfk_scale(float* p, int64_t n, float sc, hipStream_t s) { return gfk_launch_scale(p, n, sc, s); }

size_t gfk_model_struct_size() { return sizeof(GfkModel); }
size_t gfk_adam_struct_size() { return sizeof(GfkAdam); }
size_t gfk_update_struct_size() { return sizeof(GfkUpdate); }
size_t gfk_fold_struct_size() { return sizeof(GfkFold); }
size_t gfk_fold_client_struct_size() { return sizeof(GfkFoldClient); }

}  // extern "C"
