/* Learner ops of libgridenv.so: the optimizer and target-network updates of the MADDPG learner
 * (marlnav/maddpg.py) over flat float32 parameter buffers, one launch each, graph-capturable
 * (the Adam step count lives on the device).  Plain device pointers; enqueued on `stream`. */
#ifndef LEARNER_OPS_H
#define LEARNER_OPS_H

#include <stdint.h>

#include "actor_ops.h"
#include "gridenv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* torch.optim.Adam (no weight decay, no amsgrad; torch/optim/adam.py _single_tensor_adam) on n
 * elements:  m = lerp(m, g, 1 - beta1);  v = beta2 * v + (1 - beta2) * g * g;  s = step[0] + 1
 *   p -= lr / (1 - beta1^s) * (m / (sqrt(v) / sqrt(1 - beta2^s) + eps));   then step[0] = s.
 * step: int32 [2] device memory, [0] the steps taken, [1] zero (the launch's arrival counter: the
 * last block to finish advances step[0], so the step is ONE launch).
 * advanced != 0: step[0] already counts this step (a preceding launch on the stream advanced it,
 * e.g. gw_maddpg_critic_grads / gw_maddpg_actor_grads' adam_step): s = step[0], no arrival
 * counter (its same-address atomics from every block cost ~30 us per launch on a 0.5 M-element
 * buffer). 
 * The scalar hyper-parameters are doubles and the bias corrections are formed in double, as
 * torch forms them from Python floats, then rounded to float against the f32 tensors. */
gw_status gw_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                       int64_t n, double lr, double beta1, double beta2, double eps, int32_t advanced, void *stream);

/* gw_adam_step on param[0, n), then in the same launch the soft target updates that end
 * MADDPG.learn: target[i] = tau * param[i] + (1 - tau) * target[i] with the stepped param, and
 * target2 = tau * online2 + (1 - tau) * target2 on n2 elements (the other network, stepped
 * earlier; n2 = 0: none).  Same arithmetic as gw_adam_step followed by gw_soft_update2. */
gw_status gw_adam_soft_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                            int64_t n, double lr, double beta1, double beta2, double eps, float *target, float tau,
                            float *target2, const float *online2, int64_t n2, int32_t advanced, void *stream);

/* agilerl soft_update: target = tau * online + (1 - tau) * target on n elements. */
gw_status gw_soft_update(float *target, const float *online, int64_t n, float tau, void *stream);

/* Both soft target updates of one learn (the actor and critic buffers) in one launch. */
gw_status gw_soft_update2(float *target1, const float *online1, int64_t n1, float *target2, const float *online2,
                          int64_t n2, float tau, void *stream);

/* TD target of MADDPG.learn (agilerl: y = r + (1 - d) * gamma * Q'(s', a')):  rewards [B, K] f64
 * (shaped), dones [B, K] u8 (termination), q_next / y [K, B] f32;  y[k, b] = f32(r[b, k]) +
 * ((1 - d[b, k]) * gamma) * q_next[k, b], one f32 rounding per op as torch evaluates it. */
gw_status gw_td_target(const double *rewards, const uint8_t *dones, const float *q_next, float gamma, float *y,
                       int32_t K, int64_t B, void *stream);

/* The per-agent losses of MADDPG.learn over q [K, B] (one value per row):  mode 0 the critic's
 * MSELoss  loss[k] = mean_b (q - y)^2;  mode 1 the actor's  loss[k] = -mean_b q  (y unused).
 * The backward writes dq [K, B] from grad_loss [K]:  (g / B) * (2 (q - y))  or  -(g / B), the
 * op order of torch's mean / pow / neg backward. */
gw_status gw_mean_loss_fwd(const float *q, const float *y, float *loss, int32_t K, int64_t B, int32_t mode,
                           void *stream);
gw_status gw_mean_loss_bwd(const float *q, const float *y, const float *grad_loss, float *dq, int32_t K, int64_t B,
                           int32_t mode, void *stream);

/* Hidden-layer epilogue of the stacked MLPs (agilerl EvolvableMLP: Linear -> LayerNorm -> ReLU;
 * marlnav/actor.py StackedMLPActors.forward, replacing F.layer_norm + addcmul + relu, three
 * launches, by one).  z, y [K, R, h] contiguous, ln_w / ln_b [K, h]; 0 < h <= 512.
 *   y = relu(ln_b + ((z - mean) * rstd) * ln_w),  mean / rstd over h (biased variance, eps).
 * mean / rstd [K, R] receive the row statistics for the backward (both NULL: not saved). */
gw_status gw_ln_relu_fwd(const float *z, const float *ln_w, const float *ln_b, float *y, float *mean, float *rstd,
                         int32_t K, int64_t R, int32_t h, float eps, void *stream);

/* Its backward from the saved z, y, mean, rstd: dz [K, R, h] is written (one launch, a wave per
 * row); the ln_w / ln_b gradients, summed over the R rows in a fixed order, are ADDED into
 * dw_acc / db_acc [K, h] (a second launch; the parameters' existing .grad, as autograd
 * accumulates; either may be NULL). */
gw_status gw_ln_relu_bwd(const float *dy, const float *z, const float *y, const float *ln_w, const float *mean,
                         const float *rstd, float *dz, float *dw_acc, float *db_acc, int32_t K, int64_t R,
                         int32_t h, void *stream);

/* The affine + ReLU half of that epilogue after torch's own (non-affine) F.layer_norm, so the
 * normalised rows stay torch's bit for bit (the default learner path): xhat, y [K, R, h],
 * ln_w / ln_b [K, h];  y = relu(fma(xhat, ln_w, ln_b))  (torch.addcmul contracted, then relu). */
gw_status gw_affine_relu_fwd(const float *xhat, const float *ln_w, const float *ln_b, float *y, int32_t K, int64_t R,
                             int32_t h, void *stream);

/* Its backward: g = dy * (y > 0);  dxhat = g * ln_w (if dxhat != NULL);  the row sums of g * xhat
 * and g ADDED into dw_acc / db_acc [K, h] (either may be NULL), in a fixed order. */
gw_status gw_affine_relu_bwd(const float *dy, const float *xhat, const float *y, const float *ln_w, float *dxhat,
                             float *dw_acc, float *db_acc, int32_t K, int64_t R, int32_t h, void *stream);

/* agilerl GumbelSoftmax (no gradient; the target actors' next actions in MADDPG.learn) over
 * [rows, n] logits with uniforms u:  out = softmax((logits - log(-log(u + eps) + eps)) / tau).
 * out_ld == 0: out is [rows, n].  out_ld > 0: row r = k * out_b + b is written at
 * out + b * out_ld + k * n (straight into the action slots of the critic's input rows). */
gw_status gw_gumbel_softmax(const float *logits, const float *u, float *out, int64_t rows, int32_t n, float tau,
                            float eps, int64_t out_b, int64_t out_ld, void *stream);

/* ---- the fused MADDPG update (csrc/maddpg_ops.hip) ------------------------------------------
 * agilerl 1.0.15 MADDPG.learn (maddpg/agent.py:199-224; restated in marlnav/maddpg.py) on a
 * sampled batch for K stacked agents, networks in StackedMLPActors' layout (gw_mlp_actors: in ->
 * 128 -> LayerNorm -> ReLU -> 128 -> LayerNorm -> ReLU -> out; actors out = 9 over D = H*W obs
 * floats, critics out = 1 over the critic rows [s_1 .. s_K, a_1 .. a_K]).  Two calls carry the
 * update's two backward passes; between them the caller runs the critic's Adam step
 * (gw_adam_step), and after the second the actor's Adam step and the soft update
 * (gw_soft_update2); with several ranks each call's gradients are all-reduced before its Adam
 * step.  Gradients are WRITTEN (not accumulated) through the *_grad views, losses [K] f32. */
typedef struct gw_maddpg_batch {
    int32_t K, B, D;       /* agents, rows (a positive multiple of 16), obs floats per agent       */
    const float *x;        /* [B][K*D + 9K] critic input rows: states, stored action probabilities */
    float *x_next;         /* [B][K*D + 9K] next states; the target actions are written into its
                            * action slots by gw_maddpg_critic_grads                              */
    const double *reward;  /* [B][K] shaped rewards                                                */
    const uint8_t *done;   /* [B][K] terminations                                                  */
    const float *u;        /* [K][B][9] the call's Gumbel uniforms (u_next, then u_cur), or NULL:    */
    uint64_t seed;         /*   drawn in the kernels, Philox4x32-10(key seed; counter (row, *ctr,     */
    const int32_t *ctr;    /*   'GUM' + phase, 4 agent + j)); ctr: a device int32 that changes per    */
                           /*   update (e.g. the critic optimizer's step count)                       */
} gw_maddpg_batch;

/* Workspace (floats) both calls share: layer-1 partial sums and the rows' saved activations. */
int64_t gw_maddpg_workspace_floats(int32_t K, int32_t B, int32_t D);

/* a'_k = GumbelSoftmax(actor_target_k(s'_k)) into x_next's slots; y = r + (1 - d) gamma
 * critic_target_k(x_next); critic_grad = d/dtheta of mean_b (critic_k(x) - y)^2 per agent;
 * loss [K] the MSE values.  adam_step (may be NULL): the critic optimizer's step count
 * (gw_adam_step's int32 [2]), advanced by one in this call's last launch, so the Adam step that
 * follows runs with advanced = 1. */
gw_status gw_maddpg_critic_grads(const gw_mlp_actors *actor_target, const gw_mlp_actors *critic_target,
                                 const gw_mlp_actors *critic, const gw_mlp_actors *critic_grad,
                                 const gw_maddpg_batch *batch, float gamma, float *ws, float *loss,
                                 int32_t *adam_step, void *stream);

/* probs_k = GumbelSoftmax(actor_k(s_k)) (probs [K][B][9], may be NULL); actor_grad = d/dtheta of
 * -mean_b critic_k(s, a with a_k := probs_k) per agent (adam_step: the actor optimizer's count,
 * as gw_maddpg_critic_grads') (the critic as given, i.e. after its Adam
 * step; no critic gradients); loss [K]. */
gw_status gw_maddpg_actor_grads(const gw_mlp_actors *actor, const gw_mlp_actors *critic,
                                const gw_mlp_actors *actor_grad, const gw_maddpg_batch *batch, float *ws, float *loss,
                                float *probs, int32_t *adam_step, void *stream);

/* ---- the descriptor learner (csrc/maddpg_ops.hip, round 5) ----------------------------------
 * The same MADDPG update on a replay ring of obs DESCRIPTORS (Rollout(desc_ring=True): per slot the
 * 48-byte descriptors gw_obs_desc_copy stores, plus probs / rewards / terminations / dones), with
 * the sample drawn inside (gw_replay_gather_desc's Philox draws keyed by `seed` and the critic's
 * step count) and both Adam steps and the soft target updates inside: FOUR launches per update,
 * one rank (the data-parallel learner all-reduces between the gradients and Adam: the two calls
 * above).  Layer 1 is the map part c1 = b1 + map . W1 (kept in the workspace as 64-row partial
 * sums, refreshed by the launch that changes W1) plus the <= N + 1 patched cells of each obs, and
 * the W1 gradient is map (x) colsum(dZ1) plus the patched cells' terms: no layer-1 GEMM and no
 * dense rows.  Differs from the dense update (gw_maddpg_critic_grads / _actor_grads + gw_adam_step
 * + gw_soft_update2) by f32 summation order only. */
typedef struct gw_adam_buf {
    float *param;            /* the network's flat parameter buffer (its gw_mlp_actors point into it) */
    float *grad;             /* the flat gradient buffer (same layout): the update's gradients, written */
    float *exp_avg, *exp_avg_sq;
    int32_t *step;           /* int32 [2], gw_adam_step's count: [0] advanced by the update, [1] untouched */
    int64_t n;               /* elements */
    double lr, beta1, beta2, eps;
} gw_adam_buf;
typedef struct gw_desc_ring {
    const uint32_t *desc;    /* [S][E][12] every slot's obs descriptors (gw_obs_desc_copy)           */
    const float *probs;      /* [S][K][E][9] stored action probabilities                            */
    const double *reward;    /* [S][E][K] shaped rewards                                            */
    const uint8_t *term;     /* [S][E][K] terminations                                              */
    const uint8_t *done;     /* [S][E] env done (the next state is then the terminal obs)           */
    const int64_t *t_dev;    /* transitions stored (device)                                         */
    int64_t S;               /* slots                                                               */
} gw_desc_ring;
/* Workspace floats of a batch of B rows (16 <= B <= 256, B % 16 == 0); -1 on bad arguments. */
int64_t gw_maddpg_desc_workspace_floats(int32_t K, int32_t B, int32_t H, int32_t W);
/* (Re)derive the c1 partial sums of all four networks from their current W1 into ws: before the
 * first update and after any change of the weights other than gw_maddpg_desc_update's own. */
gw_status gw_maddpg_desc_prime(const gw_obs_source *src, const gw_mlp_actors *actor, const gw_mlp_actors *actor_target,
                               const gw_mlp_actors *critic, const gw_mlp_actors *critic_target, int32_t B, float *ws,
                               void *stream);
/* One whole update: sample B rows, critic gradients + Adam, actor gradients + Adam, the soft
 * updates of both targets (their flat buffers share the online layout), losses [K] f32.  The
 * optimizers' counts advance by one each (opt_critic's also keys the draws); gradients are left
 * in the grad buffers; ws keeps the rows' records (layout: csrc/maddpg_ops.hip dws_layout).
 * prof_env (may be NULL): a gw_create handle whose gw_profile spans take the update's four
 * launches as one GW_SPAN_LEARN span while it profiles. */
gw_status gw_maddpg_desc_update(const gw_obs_source *src, const gw_desc_ring *ring, const gw_mlp_actors *actor,
                                const gw_mlp_actors *actor_target, const gw_mlp_actors *critic,
                                const gw_mlp_actors *critic_target, const gw_adam_buf *opt_actor,
                                const gw_adam_buf *opt_critic, float *actor_target_flat, float *critic_target_flat,
                                float gamma, float tau, int32_t B, uint64_t seed, float *ws, float *actor_loss,
                                float *critic_loss, void *prof_env, void *stream);
/* gw_maddpg_desc_update that also leaves the stepped actor's gw_actor_act workspace parts (img,
 * from gw_actor_images_view of the workspace gw_actor_act reads; NULL = none): the row slices from
 * the actor W1 blocks, the W2 / W3 images from the blocks that step those layers -- the values
 * gw_actor_prepare would derive, bit for bit, without its two launches after the update. */
gw_status gw_maddpg_desc_update_img(const gw_obs_source *src, const gw_desc_ring *ring, const gw_mlp_actors *actor,
                                    const gw_mlp_actors *actor_target, const gw_mlp_actors *critic,
                                    const gw_mlp_actors *critic_target, const gw_adam_buf *opt_actor,
                                    const gw_adam_buf *opt_critic, float *actor_target_flat, float *critic_target_flat,
                                    float gamma, float tau, int32_t B, uint64_t seed, float *ws, float *actor_loss,
                                    float *critic_loss, const gw_actor_images *img, void *prof_env, void *stream);
#ifdef __cplusplus
}
#endif
#endif
