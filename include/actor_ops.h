/* Actor ops of libgridenv.so: the MADDPG actors' get_action fused into one MI355X kernel.
 *
 * Replaces, for every env of a grid-env handle at once, the per-step actor call of the
 * reference rollout:
 *   maddpg/agent.py:109-122   state flattening, agilerl MADDPG.get_action, argmax -> action ids
 * with agilerl 1.0.15's MLP actor (EvolvableMLP: Linear -> LayerNorm -> ReLU -> Linear ->
 * LayerNorm -> ReLU -> Linear, GumbelSoftmax output; layout from the shipped checkpoints,
 * SURVEY.md §8c) and the env's action mask (ma_customenv.py:467-506).
 *
 * The observation an env last wrote (gw_reset / gw_step) is the static map plus at most N+1
 * patched cells per RL agent (own apple, agents; ma_customenv.py:303-322), so the first layer
 *   h1 = b1 + obs . W1  =  (b1 + map . W1)  +  sum over patched cells c of (obs[c] - map[c]) W1[c,:]
 * is evaluated from the env's obs descriptors: no observation is read back from HBM.  Layers 2
 * and 3 run on f32 MFMA (v_mfma_f32_16x16x4_f32: exact f32 products, k-ordered f32 sums),
 * LayerNorm / ReLU / Gumbel noise / softmax / mask / argmax in registers.
 *
 * Shapes: hidden 128 (both layers), 9 actions, in_dim = H*W of the env, f32 parameters in
 * the stacked [K][in][out] layout (torch.bmm), 16-byte aligned.  Plain device pointers;
 * enqueued on `stream`; statuses as in gridenv.h.
 */
#ifndef ACTOR_OPS_H
#define ACTOR_OPS_H

#include <stdint.h>

#include "gridenv.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gw_mlp_actors {
    int32_t K;            /* RL agents (must equal the env's K)                         */
    int32_t in_dim;       /* H*W                                                        */
    int32_t hidden;       /* 128                                                        */
    int32_t n_actions;    /* 9                                                          */
    int32_t layer_norm;   /* LayerNorm(eps 1e-5) + affine after layers 1 and 2           */
    const float *w1;      /* [K][in_dim][128]                                           */
    const float *b1;      /* [K][128]                                                   */
    const float *ln1_w, *ln1_b;  /* [K][128] (unused without layer_norm)                */
    const float *w2;      /* [K][128][128]                                              */
    const float *b2;      /* [K][128]                                                   */
    const float *ln2_w, *ln2_b;  /* [K][128]                                            */
    const float *w3;      /* [K][128][9]                                                */
    const float *b3;      /* [K][9]                                                     */
} gw_mlp_actors;

/* Size (floats) of the workspace the two calls below share: per agent c1 = b1 + map . W1 (128),
 * the W2 / W3 images the kernel stages in LDS, and map . W1 row slices. */
int64_t gw_actor_workspace_floats(int32_t in_dim, int32_t K);

/* Derive the workspace from the parameters (c1 and the MFMA-operand images of W2 / W3).  Enqueue
 * it again after every change of the parameters (optimizer step, load); ws 16-byte aligned. */
gw_status gw_actor_prepare(void *env, const gw_mlp_actors *net, float *ws, void *stream);

/* The parts of a gw_actor_prepare workspace a learner may write directly after its actor update
 * (gw_maddpg_desc_update_img), instead of a gw_actor_prepare launch pair: the map . W1 row slices
 * (slice sl = rows [32 sl, 32 sl + 32), an f32 fma chain in row order from 0 -- gw_actor_act sums
 * them in slice order onto b1) and the MFMA-operand images of W2 (f32 and bf16x3) and W3. */
typedef struct {
    float *part;     /* [K][nslices][128] */
    int32_t nslices; /* ceil(in_dim / 32) */
    float *w2img;    /* [K][128 * 128] */
    void *w2bimg;    /* [K][3 * 8 * 4 * 64 * 4] u32: the bf16x3 image */
    float *w3img;    /* [K][8 * 4 * 9 * 4] */
} gw_actor_images;
/* ws: a gw_actor_workspace_floats(in_dim, K) workspace. */
gw_status gw_actor_images_view(float *ws, int32_t in_dim, int32_t K, gw_actor_images *out);

/* For every env e and RL agent k, on the observation the env last wrote:
 *   logits = actor_k(obs_k);  training: logits -= log(-log(u + 1e-20) + 1e-20)  (Gumbel noise;
 *   u = uniform[k][e][a] if `uniform` is given, else Philox(seed; global env id, c, k) with
 *   c = counter + *counter_dev (counter_dev: a device int64 read at launch time, e.g. the replay
 *   ring's step count, so the replays of a captured HIP graph draw fresh noise; NULL = 0));
 *   probs = softmax(logits / tau);  action = argmax over the actions allowed by mask[e][k]
 *   (first maximum; mask NULL = all allowed).
 * Outputs: actions [E][K] int32 (gw_step's rl_actions layout), probs [K][E][9] f32 (the
 * continuous actions agilerl stores in replay), logits [K][E][9] f32 before the noise (may be
 * NULL).  ws: prepared by gw_actor_prepare for the current parameters. */
gw_status gw_actor_act(void *env, const gw_mlp_actors *net, const float *ws, int training, float tau,
                       uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                       const uint16_t *mask,
                       int32_t *actions, float *probs, float *logits, void *stream);

/* ---- local windows (X1: not a reference format) ---------------------------------------------
 * The same MLP actors over each RL agent's P x P egocentric window of its observation (the layout
 * of gw_obs_patch: rows / cols -P/2 .. P-1-P/2 around the agent's own cell, -1 outside the grid);
 * net->in_dim = P*P.  The window's static part depends only on its centre cell, so
 *   h1 = T_k[centre] + sum over patched cells c inside the window of (obs[c] - map[c]) W1[pos(c), :]
 * with T_k[c] = b1 + (the -1-padded map window centred on c) . W1 derived for every cell by
 * gw_patch_actor_prepare.  No window is read back from HBM (gw_obs_patch writes them for the
 * replay ring only).  Tolerance against torch on the cropped windows: tests/test_gpu_patch_actor.py. */
int64_t gw_patch_actor_workspace_floats(int32_t P, int32_t H, int32_t W, int32_t K);
gw_status gw_patch_actor_prepare(void *env, int32_t P, const gw_mlp_actors *net, float *ws, void *stream);
gw_status gw_patch_actor_act(void *env, int32_t P, const gw_mlp_actors *net, const float *ws, int training, float tau,
                             uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                             const uint16_t *mask,
                             int32_t *actions, float *probs, float *logits, void *stream);

/* ---- the configs/cnn.yaml actor head ------------------------------------------------------
 * Conv2d(1, 32, 2, stride 2) - ReLU - Conv2d(32, 64, 2, stride 2) - ReLU - flatten (c, y, x)
 * - Linear(64 (H/4) (W/4), 128) - ReLU - Linear(128, 128) - ReLU - Linear(128, 9), per RL agent
 * (maddpg/agent.py:94-100 with configs/cnn.yaml:2-6; agilerl's EvolvableCNN, parity unpinned).
 *
 * Both convolutions have kernel == stride, so conv-2 output position (Y, X) sees exactly the 4x4
 * obs cells [4Y, 4Y + 4) x [4X, 4X + 4), and an observation (static map + at most N + 1 patched
 * cells) changes at most N + 1 of the (H/4)(W/4) positions.  The first Linear is therefore
 *   z = z_map + sum over changed positions P of Wl[:, P] . (a2(P) - a2_map(P))
 * with z_map = b + Wl . a2(map) derived once per weight version.  A position holding ONE patched
 * cell (the common case) reads its 128-float delta from a table built by gw_cnn_prepare for every
 * (agent, position, cell, value); a position holding several is recomputed (conv 1, conv 2 on
 * its 16 cells, then its 64 x 128 block of Wl).  No observation is read back from HBM. */
typedef struct gw_cnn_actors {
    int32_t K;            /* RL agents (must equal the env's K)                          */
    int32_t H, W;         /* obs grid (the env's), multiples of 4                        */
    int32_t c1, c2;       /* conv channels: 32, 64                                       */
    int32_t hidden;       /* 128                                                         */
    int32_t n_actions;    /* 9                                                           */
    const float *conv1_w; /* [K][c1][1][2][2]  (torch Conv2d weight)                     */
    const float *conv1_b; /* [K][c1]                                                     */
    const float *conv2_w; /* [K][c2][c1][2][2]                                           */
    const float *conv2_b; /* [K][c2]                                                     */
    const float *lin1_w;  /* [K][128][c2 (H/4) (W/4)]  (torch Linear weight, out x in)    */
    const float *lin1_b;  /* [K][128]                                                    */
    const float *w2;      /* [K][128][128]  ([in][out], the stacked torch.bmm layout)     */
    const float *b2;      /* [K][128]                                                    */
    const float *w3;      /* [K][128][9]                                                 */
    const float *b3;      /* [K][9]                                                      */
} gw_cnn_actors;

/* Workspace (floats) of the CNN calls for E envs: the delta table (K (H/4)(W/4) 16 19 128
 * floats: 40 MB at 64x64, K = 2), the transposed Linear-1 weight, the map activations, the
 * layer-2/3 MFMA images and a [K][E][128] layer-1 buffer. */
int64_t gw_cnn_workspace_floats(int32_t H, int32_t W, int32_t K, int64_t E);

/* Derive the workspace from the parameters; enqueue again after every parameter change. */
gw_status gw_cnn_prepare(void *env, const gw_cnn_actors *net, float *ws, void *stream);

/* gw_actor_act with the CNN head: the same noise, softmax, mask, argmax and outputs. */
gw_status gw_cnn_act(void *env, const gw_cnn_actors *net, const float *ws, int training, float tau,
                     uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                     const uint16_t *mask,
                     int32_t *actions, float *probs, float *logits, void *stream);

/* ---- the CNN head on local windows (X1: not a reference format) -----------------------------
 * The configs/cnn.yaml head built for P x P inputs (net->H = net->W = P; P = 4, 8, 12, 16) over
 * each RL agent's gw_obs_patch window.  The window centred on cell c differs from its BASE window
 * (the -1-padded map under it, with the agent's usual own value -- 1, or k + 1 in variant 1 -- at
 * the centre) only at patched cells, so
 *   z = tbl_k[c] + sum over the positions Q where the window differs of Wl[:, Q] . (a2(Q) - a2b_k[c][Q])
 * with tbl_k[c] = b + Wl . a2(base window of c) and a2b derived for every cell by
 * gw_patch_cnn_prepare (K H W (P/4)^2 64 + K H W 128 floats).  Differing positions (typically
 * 0-2 per (env, agent)) are recomputed from the obs descriptors; no window is read back.  Workspace
 * (floats) for E envs: gw_patch_cnn_workspace_floats (includes a [K][E][N + 1][128] buffer of the
 * recomputed positions' terms).  Tolerance against nn.Conv2d on the written windows:
 * tests/test_gpu_patch_cnn.py. */
int64_t gw_patch_cnn_workspace_floats(int32_t P, int32_t H, int32_t W, int32_t K, int64_t E);
gw_status gw_patch_cnn_prepare(void *env, int32_t P, const gw_cnn_actors *net, float *ws, void *stream);
gw_status gw_patch_cnn_act(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, int training, float tau,
                           uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                           const uint16_t *mask,
                           int32_t *actions, float *probs, float *logits, void *stream);
/* A rollout's step in fewer launches: gw_patch_cnn_write_list writes the env's windows exactly as
 * gw_obs_patch(env, P, patch, final_patch) does (the row writer; E % 4 == 0) and, in the SAME launch,
 * lists the positions the next act recomputes for those descriptors (the first part of
 * gw_patch_cnn_act); gw_patch_cnn_act_listed is the rest of gw_patch_cnn_act on that listing
 * (ordered after it, no env step or reset in between, the same workspace derivation).  Together
 * they equal gw_obs_patch + gw_patch_cnn_act bit for bit (tests/test_gpu_patch_cnn.py).  The
 * listing adds into bucket counters that the act kernel zeroes once the rare kernel has read them:
 * between two gw_patch_cnn_write_list calls there must be an act (either form; gw_patch_cnn_act
 * also zeroes them before its own listing, so a listing followed by an env reset and a
 * gw_patch_cnn_act is fine). */
gw_status gw_patch_cnn_write_list(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, float *patch,
                                  float *final_patch, void *stream);
gw_status gw_patch_cnn_act_listed(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, int training,
                                  float tau, uint64_t seed, uint64_t counter, const int64_t *counter_dev,
                                  const float *uniform, const uint16_t *mask, int32_t *actions, float *probs,
                                  float *logits, void *stream);

#ifdef __cplusplus
}
#endif
#endif
