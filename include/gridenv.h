/*
 * gridenv.h — C ABI of the MI355X-native vectorised grid world (libgridenv.so).
 *
 * Drop-in boundary for the reference's hot path (Henweiz/MARL-Responsible-Nav):
 *   CustomMAEnv.__init__/reset/step   custom/ma_customenv.py:74-108, 169-215, 217-334
 *   GWorld.UpdateGWorld               custom/grid_world.py:424-563
 *   Responsibility.FeAR_4_one_actor   custom/Responsibility.py:135-210
 *   MADDPGAgent.train per-step reward/score arithmetic   maddpg/agent.py:120-173, 226-243
 * The reference has no FFI of its own (pure Python); these entry points are what its
 * PettingZoo surface binds to through the ctypes layer in marlnav/_lib.py.
 *
 * One handle = E independent envs resident in HBM (structure of arrays).  All device
 * pointers are plain HIP device addresses (e.g. torch.Tensor.data_ptr()); `stream` is a
 * hipStream_t passed as void*.  Calls only enqueue work on `stream`; there is no implicit
 * host synchronisation.  Statuses are negative on error; gw_last_error() explains.
 * Layout: obs are agent-major [K][E][H*W] float32 (each RL agent's actor reads one
 * contiguous [E, H*W] matrix); per-env per-agent outputs are [E][K].
 */
#ifndef GRIDENV_H
#define GRIDENV_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GW_MAX_AGENTS 8
#define GW_N_ACTIONS 9

typedef enum gw_status {
    GW_OK = 0,
    GW_ERR_ARG = -1,    /* invalid argument / scenario                        */
    GW_ERR_HIP = -2,    /* HIP runtime error                                  */
    GW_ERR_ALLOC = -3,  /* device allocation failed                           */
    GW_ERR_STATE = -4   /* call order (e.g. gw_step before the first reset)   */
} gw_status;

/* Static scenario tables (host pointers, copied by gw_create).
 * Replaces LoadJsonScenario + CustomMAEnv.setup_env's map build
 * (custom/grid_world.py:621-674, custom/ma_customenv.py:338-365, 422). */
typedef struct gw_scenario {
    int32_t H, W;               /* grid rows, columns (H*W <= 4096, W >= 2)             */
    const uint8_t *region;      /* [H*W] 1 active road, 0 inactive                      */
    const uint8_t *policy_id;   /* [H*W] policy index                                   */
    int32_t n_policies;
    const double *policy_cdf;   /* [n_policies][2][9] choice CDFs; [.][1] = the 25 %
                                   uniform-direction branch (ma_customenv.py:441-443)   */
    const uint8_t *mdr;         /* [H*W] MdR action per cell                            */
    const int32_t *apples;      /* [K] apple cell of RL agent k                         */
} gw_scenario;

typedef struct gw_config {
    int32_t N;                  /* world agents  (Scenario N_Agents)          1..8      */
    int32_t K;                  /* RL agents     (N_INTELLIGENT_AGENTS)       1..N      */
    int64_t num_envs;           /* E, envs owned by this handle                          */
    int64_t env_offset;         /* global id of local env 0 (RNG counter; sharding)      */
    int32_t fear;               /* CustomMAEnv(fear=...)                                 */
    double fear_weight;         /* INIT_HP["FeAR_weight"] (maddpg/agent.py:125)          */
    int32_t max_steps;          /* TRAIN_STEPS episode cap; 0 = none                     */
    int32_t auto_reset;         /* reset done envs inside gw_step                        */
    uint64_t seed;              /* Philox key (spawns, scripted policy, random RL policy)*/
    int32_t variant;            /* 0: CustomMAEnv (custom/ma_customenv.py); 1: the single-
                                   agent CustomEnv (custom/customenv.py:78-183): K must be 1,
                                   rewards -10 crash (terminated only) / +20 apple (exactly one
                                   apples_caught entry; truncated) / +0.1 closer to the apple,
                                   step obs = raw WorldState ids (no relabel), prev distance set
                                   at reset.  Everything else is shared.                    */
} gw_config;

/* Per-step outputs: device pointers, any may be NULL (not written). */
typedef struct gw_step_out {
    float *obs;          /* [K][E][H*W] obs after the step (reset obs if auto-reset)  */
    float *final_obs;    /* [K][E][H*W] terminal obs; rows written only for done envs */
    double *reward;      /* [E][K] env reward                (ma_customenv.py:258-302) */
    double *fear;        /* [E][K] info["fear"]              (ma_customenv.py:245-252) */
    double *shaped;      /* [E][K] FeAR_weight*FeAR + reward (maddpg/agent.py:130)     */
    uint8_t *term;       /* [E][K] terminations                                         */
    uint8_t *trunc;      /* [E][K] truncations                                          */
    uint8_t *done;       /* [E]   all(term) | all(trunc) | t >= max_steps               */
    uint16_t *mask;      /* [E][K] 9-bit action mask of the returned obs                */
    int32_t *crashes;    /* [E]   info["agent_crashes"]                                 */
    int32_t *apples;     /* [E]   info["apples_caught"]                                 */
    double *ep_return;   /* [E]   episode score incl. this step (maddpg/agent.py:173)   */
    double *ep_fear;     /* [E]   episode fear_score (maddpg/agent.py:141)              */
    int32_t *ep_len;     /* [E]   steps in the episode incl. this one                   */
    int32_t *actions;    /* [E][N] joint action applied (env.Action4Agents)             */
    int32_t *mdr;        /* [E][N] MdR4Agents                                           */
    int32_t *final_pos;  /* [E][N] positions after the move, before any auto-reset      */
    uint8_t *crash_bits; /* [E]   bit n: agent n crashed (UpdateGWorld agent_crashes)   */
    uint8_t *restr_bits; /* [E]   bit n: restricted move                                */
    double *stats;       /* [gw_stats_rows()][GW_STATS] per-block partial sums of this step:
                            completed-episode returns, episodes completed, FeAR, crashes,
                            apples caught, shaped rewards, completed-episode lengths, envs.
                            Deterministic (fixed reduction tree); fed to the RCCL
                            reduction of the multi-GPU rollout.                          */
    uint8_t *done_copy;  /* [E]   a second destination of `done` (e.g. the per-step return
                            gather's send buffer beside the replay ring's done slot)     */
    double *stats_acc;   /* [gw_stats_rows()][GW_STATS]: every step ADDS its per-block rows
                            (a running total without a per-step reduction launch; one
                            block owns each row, so the sums are deterministic)          */
    int64_t *tick;       /* [1]   += 1 per gw_step (e.g. the replay ring's step count)   */
    uint32_t *desc_copy; /* [E][12] a second destination of the step's obs descriptors
                            (gw_obs_view's layout; e.g. a descriptor replay ring's slot,
                            include/rollout_ops.h gw_replay_gather_desc); the terminal half
                            (words 8-11) only for envs that ended                         */
} gw_step_out;

#define GW_STATS 8

/* Env state (device arrays owned by the handle), structure of arrays. */
typedef struct gw_state {
    int32_t *pos;        /* [N][E] cell r*W+c of agent n            (World.AgentLocations) */
    uint32_t *flags;     /* [E] bits 0-7 apples present, 8-15 terminations, 16-23 truncations */
    int32_t *t;          /* [E] moves in the episode                 (num_moves)          */
    uint32_t *episode;   /* [E] episode counter (RNG)                                     */
    int32_t *prev_dist;  /* [K][E] previous distance to own apple, -1 = None              */
    double *score;       /* [E] running episode score                                     */
    double *fear_score;  /* [E] running episode fear score                                */
} gw_state;

/* CustomMAEnv(render=False, fear=cfg->fear, seed=cfg->seed) x E  (ma_customenv.py:74-108).
 * Allocates the state on `device`.  The envs are unusable until gw_reset. */
gw_status gw_create(const gw_scenario *sc, const gw_config *cfg, int device, void **out_env);

/* CustomMAEnv.reset (ma_customenv.py:169-215) for every env with env_mask[e] != 0
 * (env_mask NULL = all).  spawn_cells: [E][N] sorted road cells (replay) or NULL (Philox
 * spawn).  obs [K][E][H*W] and mask [E][K] are written for the reset envs (either may be
 * NULL). */
gw_status gw_reset(void *env, const uint8_t *env_mask, const int32_t *spawn_cells, float *obs,
                   uint16_t *mask, void *stream);

/* CustomMAEnv.step (ma_customenv.py:217-334) on all E envs at once.
 *   rl_actions [E][K] int32 in 0..8, or NULL = uniform random RL policy (Philox)
 *   scripted   [E][N-K] int32 actions of the scripted agents (replay), or NULL = the
 *              scenario policy sampled on device (ma_customenv.py:432-452)
 *   spawn      [E][N] spawn cells for envs that auto-reset (replay), or NULL = Philox */
gw_status gw_step(void *env, const int32_t *rl_actions, const int32_t *scripted,
                  const int32_t *spawn, const gw_step_out *out, void *stream);

/* Device pointers of the state arrays (valid until gw_destroy). */
gw_status gw_state_view(void *env, gw_state *out);

/* Copy the whole state to (to_env = 0) or from (to_env = 1) caller buffers with the
 * gw_state layout (device or pinned host memory), enqueued on stream. */
gw_status gw_copy_state(void *env, const gw_state *buf, int to_env, void *stream);

/* Per-launch timing: while enabled, the env's kernels carry HIP timing events in their dispatch
 * (start / stop of the launch itself, on the stream each is launched on), one span per launch
 * group of a kind: GW_SPAN_STEP the world-update kernel (step_v2), GW_SPAN_OBS the obs writer
 * (obs_kernel; the merged path's step_obs), GW_SPAN_FEAR the deferred FeAR kernel (fear_v2,
 * GW_KERNEL=defer only; it runs concurrently with the writer), and the ops that take this env's
 * handle: GW_SPAN_ACT the fused actors' MLP kernel (act_kernel of gw_actor_act,
 * gw_patch_actor_act, gw_cnn_act, gw_patch_cnn_act), GW_SPAN_CNN_L1 the CNN heads' layer-1
 * listing kernel, GW_SPAN_CNN_LIST their bucket scan + unit plan and scatter (two launches), GW_SPAN_CNN_RARE
 * their recompute of the listed conv positions, GW_SPAN_WINDOW the window writer (gw_obs_patch),
 * GW_SPAN_LEARN one whole descriptor-learner update (gw_maddpg_desc_update's four launches).
 * enable > 1 also makes sure `enable` timing events exist now (creating them inside a profiled
 * step would put their host cost between its launches).  gw_profile_read synchronises on those
 * events, returns the summed elapsed milliseconds of the first three kinds and the number of
 * gw_step calls timed, and clears every span.  Used by bench.py for the live roofline. */
enum {
    GW_SPAN_STEP = 0, GW_SPAN_OBS = 1, GW_SPAN_FEAR = 2, GW_SPAN_ACT = 3, GW_SPAN_CNN_L1 = 4,
    GW_SPAN_CNN_LIST = 5, GW_SPAN_CNN_RARE = 6, GW_SPAN_WINDOW = 7, GW_SPAN_LEARN = 8
};
gw_status gw_profile(void *env, int enable);
gw_status gw_profile_read(void *env, double out_ms[3], int64_t *n_steps);
/* The spans gw_profile_read would sum, one by one (call it first: gw_profile_read clears them):
 * out[3 i + 0] = kind (GW_SPAN_*), out[3 i + 1] / [3 i + 2] = the
 * launch's start / end in milliseconds after the first span's start; at most cap spans are
 * written, *n_spans = how many exist.  Synchronises on their events.  bench.py merges the obs
 * writers' intervals (writers of consecutive steps overlap on two streams) into the writer's
 * busy time per launch. */
gw_status gw_profile_spans(void *env, double *out, int64_t cap, int64_t *n_spans);

/* Responsibility.FeAR (custom/Responsibility.py:57-132: the N x N Resp matrix, every agent as
 * actor) and FeAL (:213-303) for n world snapshots of this env's map and N, on the device:
 *   cells [n][N] agent cells, actions [n][N] the joint action, mdr [n][N] moves de rigueur
 *   (NULL = the scenario's per-cell MdR), in_list [n] bit a = agent a is in ActionID4Agents
 *   (unlisted agents stay and ignore swaps, as CustomMAEnv's close_agents lists; NULL = all);
 *   resp [n][N][N] f64, vm / va [n][N][N] ValidMoves_moveDeRigueur / _action, feal [n][N] f64,
 *   feal_vm / feal_va [n][N] (each output but resp may be NULL).  Enqueued on stream. */
gw_status gw_fear_matrix(void *env, int64_t n, const int32_t *cells, const int32_t *actions,
                         const int32_t *mdr, const uint8_t *in_list, double *resp, int32_t *vm,
                         int32_t *va, double *feal, int32_t *feal_vm, int32_t *feal_va, void *stream);

/* Rows of the gw_step_out.stats buffer (one per kernel block; GW_KERNEL=defer: the world-update
 * kernel's rows then fear_v2's rows, each kernel filling the fields it owns, zeros elsewhere). */
int64_t gw_stats_rows(void *env);

/* The kernel path gw_create chose: 3 "defer", 4 "merged" (values 0-2 named the round-1..5 A/B
 * paths "v1", "split", "fused", removed in round 6).  "merged" when a step's obs is at most
 * GW_MERGE_BYTES (default 160 MiB: small batches, bound by the step's latency chain, gain from
 * one step_obs launch per pipelined step), else "defer"; GW_KERNEL=defer|merged forces one (both
 * produce the same results).  -1 on a null handle. */
int64_t gw_kernel_path(void *env);

/* After replaying (on `stream`) a HIP graph of captured gw_step calls: the env's host-side
 * pipeline state is again the one the capture ended in (merged path with async obs: the
 * writer of the last captured step is queued, for the next gw_step or fence).  The capture
 * itself leaves that state; a fence between replays clears it, this re-arms it. */
gw_status gw_graph_replayed(void *env, void *stream);

/* The host-side pipeline state of the merged path's async obs (the queued writer's parameters,
 * the descriptor buffer in use) as an opaque blob of gw_pipeline_state_bytes() bytes.  For callers
 * that capture several HIP graphs of steps writing DIFFERENT buffers (a replay ring's slots, one
 * graph per ring phase): save the state after capturing each graph and load it after replaying
 * that graph, so the next eager step, graph or fence launches the right queued writer (on
 * `stream`).  Synchronous obs leaves nothing queued; the defer path's pipeline is not capturable. */
int64_t gw_pipeline_state_bytes(void);
gw_status gw_pipeline_save(void *env, void *buf);
gw_status gw_pipeline_load(void *env, const void *buf, void *stream);

/* What the observation an env last wrote (gw_reset / gw_step) is made of, for ops that work
 * on it without reading it back (actor_ops.h): the static step-encoding map plus, per env, a
 * 48-byte descriptor (agent cells, reset / apple flags; ma_customenv.py:197-209, 303-322).
 * Device pointers owned by the handle, valid until gw_destroy; contents change with every
 * gw_reset / gw_step (stream-ordered; with async obs the desc pointer alternates per step). */
typedef struct gw_obs_source {
    const uint32_t *desc;      /* [E][12] u32: words 0-3 agent cells (16 bits each), word 4
                                  flags (bit 0 reset encoding, bits 8-15 apples present)      */
    const float *base;         /* [H*W] 0 road, -1 inactive                                   */
    int32_t apples[GW_MAX_AGENTS];  /* apple cell of RL agent k                               */
    int32_t N, K, H, W, variant;
    int64_t E, env_offset;
} gw_obs_source;
gw_status gw_obs_view(void *env, gw_obs_source *out);

/* Copy the descriptors of the last gw_reset / gw_step ([E][12] u32, as gw_obs_view's desc) to
 * dst, enqueued on stream after that step (a replay ring of descriptors: gw_replay_gather_desc,
 * include/rollout_ops.h). */
gw_status gw_obs_desc_copy(void *env, uint32_t *dst, void *stream);

/* Count the FeAR counterfactual world updates (custom/Responsibility.py:16-54's sims, after the
 * exact de-duplication of DESIGN §5.2: one base sim per (actor, variant) and the 8 other actions of
 * each close affected agent per variant) the env's FeAR kernels run from now on: every block adds
 * its task count to *counter (device uint64, one atomic per block per step).  counter NULL: stop
 * counting (the default).  bench.py reports sims/s from it beside the VALU roofline. */
gw_status gw_count_sims(void *env, uint64_t *counter);

/* Egocentric local patches of the env's last observation (an opt-in input format; the
 * reference observes the whole grid, ma_customenv.py:303-322): for every env and RL agent k the
 * P x P window of that agent's obs centred on its own cell (rows / cols -P/2 .. P-1-P/2), cells
 * outside the grid -1.  patch [K][E][P][P] f32 (envs whose obs the last gw_step / gw_reset
 * wrote), final_patch [K][E][P][P] (the terminal obs of envs done at the last step, centred on
 * the terminal cell); either may be NULL.  Works from the descriptors, so it needs no full obs
 * (gw_step_out.obs may be NULL).  Enqueued on stream, after the step on the same stream. */
gw_status gw_obs_patch(void *env, int32_t P, float *patch, float *final_patch, void *stream);
/* Arm the NEXT gw_step to also write its P x P windows exactly as gw_obs_patch(env, P, patch,
 * final_patch) right after it would: with FeAR on (joined) and the row writer's conditions
 * (2 <= P <= 16, E % 4 == 0) inside the FeAR launch (both read only the world update's outputs),
 * else as that gw_obs_patch on the step's stream.  One request per step (cleared by gw_step). */
gw_status gw_step_patch_next(void *env, int32_t P, float *patch, float *final_patch);

/* Async observation writes (a software pipeline across steps; default off).  While enabled,
 * gw_step enqueues the world update (+ FeAR) on an internal stream that waits for the caller's
 * prior work on `stream`, and `stream` joins it: rewards, dones, masks, state and stats are
 * stream-ordered as in the synchronous mode.  The observation writer of the step runs on a
 * second internal stream and overlaps the NEXT step's world update (which reads only the
 * state).  The obs / final_obs buffers of a step are therefore ready on `stream` only after
 * gw_obs_fence(env, stream) (or gw_reset, which fences itself).  The obs descriptor alternates
 * between two buffers: re-read gw_obs_view after every gw_step.  Disabling drains the writer.
 * enable = 1: the writer starts right after the step's world update; enable = 2 (lazy): it is
 * launched at the start of the next gw_step (behind the caller's work between the steps, e.g.
 * an actor kernel that should not share the CUs with it) or at a fence.
 * enable | 4 (defer path, FeAR on): `stream` joins only the world update; fear_v2 (fear,
 * shaped, ep_return, ep_fear, the FeAR stats rows, score / fear_score) finishes on the internal
 * stream and overlaps the caller's next work (an actor that needs only the descriptors and
 * masks); those outputs are ready on `stream` after gw_fear_fence (gw_reset, gw_copy_state
 * and the next gw_step order themselves).
 * Both kernel paths pipeline (defer: the writer on its own streams; merged: one step_obs launch). */
gw_status gw_set_obs_async(void *env, int enable);

/* Observation element type of every obs / final_obs buffer the env writes (gw_reset, gw_step):
 * GW_OBS_F32 (default; the reference's values as float32) or GW_OBS_BF16 (the same values as
 * bfloat16 bits, [K][E][H*W] uint16: every value the env produces is exact in bf16, so this is
 * lossless and halves the obs bytes; needs H*W % 8 == 0).
 * The float* obs pointers then address bf16 buffers.  Called before the first gw_reset it may
 * also change gw_stats_rows (the FeAR kernel's envs per block follow the format's best choice):
 * size the stats buffer after it. */
enum { GW_OBS_F32 = 0, GW_OBS_BF16 = 1 };
gw_status gw_set_obs_dtype(void *env, int dtype);

/* The FeAR kernel's envs per block, before the first gw_reset (it fixes gw_stats_rows: size the
 * stats buffer after it): wide = 1 (the default: half the resident waves, best beside the full-obs
 * writer), 0 = narrow (twice the waves, best where FeAR is on the critical path: an env that writes
 * no full obs, e.g. the local-window rollouts; c5patch 115 -> 111-112 us per step).
 * GW_FEAR_BE=wide|narrow in the environment overrides it.  GW_ERR_STATE after gw_reset. */
gw_status gw_set_fear_blocks(void *env, int wide);
gw_status gw_obs_fence(void *env, void *stream);
gw_status gw_fear_fence(void *env, void *stream);
/* Set the thread-local error text returned by gw_last_error (for the library's other
 * translation units: learner_ops, actor_ops). */
void gw_set_last_error(const char *msg);
/* Sizes: H, W, N, K, E (out[0..4]). */
gw_status gw_dims(void *env, int64_t out[5]);

/* Thread-local description of the last error. */
const char *gw_last_error(void);

void gw_destroy(void *env);

#ifdef __cplusplus
}
#endif
#endif /* GRIDENV_H */
