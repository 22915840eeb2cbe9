/*
 * oracle/gw_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference grid-world hot path
 * (Henweiz/MARL-Responsible-Nav: custom/grid_world.py, custom/Responsibility.py,
 * custom/ma_customenv.py, and the rollout arithmetic of maddpg/agent.py).
 *
 * It is the CHECKER for the HIP path, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Parity of this restatement is pinned against golden vectors generated from
 * the reference Python itself (tests/golden/make_golden.py); see DESIGN.md §3.
 *
 * Conventions: a cell is r*W + c (row-major, rows grow downward).
 * Action ids follow custom/custom_agent.py:41-178:
 *   0 Stay, 1 Up1, 2 Down1, 3 Left1, 4 Right1, 5 Up2, 6 Down2, 7 Left2, 8 Right2.
 */
#ifndef GW_ORACLE_H
#define GW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_N 8
#define ORC_NA 9

/* Static world description shared by all envs (scenario compiled on the host). */
typedef struct orc_world {
    int32_t H, W, N, K;
    const uint8_t *region;     /* [H*W] 1 active road, 0 inactive      grid_world.py:29-30   */
    const uint8_t *policy_id;  /* [H*W] policy index                   ma_customenv.py:346-354 */
    const double *policy_cdf;  /* [P][2][9] numpy-legacy-choice CDFs: [.][0] scenario weights,
                                  [.][1] uniform-direction branch      ma_customenv.py:441-449 */
    const uint8_t *mdr;        /* [H*W] MdR action id per cell          ma_customenv.py:357-365 */
    const int32_t *apples;     /* [K] apple cell of RL agent k          ma_customenv.py:422     */
    int32_t n_free;            /* number of road cells                  ma_customenv.py:373     */
    const int32_t *free_cells; /* [n_free] road cells, row-major order                          */
    int32_t fear;              /* compute FeAR (CustomMAEnv(fear=...))  ma_customenv.py:246     */
    double fear_weight;        /* INIT_HP["FeAR_weight"]                maddpg/agent.py:125     */
    int32_t max_steps;         /* TRAIN_STEPS episode cap               maddpg/agent.py:85,243  */
    uint64_t seed;             /* Philox key for native-RNG mode                                */
    int64_t env_offset;        /* global id of env 0 (RNG counter)                              */
    int32_t variant;           /* 0 CustomMAEnv (ma_customenv.py), 1 single-agent CustomEnv
                                  (customenv.py:78-183): K = 1, float rewards, no relabel       */
} orc_world;

/* Per-env mutable state. */
typedef struct orc_env {
    int32_t pos[ORC_MAX_N];       /* World.AgentLocations as cells                  */
    uint32_t apples;              /* bit k: "apple_k" still in self.apples          */
    uint32_t term;                /* bit k: self.terminations[agent_k] (persists)   */
    uint32_t trunc;               /* bit k: self.truncation[agent_k]  (persists)    */
    int32_t prev_dist[ORC_MAX_N]; /* self.prev_distance, -1 = None                   */
    int32_t t;                    /* self.num_moves                                  */
    uint32_t episode;             /* episodes started on this env (RNG counter)      */
    double score;                 /* maddpg/agent.py:173 scores[i]                   */
    double fear_score;            /* maddpg/agent.py:141 fear_score                  */
} orc_env;

/* Outputs of one env step. */
typedef struct orc_step_out {
    int32_t actions[ORC_MAX_N];   /* env.Action4Agents after the RL override          */
    int32_t mdr[ORC_MAX_N];       /* env.MdR4Agents                                   */
    int32_t final_pos[ORC_MAX_N]; /* positions after the move (before any auto-reset) */
    uint32_t crash_bits;          /* agent_crashes of UpdateGWorld (all N agents)     */
    uint32_t restricted_bits;     /* restricted_moves of UpdateGWorld                 */
    double reward[ORC_MAX_N];     /* env reward (int valued)                          */
    double fear[ORC_MAX_N];       /* info["fear"][agent]                              */
    double shaped[ORC_MAX_N];     /* FeAR_weight*FeAR + reward (maddpg/agent.py:130)  */
    uint8_t term[ORC_MAX_N];
    uint8_t trunc[ORC_MAX_N];
    uint16_t mask[ORC_MAX_N];     /* action mask (9 bits) of the obs returned          */
    int32_t crashes;              /* info["agent_crashes"]                            */
    int32_t apples_caught;        /* info["apples_caught"]                            */
    uint8_t done;                 /* all(term) or all(trunc) or t >= max_steps        */
    double ep_return;             /* score of the episode including this step          */
    double ep_fear;
    int32_t ep_len;
} orc_step_out;

/* ---- primitives ------------------------------------------------------------------ */

/* Philox4x32-10 (Salmon et al., SC'11). */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* numpy float64 np.sum(a) over a C-contiguous array of n elements
 * (0.0 + numpy pairwise_sum; 8-accumulator blocks, PW_BLOCKSIZE 128). */
double orc_np_sum(const double *a, int n);

/* GWorld.UpdateGWorld (custom/grid_world.py:424-563).  eaters are agents 0..n_eaters-1,
 * apple_cells[k] is apple k's cell or -1 if it has been eaten.  caught_pairs receives
 * (agent, apple) pairs in the order grid_world.py:533-540 appends them. Returns the total
 * number of collision-resolution passes over the 4 sub-steps. */
int orc_update_world(int H, int W, const uint8_t *region, int N, const int32_t *loc,
                     const int32_t *act, int n_eaters, const int32_t *apple_cells,
                     uint8_t *crash, uint8_t *restricted, int32_t *final_loc,
                     int32_t *caught_pairs, int32_t *n_caught);

/* Responsibility.FeAR_4_one_actor (custom/Responsibility.py:135-210) for the action list
 * (list_ids[i], list_acts[i]) produced by CustomMAEnv.close_agents.  resp is [N*N]
 * (only row `actor` is filled), vm/va are [N] (ValidMoves_moveDeRigueur / _action row).
 * Returns np.sum(resp) as ma_customenv.py:252 does. */
double orc_fear_one_actor(int H, int W, const uint8_t *region, int N, const int32_t *loc,
                          int list_len, const int32_t *list_ids, const int32_t *list_acts,
                          const int32_t *mdr_acts, int actor, double *resp, int32_t *vm,
                          int32_t *va);

/* Responsibility.FeAR (custom/Responsibility.py:57-132): the full N x N Resp matrix with every
 * agent as actor, for the action list (list_ids, list_acts); resp/vm/va are [N*N]. */
void orc_fear_matrix(int H, int W, const uint8_t *region, int N, const int32_t *loc, int list_len,
                     const int32_t *list_ids, const int32_t *list_acts, const int32_t *mdr_acts,
                     double *resp, int32_t *vm, int32_t *va);

/* Responsibility.FeAL (custom/Responsibility.py:213-303); feal/vm/va are [N]. */
void orc_feal(int H, int W, const uint8_t *region, int N, const int32_t *loc, int list_len,
              const int32_t *list_ids, const int32_t *list_acts, const int32_t *mdr_acts, double *feal,
              int32_t *vm, int32_t *va);

/* get_action_mask (custom/ma_customenv.py:467-506) as a 9-bit mask. */
uint16_t orc_action_mask(int H, int W, const uint8_t *region, int cell);

/* ---- env level ----------------------------------------------------------------- */

/* CustomMAEnv.reset (ma_customenv.py:169-215).  spawn: N cells (replay mode) or NULL
 * (native mode: Philox Floyd sampling, sorted).  obs: [K][H*W] f32 or NULL; mask: [K]. */
void orc_env_reset(const orc_world *w, int64_t env_id, orc_env *s, const int32_t *spawn,
                   float *obs, uint16_t *mask);

/* CustomMAEnv.step (ma_customenv.py:217-334) + the per-step rollout arithmetic of
 * MADDPGAgent.train (maddpg/agent.py:120-173, 226-243).
 *   rl_act   [K]   RL actions, or NULL = Philox-uniform random policy
 *   scripted [N-K] scripted actions (replay), or NULL = Philox scripted policy
 *   spawn    [N]   spawn for the auto-reset (replay), or NULL = Philox
 *   obs      [K][H*W] obs returned (reset obs when the env auto-reset), or NULL
 *   final_obs[K][H*W] terminal obs (written only when done), or NULL */
void orc_env_step(const orc_world *w, int64_t env_id, orc_env *s, const int32_t *rl_act,
                  const int32_t *scripted, const int32_t *spawn, int auto_reset, float *obs,
                  float *final_obs, orc_step_out *out);

/* Batched CPU step over E envs (the CPU baseline).  obs is [K][E][H*W] or NULL; the
 * per-env outputs are written to outs[E] (may be NULL).  nthreads OpenMP threads. */
void orc_vec_step(const orc_world *w, orc_env *envs, int64_t E, const int32_t *rl_act,
                  int auto_reset, float *obs, orc_step_out *outs, int nthreads);
/* The same; final_obs [K][E][H*W] (or NULL) receives the terminal obs of the envs that ended
 * this step (their rows are left untouched otherwise). */
void orc_vec_step_final(const orc_world *w, orc_env *envs, int64_t E, const int32_t *rl_act,
                        int auto_reset, float *obs, float *final_obs, orc_step_out *outs, int nthreads);
void orc_vec_reset(const orc_world *w, orc_env *envs, int64_t E, float *obs, int nthreads);

int orc_sizeof_env(void);
int orc_sizeof_step_out(void);

#ifdef __cplusplus
}
#endif
#endif
