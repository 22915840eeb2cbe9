/* Rollout bookkeeping ops of libgridenv.so (marlnav/rollout.py, marlnav/parallel.py).
 *
 * Per step the batched rollout (maddpg/agent.py:124-173 over E envs) folds the step kernels'
 * per-block partial sums (gw_step_out.stats: completed-episode returns, episodes, FeAR, crashes,
 * apples, shaped rewards, lengths, env-steps) into running totals and advances the replay
 * ring's device-side step count.  As PyTorch ops that is a generic reduction, an add and an
 * increment (three launches, ~20 us at 65,536 envs); here it is one single-block launch.
 * Plain device pointers; enqueued on `stream`; statuses as in gridenv.h. */
#ifndef ROLLOUT_OPS_H
#define ROLLOUT_OPS_H

#include <stdint.h>

#include "gridenv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* s[f] = sum over r of partials[r][f] (r ascending per lane stride, then a fixed tree: the
 * result is deterministic); row_sum[f] = s[f] if row_sum != NULL; totals[f] += s[f] if
 * totals != NULL; *counter += 1 if counter != NULL.  n_fields <= 64. */
gw_status gw_rollout_tick(const double *partials, int64_t rows, int32_t n_fields, double *row_sum,
                          double *totals, int64_t *counter, void *stream);

/* Completed-episode return compaction of a window of gathered steps (marlnav/parallel.py
 * ReturnGather.compact; the reference appends scores[i] to completed_episode_scores for every
 * env done this step, maddpg/agent.py:229-247).  recv holds `steps` x `world` slots of
 * slot_bytes bytes: [emax] f64 returns, then [emax] u8 done flags (slot_bytes % 8 == 0,
 * slot_bytes >= 9 * emax).  Every done element, in (step, rank, env) order, is appended to the
 * ring scores[capacity] at (*n_completed + its rank) % capacity (only the last `capacity` of
 * the window are written), and *n_completed grows by the window's count.  scratch:
 * gw_return_compact_scratch(steps, world, emax) int32 words of device memory.  Two launches,
 * deterministic, no host synchronisation (graph-capturable). */
gw_status gw_return_compact(const uint8_t *recv, int64_t steps, int32_t world, int64_t emax,
                            int64_t slot_bytes, double *scores, int64_t capacity,
                            int64_t *n_completed, int32_t *scratch, void *stream);
int64_t gw_return_compact_scratch(int64_t steps, int32_t world, int64_t emax);

/* The packed per-step return gather of several ranks (marlnav/parallel.py ReturnGather, world > 1;
 * the reference's completed_episode_scores, maddpg/agent.py:229-247).  Instead of every env's
 * return + done flag (9 B per env per step), a rank sends only its completed episodes' returns:
 *
 * gw_gather_pack (sender, per step): this step's done envs' ep_return (env order) are appended to
 * the rank's FIFO fifo[fifo_cap] (ring, state ctl[4] = {head, tail, overflow, 0} int64, zeroed at
 * start); the send slot (32 + 8 cap bytes) gets the header {count, sent, backlog after, overflow}
 * (int64) and the FIFO's first sent = min(backlog, cap) entries.  scratch:
 * gw_gather_pack_scratch(E) int32 words.  Two launches, no host synchronisation.
 *
 * gw_gather_unpack (receiver, per window of `steps` gathered slots [steps][world][slot_bytes]):
 * appends every rank's payload to its mirror FIFO (mirror[world][mirror_cap]), queues the per-step
 * counts in pend[pend_cap][world], and appends to the score ring scores[capacity] (the last
 * `capacity` kept; *n_completed = completions ever) every pending step whose entries have all
 * arrived, in (step, rank, env) order: the reference's order with rank-major contiguous shards.
 * rstate: int64 [2 world + 4] = {received per rank, emitted per rank, pending head, pending tail,
 * overflow (sticky: a FIFO, mirror or pending ring ran out), max sender backlog of the window},
 * zeroed at start.  plan: gw_gather_unpack_plan_cap(steps, world, pend_cap) segments of 40 bytes
 * + 32 bytes.  Three launches, no host synchronisation. */
int64_t gw_gather_pack_scratch(int64_t E);
gw_status gw_gather_pack(const double *ep_return, const uint8_t *done, int64_t E, int64_t cap, double *fifo,
                         int64_t fifo_cap, int64_t *ctl, int32_t *scratch, uint8_t *slot, void *stream);
int64_t gw_gather_unpack_plan_cap(int64_t steps, int32_t world, int64_t pend_cap);
gw_status gw_gather_unpack(const uint8_t *recv, int64_t steps, int32_t world, int64_t slot_bytes, double *mirror,
                           int64_t mirror_cap, int64_t *rstate, int32_t *pend, int64_t pend_cap, void *plan,
                           int64_t plan_cap, double *scores, int64_t capacity, int64_t *n_completed, void *stream);

/* Replay-ring sample (agilerl MultiAgentReplayBuffer.sample, uniform; called at
 * maddpg/agent.py:209-211; marlnav/rollout.py ReplayRing.sample) as ONE gather launch.  Ring
 * layout: obs / final_obs [S, K, E, HW] (f32, or bf16 if obs_bf16), probs [S, K, E, 9] f32,
 * reward [S, E, K] f64, term [S, E, K] u8, done [S, E] u8; *t_dev = transitions stored.  For each
 * b < B:  n = clamp(*t_dev, 1, S - 1);  step = min((int64)(u[b] * (float)n), n - 1);
 * tr = (*t_dev - 1 - step) mod S;  nx = (tr + 1) mod S;  e = env[b];  then
 *   state[k, b] = obs[tr, k, e];  next[k, b] = done[tr, e] ? final_obs[tr, k, e] : obs[nx, k, e]
 *   probs_out[k, b] = probs[tr, k, e];  reward_out[b] = reward[tr, e];  term_out[b] = term[tr, e]
 * (outputs f32 [K, B, HW], [K, B, 9], f64 [B, K], u8 [B, K]); tr_out[b] = tr if tr_out != NULL.
 * x_out / xn_out (may be NULL): the critic's input rows [B, K*HW + K*9] of MADDPG.learn, agent-major
 * states then the K action slots (agilerl's torch.cat of states and actions):
 *   x_out[b] = [state[0, b] .. state[K-1, b], probs_out[0, b] .. probs_out[K-1, b]];
 *   xn_out[b][0, K*HW) = next_state[., b] (its action slots are left to the caller).
 * u = env = NULL: u[b] and e drawn in the kernel from Philox4x32-10(key seed; counter (b, *ctr,
 * 'SAMP', 0)) (the uniform from the first word, e = (second word * E) >> 32), as
 * gw_replay_gather_desc does, so both samplers pick the same rows. */
gw_status gw_replay_gather(const void *obs, const void *final_obs, int32_t obs_bf16, const float *probs,
                           const double *reward, const uint8_t *term, const uint8_t *done, const int64_t *t_dev,
                           const float *u, const int64_t *env, int64_t S, int32_t K, int64_t E, int64_t HW,
                           int64_t B, float *state, float *next_state, float *probs_out, double *reward_out,
                           uint8_t *term_out, int64_t *tr_out, float *x_out, float *xn_out, uint64_t seed,
                           const int32_t *ctr, void *stream);

/* gw_replay_gather with the obs rows expanded from a ring of obs descriptors instead of read
 * from the dense obs / final_obs slots (the learner then never waits for the obs writer of the
 * step it follows; the rows are bit for bit the ones the obs writer put in the ring).
 * desc [S][E][12] u32: slot j holds the descriptors of the step whose obs went to obs slot j
 * (gw_obs_desc_copy after that step, into slot j); the terminal obs of transition slot tr
 * comes from the terminal half of descriptor slot tr + 1.  src: gw_obs_view of the env
 * (base map, apple cells, N, K, H, W, variant, E; its desc pointer is not used).  Every other
 * argument and output as gw_replay_gather (f32 rows; K = src->K, HW = src->H * src->W <= 4096).
 * u = env = NULL: the (transition, env) draws are made in the kernel instead of read: row b's
 * uniform and env index from Philox4x32-10(key seed; counter (b, *ctr, 'SAMP', 0)), the env as
 * the multiply-high of a 32-bit draw and E (ctr: a device int32 that changes per sample, e.g.
 * the critic optimizer's step count before the update advances it).  state / next_state may be
 * NULL when x_out and xn_out are given (the fused learner reads only the critic rows). */
gw_status gw_replay_gather_desc(const gw_obs_source *src, const uint32_t *desc, const float *probs,
                                const double *reward, const uint8_t *term, const uint8_t *done, const int64_t *t_dev,
                                const float *u, const int64_t *env, int64_t S, int64_t B, float *state,
                                float *next_state, float *probs_out, double *reward_out, uint8_t *term_out,
                                int64_t *tr_out, float *x_out, float *xn_out, uint64_t seed, const int32_t *ctr,
                                void *stream);

/* One evaluation step's totals (customeval.py:70-133 over E episodes at once; marlnav/evaluate.py):
 * for every env e with active[e]:  counts[0] += crashes[e];  counts[1] += apples[e];
 * counts[2] += 1;  *fear_total += sum_k fear[e, k];  then active[e] = 0 if done[e].
 * crashes / apples [E] i32, fear [E, K] f64, done / active [E] u8.  One block, fixed order. */
gw_status gw_eval_accum(const int32_t *crashes, const int32_t *apples, const double *fear, const uint8_t *done,
                        uint8_t *active, int64_t *counts, double *fear_total, int64_t E, int32_t K, void *stream);

#ifdef __cplusplus
}
#endif
#endif
