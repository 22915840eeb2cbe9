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

#ifdef __cplusplus
}
#endif
#endif
