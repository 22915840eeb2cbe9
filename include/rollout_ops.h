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

#ifdef __cplusplus
}
#endif
#endif
