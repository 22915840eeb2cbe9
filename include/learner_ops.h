/* Learner ops of libgridenv.so: the optimizer and target-network updates of the MADDPG learner
 * (marlnav/maddpg.py) over flat float32 parameter buffers, one launch each, graph-capturable
 * (the Adam step count lives on the device).  Plain device pointers; enqueued on `stream`. */
#ifndef LEARNER_OPS_H
#define LEARNER_OPS_H

#include <stdint.h>

#include "gridenv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* torch.optim.Adam (no weight decay, no amsgrad; torch/optim/adam.py _single_tensor_adam) on n
 * elements:  m = lerp(m, g, 1 - beta1);  v = beta2 * v + (1 - beta2) * g * g;  s = step[0] + 1
 *   p -= lr / (1 - beta1^s) * (m / (sqrt(v) / sqrt(1 - beta2^s) + eps));   then step[0] = s.
 * The scalar hyper-parameters are doubles and the bias corrections are formed in double, as
 * torch forms them from Python floats, then rounded to float against the f32 tensors. */
gw_status gw_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                       int64_t n, double lr, double beta1, double beta2, double eps, void *stream);

/* agilerl soft_update: target = tau * online + (1 - tau) * target on n elements. */
gw_status gw_soft_update(float *target, const float *online, int64_t n, float tau, void *stream);

#ifdef __cplusplus
}
#endif
#endif
