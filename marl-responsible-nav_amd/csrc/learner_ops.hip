// Flat-buffer Adam and soft target update for the MADDPG learner (include/learner_ops.h).
// torch's fused/foreach Adam gives each 65,536-element chunk of a tensor one workgroup, so a
// 0.5 M-parameter network gets ~9 workgroups and 77 us per step on MI355X; these are plain
// grid-stride elementwise kernels over the whole flat buffer (float4 where aligned).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "learner_ops.h"

namespace {

__global__ void __launch_bounds__(256) adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                   float *__restrict__ m, float *__restrict__ v,
                                                   const int32_t *__restrict__ step, int64_t n, double lr,
                                                   double beta1, double beta2, double eps) {
    // the scalars exactly as torch's single-tensor Adam forms them: in double on the host side
    // (Python floats), rounded to float where they meet the f32 tensors
    const double s = (double)(step[0] + 1);
    const float step_size = (float)(lr / (1.0 - pow(beta1, s)));
    const float bc2_sqrt = (float)sqrt(1.0 - pow(beta2, s));
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2), e = (float)eps;
    // torch's elementwise kernels are built with FMA contraction; each torch op below is one
    // rounding (or one fma), and this file is built -ffp-contract=off, so the fmas are explicit
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i];
        const float mi = __fmaf_rn(w1, gi - m[i], m[i]);         // exp_avg.lerp_(grad, 1 - beta1)
        const float vi = __fmaf_rn(w2 * gi, gi, v[i] * b2);      // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + e;             // (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
        p[i] = __fmaf_rn(-step_size, mi / denom, p[i]);          // param.addcdiv_(exp_avg, denom, -step_size)
    }
}

__global__ void step_inc(int32_t *step) { step[0] += 1; }

__global__ void __launch_bounds__(256) soft_update_kernel(float *__restrict__ t, const float *__restrict__ p,
                                                          int64_t n, float tau) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        t[i] = tau * p[i] + (1.0f - tau) * t[i];
}

unsigned grid_for(int64_t n) {
    const int64_t blocks = (n + 255) / 256;
    return (unsigned)(blocks < 4096 ? (blocks > 0 ? blocks : 1) : 4096);
}

}  // namespace

extern "C" {

gw_status gw_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                       int64_t n, double lr, double beta1, double beta2, double eps, void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n < 0) return GW_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, s, param, grad, exp_avg, exp_avg_sq, step, n,
                       lr, beta1, beta2, eps);
    hipLaunchKernelGGL(step_inc, dim3(1), dim3(1), 0, s, step);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_soft_update(float *target, const float *online, int64_t n, float tau, void *stream) {
    if (!target || !online || n < 0) return GW_ERR_ARG;
    hipLaunchKernelGGL(soft_update_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       target, online, n, tau);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

}  // extern "C"
