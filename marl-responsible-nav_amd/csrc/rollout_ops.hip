// rollout_ops.hip — the batched rollout's per-step bookkeeping in one launch (include/rollout_ops.h).
#include <hip/hip_runtime.h>

#include <string>

#include "rollout_ops.h"

namespace {

constexpr int T = 1024, MAXF = 64, U = 8;

// one block: lane group g = tid / n_fields sums rows g, g + G, ... of field tid % n_fields (U
// loads in flight per lane, added in row order), then the G group sums of each field meet in a
// fixed binary tree: deterministic
__global__ void __launch_bounds__(T) tick_kernel(const double *__restrict__ partials, int64_t rows, int nf,
                                                 double *__restrict__ row_sum, double *__restrict__ totals,
                                                 int64_t *__restrict__ counter) {
    __shared__ double part[T];
    const int tid = threadIdx.x, groups = T / nf, g = tid / nf, f = tid % nf;
    double s = 0.0;
    if (g < groups) {
        for (int64_t r0 = g; r0 < rows; r0 += (int64_t)U * groups) {
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = r0 + (int64_t)u * groups;
                v[u] = r < rows ? partials[r * nf + f] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) s = __dadd_rn(s, v[u]);
        }
    }
    part[tid] = s;
    __syncthreads();
    int pow2 = 1;
    while (pow2 * 2 <= groups) pow2 *= 2;
    if (g >= pow2 && g < groups) part[(g - pow2) * nf + f] = __dadd_rn(part[(g - pow2) * nf + f], s);
    __syncthreads();
    for (int stride = pow2 / 2; stride >= 1; stride /= 2) {
        if (g < stride) part[g * nf + f] = __dadd_rn(part[g * nf + f], part[(g + stride) * nf + f]);
        __syncthreads();
    }
    if (tid < nf) {
        const double t = part[tid];
        if (row_sum) row_sum[tid] = t;
        if (totals) totals[tid] = __dadd_rn(totals[tid], t);
    }
    if (tid == 0 && counter) counter[0] += 1;
}

}  // namespace

extern "C" {

gw_status gw_rollout_tick(const double *partials, int64_t rows, int32_t n_fields, double *row_sum, double *totals,
                          int64_t *counter, void *stream) {
    if ((rows > 0 && !partials) || n_fields < 1 || n_fields > MAXF || rows < 0) {
        gw_set_last_error("gw_rollout_tick: bad argument");
        return GW_ERR_ARG;
    }
    hipLaunchKernelGGL(tick_kernel, dim3(1), dim3(T), 0, static_cast<hipStream_t>(stream), partials, rows, n_fields,
                       row_sum, totals, counter);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gw_set_last_error((std::string("gw_rollout_tick: ") + hipGetErrorString(e)).c_str());
        return GW_ERR_HIP;
    }
    return GW_OK;
}

}  // extern "C"
