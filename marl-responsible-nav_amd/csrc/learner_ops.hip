// Flat-buffer Adam and soft target update for the MADDPG learner (include/learner_ops.h).
// torch's fused/foreach Adam gives each 65,536-element chunk of a tensor one workgroup, so a
// 0.5 M-parameter network gets ~9 workgroups and 77 us per step on MI355X; these are plain
// grid-stride elementwise kernels over the whole flat buffer (float4 where aligned).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "learner_ops.h"

namespace {

// torch.optim.Adam on p[0, n) and, when t1 != null, the soft target update that follows it in
// MADDPG.learn (agilerl soft_update, both networks): t1[i] = tau p[i] + (1 - tau) t1[i] with the
// just-updated p[i] (same element, same thread), and t2 = tau p2 + (1 - tau) t2 on [n, n + n2)
// (the other network, already stepped): one launch instead of an Adam and a soft-update launch.
__global__ void __launch_bounds__(256) adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                   float *__restrict__ m, float *__restrict__ v,
                                                   int32_t *__restrict__ step, int64_t n, double lr,
                                                   double beta1, double beta2, double eps, float *__restrict__ t1,
                                                   float *__restrict__ t2, const float *__restrict__ p2, int64_t n2,
                                                   float tau, int advanced) {
    // the scalars exactly as torch's single-tensor Adam forms them: in double on the host side
    // (Python floats), rounded to float where they meet the f32 tensors
    // advanced: the count already includes this step (the caller's preceding launch advanced it);
    // else read by every block before the last one advances it (below)
    // the two bias corrections (double pow) once per block, not per thread
    __shared__ float s_sc[2];
    const int32_t st = step[0];
    if (threadIdx.x == 0) {
        const double s = (double)(advanced ? st : st + 1);
        s_sc[0] = (float)(lr / (1.0 - pow(beta1, s)));
        s_sc[1] = (float)sqrt(1.0 - pow(beta2, s));
    }
    __syncthreads();
    const float step_size = s_sc[0], bc2_sqrt = s_sc[1];
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2), e = (float)eps;
    const int64_t total = n + (t1 ? n2 : 0);
    // torch's elementwise kernels are built with FMA contraction; each torch op below is one
    // rounding (or one fma), and this file is built -ffp-contract=off, so the fmas are explicit
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        if (i >= n) {  // the other network's soft update (the soft_update2_kernel's op order)
            const int64_t j = i - n;
            t2[j] = tau * p2[j] + (1.0f - tau) * t2[j];
            continue;
        }
        const float gi = g[i];
        const float mi = __fmaf_rn(w1, gi - m[i], m[i]);         // exp_avg.lerp_(grad, 1 - beta1)
        const float vi = __fmaf_rn(w2 * gi, gi, v[i] * b2);      // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + e;             // (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
        const float pi = __fmaf_rn(-step_size, mi / denom, p[i]);  // param.addcdiv_(exp_avg, denom, -step_size)
        p[i] = pi;
        if (t1) t1[i] = tau * pi + (1.0f - tau) * t1[i];
    }
    // the last block to finish advances the step count: every block has read it by then (no
    // separate increment launch); step[1] counts the arrivals and is left at 0.  No fences: no
    // block reads what another block wrote (each block's read of step[0] completed before its
    // arrival: the loop above consumed it), and the kernel's end publishes the last block's
    // stores.  A device-scope fence per block writes back the XCD's L2 on gfx950 (~2,200 blocks
    // of this launch took 79 us instead of 9)
    // (same-address atomics from ~2,200 blocks still serialise: ~36 us per launch, so the learner
    // advances its counts in the gradient launch before the step instead: advanced = 1)
    if (advanced) return;
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(&step[1], 1) == (int32_t)gridDim.x - 1) {
        step[0] = st + 1;
        step[1] = 0;
    }
}

__global__ void __launch_bounds__(256) soft_update_kernel(float *__restrict__ t, const float *__restrict__ p,
                                                          int64_t n, float tau) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        t[i] = tau * p[i] + (1.0f - tau) * t[i];
}

// ---- hidden-layer epilogue of StackedMLPActors: y = relu(ln_b + layer_norm(z) * ln_w) ----------
// One 64-lane wave per row (h <= LN_MAXV * 64 features, lane j holds features j, j + 64, ...);
// the sums are wave butterflies in a fixed order, so results do not depend on the launch shape.
constexpr int LN_MAXV = 8;

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ void __launch_bounds__(256) ln_relu_fwd_kernel(const float *__restrict__ z, const float *__restrict__ w,
                                                          const float *__restrict__ b, float *__restrict__ y,
                                                          float *__restrict__ mean_out, float *__restrict__ rstd_out,
                                                          int64_t R, int64_t rows, int h, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= rows) return;  // uniform per wave
    const int64_t k = row / R;
    const float *zr = z + row * h;
    float v[LN_MAXV];
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int j = lane + 64 * i;
        v[i] = j < h ? zr[j] : 0.0f;
        s += v[i];
    }
    const float inv_h = 1.0f / (float)h;
    const float mean = wave_sum(s) * inv_h;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const float d = lane + 64 * i < h ? v[i] - mean : 0.0f;
        q = __fmaf_rn(d, d, q);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) * inv_h + eps);  // biased variance, as nn.LayerNorm
    float *yr = y + row * h;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int j = lane + 64 * i;
        if (j < h) {
            const float o = (v[i] - mean) * rstd * w[k * h + j] + b[k * h + j];  // addcmul: two roundings
            yr[j] = o > 0.0f ? o : 0.0f;
        }
    }
    if (mean_out && lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

// Backward of the epilogue, two launches:
//   rows (one wave per row, any number of rows in flight):
//     g = dy * (y > 0);  xhat = (z - mean) * rstd;  dxhat = g * w
//     dz = rstd * (dxhat - mean_j(dxhat) - xhat * mean_j(dxhat * xhat))
//   columns (block = 64 columns x 16 row groups of agent k, fixed-order sums: deterministic):
//     dW += sum_r g * xhat;  dB += sum_r g
__global__ void __launch_bounds__(256) ln_relu_bwd_rows_kernel(
    const float *__restrict__ dy, const float *__restrict__ z, const float *__restrict__ y,
    const float *__restrict__ w, const float *__restrict__ mean, const float *__restrict__ rstd,
    float *__restrict__ dz, int64_t R, int64_t rows, int h) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= rows) return;  // uniform per wave
    const int64_t k = row / R;
    const float m = mean[row], rs = rstd[row];
    float xh[LN_MAXV], dxh[LN_MAXV];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int j = lane + 64 * i;
        xh[i] = dxh[i] = 0.0f;
        if (j < h) {
            const int64_t o = row * h + j;
            const float g = y[o] > 0.0f ? dy[o] : 0.0f;
            xh[i] = (z[o] - m) * rs;
            dxh[i] = g * w[k * h + j];
            s1 += dxh[i];
            s2 = __fmaf_rn(dxh[i], xh[i], s2);
        }
    }
    const float inv_h = 1.0f / (float)h;
    const float m1 = wave_sum(s1) * inv_h, m2 = wave_sum(s2) * inv_h;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int j = lane + 64 * i;
        if (j < h) dz[row * h + j] = rs * (dxh[i] - m1 - xh[i] * m2);
    }
}

constexpr int LN_RG = 16;

__global__ void __launch_bounds__(LN_RG * 64) ln_relu_bwd_cols_kernel(
    const float *__restrict__ dy, const float *__restrict__ z, const float *__restrict__ y,
    const float *__restrict__ mean, const float *__restrict__ rstd, float *__restrict__ dw_acc,
    float *__restrict__ db_acc, int64_t R, int h) {
    __shared__ float s_dw[LN_RG][64], s_db[LN_RG][64];
    const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    const int64_t k = blockIdx.y;
    const bool ok = j < h;
    float pdw = 0.0f, pdb = 0.0f;
    if (ok) {
#pragma unroll 4
        for (int64_t r = rg; r < R; r += LN_RG) {
            const int64_t row = k * R + r, o = row * h + j;
            const float g = y[o] > 0.0f ? dy[o] : 0.0f;
            pdw = __fmaf_rn(g, (z[o] - mean[row]) * rstd[row], pdw);
            pdb += g;
        }
    }
    s_dw[rg][c] = pdw;
    s_db[rg][c] = pdb;
    __syncthreads();
    if (rg == 0 && ok) {
        float a = 0.0f, d = 0.0f;
        for (int q = 0; q < LN_RG; ++q) {
            a += s_dw[q][c];
            d += s_db[q][c];
        }
        if (dw_acc) dw_acc[k * h + j] += a;
        if (db_acc) db_acc[k * h + j] += d;
    }
}

// agilerl GumbelSoftmax sample without gradient (the target actors' next actions):
//   softmax((logits - log(-log(u + eps) + eps)) / tau) over the n entries of each row, each torch
//   op one f32 rounding; one lane per row.
__global__ void __launch_bounds__(256) gumbel_softmax_kernel(const float *__restrict__ logits,
                                                             const float *__restrict__ u, float *__restrict__ out,
                                                             int64_t rows, int n, float tau, float eps,
                                                             int64_t out_b, int64_t out_ld) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const float *lr = logits + r * n;
    const float *ur = u + r * n;
    // out_ld > 0: row r = k * out_b + b goes to out + b * out_ld + k * n (a critic-input slot)
    float *o = out_ld > 0 ? out + (r % out_b) * out_ld + (r / out_b) * n : out + r * n;
    float mx = -INFINITY;
    for (int j = 0; j < n; ++j) {
        const float g = logf(-logf(ur[j] + eps) + eps);
        const float v = (lr[j] - g) / tau;
        o[j] = v;
        mx = fmaxf(mx, v);
    }
    float sum = 0.0f;
    for (int j = 0; j < n; ++j) {
        const float e = expf(o[j] - mx);
        o[j] = e;
        sum += e;
    }
    for (int j = 0; j < n; ++j) o[j] = o[j] / sum;
}

// ---- affine + ReLU after torch's (non-affine) layer_norm: y = relu(ln_b + xhat * ln_w) ----------
// Forward: torch's addcmul (self + t1 * t2: the product rounded, then the sum) then relu, one launch.
__global__ void __launch_bounds__(256) affine_relu_fwd_kernel(const float *__restrict__ xh, const float *__restrict__ w,
                                                              const float *__restrict__ b, float *__restrict__ y,
                                                              int64_t R, int64_t n, int h) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / (R * h);
        const int j = (int)(i % h);
        const float o = xh[i] * w[k * h + j] + b[k * h + j];  // two roundings (file built -ffp-contract=off)
        y[i] = o > 0.0f ? o : 0.0f;
    }
}

// Backward for block (column chunk of 64, agent k): g = dy * (y > 0); dxh = g * w;
// dW += sum_r g * xh; dB += sum_r g.  AR_RG row groups of 64 columns each (1024 threads), rows
// strided over the groups with the loads of 4 rows in flight per thread; the group partials are
// combined in a fixed order (deterministic).
constexpr int AR_RG = 16;

__global__ void __launch_bounds__(AR_RG * 64) affine_relu_bwd_kernel(const float *__restrict__ dy,
                                                                    const float *__restrict__ xh,
                                                                    const float *__restrict__ y,
                                                                    const float *__restrict__ w,
                                                                    float *__restrict__ dxh, float *__restrict__ dw_acc,
                                                                    float *__restrict__ db_acc, int64_t R, int h) {
    __shared__ float s_dw[AR_RG][64], s_db[AR_RG][64];
    const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    const int64_t k = blockIdx.y;
    const bool ok = j < h;
    const float wj = ok ? w[k * h + j] : 0.0f;
    float pdw = 0.0f, pdb = 0.0f;
    if (ok) {
        const int64_t base = k * R * h + j;
#pragma unroll 4
        for (int64_t r = rg; r < R; r += AR_RG) {
            const int64_t o = base + r * h;
            const float g = y[o] > 0.0f ? dy[o] : 0.0f;
            if (dxh) dxh[o] = g * wj;
            pdw = __fmaf_rn(g, xh[o], pdw);
            pdb += g;
        }
    }
    s_dw[rg][c] = pdw;
    s_db[rg][c] = pdb;
    __syncthreads();
    if (rg == 0 && ok) {
        float a = 0.0f, d = 0.0f;
        for (int q = 0; q < AR_RG; ++q) {
            a += s_dw[q][c];
            d += s_db[q][c];
        }
        if (dw_acc) dw_acc[k * h + j] += a;
        if (db_acc) db_acc[k * h + j] += d;
    }
}

// Two soft target updates (actor and critic buffers) in one launch.
__global__ void __launch_bounds__(256) soft_update2_kernel(float *__restrict__ t1, const float *__restrict__ p1, int64_t n1,
                                                           float *__restrict__ t2, const float *__restrict__ p2, int64_t n2,
                                                           float tau) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < n1)
            t1[i] = tau * p1[i] + (1.0f - tau) * t1[i];
        else
            t2[i - n1] = tau * p2[i - n1] + (1.0f - tau) * t2[i - n1];
    }
}

// TD target of MADDPG.learn: y[k, b] = r + (1 - d) * gamma * q_next in torch's op order, one
// f32 rounding per op (r: the f64 shaped reward rounded to f32).
__global__ void __launch_bounds__(256) td_target_kernel(const double *__restrict__ r, const uint8_t *__restrict__ d,
                                                        const float *__restrict__ q_next, float gamma,
                                                        float *__restrict__ y, int K, int64_t B) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // i = k * B + b
    if (i >= (int64_t)K * B) return;
    const int64_t k = i / B, b = i % B;
    const float t1 = 1.0f - (float)d[b * K + k];
    const float t2 = t1 * gamma;
    const float t3 = t2 * q_next[i];
    y[i] = (float)r[b * K + k] + t3;
}

// Per-agent losses of MADDPG.learn over q [K, B]: mode 0 MSE (mean_b (q - y)^2, the critic),
// mode 1 -mean_b q (the actor).  Forward: one 256-thread block per agent (fixed-order sum).
// Backward: dq[k, b] = (g[k] / B) * (2 (q - y)) or -(g[k] / B), torch's op order bit for bit.
__global__ void __launch_bounds__(256) mean_loss_fwd_kernel(const float *__restrict__ q, const float *__restrict__ y,
                                                            float *__restrict__ loss, int64_t B, int mode) {
    __shared__ float part[256];
    const int64_t k = blockIdx.x;
    float acc = 0.0f;
    for (int64_t b = threadIdx.x; b < B; b += 256) {
        const float v = q[k * B + b];
        if (mode == 0) {
            const float d = v - y[k * B + b];
            acc += d * d;
        } else {
            acc += v;
        }
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[k] = mode == 0 ? part[0] / (float)B : -(part[0] / (float)B);
}

__global__ void __launch_bounds__(256) mean_loss_bwd_kernel(const float *__restrict__ q, const float *__restrict__ y,
                                                            const float *__restrict__ g, float *__restrict__ dq,
                                                            int64_t B, int64_t n, int mode) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = g[i / B] / (float)B;
    dq[i] = mode == 0 ? a * (2.0f * (q[i] - y[i])) : -a;
}

unsigned grid_for(int64_t n) {
    const int64_t blocks = (n + 255) / 256;
    return (unsigned)(blocks < 4096 ? (blocks > 0 ? blocks : 1) : 4096);
}

}  // namespace

extern "C" {

gw_status gw_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                       int64_t n, double lr, double beta1, double beta2, double eps, int32_t advanced, void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n < 0) return GW_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, s, param, grad, exp_avg, exp_avg_sq, step, n,
                       lr, beta1, beta2, eps, nullptr, nullptr, nullptr, (int64_t)0, 0.0f, (int)(advanced != 0));
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_adam_soft_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t *step,
                            int64_t n, double lr, double beta1, double beta2, double eps, float *target, float tau,
                            float *target2, const float *online2, int64_t n2, int32_t advanced, void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n < 0 || !target || n2 < 0 ||
        (n2 > 0 && (!target2 || !online2)))
        return GW_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n + n2)), dim3(256), 0, s, param, grad, exp_avg, exp_avg_sq, step, n,
                       lr, beta1, beta2, eps, target, target2, online2, n2, tau, (int)(advanced != 0));
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_soft_update(float *target, const float *online, int64_t n, float tau, void *stream) {
    if (!target || !online || n < 0) return GW_ERR_ARG;
    hipLaunchKernelGGL(soft_update_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       target, online, n, tau);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_ln_relu_fwd(const float *z, const float *ln_w, const float *ln_b, float *y, float *mean, float *rstd,
                         int32_t K, int64_t R, int32_t h, float eps, void *stream) {
    if (!z || !ln_w || !ln_b || !y || K < 0 || R < 0 || h <= 0 || h > LN_MAXV * 64 || (!mean) != (!rstd))
        return GW_ERR_ARG;
    const int64_t rows = (int64_t)K * R;
    if (rows == 0) return GW_OK;
    hipLaunchKernelGGL(ln_relu_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), z, ln_w, ln_b, y, mean, rstd, R, rows, (int)h, eps);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_ln_relu_bwd(const float *dy, const float *z, const float *y, const float *ln_w, const float *mean,
                         const float *rstd, float *dz, float *dw_acc, float *db_acc, int32_t K, int64_t R,
                         int32_t h, void *stream) {
    if (!dy || !z || !y || !ln_w || !mean || !rstd || !dz || K < 0 || R < 0 || h <= 0 || h > LN_MAXV * 64)
        return GW_ERR_ARG;
    if (K == 0) return GW_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t rows = (int64_t)K * R;
    if (rows == 0) return GW_OK;
    hipLaunchKernelGGL(ln_relu_bwd_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, dy, z, y, ln_w,
                       mean, rstd, dz, R, rows, (int)h);
    if (dw_acc || db_acc)
        hipLaunchKernelGGL(ln_relu_bwd_cols_kernel, dim3((unsigned)((h + 63) / 64), (unsigned)K), dim3(LN_RG * 64), 0,
                           st, dy, z, y, mean, rstd, dw_acc, db_acc, R, (int)h);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_gumbel_softmax(const float *logits, const float *u, float *out, int64_t rows, int32_t n, float tau,
                            float eps, int64_t out_b, int64_t out_ld, void *stream) {
    if (!logits || !u || !out || rows < 0 || n <= 0 || !(tau > 0.0f) || (out_ld > 0 && out_b <= 0)) return GW_ERR_ARG;
    if (rows == 0) return GW_OK;
    hipLaunchKernelGGL(gumbel_softmax_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), logits, u, out, rows, (int)n, tau, eps, out_b, out_ld);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_affine_relu_fwd(const float *xhat, const float *ln_w, const float *ln_b, float *y, int32_t K, int64_t R,
                             int32_t h, void *stream) {
    if (!xhat || !ln_w || !ln_b || !y || K < 0 || R < 0 || h <= 0) return GW_ERR_ARG;
    const int64_t n = (int64_t)K * R * h;
    if (n == 0) return GW_OK;
    hipLaunchKernelGGL(affine_relu_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream), xhat,
                       ln_w, ln_b, y, R, n, (int)h);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_affine_relu_bwd(const float *dy, const float *xhat, const float *y, const float *ln_w, float *dxhat,
                             float *dw_acc, float *db_acc, int32_t K, int64_t R, int32_t h, void *stream) {
    if (!dy || !xhat || !y || !ln_w || K < 0 || R < 0 || h <= 0) return GW_ERR_ARG;
    if ((int64_t)K * R == 0) return GW_OK;
    hipLaunchKernelGGL(affine_relu_bwd_kernel, dim3((unsigned)((h + 63) / 64), (unsigned)K), dim3(AR_RG * 64), 0,
                       static_cast<hipStream_t>(stream), dy, xhat, y, ln_w, dxhat, dw_acc, db_acc, R, (int)h);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_soft_update2(float *target1, const float *online1, int64_t n1, float *target2, const float *online2,
                          int64_t n2, float tau, void *stream) {
    if (!target1 || !online1 || !target2 || !online2 || n1 < 0 || n2 < 0) return GW_ERR_ARG;
    hipLaunchKernelGGL(soft_update2_kernel, dim3(grid_for(n1 + n2)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       target1, online1, n1, target2, online2, n2, tau);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_td_target(const double *rewards, const uint8_t *dones, const float *q_next, float gamma, float *y,
                       int32_t K, int64_t B, void *stream) {
    if (!rewards || !dones || !q_next || !y || K <= 0 || B < 0) return GW_ERR_ARG;
    const int64_t n = (int64_t)K * B;
    if (n == 0) return GW_OK;
    hipLaunchKernelGGL(td_target_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), rewards, dones, q_next, gamma, y, (int)K, B);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_mean_loss_fwd(const float *q, const float *y, float *loss, int32_t K, int64_t B, int32_t mode,
                           void *stream) {
    if (!q || !loss || (mode == 0 && !y) || mode < 0 || mode > 1 || K <= 0 || B <= 0) return GW_ERR_ARG;
    hipLaunchKernelGGL(mean_loss_fwd_kernel, dim3((unsigned)K), dim3(256), 0, static_cast<hipStream_t>(stream), q, y,
                       loss, B, (int)mode);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_mean_loss_bwd(const float *q, const float *y, const float *grad_loss, float *dq, int32_t K, int64_t B,
                           int32_t mode, void *stream) {
    if (!q || !grad_loss || !dq || (mode == 0 && !y) || mode < 0 || mode > 1 || K <= 0 || B <= 0) return GW_ERR_ARG;
    const int64_t n = (int64_t)K * B;
    hipLaunchKernelGGL(mean_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), q, y, grad_loss, dq, B, n, (int)mode);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

}  // extern "C"
