// rollout_ops.hip — the batched rollout's per-step bookkeeping in one launch (include/rollout_ops.h).
#include <hip/hip_runtime.h>

#include <string>

#include "rollout_ops.h"

namespace {

// One block of 256 threads (4 waves: it finds a CU slot even while a concurrent obs writer
// fills the chip; the 1024-thread form waited up to 40 us for 16 free wave slots, profiles/r2_c5)
constexpr int T = 256, MAXF = 64, U = 16;

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

// ---- completed-episode return compaction (parallel.ReturnGather.compact) ----
// Element i of a window = (step t, rank r, env e) in that order, e fastest: slot (t, r) starts
// at byte (t * world + r) * slot_bytes and holds [emax] f64 returns then [emax] u8 done flags.
// Pass 1 counts each chunk's done flags; pass 2 gives every chunk its exclusive prefix (a sum
// over the previous chunks' counts), scans the chunk in the block, and scatters the last
// `capacity` completions into the ring in element order.  Deterministic; two launches.
constexpr int CT = 256, CPT = 16, CCH = CT * CPT;  // threads, elements per thread, per chunk

__device__ __forceinline__ uint32_t done_at(const uint8_t *__restrict__ recv, int64_t i, int64_t emax,
                                            int64_t slot_bytes) {
    const int64_t slot = i / emax, e = i - slot * emax;
    return recv[slot * slot_bytes + 8 * emax + e] != 0;
}

__device__ __forceinline__ int block_sum_int(int v, int *red) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    const int tid = threadIdx.x;
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int w = 0; w < CT / 64; ++w) s += red[w];
    return s;
}

__global__ void __launch_bounds__(CT) compact_count(const uint8_t *__restrict__ recv, int64_t n, int64_t emax,
                                                    int64_t slot_bytes, int32_t *__restrict__ counts,
                                                    const int64_t *__restrict__ n_completed,
                                                    int64_t *__restrict__ base) {
    __shared__ int red[CT / 64];
    const int64_t i0 = (int64_t)blockIdx.x * CCH + (int64_t)threadIdx.x * CPT;
    int c = 0;
#pragma unroll
    for (int u = 0; u < CPT; ++u)
        if (i0 + u < n) c += (int)done_at(recv, i0 + u, emax, slot_bytes);
    c = block_sum_int(c, red);
    if (threadIdx.x == 0) {
        counts[blockIdx.x] = c;
        if (blockIdx.x == 0) base[0] = n_completed[0];  // snapshot: pass 2 updates n_completed
    }
}

__global__ void __launch_bounds__(CT) compact_scatter(const uint8_t *__restrict__ recv, int64_t n, int64_t emax,
                                                      int64_t slot_bytes, const int32_t *__restrict__ counts,
                                                      int32_t nchunks, const int64_t *__restrict__ base,
                                                      double *__restrict__ scores, int64_t capacity,
                                                      int64_t *__restrict__ n_completed) {
    __shared__ int red[CT / 64];
    __shared__ int wsum[CT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // prefix of this chunk and the window's total
    int pre = 0, tot = 0;
    for (int b = tid; b < nchunks; b += CT) {
        const int c = counts[b];
        tot += c;
        if (b < (int)blockIdx.x) pre += c;
    }
    pre = block_sum_int(pre, red);
    tot = block_sum_int(tot, red);
    const int64_t n0 = base[0];
    if (blockIdx.x == 0 && tid == 0) n_completed[0] = n0 + tot;
    // this thread's flags and its exclusive rank inside the chunk
    const int64_t i0 = (int64_t)blockIdx.x * CCH + (int64_t)tid * CPT;
    uint32_t bits = 0;
#pragma unroll
    for (int u = 0; u < CPT; ++u)
        if (i0 + u < n) bits |= done_at(recv, i0 + u, emax, slot_bytes) << u;
    const int mine = __popc(bits);
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int woff = 0;
#pragma unroll
    for (int w = 0; w < CT / 64; ++w) woff += (w < wv) ? wsum[w] : 0;
    int64_t pos = (int64_t)pre + woff + incl - mine;  // completions before this thread's first
    // kept: the last `capacity` completions of the window (older ones would be overwritten)
    const int64_t first_kept = (int64_t)tot - capacity;
    while (bits) {
        const int u = __ffs(bits) - 1;
        bits &= bits - 1;
        if (pos >= first_kept) {
            const int64_t i = i0 + u, slot = i / emax, e = i - slot * emax;
            const double r = reinterpret_cast<const double *>(recv + slot * slot_bytes)[e];
            scores[(n0 + pos) % capacity] = r;
        }
        ++pos;
    }
}

// ---- replay-ring sample: one block per (agent k, sample b) ----------------------------------
__device__ inline float ring_obs(const void *p, int bf16, int64_t i) {
    if (bf16) return __uint_as_float((uint32_t)static_cast<const uint16_t *>(p)[i] << 16);
    return static_cast<const float *>(p)[i];
}

__global__ void __launch_bounds__(256) replay_gather_kernel(
    const void *__restrict__ obs, const void *__restrict__ final_obs, int bf16, const float *__restrict__ probs,
    const double *__restrict__ reward, const uint8_t *__restrict__ term, const uint8_t *__restrict__ done,
    const int64_t *__restrict__ t_dev, const float *__restrict__ u, const int64_t *__restrict__ env, int64_t S,
    int K, int64_t E, int64_t HW, int64_t B, float *__restrict__ state, float *__restrict__ next_state,
    float *__restrict__ probs_out, double *__restrict__ reward_out, uint8_t *__restrict__ term_out,
    int64_t *__restrict__ tr_out, float *__restrict__ x_out, float *__restrict__ xn_out) {
    const int64_t b = blockIdx.x;
    const int k = blockIdx.y;
    const int64_t t = t_dev[0];
    const int64_t n = t < 1 ? 1 : (t > S - 1 ? S - 1 : t);
    int64_t step = (int64_t)(u[b] * (float)n);  // torch: (rand * n).long(), then minimum(., n - 1)
    if (step > n - 1) step = n - 1;
    int64_t tr = (t - 1 - step) % S;
    if (tr < 0) tr += S;  // Python / torch modulo
    const int64_t nx = (tr + 1) % S;
    const int64_t e = env[b];
    const bool dn = done[tr * E + e] != 0;
    const int64_t src = ((tr * K + k) * E + e) * HW;
    const int64_t nsrc = dn ? src : ((nx * K + k) * E + e) * HW;
    const void *nbuf = dn ? final_obs : obs;
    float *so = state + (k * B + b) * HW;
    float *no = next_state + (k * B + b) * HW;
    // the critic's input rows [B, K*HW + K*9] (agent-major states, then the K action slots)
    const int64_t ldx = (int64_t)K * HW + (int64_t)K * 9;
    float *xo = x_out ? x_out + b * ldx + (int64_t)k * HW : nullptr;
    float *xno = xn_out ? xn_out + b * ldx + (int64_t)k * HW : nullptr;
    for (int64_t i = threadIdx.x; i < HW; i += blockDim.x) {
        const float sv = ring_obs(obs, bf16, src + i), nv = ring_obs(nbuf, bf16, nsrc + i);
        so[i] = sv;
        no[i] = nv;
        if (xo) xo[i] = sv;
        if (xno) xno[i] = nv;
    }
    if (threadIdx.x < 9) {
        const float pv = probs[((tr * K + k) * E + e) * 9 + threadIdx.x];
        probs_out[(k * B + b) * 9 + threadIdx.x] = pv;
        if (x_out) x_out[b * ldx + (int64_t)K * HW + k * 9 + threadIdx.x] = pv;
    }
    if (k == 0 && threadIdx.x >= 64 && threadIdx.x < 64 + K) {
        const int j = threadIdx.x - 64;
        reward_out[b * K + j] = reward[(tr * E + e) * K + j];
        term_out[b * K + j] = term[(tr * E + e) * K + j];
    }
    if (k == 0 && threadIdx.x == 128 && tr_out) tr_out[b] = tr;
}

// ---- evaluation totals (customeval.py:70-133): one 1024-thread block, fixed-order sums ------------
constexpr int EV_T = 1024;

__global__ void __launch_bounds__(EV_T) eval_accum_kernel(const int32_t *__restrict__ crashes,
                                                           const int32_t *__restrict__ apples,
                                                           const double *__restrict__ fear, const uint8_t *__restrict__ done,
                                                           uint8_t *__restrict__ active, int64_t *__restrict__ counts,
                                                           double *__restrict__ fear_total, int64_t E, int K) {
    __shared__ int64_t s_c[EV_T], s_a[EV_T], s_s[EV_T];
    __shared__ double s_f[EV_T];
    int64_t c = 0, a = 0, n = 0;
    double fs = 0.0;
    for (int64_t e = threadIdx.x; e < E; e += EV_T) {
        if (active[e]) {
            c += crashes[e];
            a += apples[e];
            n += 1;
            double fe = 0.0;
            for (int k = 0; k < K; ++k) fe += fear[e * K + k];
            fs += fe;
            if (done[e]) active[e] = 0;
        }
    }
    const int t = threadIdx.x;
    s_c[t] = c;
    s_a[t] = a;
    s_s[t] = n;
    s_f[t] = fs;
    __syncthreads();
    for (int o = EV_T / 2; o > 0; o >>= 1) {
        if (t < o) {
            s_c[t] += s_c[t + o];
            s_a[t] += s_a[t + o];
            s_s[t] += s_s[t + o];
            s_f[t] += s_f[t + o];
        }
        __syncthreads();
    }
    if (t == 0) {
        counts[0] += s_c[0];
        counts[1] += s_a[0];
        counts[2] += s_s[0];
        fear_total[0] += s_f[0];
    }
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

gw_status gw_return_compact(const uint8_t *recv, int64_t steps, int32_t world, int64_t emax, int64_t slot_bytes,
                            double *scores, int64_t capacity, int64_t *n_completed, int32_t *scratch,
                            void *stream) {
    if (steps < 0 || world < 1 || emax < 1 || slot_bytes < 9 * emax || slot_bytes % 8 || capacity < 1 ||
        !scores || !n_completed || !scratch || (steps > 0 && !recv)) {
        gw_set_last_error("gw_return_compact: bad argument");
        return GW_ERR_ARG;
    }
    const int64_t n = steps * world * emax;
    if (n == 0) return GW_OK;
    const int64_t nchunks = (n + CCH - 1) / CCH;
    if (nchunks > (int64_t)1 << 30) {
        gw_set_last_error("gw_return_compact: window too large");
        return GW_ERR_ARG;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    int64_t *base = reinterpret_cast<int64_t *>(scratch);  // scratch: [2] i32 (base), then counts
    int32_t *counts = scratch + 2;
    hipLaunchKernelGGL(compact_count, dim3((unsigned)nchunks), dim3(CT), 0, s, recv, n, emax, slot_bytes, counts,
                       n_completed, base);
    hipLaunchKernelGGL(compact_scatter, dim3((unsigned)nchunks), dim3(CT), 0, s, recv, n, emax, slot_bytes, counts,
                       (int32_t)nchunks, base, scores, capacity, n_completed);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gw_set_last_error((std::string("gw_return_compact: ") + hipGetErrorString(e)).c_str());
        return GW_ERR_HIP;
    }
    return GW_OK;
}

int64_t gw_return_compact_scratch(int64_t steps, int32_t world, int64_t emax) {
    const int64_t n = steps * (int64_t)world * emax;
    return 2 + (n + CCH - 1) / CCH;
}

gw_status gw_replay_gather(const void *obs, const void *final_obs, int32_t obs_bf16, const float *probs,
                           const double *reward, const uint8_t *term, const uint8_t *done, const int64_t *t_dev,
                           const float *u, const int64_t *env, int64_t S, int32_t K, int64_t E, int64_t HW,
                           int64_t B, float *state, float *next_state, float *probs_out, double *reward_out,
                           uint8_t *term_out, int64_t *tr_out, float *x_out, float *xn_out, void *stream) {
    if (!obs || !final_obs || !probs || !reward || !term || !done || !t_dev || !u || !env || !state || !next_state ||
        !probs_out || !reward_out || !term_out || S < 2 || K <= 0 || K > 64 || E <= 0 || HW <= 0 || B < 0 ||
        B > 0x7fffffff)
        return GW_ERR_ARG;
    if (B == 0) return GW_OK;
    hipLaunchKernelGGL(replay_gather_kernel, dim3((unsigned)B, (unsigned)K), dim3(256), 0,
                       static_cast<hipStream_t>(stream), obs, final_obs, (int)obs_bf16, probs, reward, term, done,
                       t_dev, u, env, S, (int)K, E, HW, B, state, next_state, probs_out, reward_out, term_out, tr_out,
                       x_out, xn_out);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_eval_accum(const int32_t *crashes, const int32_t *apples, const double *fear, const uint8_t *done,
                        uint8_t *active, int64_t *counts, double *fear_total, int64_t E, int32_t K, void *stream) {
    if (!crashes || !apples || !fear || !done || !active || !counts || !fear_total || E < 0 || K <= 0)
        return GW_ERR_ARG;
    hipLaunchKernelGGL(eval_accum_kernel, dim3(1), dim3(EV_T), 0, static_cast<hipStream_t>(stream), crashes, apples,
                       fear, done, active, counts, fear_total, E, (int)K);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

}  // extern "C"
