// rollout_ops.hip — the batched rollout's per-step bookkeeping in one launch (include/rollout_ops.h).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <string>

#include "philox.h"
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
    int64_t *__restrict__ tr_out, float *__restrict__ x_out, float *__restrict__ xn_out, uint64_t seed,
    const int32_t *__restrict__ ctr) {
    const int64_t b = blockIdx.x;
    const int k = blockIdx.y;
    const int64_t t = t_dev[0];
    float ub;
    int64_t e;
    if (u) {
        ub = u[b];
        e = env[b];
    } else {  // in-kernel draws, as replay_gather_desc_kernel
        const uint4 r = gwrng::philox((uint32_t)b, (uint32_t)ctr[0], gwrng::TAG_SAMPLE, 0u, (uint32_t)seed,
                                      (uint32_t)(seed >> 32));
        ub = gwrng::unit(r.x);
        e = (int64_t)(((uint64_t)r.y * (uint64_t)E) >> 32);
    }
    const int64_t n = t < 1 ? 1 : (t > S - 1 ? S - 1 : t);
    int64_t step = (int64_t)(ub * (float)n);  // torch: (rand * n).long(), then minimum(., n - 1)
    if (step > n - 1) step = n - 1;
    int64_t tr = (t - 1 - step) % S;
    if (tr < 0) tr += S;  // Python / torch modulo
    const int64_t nx = (tr + 1) % S;
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

// ---- replay-ring sample from the descriptor ring: the same rows, expanded from 48-byte obs
// descriptors instead of read from the dense obs slots (so the learner never waits for the obs
// writer of the step it follows).  The cell values restate the obs writer (gridenv.hip obs_block;
// ma_customenv.py:197-209 reset encoding, :303-322 step encoding): map 0 / -1, own apple
// +9 first, then agent n's cell (a later patch overrides an earlier one) ----
constexpr int DESC_WORDS = 12;  // gridenv.hip NDESC
constexpr uint32_t DF_RESET = 1u;

__device__ __forceinline__ float desc_agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;
    if (v == k + 1) v = 1;
    return (float)v;
}

struct DescSrc {
    const float *base;
    int apples[GW_MAX_AGENTS];
    int N, K, HW, variant;
    int64_t E;
};

// patches of (descriptor words d[0..11], agent k): which 0 = the obs, 1 = the terminal obs (words
// 8-11); apple_map = the map value under agent k's apple cell
__device__ __forceinline__ int desc_patches(const DescSrc &q, const uint32_t (&d)[DESC_WORDS], int which, int k,
                                            float apple_map, int *pc, float *pv) {
    const uint32_t f = d[4];
    const bool reset = which == 0 && (f & DF_RESET);
    const uint32_t apples = which == 0 ? (f >> 8) & 0xFFu : (f >> 16) & 0xFFu;
    const int ac = ((apples >> k) & 1u) ? q.apples[k] : -1;
    int np = 0;
    if (ac >= 0) {
        float av = apple_map + 9.0f;
        if (!reset && av == (float)(k + 1)) av = 1.0f;
        pc[np] = ac;
        pv[np] = av;
        ++np;
    }
    for (int n = 0; n < q.N; ++n) {
        const uint32_t w = which == 0 ? d[n >> 1] : d[8 + (n >> 1)];
        const int c = (int)((w >> (16 * (n & 1))) & 0xFFFFu);
        pc[np] = c;
        pv[np] = desc_agent_value(reset, n, k, c == ac, q.variant);
        ++np;
    }
    return np;
}

constexpr int GD_CELLS = 16;  // map cells per thread prefetched (HW <= 256 * GD_CELLS = 4096)

// Every load of a block is issued in two waves: (t, u, env, the apple's map value, this thread's
// map cells), then (done, both descriptors whole, probs, reward, term); the rest is register / LDS
// work (each dependent global round trip costs ~1-2 us).
// KB agents per block (256 threads each; one: both agents of a row in one block measured slower)
template <int KB>
__global__ void __launch_bounds__(256 * KB) replay_gather_desc_kernel(
    DescSrc q, const uint32_t *__restrict__ desc, const float *__restrict__ probs, const double *__restrict__ reward,
    const uint8_t *__restrict__ term, const uint8_t *__restrict__ done, const int64_t *__restrict__ t_dev,
    const float *__restrict__ u, const int64_t *__restrict__ env, int64_t S, int64_t B, float *__restrict__ state,
    float *__restrict__ next_state, float *__restrict__ probs_out, double *__restrict__ reward_out,
    uint8_t *__restrict__ term_out, int64_t *__restrict__ tr_out, float *__restrict__ x_out,
    float *__restrict__ xn_out, uint64_t seed, const int32_t *__restrict__ ctr) {
    __shared__ int s_pcb[KB][2][GW_MAX_AGENTS + 1];
    __shared__ float s_pvb[KB][2][GW_MAX_AGENTS + 1];
    __shared__ int s_npb[KB][2];
    const int64_t b = blockIdx.x;
    const int kb = KB > 1 ? (int)(threadIdx.x >> 8) : 0;
    const int k = blockIdx.y * KB + kb, K = q.K, tid = threadIdx.x & 255;
    int (*s_pc)[GW_MAX_AGENTS + 1] = s_pcb[kb];
    float (*s_pv)[GW_MAX_AGENTS + 1] = s_pvb[kb];
    int *s_np = s_npb[kb];
    const int64_t E = q.E, HW = q.HW;
    // wave 1
    const int64_t t = t_dev[0];
    float ub;
    int64_t e;
    if (u) {
        ub = u[b];
        e = env[b];
    } else {  // in-kernel draws: Philox(seed; row, *ctr, tag), the env by a multiply-high of E
        const uint4 r = gwrng::philox((uint32_t)b, (uint32_t)ctr[0], gwrng::TAG_SAMPLE, 0u, (uint32_t)seed,
                                      (uint32_t)(seed >> 32));
        ub = gwrng::unit(r.x);
        e = (int64_t)(((uint64_t)r.y * (uint64_t)E) >> 32);
    }
    const float apple_map = q.apples[k] >= 0 ? q.base[q.apples[k]] : 0.0f;
    float mv[GD_CELLS];
#pragma unroll
    for (int c = 0; c < GD_CELLS; ++c) {
        const int64_t i = tid + 256 * c;
        mv[c] = i < HW ? q.base[i] : 0.0f;
    }
    const int64_t n = t < 1 ? 1 : (t > S - 1 ? S - 1 : t);
    int64_t step = (int64_t)(ub * (float)n);  // as replay_gather_kernel (torch's draw)
    if (step > n - 1) step = n - 1;
    int64_t tr = (t - 1 - step) % S;
    if (tr < 0) tr += S;
    const int64_t nx = (tr + 1) % S;
    // wave 2: obs slot j of the ring was written from descriptor slot j; the terminal obs of the
    // transition in slot tr (its final_obs slot) from the terminal half of descriptor slot tr + 1
    const bool dn = done[tr * E + e] != 0;
    if (tid < 2) {
        const uint4 *d4 = reinterpret_cast<const uint4 *>(desc + ((tid == 0 ? tr : nx) * E + e) * DESC_WORDS);
        const uint4 a = d4[0], bq = d4[1], c = d4[2];
        const uint32_t d[DESC_WORDS] = {a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c.x, c.y, c.z, c.w};
        s_np[tid] = desc_patches(q, d, tid == 0 ? 0 : (dn ? 1 : 0), k, apple_map, s_pc[tid], s_pv[tid]);
    }
    const int64_t ldx = (int64_t)K * HW + (int64_t)K * 9;
    if (tid < 9) {
        const float pv = probs[((tr * K + k) * E + e) * 9 + tid];
        probs_out[(k * B + b) * 9 + tid] = pv;
        if (x_out) x_out[b * ldx + (int64_t)K * HW + k * 9 + tid] = pv;
    }
    if (k == 0 && tid >= 64 && tid < 64 + K) {
        const int j = tid - 64;
        reward_out[b * K + j] = reward[(tr * E + e) * K + j];
        term_out[b * K + j] = term[(tr * E + e) * K + j];
    }
    if (k == 0 && tid == 128 && tr_out) tr_out[b] = tr;
    __syncthreads();
    const int np0 = s_np[0], np1 = s_np[1];
    // state / next_state may be NULL when the critic rows are all the caller needs
    float *so = state ? state + (k * B + b) * HW : nullptr;
    float *no = next_state ? next_state + (k * B + b) * HW : nullptr;
    float *xo = x_out ? x_out + b * ldx + (int64_t)k * HW : nullptr;
    float *xno = xn_out ? xn_out + b * ldx + (int64_t)k * HW : nullptr;
#pragma unroll
    for (int c = 0; c < GD_CELLS; ++c) {
        const int64_t i = tid + 256 * c;
        if (i >= HW) break;
        float sv = mv[c], nv = mv[c];
        for (int j = 0; j < np0; ++j)
            if (s_pc[0][j] == i) sv = s_pv[0][j];
        for (int j = 0; j < np1; ++j)
            if (s_pc[1][j] == i) nv = s_pv[1][j];
        if (so) so[i] = sv;
        if (no) no[i] = nv;
        if (xo) xo[i] = sv;
        if (xno) xno[i] = nv;
    }
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

// ---- the packed per-step return gather (parallel.ReturnGather, world > 1) ----
// Sender: this step's completed-episode returns (done envs, env order) are appended to a FIFO;
// the send slot carries a 32-byte header {count, sent, backlog after, overflow} and the FIFO's
// first `sent` = min(backlog, cap) entries.  Receiver: per source rank, a mirror FIFO of the
// entries received and a ring of per-step counts; a step is emitted into the score ring, in
// (step, rank, env) order, once every rank's entries of it have arrived.
constexpr int PT = 256, PPT = 4, PCH = PT * PPT;  // pack: threads, envs per thread, envs per chunk
constexpr int HDR = 32;                           // slot header bytes

__device__ __forceinline__ int block_excl_scan(int v, int *red, int &total) {
    // exclusive prefix of v over the block's threads (in thread order) and the block total
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    __syncthreads();
    if (lane == 63) red[wave] = incl;
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < PT / 64; ++w) {
        const int x = red[w];
        if (w < wave) before += x;
        total += x;
    }
    return before + incl - v;
}

__global__ void __launch_bounds__(PT) pack_count(const uint8_t *__restrict__ done, int64_t E,
                                                 const int64_t *__restrict__ ctl, int32_t *__restrict__ scratch) {
    __shared__ int red[PT / 64];
    const int64_t e0 = (int64_t)blockIdx.x * PCH + (int64_t)threadIdx.x * PPT;
    int c = 0;
#pragma unroll
    for (int j = 0; j < PPT; ++j) c += (e0 + j < E && done[e0 + j]) ? 1 : 0;
    int total = 0;
    (void)block_excl_scan(c, red, total);
    int64_t *snap = reinterpret_cast<int64_t *>(scratch);
    if (threadIdx.x == 0) {
        scratch[4 + blockIdx.x] = total;
        if (blockIdx.x == 0) {
            snap[0] = ctl[0];
            snap[1] = ctl[1];
        }
    }
}

__global__ void __launch_bounds__(PT) pack_scatter(const double *__restrict__ ret, const uint8_t *__restrict__ done,
                                                   int64_t E, int nchunks, int64_t cap, double *__restrict__ fifo,
                                                   int64_t fifo_cap, int64_t *__restrict__ ctl,
                                                   const int32_t *__restrict__ scratch, uint8_t *__restrict__ slot) {
    __shared__ int red[PT / 64];
    const int tid = threadIdx.x, b = blockIdx.x;
    const int64_t *snap = reinterpret_cast<const int64_t *>(scratch);
    const int32_t *counts = scratch + 4;
    const int64_t head = snap[0], tail = snap[1];
    // this step's total and (chunk blocks) the chunk's prefix over the earlier chunks
    int pre = 0, all = 0;
    for (int i = tid; i < nchunks; i += PT) {
        const int x = counts[i];
        all += x;
        if (i < b) pre += x;
    }
    int tot_all = 0, tot_pre = 0;
    (void)block_excl_scan(all, red, tot_all);
    (void)block_excl_scan(pre, red, tot_pre);
    const int64_t c = tot_all, backlog0 = tail - head;
    const int64_t nsend = min(backlog0 + c, cap);
    double *payload = reinterpret_cast<double *>(slot + HDR);
    if (b < nchunks) {
        const int64_t e0 = (int64_t)b * PCH + (int64_t)tid * PPT;
        uint32_t bits = 0;
        double v[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const bool d = e0 + j < E && done[e0 + j];
            bits |= (d ? 1u : 0u) << j;
            v[j] = d ? ret[e0 + j] : 0.0;
        }
        int total = 0;
        int pos = tot_pre + block_excl_scan(__popc(bits), red, total);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            if (!((bits >> j) & 1u)) continue;
            const int64_t at = tail + pos;  // FIFO position of this completion
            fifo[at % fifo_cap] = v[j];
            const int64_t q = at - head;
            if (q < nsend) payload[q] = v[j];
            ++pos;
        }
    } else {  // the old backlog's entries that go out this step
        const int64_t nold = min(backlog0, nsend);
        for (int64_t i = (int64_t)(b - nchunks) * PT + tid; i < nold; i += (int64_t)(gridDim.x - nchunks) * PT)
            payload[i] = fifo[(head + i) % fifo_cap];
    }
    if (b == 0 && tid == 0) {
        const int64_t backlog1 = backlog0 + c - nsend;
        const int64_t ovf = (ctl[2] != 0 || backlog0 + c > fifo_cap) ? 1 : 0;
        int64_t *hdr = reinterpret_cast<int64_t *>(slot);
        hdr[0] = c;
        hdr[1] = nsend;
        hdr[2] = backlog1;
        hdr[3] = ovf;
        ctl[0] = head + nsend;
        ctl[1] = tail + c;
        ctl[2] = ovf;
    }
}

// receiver plan: one thread walks the window's headers (steps x world) and the pending steps;
// segments: {kind (0 payload -> mirror, 1 mirror -> scores), rank, src, len, dst}
struct Seg {
    int64_t kind, rank, src, len, dst;
};

__global__ void unpack_plan(const uint8_t *__restrict__ recv, int64_t steps, int world, int64_t slot_bytes,
                            int64_t *__restrict__ rst, int32_t *__restrict__ pend, int64_t pend_cap,
                            Seg *__restrict__ plan, int64_t plan_cap, int64_t *__restrict__ n_completed,
                            int64_t *__restrict__ plan_meta) {
    if (threadIdx.x != 0) return;
    int64_t *recv_tot = rst, *emitted = rst + world, *ph = rst + 2 * world, *pt = ph + 1, *ovf = pt + 1,
            *maxb = ovf + 1;
    int64_t na = 0, nb = 0, mb = 0, bad = *ovf;
    for (int64_t s = 0; s < steps; ++s) {
        if (*pt - *ph >= pend_cap) bad = 1;
        for (int r = 0; r < world; ++r) {
            const int64_t *hdr = reinterpret_cast<const int64_t *>(recv + (s * world + r) * slot_bytes);
            const int64_t c = hdr[0], n = hdr[1];
            mb = max(mb, hdr[2]);
            bad |= hdr[3];
            if (n > 0 && na < plan_cap) {
                plan[na] = Seg{0, r, (s * world + r) * slot_bytes + HDR, n, recv_tot[r]};
                ++na;
            }
            recv_tot[r] += n;
            pend[(*pt % pend_cap) * world + r] = (int32_t)c;
        }
        *pt += 1;
    }
    // emit every pending step whose entries have all arrived, in order
    const int64_t base = *n_completed;
    int64_t off = 0;
    while (*ph < *pt) {
        const int32_t *cs = pend + (*ph % pend_cap) * world;
        bool ready = true;
        for (int r = 0; r < world; ++r) ready = ready && emitted[r] + cs[r] <= recv_tot[r];
        if (!ready) break;
        for (int r = 0; r < world; ++r) {
            if (cs[r] > 0 && na + nb < plan_cap) {
                plan[na + nb] = Seg{1, r, emitted[r], cs[r], base + off};
                ++nb;
            }
            emitted[r] += cs[r];
            off += cs[r];
        }
        *ph += 1;
    }
    if (na + nb >= plan_cap) bad = 1;
    *n_completed = base + off;
    *maxb = mb;
    *ovf = bad;
    plan_meta[0] = na;
    plan_meta[1] = nb;
    plan_meta[2] = base + off;  // the new total: entries before total - capacity are not kept
}

// grid (G, CPB): block (g, j) copies elements j, j + CPB * T, ... of segments g, g + G, ... of `kind`
constexpr int CPB = 8;

__global__ void __launch_bounds__(PT) unpack_copy(const uint8_t *__restrict__ recv, double *__restrict__ mirror,
                                                  int64_t mirror_cap, const Seg *__restrict__ plan,
                                                  const int64_t *__restrict__ plan_meta, int kind,
                                                  double *__restrict__ scores, int64_t capacity) {
    const int64_t na = plan_meta[0], nb = plan_meta[1], total = plan_meta[2];
    const int64_t nseg = kind == 0 ? na : nb, first = kind == 0 ? 0 : na;
    for (int64_t g = blockIdx.x; g < nseg; g += gridDim.x) {
        const Seg sg = plan[first + g];
        double *mr = mirror + sg.rank * mirror_cap;
        for (int64_t i = (int64_t)blockIdx.y * PT + threadIdx.x; i < sg.len; i += (int64_t)CPB * PT) {
            if (kind == 0) {
                mr[(sg.dst + i) % mirror_cap] = reinterpret_cast<const double *>(recv + sg.src)[i];
            } else {
                const int64_t d = sg.dst + i;
                if (d >= total - capacity) scores[d % capacity] = mr[(sg.src + i) % mirror_cap];
            }
        }
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

int64_t gw_gather_pack_scratch(int64_t E) { return 4 + (E + PCH - 1) / PCH; }

gw_status gw_gather_pack(const double *ep_return, const uint8_t *done, int64_t E, int64_t cap, double *fifo,
                         int64_t fifo_cap, int64_t *ctl, int32_t *scratch, uint8_t *slot, void *stream) {
    if (!ep_return || !done || E < 1 || cap < 1 || !fifo || fifo_cap < cap || !ctl || !scratch || !slot) {
        gw_set_last_error("gw_gather_pack: bad argument");
        return GW_ERR_ARG;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t nchunks = (E + PCH - 1) / PCH;
    const int64_t ncopy = std::min<int64_t>((cap + PT * 4 - 1) / (PT * 4), 64);
    hipLaunchKernelGGL(pack_count, dim3((unsigned)nchunks), dim3(PT), 0, s, done, E, ctl, scratch);
    hipLaunchKernelGGL(pack_scatter, dim3((unsigned)(nchunks + ncopy)), dim3(PT), 0, s, ep_return, done, E,
                       (int)nchunks, cap, fifo, fifo_cap, ctl, scratch, slot);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gw_set_last_error((std::string("gw_gather_pack: ") + hipGetErrorString(e)).c_str());
        return GW_ERR_HIP;
    }
    return GW_OK;
}

int64_t gw_gather_unpack_plan_cap(int64_t steps, int32_t world, int64_t pend_cap) {
    return (steps + pend_cap) * (int64_t)world + 1;
}

gw_status gw_gather_unpack(const uint8_t *recv, int64_t steps, int32_t world, int64_t slot_bytes, double *mirror,
                           int64_t mirror_cap, int64_t *rstate, int32_t *pend, int64_t pend_cap, void *plan,
                           int64_t plan_cap, double *scores, int64_t capacity, int64_t *n_completed, void *stream) {
    if (steps < 0 || world < 1 || slot_bytes < HDR + 8 || slot_bytes % 8 || !mirror || mirror_cap < 1 || !rstate ||
        !pend || pend_cap < 1 || !plan || plan_cap < 2 || !scores || capacity < 1 || !n_completed ||
        (steps > 0 && !recv)) {
        gw_set_last_error("gw_gather_unpack: bad argument");
        return GW_ERR_ARG;
    }
    if (steps == 0) return GW_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // plan: [plan_cap] segments, then 4 int64 of metadata
    Seg *segs = static_cast<Seg *>(plan);
    int64_t *meta = reinterpret_cast<int64_t *>(segs + plan_cap);
    hipLaunchKernelGGL(unpack_plan, dim3(1), dim3(64), 0, s, recv, steps, (int)world, slot_bytes, rstate, pend,
                       pend_cap, segs, plan_cap, n_completed, meta);
    const unsigned na = (unsigned)std::min<int64_t>(std::min<int64_t>(steps * world, plan_cap), 512);
    const unsigned nb = (unsigned)std::min<int64_t>(std::min<int64_t>(pend_cap * world, plan_cap), 512);
    hipLaunchKernelGGL(unpack_copy, dim3(na, CPB), dim3(PT), 0, s, recv, mirror, mirror_cap, segs, meta, 0, scores,
                       capacity);
    hipLaunchKernelGGL(unpack_copy, dim3(nb, CPB), dim3(PT), 0, s, recv, mirror, mirror_cap, segs, meta, 1, scores,
                       capacity);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gw_set_last_error((std::string("gw_gather_unpack: ") + hipGetErrorString(e)).c_str());
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
                           uint8_t *term_out, int64_t *tr_out, float *x_out, float *xn_out, uint64_t seed,
                           const int32_t *ctr, void *stream) {
    if (!obs || !final_obs || !probs || !reward || !term || !done || !t_dev || (!u != !env) || (!u && !ctr) ||
        !state || !next_state ||
        !probs_out || !reward_out || !term_out || S < 2 || K <= 0 || K > 64 || E <= 0 || HW <= 0 || B < 0 ||
        B > 0x7fffffff)
        return GW_ERR_ARG;
    if (B == 0) return GW_OK;
    hipLaunchKernelGGL(replay_gather_kernel, dim3((unsigned)B, (unsigned)K), dim3(256), 0,
                       static_cast<hipStream_t>(stream), obs, final_obs, (int)obs_bf16, probs, reward, term, done,
                       t_dev, u, env, S, (int)K, E, HW, B, state, next_state, probs_out, reward_out, term_out, tr_out,
                       x_out, xn_out, seed, ctr);
    return hipGetLastError() == hipSuccess ? GW_OK : GW_ERR_HIP;
}

gw_status gw_replay_gather_desc(const gw_obs_source *src, const uint32_t *desc, const float *probs,
                                const double *reward, const uint8_t *term, const uint8_t *done, const int64_t *t_dev,
                                const float *u, const int64_t *env, int64_t S, int64_t B, float *state,
                                float *next_state, float *probs_out, double *reward_out, uint8_t *term_out,
                                int64_t *tr_out, float *x_out, float *xn_out, uint64_t seed, const int32_t *ctr,
                                void *stream) {
    if (!src || !src->base || !desc || !probs || !reward || !term || !done || !t_dev || (!u != !env) ||
        (!u && !ctr) || ((!state || !next_state) && (!x_out || !xn_out)) || !probs_out || !reward_out ||
        !term_out || S < 2 || src->K <= 0 || src->K > GW_MAX_AGENTS ||
        src->N < src->K || src->N > GW_MAX_AGENTS || src->E <= 0 || src->H <= 0 || src->W <= 0 || B < 0 ||
        B > 0x7fffffff || (int64_t)src->H * src->W > 256 * GD_CELLS)
        return GW_ERR_ARG;
    if (B == 0) return GW_OK;
    DescSrc q;
    q.base = src->base;
    for (int k = 0; k < GW_MAX_AGENTS; ++k) q.apples[k] = src->apples[k];
    q.N = src->N;
    q.K = src->K;
    q.HW = src->H * src->W;
    q.variant = src->variant;
    q.E = src->E;
    hipLaunchKernelGGL(replay_gather_desc_kernel<1>, dim3((unsigned)B, (unsigned)q.K), dim3(256), 0,
                       static_cast<hipStream_t>(stream), q, desc, probs, reward, term, done, t_dev, u, env, S, B,
                       state, next_state, probs_out, reward_out, term_out, tr_out, x_out, xn_out, seed, ctr);
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
