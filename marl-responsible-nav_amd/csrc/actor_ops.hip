// actor_ops.hip — the MADDPG actors' get_action for every env of a grid-env handle in one
// MI355X kernel (include/actor_ops.h).  Reference: maddpg/agent.py:109-122 (get_action over the
// flattened obs, argmax), agilerl 1.0.15 MADDPG.get_action with an EvolvableMLP actor
// (Linear-LayerNorm-ReLU x2, Linear, GumbelSoftmax; parity of agilerl itself unpinned).
//
// Work split (block = 4 waves = one RL agent k, persistent over 32-env tiles, one tile per wave):
//   layer 1   from the obs descriptors: h1 = c1_k + sum_{patched cells c} delta_c * W1_k[c, :],
//             c1_k = b1_k + map . W1_k (prologue kernel).  Lane (env = l & 31, half = l >> 5)
//             accumulates features [64 half, 64 half + 64) of its env (W1 rows are L2 resident).
//   LN1/ReLU  in registers; the two halves of an env meet through one cross-half shuffle.
//   layer 2   transposed f32 MFMA: H2^T = W2^T A1^T with v_mfma_f32_32x32x2_f32.  The lane's 64
//             layer-1 registers ARE the B operand (k-step s pairs feature s of half 0 with feature
//             64 + s of half 1), W2 is the A operand from LDS; the result has env on the lane and
//             features in the registers, so LN2 again needs only the cross-half shuffle.
//   layer 3   the same with A = W3^T (9 of 32 rows live), B = the LN2 registers in D order.
//   epilogue  logits -> LDS -> one lane per env: Gumbel noise, softmax, mask, argmax.
// f32 throughout: every product exact, k-ordered f32 sums (MFMA), so the result differs from a
// torch fp32 forward only by summation order (tests/test_actor_ops.py states the tolerance).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "actor_ops.h"

namespace {

constexpr int HID = 128, NA = 9, TILE = 32, WAVES = 4, THREADS = 64 * WAVES, MAXN = GW_MAX_AGENTS;
constexpr int NDESC = 12;
constexpr uint32_t D_RESET = 1u;
constexpr float LN_EPS = 1e-5f, G_EPS = 1e-20f;
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ActParams {
    gw_mlp_actors net;
    float *c1;                // [K][128] (written by c1_kernel)
    const uint32_t *desc;     // [E][12]
    const float *base;        // [HW]
    const uint16_t *mask;     // [E][K] or null
    const float *uniform;     // [K][E][9] or null
    int32_t *actions;         // [E][K]
    float *probs;             // [K][E][9]
    float *logits;            // [K][E][9] or null
    int64_t E, env_offset;
    int N, K, HW, variant, training, tiles;
    float tau;
    uint32_t key0, key1, ctr0, ctr1;
    int apples[MAXN];
};

// Philox4x32-10, the same generator as gridenv.hip (keyed draws, graph- and shard-invariant)
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                        uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    return make_uint4(c0, c1, c2, c3);
}

// obs value of agent n in RL agent k's observation (ma_customenv.py:197-209 reset encoding,
// :303-322 step encoding incl. the hard-coded relabel list [1, 2, 3, 4]); the same rule as
// gridenv.hip's obs writer (agent_value)
__device__ __forceinline__ float agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;
    if (v == k + 1) v = 1;
    return (float)v;
}

// c1[k][j] = b1[k][j] + sum_c map[c] * W1[k][c][j]; block (k, 32-column group), 8 row slices
__global__ void __launch_bounds__(256) c1_kernel(ActParams p) {
    __shared__ float part[8][32];
    const int k = blockIdx.y, j = blockIdx.x * 32 + (threadIdx.x & 31), sl = threadIdx.x >> 5;
    const float *w1 = p.net.w1 + (size_t)k * p.HW * HID;
    float acc = 0.0f;
    for (int c = sl; c < p.HW; c += 8) acc = fmaf(p.base[c], w1[(size_t)c * HID + j], acc);
    part[sl][threadIdx.x & 31] = acc;
    __syncthreads();
    if (sl == 0) {
        float s = 0.0f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s += part[q][threadIdx.x];
        p.c1[k * HID + j] = p.net.b1[k * HID + j] + s;
    }
}

__device__ __forceinline__ float half_sum(float s) {  // sum over the two lanes of an env
    return s + __shfl_xor(s, 32, 64);
}

__global__ void __launch_bounds__(THREADS, 2) act_kernel(ActParams p) {
    __shared__ float s_w2[HID * HID];        // [in][out], 64 KB
    __shared__ float s_w3[HID * NA];         // [in][a]
    __shared__ float s_vec[8][HID];          // c1, ln1_w, ln1_b, b2, ln2_w, ln2_b
    __shared__ float s_b3[12];
    __shared__ float s_lg[WAVES][TILE][NA + 1];

    const int k = blockIdx.y, tid = threadIdx.x;
    const bool ln = p.net.layer_norm != 0;
    {   // stage this agent's layer-2/3 weights and vectors (all loads of a lane issued first)
        const float4 *w2 = reinterpret_cast<const float4 *>(p.net.w2 + (size_t)k * HID * HID);
        float4 r[HID * HID / 4 / THREADS];
#pragma unroll
        for (int i = 0; i < HID * HID / 4 / THREADS; ++i) r[i] = w2[i * THREADS + tid];
#pragma unroll
        for (int i = 0; i < HID * HID / 4 / THREADS; ++i) reinterpret_cast<float4 *>(s_w2)[i * THREADS + tid] = r[i];
        for (int i = tid; i < HID * NA; i += THREADS) s_w3[i] = p.net.w3[(size_t)k * HID * NA + i];
        if (tid < HID) {
            s_vec[0][tid] = p.c1[k * HID + tid];
            s_vec[1][tid] = ln ? p.net.ln1_w[k * HID + tid] : 1.0f;
            s_vec[2][tid] = ln ? p.net.ln1_b[k * HID + tid] : 0.0f;
            s_vec[3][tid] = p.net.b2[k * HID + tid];
            s_vec[4][tid] = ln ? p.net.ln2_w[k * HID + tid] : 1.0f;
            s_vec[5][tid] = ln ? p.net.ln2_b[k * HID + tid] : 0.0f;
        }
        if (tid < NA) s_b3[tid] = p.net.b3[k * NA + tid];
    }
    __syncthreads();

    const int wave = tid >> 6, lane = tid & 63, el = lane & 31, h = lane >> 5;
    const float *w1 = p.net.w1 + (size_t)k * p.HW * HID + 64 * h;
    const int K = p.K, N = p.N;
    const int ac_k = p.apples[k];

    for (int tile = blockIdx.x * WAVES + wave; tile < p.tiles; tile += gridDim.x * WAVES) {
        const int64_t e = (int64_t)tile * TILE + el;
        const bool valid = e < p.E;
        // ---- obs patches of (e, k): slot 0 own apple, slot 1 + n agent n; a later slot on
        //      the same cell overrides an earlier one (the obs writer's order) ----
        int pc[MAXN + 1];
        float pv[MAXN + 1];
#pragma unroll
        for (int q = 0; q <= MAXN; ++q) {
            pc[q] = -1;
            pv[q] = 0.0f;
        }
        if (valid) {
            const uint4 d03 = *reinterpret_cast<const uint4 *>(p.desc + e * NDESC);
            const uint32_t f = p.desc[e * NDESC + 4];
            const bool reset = (f & D_RESET) != 0;
            const int ac = ((f >> (8 + k)) & 1u) ? ac_k : -1;
            if (ac >= 0) {
                float av = p.base[ac] + 9.0f;
                if (!reset && av == (float)(k + 1)) av = 1.0f;  // relabel of :321 (apple on a wall)
                pc[0] = ac;
                pv[0] = av;
            }
            const uint32_t dw[4] = {d03.x, d03.y, d03.z, d03.w};
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
                if (n < N) {
                    const int c = (int)((dw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                    pc[1 + n] = c;
                    pv[1 + n] = agent_value(reset, n, k, c == ac, p.variant);
                }
            }
        }
        // ---- layer 1: c1 + sum of (value - map) * W1 row over the distinct patched cells ----
        float a[64];
#pragma unroll
        for (int i = 0; i < 64; ++i) a[i] = s_vec[0][64 * h + i];
#pragma unroll
        for (int q = 0; q <= MAXN; ++q) {
            const int c = pc[q];
            bool last = (unsigned)c < (unsigned)p.HW;
#pragma unroll
            for (int r = q + 1; r <= MAXN; ++r) last = last && pc[r] != c;
            const float dlt = last ? pv[q] - p.base[c] : 0.0f;
            if (dlt != 0.0f) {
                const float4 *row = reinterpret_cast<const float4 *>(w1 + (size_t)c * HID);
                float4 wr[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) wr[i] = row[i];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    a[4 * i + 0] = fmaf(dlt, wr[i].x, a[4 * i + 0]);
                    a[4 * i + 1] = fmaf(dlt, wr[i].y, a[4 * i + 1]);
                    a[4 * i + 2] = fmaf(dlt, wr[i].z, a[4 * i + 2]);
                    a[4 * i + 3] = fmaf(dlt, wr[i].w, a[4 * i + 3]);
                }
            }
        }
        // ---- LN1 + ReLU (nn.LayerNorm(128), eps 1e-5, biased variance) ----
        if (ln) {
            float s = 0.0f;
#pragma unroll
            for (int i = 0; i < 64; ++i) s += a[i];
            const float mean = half_sum(s) * (1.0f / HID);
            float v = 0.0f;
#pragma unroll
            for (int i = 0; i < 64; ++i) v = fmaf(a[i] - mean, a[i] - mean, v);
            const float rstd = rsqrtf(half_sum(v) * (1.0f / HID) + LN_EPS);
#pragma unroll
            for (int i = 0; i < 64; ++i)
                a[i] = fmaxf(fmaf((a[i] - mean) * rstd, s_vec[1][64 * h + i], s_vec[2][64 * h + i]), 0.0f);
        } else {
#pragma unroll
            for (int i = 0; i < 64; ++i) a[i] = fmaxf(a[i], 0.0f);
        }
        // ---- layer 2: D[m] (32 features x 32 envs) = W2^T[32m.., k] . A1^T ----
        f32x16 acc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] = 0.0f;
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            const float *wrow = s_w2 + (64 * h + s) * HID + el;
#pragma unroll
            for (int m = 0; m < 4; ++m)
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(wrow[32 * m], a[s], acc[m], 0, 0, 0);
        }
        // register r of tile m holds feature 32m + (r & 3) + 8 (r >> 2) + 4h of env el
#define FEAT(m, r) (32 * (m) + ((r) & 3) + 8 * ((r) >> 2) + 4 * h)
        float s2 = 0.0f;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[m][r] += s_vec[3][FEAT(m, r)];
                s2 += acc[m][r];
            }
        if (ln) {
            const float mean = half_sum(s2) * (1.0f / HID);
            float v = 0.0f;
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) v = fmaf(acc[m][r] - mean, acc[m][r] - mean, v);
            const float rstd = rsqrtf(half_sum(v) * (1.0f / HID) + LN_EPS);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    acc[m][r] = fmaxf(fmaf((acc[m][r] - mean) * rstd, s_vec[4][FEAT(m, r)], s_vec[5][FEAT(m, r)]), 0.0f);
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[m][r] = fmaxf(acc[m][r], 0.0f);
        }
        // ---- layer 3: D3 (32 action rows, 9 live x 32 envs) = W3^T . A2^T, one accumulator per
        //      feature tile (independent MFMA chains), summed in tile order ----
        f32x16 o3[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int r = 0; r < 16; ++r) o3[m][r] = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float wa = el < NA ? s_w3[FEAT(m, r) * NA + el] : 0.0f;
                o3[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa, acc[m][r], o3[m], 0, 0, 0);
            }
        }
        f32x16 out = o3[0] + o3[1] + o3[2] + o3[3];
#undef FEAT
        // D3 row (r & 3) + 8 (r >> 2) + 4h = action: h 0 -> r 0-3 (actions 0-3), r 4 (action 8);
        // h 1 -> r 0-3 (actions 4-7)
#pragma unroll
        for (int r = 0; r < 4; ++r) s_lg[wave][el][r + 4 * h] = out[r] + s_b3[r + 4 * h];
        if (h == 0) s_lg[wave][el][8] = out[4] + s_b3[8];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- epilogue: one lane per env ----
        if (h == 0 && valid) {
            float lg[NA];
#pragma unroll
            for (int a9 = 0; a9 < NA; ++a9) lg[a9] = s_lg[wave][el][a9];
            const size_t o = ((size_t)k * p.E + e) * NA;
            if (p.logits) {
#pragma unroll
                for (int a9 = 0; a9 < NA; ++a9) p.logits[o + a9] = lg[a9];
            }
            if (p.training) {  // agilerl GumbelSoftmax: logits - log(-log(u + eps) + eps)
                float u[12];
                if (p.uniform) {
#pragma unroll
                    for (int a9 = 0; a9 < NA; ++a9) u[a9] = p.uniform[o + a9];
                } else {
                    const uint32_t ge = (uint32_t)(p.env_offset + e);
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const uint4 x = philox(ge, p.ctr0, (uint32_t)k | ((uint32_t)q << 8) | (0xA7u << 24), p.ctr1,
                                               p.key0, p.key1);
                        u[4 * q + 0] = (float)(x.x >> 8) * (1.0f / 16777216.0f);
                        u[4 * q + 1] = (float)(x.y >> 8) * (1.0f / 16777216.0f);
                        u[4 * q + 2] = (float)(x.z >> 8) * (1.0f / 16777216.0f);
                        u[4 * q + 3] = (float)(x.w >> 8) * (1.0f / 16777216.0f);
                    }
                }
#pragma unroll
                for (int a9 = 0; a9 < NA; ++a9) lg[a9] = lg[a9] - logf(-logf(u[a9] + G_EPS) + G_EPS);
            }
            float z[NA], ex[NA], mx = -INFINITY, sum = 0.0f;  // softmax(logits / tau)
#pragma unroll
            for (int a9 = 0; a9 < NA; ++a9) {
                z[a9] = lg[a9] / p.tau;
                mx = fmaxf(mx, z[a9]);
            }
#pragma unroll
            for (int a9 = 0; a9 < NA; ++a9) {
                ex[a9] = expf(z[a9] - mx);
                sum += ex[a9];
            }
            const uint32_t mk = p.mask ? p.mask[e * K + k] : 0x1FFu;
            int best = 0;
            float bv = -1.0f;
#pragma unroll
            for (int a9 = 0; a9 < NA; ++a9) {
                const float pr = ex[a9] / sum;
                p.probs[o + a9] = pr;
                const float pm = ((mk >> a9) & 1u) ? pr : 0.0f;
                if (pm > bv) {
                    bv = pm;
                    best = a9;
                }
            }
            p.actions[e * K + k] = best;
        }
        __builtin_amdgcn_wave_barrier();  // s_lg is rewritten by the next tile
    }
}

gw_status err(gw_status s, const std::string &msg) {
    gw_set_last_error(msg.c_str());
    return s;
}

}  // namespace

extern "C" {

gw_status gw_actor_act(void *env, const gw_mlp_actors *net, float *c1_ws, int training, float tau, uint64_t seed,
                       uint64_t counter, const float *uniform, const uint16_t *mask, int32_t *actions, float *probs,
                       float *logits, void *stream) {
    if (!env || !net || !c1_ws || !actions || !probs) return err(GW_ERR_ARG, "gw_actor_act: null argument");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if (net->K != src.K) return err(GW_ERR_ARG, "gw_actor_act: net K != env K");
    if (net->in_dim != src.H * src.W) return err(GW_ERR_ARG, "gw_actor_act: in_dim != H*W");
    if (net->hidden != HID || net->n_actions != NA)
        return err(GW_ERR_ARG, "gw_actor_act: only hidden 128 and 9 actions are fused");
    if (!net->w1 || !net->b1 || !net->w2 || !net->b2 || !net->w3 || !net->b3 ||
        (net->layer_norm && (!net->ln1_w || !net->ln1_b || !net->ln2_w || !net->ln2_b)))
        return err(GW_ERR_ARG, "gw_actor_act: null parameter");
    if ((reinterpret_cast<uintptr_t>(net->w1) | reinterpret_cast<uintptr_t>(net->w2)) & 15u)
        return err(GW_ERR_ARG, "gw_actor_act: w1 / w2 must be 16-byte aligned");
    if (!(tau > 0.0f)) return err(GW_ERR_ARG, "gw_actor_act: tau must be > 0");
    ActParams p;
    p.net = *net;
    p.c1 = c1_ws;
    p.desc = src.desc;
    p.base = src.base;
    p.mask = mask;
    p.uniform = uniform;
    p.actions = actions;
    p.probs = probs;
    p.logits = logits;
    p.E = src.E;
    p.env_offset = src.env_offset;
    p.N = src.N;
    p.K = src.K;
    p.HW = src.H * src.W;
    p.variant = src.variant;
    p.training = training ? 1 : 0;
    p.tau = tau;
    p.key0 = (uint32_t)seed;
    p.key1 = (uint32_t)(seed >> 32);
    p.ctr0 = (uint32_t)counter;
    p.ctr1 = (uint32_t)(counter >> 32);
    for (int k = 0; k < MAXN; ++k) p.apples[k] = src.apples[k];
    const int64_t tiles = (src.E + TILE - 1) / TILE;
    p.tiles = (int)tiles;
    // 2 blocks of 4 waves per CU (77 KB LDS each): 512 resident blocks over the K agents
    const int64_t want = (tiles + WAVES - 1) / WAVES;
    const int per_agent = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(1, 512 / src.K)));
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(c1_kernel, dim3(HID / 32, src.K), dim3(256), 0, s, p);
    hipLaunchKernelGGL(act_kernel, dim3(per_agent, src.K), dim3(THREADS), 0, s, p);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_actor_act: ") + hipGetErrorString(e));
    return GW_OK;
}

}  // extern "C"
