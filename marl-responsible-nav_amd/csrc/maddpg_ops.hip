// maddpg_ops.hip — one MADDPG update (agilerl 1.0.15 MADDPG.learn as called by
// maddpg/agent.py:199-224, restated in marlnav/maddpg.py) in a handful of MI355X launches
// (include/learner_ops.h: gw_maddpg_critic_grads, gw_maddpg_actor_grads; the Adam steps and the
// soft update are gw_adam_step / gw_soft_update2).
//
// The networks are K stacked MLPs in marlnav/actor.py's StackedMLPActors layout: in -> 128 ->
// LayerNorm -> ReLU -> 128 -> LayerNorm -> ReLU -> out (9 actor logits, 1 critic value).  A batch
// of B rows (B a multiple of 16) is processed as:
//   l1_kernel       layer 1 (the only wide GEMM: in = K*D + 9K for a critic) split over
//                   64-input chunks: one workgroup per (job, agent, chunk, 128-row tile) writes
//                   the chunk's partial [rows][128]; the consumer adds the chunks in order.
//   *_tail kernels  everything per row: the chunk sum, LayerNorms, ReLUs, layers 2-3 (the
//                   block's 16 rows x 128 on v_mfma_f32_16x16x4_f32, W2 read from L2), Gumbel
//                   softmax (the critic tail computes every agent's target action itself), TD
//                   target, the loss gradient and the backward through layers 3, 2 and the
//                   LayerNorms.  One workgroup per (agent, 16 rows); a row's 128 features live on
//                   16 lanes (8 each), LayerNorm sums are 16-lane butterflies.
//   grads_kernel    the parameter gradients, reductions over the rows in row order: W1 = X^T dz1,
//                   W2 = h1^T dz2, W3 = h2^T g3, biases, LayerNorm affines, the loss value; written
//                   (not accumulated) into the flat gradient buffer's per-layer views.
// Everything is f32 with fixed summation orders (deterministic).  It differs from the torch
// composition (tests/test_maddpg_fused.py) by f32 summation order, including inside LayerNorm's
// row statistics, so a ReLU whose input sits at the rounding edge can take the other side; the
// tests state the flip-tolerant bound.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <initializer_list>
#include <string>

#include "learner_ops.h"
#include "philox.h"

namespace {

constexpr int HID = 128, NA = 9, RB = 16, TILE_R = 128, DC = 64, MAXK = GW_MAX_AGENTS, MAXJOB = 4;
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr float LN_EPS = 1e-5f, G_EPS = 1e-20f;

gw_status fail(gw_status s, const std::string &msg) {
    gw_set_last_error(msg.c_str());
    return s;
}

// ---- layer 1, split over input chunks ---------------------------------------------------------
// job: rows r of agent k read x[r * ldx + k * xk + col0 + d], weights w[k * wk + (wrow0 + d) * 128 + j]
// for d < D; part[((chunk * K + k) * B + r) * 128 + j] = sum over the chunk's inputs in order.
struct L1Job {
    const float *x;
    const float *w;
    float *part;
    int64_t ldx, xk, wk;
    int col0, wrow0, D, nchunk;
};
struct L1Params {
    L1Job job[MAXJOB];
    int njob, K, B, ntile;
    int start[MAXJOB + 1];  // first block of each job (blocks: job, k, chunk, row tile)
};

__global__ void __launch_bounds__(256) l1_kernel(L1Params p) {
    __shared__ __attribute__((aligned(16))) float s_x[DC][TILE_R + 4];  // [input][row]
    __shared__ __attribute__((aligned(16))) float s_w[DC][HID];         // [input][feature]
    int b = blockIdx.x, j = 0;
    while (j + 1 < p.njob && b >= p.start[j + 1]) ++j;
    const L1Job &jb = p.job[j];
    b -= p.start[j];
    const int tile = b % p.ntile;
    b /= p.ntile;
    const int chunk = b % jb.nchunk, k = b / jb.nchunk;
    const int tid = threadIdx.x;
    const int d0 = chunk * DC, r0 = tile * TILE_R;
    const int nd = min(DC, jb.D - d0);
    // stage x^T (rows of this tile, inputs of this chunk) and the chunk's weight rows
    // every load of a thread is issued before the first LDS store (one memory round trip: the
    // loop form waited for each of its 40 loads in turn, ~20 us per launch)
    const float *xb = jb.x + (int64_t)k * jb.xk + jb.col0 + d0;
    constexpr int XN = DC * TILE_R / 256, WN = DC * HID / 4 / 256;
    float xv[XN];
    float4 wv[WN];
#pragma unroll
    for (int t = 0; t < XN; ++t) {
        const int i = tid + 256 * t, r = i / DC, d = i % DC;  // consecutive threads: consecutive inputs of a row
        xv[t] = (d < nd && r0 + r < p.B) ? xb[(int64_t)(r0 + r) * jb.ldx + d] : 0.0f;
    }
    const float *wb = jb.w + (int64_t)k * jb.wk + (int64_t)(jb.wrow0 + d0) * HID;
#pragma unroll
    for (int t = 0; t < WN; ++t) {
        const int i = tid + 256 * t, d = i / (HID / 4), c = i % (HID / 4);
        wv[t] = d < nd ? reinterpret_cast<const float4 *>(wb + (int64_t)d * HID)[c] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < XN; ++t) {
        const int i = tid + 256 * t;
        s_x[i % DC][i / DC] = xv[t];
    }
#pragma unroll
    for (int t = 0; t < WN; ++t) {
        const int i = tid + 256 * t;
        *reinterpret_cast<float4 *>(&s_w[i / (HID / 4)][4 * (i % (HID / 4))]) = wv[t];
    }
    __syncthreads();
    // v_mfma_f32_16x16x4_f32: wave w computes rows 32 w .. 32 w + 31 (two 16-row tiles) x all 128
    // features (eight 16-column tiles) over the chunk's inputs in order, four per instruction: a
    // k-ordered f32 fma chain from 0, bit for bit the VALU loop it replaced (inputs past the
    // chunk's end are staged as zeros: fma(0, 0, acc) = acc)
    const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
    f32x4 acc[2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[a][c] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int nk = (nd + 3) / 4;
    for (int kk = 0; kk < nk; ++kk) {
        const int d = 4 * kk + lq;
        const float a0 = s_x[d][32 * wave + lr], a1 = s_x[d][32 * wave + 16 + lr];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float bw = s_w[d][16 * c + lr];
            acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bw, acc[0][c], 0, 0, 0);
            acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bw, acc[1][c], 0, 0, 0);
        }
    }
    // D: row 4 lq + i of the tile, column lr
    float *ob = jb.part + ((int64_t)chunk * p.K + k) * p.B * HID;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = r0 + 32 * wave + 16 * a + 4 * lq + i;
            if (r < p.B) {
#pragma unroll
                for (int c = 0; c < 8; ++c) ob[(int64_t)r * HID + 16 * c + lr] = acc[a][c][i];
            }
        }
}

// ---- layer-1 pre-activations: the chunk partials summed in chunk order + the bias ------------------
// z[k][r][j] = (sum over chunks c in order of part[c][k][r][j]) + b1[k][j]: the sum the tails formed
// themselves until round 4, bit for bit, now with every (k, r, 4 features) of every job in
// parallel (a thread's chunk loads 16 at a time in flight) instead of a dependent chain of L2/HBM
// round trips inside each tail (the partials come from other XCDs' L2s: ~2 us per round trip).
struct ReduceJob {
    const float *part, *b1;  // [nch][K][B][HID], [K][HID]
    float *z;                // [K][B][HID]
    int nch;
};
struct ReduceParams {
    ReduceJob job[MAXJOB];
    int njob, K, B, per_job;  // per_job: float4 outputs of one job (K B HID / 4)
};
constexpr int RED_PRE = 16;
__global__ void __launch_bounds__(256) l1_reduce(ReduceParams p) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int j = (int)(t / p.per_job);
    if (j >= p.njob) return;
    const ReduceJob &jb = p.job[j];
    const int i = (int)(t - (int64_t)j * p.per_job);  // float4 index in [K][B][HID / 4]
    const int k = i / (p.B * (HID / 4));
    const int j4 = i % (HID / 4);
    const int64_t cstride = (int64_t)p.K * p.B * (HID / 4);
    const float4 *src = reinterpret_cast<const float4 *>(jb.part) + i;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int c0 = 0; c0 < jb.nch; c0 += RED_PRE) {
        float4 v[RED_PRE];
#pragma unroll
        for (int c = 0; c < RED_PRE; ++c)
            v[c] = c0 + c < jb.nch ? src[(c0 + c) * cstride] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int c = 0; c < RED_PRE; ++c) {
            if (c0 + c < jb.nch) {  // (past the end: nothing added, not even a zero)
                acc.x += v[c].x;
                acc.y += v[c].y;
                acc.z += v[c].z;
                acc.w += v[c].w;
            }
        }
    }
    const float4 b = reinterpret_cast<const float4 *>(jb.b1 + (int64_t)k * HID)[j4];
    reinterpret_cast<float4 *>(jb.z)[i] = make_float4(acc.x + b.x, acc.y + b.y, acc.z + b.z, acc.w + b.w);
}

// ---- per-row helpers (a row = 16 lanes, lane g holds features 8 g .. 8 g + 7) ---------------------
__device__ __forceinline__ float row_sum(float v) {  // over the row's 16 lanes
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

struct Mlp {  // one agent's parameters (pointers already offset to agent k)
    const float *w1, *b1, *lw1, *lb1, *w2, *b2, *lw2, *lb2, *w3, *b3;
};
__device__ __forceinline__ Mlp mlp_k(const gw_mlp_actors &n, int k, int in_dim, int out) {
    Mlp m;
    m.w1 = n.w1 + (int64_t)k * in_dim * HID;
    m.b1 = n.b1 + k * HID;
    m.lw1 = n.ln1_w + k * HID;
    m.lb1 = n.ln1_b + k * HID;
    m.w2 = n.w2 + (int64_t)k * HID * HID;
    m.b2 = n.b2 + k * HID;
    m.lw2 = n.ln2_w + k * HID;
    m.lb2 = n.ln2_b + k * HID;
    m.w3 = n.w3 + (int64_t)k * HID * out;
    m.b3 = n.b3 + k * out;
    return m;
}

// LayerNorm (biased variance, eps 1e-5) + affine + ReLU of the 8 features z; xhat / relu output
__device__ __forceinline__ void ln_relu(const float z[8], const float *lw, const float *lb, int g, float xh[8],
                                        float y[8], float &rstd_out) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += z[i];
    const float mean = row_sum(s) * (1.0f / HID);
    float v = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = fmaf(z[i] - mean, z[i] - mean, v);
    const float rstd = rsqrtf(row_sum(v) * (1.0f / HID) + LN_EPS);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        xh[i] = (z[i] - mean) * rstd;
        const float o = xh[i] * lw[8 * g + i] + lb[8 * g + i];
        y[i] = o > 0.0f ? o : 0.0f;
    }
    rstd_out = rstd;
}

// backward of ln_relu: gy = grad at the ReLU output; gv = gy * (y > 0) (the affine output's
// gradient, kept for the LayerNorm parameter gradients); dz = rstd (dxh - mean(dxh) - xh mean(dxh xh))
__device__ __forceinline__ void ln_relu_bwd(const float gy[8], const float y[8], const float xh[8], float rstd,
                                            const float *lw, int g, float gv[8], float dz[8]) {
    float dx[8], s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        gv[i] = y[i] > 0.0f ? gy[i] : 0.0f;
        dx[i] = gv[i] * lw[8 * g + i];
        s1 += dx[i];
        s2 = fmaf(dx[i], xh[i], s2);
    }
    const float m1 = row_sum(s1) * (1.0f / HID), m2 = row_sum(s2) * (1.0f / HID);
#pragma unroll
    for (int i = 0; i < 8; ++i) dz[i] = rstd * (dx[i] - m1 - xh[i] * m2);
}

// The block's 16 rows through a 128 x 128 layer: z[r][n] = sum_c h[r][c] W[c][n] (transpose:
// W[n][c]) on v_mfma_f32_16x16x4_f32, W read straight from global memory (L2-resident: every
// block of the agent reads the same 64 KB), h from LDS.  Wave w computes columns 32 w .. 32 w +
// 31; each output is the k-ordered f32 fma chain over c = 0 .. 127 from 0 (the per-row VALU
// GEMV it replaced, bit for bit).  All threads call it; s_z [16][HP] receives z (the caller syncs
// before reading it).
constexpr int HP = HID + 4;  // padded LDS row
template <int U = HID / 4>  // k-steps per unrolled batch (U = 32: the whole layer's loads in flight)
__device__ __forceinline__ void gemv16(const float *s_h, const float *__restrict__ w, bool transpose, float *s_z) {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3, lr = lane & 15, lq = lane >> 4;
    const int n0 = 32 * wave + lr, n1 = n0 + 16;
    f32x4 acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
    // fully unrolled: the 64 weight loads of a lane are all in flight before the first MFMA
    // needs one (one L2 round trip per layer instead of one per 8 k-steps)
#pragma unroll U
    for (int kk = 0; kk < HID / 4; ++kk) {
        const int c = 4 * kk + lq;
        const float a = s_h[lr * HP + c];
        const float b0 = transpose ? w[n0 * HID + c] : w[c * HID + n0];
        const float b1 = transpose ? w[n1 * HID + c] : w[c * HID + n1];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b1, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s_z[(4 * lq + i) * HP + n0] = acc0[i];
        s_z[(4 * lq + i) * HP + n1] = acc1[i];
    }
}

// the block's rows through a 128 x 128 layer in the per-row layout (thread (rl, g) holds row rl's
// features 8 g .. 8 g + 7): v -> LDS, gemv16, back to registers (two block barriers)
template <int U = HID / 4>
__device__ __forceinline__ void rows_gemv(const float v[8], int rl, int g, const float *w, bool transpose, float *s_in,
                                          float *s_out, float out[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_in[rl * HP + 8 * g + i] = v[i];
    __syncthreads();
    gemv16<U>(s_in, w, transpose, s_out);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = s_out[rl * HP + 8 * g + i];
}

// the 8 layer-1 pre-activations of (k, row r) lane g holds, from l1_reduce's z [K][B][128]
__device__ __forceinline__ void z8(const float *zb, int B, int k, int r, int g, float z[8]) {
    const float *o = zb + ((int64_t)k * B + r) * HID + 8 * g;
    const float4 a = *reinterpret_cast<const float4 *>(o), b = *reinterpret_cast<const float4 *>(o + 4);
    z[0] = a.x; z[1] = a.y; z[2] = a.z; z[3] = a.w;
    z[4] = b.x; z[5] = b.y; z[6] = b.z; z[7] = b.w;
}

// save 8 features of row r to buf [K][B][128]
__device__ __forceinline__ void put8(float *buf, int K, int B, int k, int r, int g, const float v[8]) {
    (void)K;
    float *o = buf + ((int64_t)k * B + r) * HID + 8 * g;
    *reinterpret_cast<float4 *>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4 *>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// saved per-row quantities of one network's forward + backward (for grads_kernel)
struct Saved {
    float *h1, *h2, *xh1, *xh2, *gv1, *gv2, *dz1, *dz2;  // [K][B][128]
    float *g3;                                           // [K][B][out] gradient at layer 3's output
    float *aux;                                          // [K][B]: the loss terms
};

struct TailParams {
    gw_mlp_actors actor_t, critic_t, critic, actor;  // parameter sets
    const float *x;        // [B][ldx] critic input rows (states, stored actions)
    float *x_next;         // [B][ldx] next states; target actions written into the action slots
    const double *reward;  // [B][K]
    const uint8_t *done;   // [B][K]
    const float *u;        // [K][B][9] Gumbel uniforms of this phase's sample, or null: Philox draws
    uint64_t seed;         // (u null) key of the in-kernel draws
    const int32_t *ctr;    // (u null) a device counter that changes per update
    const float *z_a, *z_ct, *z_c;  // layer-1 pre-activations (l1_reduce: actor-like, critic target, critic)
    Saved sv;
    float gamma;
    int64_t ldx;
    int K, B, D;
    float *probs_out;      // actor phase: [K][B][9] the fresh action probabilities (tests), may be null
};

// the 9 Gumbel uniforms of (agent kk, row r) in phase ph (0: the target actions, 1: the actor's
// sample): from p.u, or Philox(seed; r, *ctr, 'GUM' + ph, 4 kk + j) when p.u is null
__device__ __forceinline__ void gumbel_uniforms(const TailParams &p, int ph, int kk, int r, float ur[NA]) {
    if (p.u) {
        const float *src = p.u + ((int64_t)kk * p.B + r) * NA;
#pragma unroll
        for (int a = 0; a < NA; ++a) ur[a] = src[a];
        return;
    }
    const uint32_t c = (uint32_t)p.ctr[0];
#pragma unroll
    for (int j = 0; j < (NA + 3) / 4; ++j) {
        const uint4 d = gwrng::philox((uint32_t)r, c, gwrng::TAG_GUMBEL + (uint32_t)ph, (uint32_t)(4 * kk + j),
                                      (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * j + i < NA) ur[4 * j + i] = gwrng::unit(w[i]);
    }
}

// ---- phase 1a: target actions a'_k = GumbelSoftmax(actor_target_k(s'_k)) -------------------
// agent kk's target action probabilities for row r (the per-row layout; all threads call it)
template <int U = HID / 4>
__device__ __forceinline__ void target_probs(const TailParams &p, int kk, int r, int rl, int g, float *s_in,
                                             float *s_out, float pr[NA]) {
    const Mlp m = mlp_k(p.actor_t, kk, p.D, NA);
    float z[8], xh[8], y[8], rs;
    z8(p.z_a, p.B, kk, r, g, z);
    ln_relu(z, m.lw1, m.lb1, g, xh, y, rs);
    rows_gemv<U>(y, rl, g, m.w2, false, s_in, s_out, z);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] += m.b2[8 * g + i];
    ln_relu(z, m.lw2, m.lb2, g, xh, y, rs);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = fmaf(y[i], m.w3[(8 * g + i) * NA + a], s);
        pr[a] = row_sum(s) + m.b3[a];
    }
    // GumbelSoftmax (tau 1): softmax(logits - log(-log(u + eps) + eps)), gw_gumbel_softmax's op order
    float ur[NA];
    gumbel_uniforms(p, 0, kk, r, ur);
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        pr[a] = (pr[a] - logf(-logf(ur[a] + G_EPS) + G_EPS)) / 1.0f;
        mx = fmaxf(mx, pr[a]);
    }
    float sum = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        pr[a] = expf(pr[a] - mx);
        sum += pr[a];
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) pr[a] = pr[a] / sum;
}

// forward of critic (m) on row r: z1 = partial sum + b1 + the action columns of `act` (9K values
// of this row, from LDS); saves into the given arrays; returns q
struct RowFwd {
    float xh1[8], y1[8], rs1, xh2[8], y2[8], rs2;
};
template <int U = HID / 4, int AU = 9>  // AU: action rows' loads in flight
__device__ __forceinline__ float critic_fwd(const Mlp &m, const float *zsrc, const TailParams &p, int k,
                                            int r, int rl, int g, const float *act, float *s_in, float *s_out,
                                            RowFwd &f) {
    float z[8];
    z8(zsrc, p.B, k, r, g, z);
    const int Ds = p.K * p.D;
#pragma unroll AU
    for (int a = 0; a < NA * p.K; ++a) {  // AU rows' loads in flight together, fmas in row order
        const float av = act[a];
        const float *wr = m.w1 + (int64_t)(Ds + a) * HID + 8 * g;
        const float4 w0 = *reinterpret_cast<const float4 *>(wr), w1 = *reinterpret_cast<const float4 *>(wr + 4);
        z[0] = fmaf(av, w0.x, z[0]); z[1] = fmaf(av, w0.y, z[1]); z[2] = fmaf(av, w0.z, z[2]); z[3] = fmaf(av, w0.w, z[3]);
        z[4] = fmaf(av, w1.x, z[4]); z[5] = fmaf(av, w1.y, z[5]); z[6] = fmaf(av, w1.z, z[6]); z[7] = fmaf(av, w1.w, z[7]);
    }
    ln_relu(z, m.lw1, m.lb1, g, f.xh1, f.y1, f.rs1);
    rows_gemv<U>(f.y1, rl, g, m.w2, false, s_in, s_out, z);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] += m.b2[8 * g + i];
    ln_relu(z, m.lw2, m.lb2, g, f.xh2, f.y2, f.rs2);
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s = fmaf(f.y2[i], m.w3[8 * g + i], s);
    return row_sum(s) + m.b3[0];
}

// backward through the critic from dq to dz1 (dh1 = dz2 W2^T on MFMA)
template <int U = HID / 4>
__device__ __forceinline__ void critic_bwd(const Mlp &m, float dq, int rl, int g, const RowFwd &f, float *s_in,
                                           float *s_out, float gv1[8], float dz1[8], float gv2[8], float dz2[8]) {
    float gy[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) gy[i] = dq * m.w3[8 * g + i];
    ln_relu_bwd(gy, f.y2, f.xh2, f.rs2, m.lw2, g, gv2, dz2);
    rows_gemv<U>(dz2, rl, g, m.w2, true, s_in, s_out, gy);
    ln_relu_bwd(gy, f.y1, f.xh1, f.rs1, m.lw1, g, gv1, dz1);
}

// ---- phase 1b: TD target from the critic target, the critic's forward, MSE gradient, backward ----
__global__ void __launch_bounds__(256) critic_tail(TailParams p) {
    __shared__ __attribute__((aligned(16))) float s_in[RB * HP];
    __shared__ __attribute__((aligned(16))) float s_out[RB * HP];
    __shared__ float s_act[RB][NA * MAXK];
    const int k = blockIdx.y, tid = threadIdx.x, rl = tid >> 4, g = tid & 15;
    const int r = blockIdx.x * RB + rl;
    const int na = NA * p.K;
    const int64_t Ds = (int64_t)p.K * p.D;
    // target critic on (s', a'): the target actions just computed
    const Mlp mt = mlp_k(p.critic_t, k, p.K * p.D + na, 1);
    const Mlp m = mlp_k(p.critic, k, p.K * p.D + na, 1);
    // every agent's target action on this block's rows (a block per agent recomputes the others':
    // K x a small MLP instead of a launch and a round trip through x_next); agent k's go to x_next
    // too (the caller's record of a')
    for (int kk = 0; kk < p.K; ++kk) {
        float pr[NA];
        target_probs(p, kk, r, rl, g, s_in, s_out, pr);
        if (g == 0) {
#pragma unroll
            for (int a = 0; a < NA; ++a) s_act[rl][NA * kk + a] = pr[a];
            if (kk == k) {
                float *o = p.x_next + (int64_t)r * p.ldx + Ds + NA * k;
#pragma unroll
                for (int a = 0; a < NA; ++a) o[a] = pr[a];
            }
        }
    }
    __syncthreads();
    RowFwd f;
    const float q_next = critic_fwd(mt, p.z_ct, p, k, r, rl, g, s_act[rl], s_in, s_out, f);
    // y = f32(r) + ((1 - d) * gamma) * q_next, gw_td_target's op order
    const float t1 = 1.0f - (float)p.done[(int64_t)r * p.K + k];
    const float y = (float)p.reward[(int64_t)r * p.K + k] + (t1 * p.gamma) * q_next;
    // online critic on (s, a): the stored actions are the x rows' action slots (in the partials)
    float z[8];
    z8(p.z_c, p.B, k, r, g, z);
    RowFwd o;
    ln_relu(z, m.lw1, m.lb1, g, o.xh1, o.y1, o.rs1);
    rows_gemv(o.y1, rl, g, m.w2, false, s_in, s_out, z);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] += m.b2[8 * g + i];
    ln_relu(z, m.lw2, m.lb2, g, o.xh2, o.y2, o.rs2);
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s = fmaf(o.y2[i], m.w3[8 * g + i], s);
    const float q = row_sum(s) + m.b3[0];
    const float diff = q - y;
    const float dq = (1.0f / (float)p.B) * (2.0f * diff);  // MSELoss backward (gw_mean_loss_bwd's order)
    float gv1[8], dz1[8], gv2[8], dz2[8];
    critic_bwd(m, dq, rl, g, o, s_in, s_out, gv1, dz1, gv2, dz2);
    const Saved &sv = p.sv;
    put8(sv.h1, p.K, p.B, k, r, g, o.y1);
    put8(sv.h2, p.K, p.B, k, r, g, o.y2);
    put8(sv.xh1, p.K, p.B, k, r, g, o.xh1);
    put8(sv.xh2, p.K, p.B, k, r, g, o.xh2);
    put8(sv.gv1, p.K, p.B, k, r, g, gv1);
    put8(sv.gv2, p.K, p.B, k, r, g, gv2);
    put8(sv.dz1, p.K, p.B, k, r, g, dz1);
    put8(sv.dz2, p.K, p.B, k, r, g, dz2);
    if (g == 0) {
        sv.g3[(int64_t)k * p.B + r] = dq;
        sv.aux[(int64_t)k * p.B + r] = diff * diff;
    }
}

// ---- phase 2: the actor's forward, GumbelSoftmax, the (updated) critic on the mixed actions,
//      -mean Q gradient, backward through the critic (no parameter gradients) and the actor ----
__global__ void __launch_bounds__(256) actor_tail(TailParams p) {
    __shared__ __attribute__((aligned(16))) float s_in[RB * HP];
    __shared__ __attribute__((aligned(16))) float s_out[RB * HP];
    __shared__ float s_act[RB][NA * MAXK];
    const int k = blockIdx.y, tid = threadIdx.x, rl = tid >> 4, g = tid & 15;
    const int r = blockIdx.x * RB + rl;
    const int na = NA * p.K;
    const int64_t Ds = (int64_t)p.K * p.D;
    const Mlp ma = mlp_k(p.actor, k, p.D, NA);
    const Mlp mc = mlp_k(p.critic, k, p.K * p.D + na, 1);
    // actor forward
    for (int i = tid; i < RB * na; i += 256) s_act[i / na][i % na] = p.x[(int64_t)(blockIdx.x * RB + i / na) * p.ldx + Ds + i % na];
    __syncthreads();
    float z[8];
    RowFwd fa;
    z8(p.z_a, p.B, k, r, g, z);
    ln_relu(z, ma.lw1, ma.lb1, g, fa.xh1, fa.y1, fa.rs1);
    rows_gemv(fa.y1, rl, g, ma.w2, false, s_in, s_out, z);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] += ma.b2[8 * g + i];
    ln_relu(z, ma.lw2, ma.lb2, g, fa.xh2, fa.y2, fa.rs2);
    float lg[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = fmaf(fa.y2[i], ma.w3[(8 * g + i) * NA + a], s);
        lg[a] = row_sum(s) + ma.b3[a];
    }
    // GumbelSoftmax (tau 1) with its gradient: torch's softmax((logits - log(-log(u + eps) + eps)) / 1)
    float ur[NA];
    gumbel_uniforms(p, 1, k, r, ur);
    float pr[NA], mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        pr[a] = (lg[a] - logf(-logf(ur[a] + G_EPS) + G_EPS)) / 1.0f;
        mx = fmaxf(mx, pr[a]);
    }
    float sum = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        pr[a] = expf(pr[a] - mx);
        sum += pr[a];
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) pr[a] = pr[a] / sum;
    if (p.probs_out && g == 0)
        for (int a = 0; a < NA; ++a) p.probs_out[((int64_t)k * p.B + r) * NA + a] = pr[a];
    // the critic k on the mixed actions (own slot: the fresh probabilities; the row's 16 lanes are
    // one wave's, whose LDS operations complete in order)
    if (g == 0)
        for (int a = 0; a < NA; ++a) s_act[rl][NA * k + a] = pr[a];
    RowFwd fc;
    const float q = critic_fwd(mc, p.z_c, p, k, r, rl, g, s_act[rl], s_in, s_out, fc);
    const float dq = -(1.0f / (float)p.B);  // -mean Q backward (gw_mean_loss_bwd mode 1)
    float gv1[8], dz1[8], gv2[8], dz2[8];
    critic_bwd(mc, dq, rl, g, fc, s_in, s_out, gv1, dz1, gv2, dz2);
    // d probs_k = dz1 . W1[the agent's action rows]^T
    float dp[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const float *wr = mc.w1 + (Ds + NA * k + a) * HID + 8 * g;
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = fmaf(dz1[i], wr[i], s);
        dp[a] = row_sum(s);
    }
    // softmax backward: dlogits = p (dp - sum p dp)  (tau 1)
    float dot = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a) dot = fmaf(pr[a], dp[a], dot);
    float dl[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) dl[a] = pr[a] * (dp[a] - dot);
    // actor backward
    float gy[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float s = 0.0f;
#pragma unroll
        for (int a = 0; a < NA; ++a) s = fmaf(dl[a], ma.w3[(8 * g + i) * NA + a], s);
        gy[i] = s;
    }
    ln_relu_bwd(gy, fa.y2, fa.xh2, fa.rs2, ma.lw2, g, gv2, dz2);
    rows_gemv(dz2, rl, g, ma.w2, true, s_in, s_out, gy);
    ln_relu_bwd(gy, fa.y1, fa.xh1, fa.rs1, ma.lw1, g, gv1, dz1);
    const Saved &sv = p.sv;
    put8(sv.h1, p.K, p.B, k, r, g, fa.y1);
    put8(sv.h2, p.K, p.B, k, r, g, fa.y2);
    put8(sv.xh1, p.K, p.B, k, r, g, fa.xh1);
    put8(sv.xh2, p.K, p.B, k, r, g, fa.xh2);
    put8(sv.gv1, p.K, p.B, k, r, g, gv1);
    put8(sv.gv2, p.K, p.B, k, r, g, gv2);
    put8(sv.dz1, p.K, p.B, k, r, g, dz1);
    put8(sv.dz2, p.K, p.B, k, r, g, dz2);
    if (g == 0) {
        for (int a = 0; a < NA; ++a) sv.g3[((int64_t)k * p.B + r) * NA + a] = dl[a];
        sv.aux[(int64_t)k * p.B + r] = q;
    }
}

// ---- parameter gradients: reductions over the B rows, in row order ---------------------------
// blocks [0, nw1): W1 rows (16 inputs each); [nw1, nw1 + 8): W2 rows; then one block for W3, the
// vectors and the loss.  x: rows r of agent k's layer-1 input at x[r * ldx + k * xk + col0 + d].
struct GradParams {
    gw_mlp_actors grad;    // the gradient views (same layout as the parameters), written
    const float *x;
    int64_t ldx, xk;
    int col0, in_dim, out, K, B, nw1, mode;  // mode 0: critic (loss mean (q - y)^2), 1: actor (-mean q)
    Saved sv;
    float *loss;           // [K]
    int32_t *adam_step;    // the following Adam step's count, advanced here (may be null)
};

constexpr int GRG = 16;  // row groups of the vector / W3 blocks (rows rg, rg + 16, ...)

__global__ void __launch_bounds__(256) grads_kernel(GradParams p) {
    if (p.adam_step && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) p.adam_step[0] += 1;
    // W blocks: s_in + s_dz; vector block: [16][6][128]; W3 block: [16][128][9] + [16][10]
    __shared__ __attribute__((aligned(16))) float smem[GRG * HID * NA + GRG * (NA + 1) > RB * (TILE_R + 4) + TILE_R * HID
                                                        ? GRG * HID * NA + GRG * (NA + 1)
                                                        : RB * (TILE_R + 4) + TILE_R * HID];
    const int k = blockIdx.y, tid = threadIdx.x;
    const int b = blockIdx.x;
    if (b < p.nw1 + HID / RB) {
        float (*s_in)[TILE_R + 4] = reinterpret_cast<float (*)[TILE_R + 4]>(smem);     // [input][row]
        float (*s_dz)[HID] = reinterpret_cast<float (*)[HID]>(smem + RB * (TILE_R + 4));  // [row][feature]
        const bool w1 = b < p.nw1;
        const int d0 = (w1 ? b : b - p.nw1) * RB;
        const int D = w1 ? p.in_dim : HID;
        const float *dz = w1 ? p.sv.dz1 : p.sv.dz2;
        // v_mfma_f32_16x16x4_f32: the block's 16 inputs x 128 features = X^T dz over the rows in
        // order (a k-ordered f32 fma chain from 0 across the row tiles); wave w owns features
        // 32 w .. 32 w + 31
        const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
        f32x4 acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
        const int n0 = 32 * wave + lr, n1 = n0 + 16;
        for (int r0 = 0; r0 < p.B; r0 += TILE_R) {
            const int nr = min(TILE_R, p.B - r0);
            __syncthreads();
            // all of a thread's loads first, then the LDS stores (one memory round trip)
            constexpr int XN = RB * TILE_R / 256, ZN = TILE_R * HID / 4 / 256;
            float xv[XN];
            float4 zv[ZN];
#pragma unroll
            for (int t = 0; t < XN; ++t) {
                const int i = tid + 256 * t, r = i / RB, d = i % RB;
                float v = 0.0f;
                if (r < nr && d0 + d < D)
                    v = w1 ? p.x[(int64_t)(r0 + r) * p.ldx + (int64_t)k * p.xk + p.col0 + d0 + d]
                           : p.sv.h1[((int64_t)k * p.B + r0 + r) * HID + d0 + d];
                xv[t] = v;
            }
#pragma unroll
            for (int t = 0; t < ZN; ++t) {
                const int i = tid + 256 * t, r = i / (HID / 4), c = i % (HID / 4);
                zv[t] = r < nr ? reinterpret_cast<const float4 *>(dz + ((int64_t)k * p.B + r0 + r) * HID)[c]
                               : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
#pragma unroll
            for (int t = 0; t < XN; ++t) {
                const int i = tid + 256 * t;
                if (i / RB < nr) s_in[i % RB][i / RB] = xv[t];
            }
#pragma unroll
            for (int t = 0; t < ZN; ++t) {
                const int i = tid + 256 * t;
                if (i / (HID / 4) < nr) *reinterpret_cast<float4 *>(&s_dz[i / (HID / 4)][4 * (i % (HID / 4))]) = zv[t];
            }
            __syncthreads();
            for (int kk = 0; kk < nr / 4; ++kk) {  // nr: a multiple of 16 (B % 16 == 0)
                const int r = 4 * kk + lq;
                const float a = s_in[lr][r];
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s_dz[r][n0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s_dz[r][n1], acc1, 0, 0, 0);
            }
        }
        float *ob = const_cast<float *>(w1 ? p.grad.w1 + (int64_t)k * p.in_dim * HID : p.grad.w2 + (int64_t)k * HID * HID);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = d0 + 4 * lq + i;
            if (d < D) {
                ob[(int64_t)d * HID + n0] = acc0[i];
                ob[(int64_t)d * HID + n1] = acc1[i];
            }
        }
        return;
    }
    // thread (row group rg, features 8 g .. 8 g + 7) sums rows rg, rg + 16, ...; the 16 partials are
    // then added in row-group order (fixed order, independent of the launch)
    const int rg = tid >> 4, g = tid & 15;
    const int64_t base = (int64_t)k * p.B * HID;
    if (b == p.nw1 + HID / RB) {  // the vectors: b1, ln1 affine, b2, ln2 affine
        float acc[6][8];
#pragma unroll
        for (int v = 0; v < 6; ++v)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[v][i] = 0.0f;
#pragma unroll 2
        for (int r = rg; r < p.B; r += GRG) {
            const int64_t o = base + (int64_t)r * HID + 8 * g;
            const float *src[6] = {p.sv.dz1 + o, p.sv.gv1 + o, p.sv.xh1 + o, p.sv.dz2 + o, p.sv.gv2 + o, p.sv.xh2 + o};
            float4 q[6][2];
#pragma unroll
            for (int v = 0; v < 6; ++v) {
                q[v][0] = *reinterpret_cast<const float4 *>(src[v]);
                q[v][1] = *reinterpret_cast<const float4 *>(src[v] + 4);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int o2 = 3 * h;  // (dz, gv, xh) of layer h + 1
                const float dzv[8] = {q[o2][0].x, q[o2][0].y, q[o2][0].z, q[o2][0].w,
                                      q[o2][1].x, q[o2][1].y, q[o2][1].z, q[o2][1].w};
                const float gvv[8] = {q[o2 + 1][0].x, q[o2 + 1][0].y, q[o2 + 1][0].z, q[o2 + 1][0].w,
                                      q[o2 + 1][1].x, q[o2 + 1][1].y, q[o2 + 1][1].z, q[o2 + 1][1].w};
                const float xhv[8] = {q[o2 + 2][0].x, q[o2 + 2][0].y, q[o2 + 2][0].z, q[o2 + 2][0].w,
                                      q[o2 + 2][1].x, q[o2 + 2][1].y, q[o2 + 2][1].z, q[o2 + 2][1].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    acc[o2][i] += dzv[i];                                  // db
                    acc[o2 + 1][i] = fmaf(gvv[i], xhv[i], acc[o2 + 1][i]);  // d ln_w
                    acc[o2 + 2][i] += gvv[i];                              // d ln_b
                }
            }
        }
        float (*part)[6][HID] = reinterpret_cast<float (*)[6][HID]>(smem);  // [rg][vector][feature]
#pragma unroll
        for (int v = 0; v < 6; ++v)
#pragma unroll
            for (int i = 0; i < 8; ++i) part[rg][v][8 * g + i] = acc[v][i];
        __syncthreads();
        for (int t = tid; t < 6 * HID; t += 256) {
            const int v = t / HID, j = t % HID;
            float sum = 0.0f;
            for (int q = 0; q < GRG; ++q) sum += part[q][v][j];
            float *dst[6] = {const_cast<float *>(p.grad.b1), const_cast<float *>(p.grad.ln1_w),
                             const_cast<float *>(p.grad.ln1_b), const_cast<float *>(p.grad.b2),
                             const_cast<float *>(p.grad.ln2_w), const_cast<float *>(p.grad.ln2_b)};
            dst[v][k * HID + j] = sum;
        }
        return;
    }
    // W3 = h2^T g3 [128][out], b3 = sum g3, the loss
    const int out = p.out;
    float acc[8][NA];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[i][a] = 0.0f;
    float bacc[NA], lacc = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a) bacc[a] = 0.0f;
#pragma unroll 4
    for (int r = rg; r < p.B; r += GRG) {
        const float *hs = p.sv.h2 + base + (int64_t)r * HID + 8 * g;
        const float4 h0 = *reinterpret_cast<const float4 *>(hs), h1 = *reinterpret_cast<const float4 *>(hs + 4);
        const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        const float *gs = p.sv.g3 + ((int64_t)k * p.B + r) * out;
        float gv[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) gv[a] = a < out ? gs[a] : 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int a = 0; a < NA; ++a) acc[i][a] = fmaf(hv[i], gv[a], acc[i][a]);
#pragma unroll
        for (int a = 0; a < NA; ++a) bacc[a] += gv[a];
        lacc += p.sv.aux[(int64_t)k * p.B + r];
    }
    float (*part)[HID][NA] = reinterpret_cast<float (*)[HID][NA]>(smem);            // [rg][feature][a]
    float (*pb)[NA + 1] = reinterpret_cast<float (*)[NA + 1]>(smem + GRG * HID * NA);  // [rg][a | loss]
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int a = 0; a < NA; ++a) part[rg][8 * g + i][a] = acc[i][a];
    if (g == 0) {
#pragma unroll
        for (int a = 0; a < NA; ++a) pb[rg][a] = bacc[a];
        pb[rg][NA] = lacc;
    }
    __syncthreads();
    for (int t = tid; t < HID * out; t += 256) {
        const int j = t / out, a = t % out;
        float sum = 0.0f;
        for (int q = 0; q < GRG; ++q) sum += part[q][j][a];
        const_cast<float *>(p.grad.w3)[((int64_t)k * HID + j) * out + a] = sum;
    }
    if (tid < out) {
        float sum = 0.0f;
        for (int q = 0; q < GRG; ++q) sum += pb[q][tid];
        const_cast<float *>(p.grad.b3)[k * out + tid] = sum;
    } else if (tid == 64 && p.loss) {
        float sum = 0.0f;
        for (int q = 0; q < GRG; ++q) sum += pb[q][NA];
        p.loss[k] = p.mode == 0 ? sum / (float)p.B : -(sum / (float)p.B);
    }
}

// ---- workspace ---------------------------------------------------------------------------------
struct Ws {
    float *part_a, *part_ct, *part_c;
    float *z_a, *z_ct, *z_c;  // [K][B][HID] each
    Saved sv;
};
inline int nchunks(int64_t D) { return (int)((D + DC - 1) / DC); }
inline Ws ws_layout(float *w, int K, int B, int D) {
    const int64_t ldx = (int64_t)K * D + (int64_t)NA * K;
    Ws s;
    s.part_a = w;
    w += (int64_t)nchunks(D) * K * B * HID;
    s.part_ct = w;
    w += (int64_t)nchunks((int64_t)K * D) * K * B * HID;
    s.part_c = w;
    w += (int64_t)nchunks(ldx) * K * B * HID;
    s.z_a = w;
    s.z_ct = w + (int64_t)K * B * HID;
    s.z_c = w + 2LL * K * B * HID;
    w += 3LL * K * B * HID;
    float **f[8] = {&s.sv.h1, &s.sv.h2, &s.sv.xh1, &s.sv.xh2, &s.sv.gv1, &s.sv.gv2, &s.sv.dz1, &s.sv.dz2};
    for (float **q : f) {
        *q = w;
        w += (int64_t)K * B * HID;
    }
    s.sv.g3 = w;
    w += (int64_t)K * B * NA;
    s.sv.aux = w;
    return s;
}
int64_t ws_floats(int K, int B, int D) {
    const int64_t ldx = (int64_t)K * D + (int64_t)NA * K;
    return ((int64_t)nchunks(D) + nchunks((int64_t)K * D) + nchunks(ldx)) * K * B * HID + 11LL * K * B * HID +
           (int64_t)K * B * NA + (int64_t)K * B + 64;
}

void add_job(L1Params &lp, int &blocks, const float *x, int64_t ldx, int64_t xk, int col0, const float *w, int64_t wk,
             int wrow0, int D, float *part) {
    L1Job &j = lp.job[lp.njob];
    j.x = x;
    j.w = w;
    j.part = part;
    j.ldx = ldx;
    j.xk = xk;
    j.wk = wk;
    j.col0 = col0;
    j.wrow0 = wrow0;
    j.D = D;
    j.nchunk = nchunks(D);
    lp.start[lp.njob] = blocks;
    blocks += j.nchunk * lp.K * lp.ntile;
    lp.njob++;
    lp.start[lp.njob] = blocks;
}

void launch_reduce(int K, int B, std::initializer_list<ReduceJob> jobs, hipStream_t s) {
    ReduceParams rp{};
    for (const ReduceJob &j : jobs) rp.job[rp.njob++] = j;
    rp.K = K;
    rp.B = B;
    rp.per_job = K * B * (HID / 4);
    const int64_t threads = (int64_t)rp.njob * rp.per_job;
    hipLaunchKernelGGL(l1_reduce, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, rp);
}

gw_status check(const gw_maddpg_batch *b, const char *who) {
    const std::string w(who);
    if (!b || !b->x || !b->x_next || (!b->u && !b->ctr)) return fail(GW_ERR_ARG, w + ": null argument");
    if (b->K < 1 || b->K > MAXK) return fail(GW_ERR_ARG, w + ": K out of range");
    if (b->B < RB || b->B % RB) return fail(GW_ERR_ARG, w + ": B must be a positive multiple of 16");
    if (b->D < 1) return fail(GW_ERR_ARG, w + ": D must be >= 1");
    if ((reinterpret_cast<uintptr_t>(b->x) | reinterpret_cast<uintptr_t>(b->x_next)) & 3u)
        return fail(GW_ERR_ARG, w + ": misaligned rows");
    return GW_OK;
}

gw_status check_net(const gw_mlp_actors &n, int K, int in_dim, int out, const std::string &w) {
    if (n.K != K || n.in_dim != in_dim || n.hidden != HID || n.n_actions != out || !n.layer_norm)
        return fail(GW_ERR_ARG, w + ": network shape (needs K, in_dim, hidden 128, LayerNorm, out)");
    if (!n.w1 || !n.b1 || !n.ln1_w || !n.ln1_b || !n.w2 || !n.b2 || !n.ln2_w || !n.ln2_b || !n.w3 || !n.b3)
        return fail(GW_ERR_ARG, w + ": null parameter");
    if ((reinterpret_cast<uintptr_t>(n.w1) | reinterpret_cast<uintptr_t>(n.w2)) & 15u)
        return fail(GW_ERR_ARG, w + ": w1 / w2 must be 16-byte aligned");
    return GW_OK;
}

}  // namespace

extern "C" {

int64_t gw_maddpg_workspace_floats(int32_t K, int32_t B, int32_t D) { return ws_floats(K, B, D); }

gw_status gw_maddpg_critic_grads(const gw_mlp_actors *actor_target, const gw_mlp_actors *critic_target,
                                 const gw_mlp_actors *critic, const gw_mlp_actors *critic_grad,
                                 const gw_maddpg_batch *batch, float gamma, float *ws, float *loss,
                                 int32_t *adam_step, void *stream) {
    gw_status st = check(batch, "gw_maddpg_critic_grads");
    if (st != GW_OK) return st;
    if (!actor_target || !critic_target || !critic || !critic_grad || !ws || !batch->reward || !batch->done)
        return fail(GW_ERR_ARG, "gw_maddpg_critic_grads: null argument");
    const int K = batch->K, B = batch->B, D = batch->D;
    const int64_t ldx = (int64_t)K * D + (int64_t)NA * K;
    const std::string who("gw_maddpg_critic_grads");
    if ((st = check_net(*actor_target, K, D, NA, who)) != GW_OK) return st;
    if ((st = check_net(*critic_target, K, (int)ldx, 1, who)) != GW_OK) return st;
    if ((st = check_net(*critic, K, (int)ldx, 1, who)) != GW_OK) return st;
    const Ws w = ws_layout(ws, K, B, D);
    hipStream_t s = static_cast<hipStream_t>(stream);
    L1Params lp{};
    lp.K = K;
    lp.B = B;
    lp.ntile = (B + TILE_R - 1) / TILE_R;
    int blocks = 0;
    add_job(lp, blocks, batch->x_next, ldx, D, 0, actor_target->w1, (int64_t)D * HID, 0, D, w.part_a);
    add_job(lp, blocks, batch->x_next, ldx, 0, 0, critic_target->w1, ldx * HID, 0, K * D, w.part_ct);
    add_job(lp, blocks, batch->x, ldx, 0, 0, critic->w1, ldx * HID, 0, (int)ldx, w.part_c);
    hipLaunchKernelGGL(l1_kernel, dim3(blocks), dim3(256), 0, s, lp);
    launch_reduce(K, B, {{w.part_a, actor_target->b1, w.z_a, nchunks(D)},
                         {w.part_ct, critic_target->b1, w.z_ct, nchunks((int64_t)K * D)},
                         {w.part_c, critic->b1, w.z_c, nchunks(ldx)}}, s);
    TailParams tp{};
    tp.actor_t = *actor_target;
    tp.critic_t = *critic_target;
    tp.critic = *critic;
    tp.x = batch->x;
    tp.x_next = batch->x_next;
    tp.reward = batch->reward;
    tp.done = batch->done;
    tp.u = batch->u;
    tp.seed = batch->seed;
    tp.ctr = batch->ctr;
    tp.z_a = w.z_a;
    tp.z_ct = w.z_ct;
    tp.z_c = w.z_c;
    tp.sv = w.sv;
    tp.gamma = gamma;
    tp.ldx = ldx;
    tp.K = K;
    tp.B = B;
    tp.D = D;
    hipLaunchKernelGGL(critic_tail, dim3(B / RB, K), dim3(256), 0, s, tp);
    GradParams gp{};
    gp.grad = *critic_grad;
    gp.x = batch->x;
    gp.ldx = ldx;
    gp.xk = 0;
    gp.col0 = 0;
    gp.in_dim = (int)ldx;
    gp.out = 1;
    gp.K = K;
    gp.B = B;
    gp.nw1 = (int)((ldx + RB - 1) / RB);
    gp.mode = 0;
    gp.sv = w.sv;
    gp.loss = loss;
    gp.adam_step = adam_step;
    hipLaunchKernelGGL(grads_kernel, dim3(gp.nw1 + HID / RB + 2, K), dim3(256), 0, s, gp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GW_ERR_HIP, who + ": " + hipGetErrorString(e));
    return GW_OK;
}

gw_status gw_maddpg_actor_grads(const gw_mlp_actors *actor, const gw_mlp_actors *critic,
                                const gw_mlp_actors *actor_grad, const gw_maddpg_batch *batch, float *ws, float *loss,
                                float *probs, int32_t *adam_step, void *stream) {
    gw_status st = check(batch, "gw_maddpg_actor_grads");
    if (st != GW_OK) return st;
    if (!actor || !critic || !actor_grad || !ws) return fail(GW_ERR_ARG, "gw_maddpg_actor_grads: null argument");
    const int K = batch->K, B = batch->B, D = batch->D;
    const int64_t ldx = (int64_t)K * D + (int64_t)NA * K;
    const std::string who("gw_maddpg_actor_grads");
    if ((st = check_net(*actor, K, D, NA, who)) != GW_OK) return st;
    if ((st = check_net(*critic, K, (int)ldx, 1, who)) != GW_OK) return st;
    const Ws w = ws_layout(ws, K, B, D);
    hipStream_t s = static_cast<hipStream_t>(stream);
    L1Params lp{};
    lp.K = K;
    lp.B = B;
    lp.ntile = (B + TILE_R - 1) / TILE_R;
    int blocks = 0;
    add_job(lp, blocks, batch->x, ldx, D, 0, actor->w1, (int64_t)D * HID, 0, D, w.part_a);
    add_job(lp, blocks, batch->x, ldx, 0, 0, critic->w1, ldx * HID, 0, K * D, w.part_c);  // state columns
    hipLaunchKernelGGL(l1_kernel, dim3(blocks), dim3(256), 0, s, lp);
    launch_reduce(K, B, {{w.part_a, actor->b1, w.z_a, nchunks(D)}, {w.part_c, critic->b1, w.z_c, nchunks((int64_t)K * D)}}, s);
    TailParams tp{};
    tp.actor = *actor;
    tp.critic = *critic;
    tp.x = batch->x;
    tp.x_next = batch->x_next;
    tp.u = batch->u;
    tp.seed = batch->seed;
    tp.ctr = batch->ctr;
    tp.z_a = w.z_a;
    tp.z_c = w.z_c;
    tp.sv = w.sv;
    tp.ldx = ldx;
    tp.K = K;
    tp.B = B;
    tp.D = D;
    tp.probs_out = probs;
    hipLaunchKernelGGL(actor_tail, dim3(B / RB, K), dim3(256), 0, s, tp);
    GradParams gp{};
    gp.grad = *actor_grad;
    gp.x = batch->x;
    gp.ldx = ldx;
    gp.xk = D;
    gp.col0 = 0;
    gp.in_dim = D;
    gp.out = NA;
    gp.K = K;
    gp.B = B;
    gp.nw1 = (D + RB - 1) / RB;
    gp.mode = 1;
    gp.sv = w.sv;
    gp.loss = loss;
    gp.adam_step = adam_step;
    hipLaunchKernelGGL(grads_kernel, dim3(gp.nw1 + HID / RB + 2, K), dim3(256), 0, s, gp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GW_ERR_HIP, who + ": " + hipGetErrorString(e));
    return GW_OK;
}

}  // extern "C"
