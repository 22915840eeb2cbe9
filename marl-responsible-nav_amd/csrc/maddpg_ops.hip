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
#include <vector>
#include <cstdio>

#include "learner_ops.h"
#include "philox.h"
#include "prof.h"
#include "measure.h"

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
// v from the lane the DPP control names (within the lane's 16-lane row)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// over the row's 16 lanes, a butterfly on DPP lane moves (VALU, no LDS round trip): pairs (xor 1),
// quads (xor 2), half rows (mirror within 8) and rows (mirror within 16); every lane ends with the
// same sum (each step adds two equal-valued partials in either order), the xor butterfly's values
__device__ __forceinline__ float row_sum(float v) {
    v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_f<0x141>(v);  // row_half_mirror
    v += dpp_f<0x140>(v);  // row_mirror
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
// gemv_t4 (round 5): the transposed layer (W^T, the backward) feeds k-step 4 t + s with input
// c = 16 t + 4 lq + s, so a lane's four values of a step group are ONE float4 of its W row (and of
// its LDS row): 8 instead of 32 loads per column, each a contiguous 16 bytes (the strided c = 4 kk
// + lq order touched 16 rows' lines per load instruction: ~7 us per layer on freshly updated
// weights vs ~1.7 us forward).  The k order differs from the VALU loop's, so the backward layers
// are deterministic but no longer the loop's bits (the parity tests bound them against torch).
constexpr int HP = HID + 4;  // padded LDS row
template <int U = HID / 4>  // k-steps per unrolled batch (U = 32: the whole layer's loads in flight)
__device__ __forceinline__ void gemv16(const float *s_h, const float *__restrict__ w, bool transpose, float *s_z) {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3, lr = lane & 15, lq = lane >> 4;
    const int n0 = 32 * wave + lr, n1 = n0 + 16;
    f32x4 acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
    if (transpose) {  // W^T: k-step 4 t + s takes c = 16 t + 4 lq + s (gemv_t4)
        float4 w0[HID / 16], w1[HID / 16];
#pragma unroll
        for (int t = 0; t < HID / 16; ++t) {
            w0[t] = *reinterpret_cast<const float4 *>(w + n0 * HID + 16 * t + 4 * lq);
            w1[t] = *reinterpret_cast<const float4 *>(w + n1 * HID + 16 * t + 4 * lq);
        }
#pragma unroll
        for (int t = 0; t < HID / 16; ++t) {
            const float4 a = *reinterpret_cast<const float4 *>(s_h + lr * HP + 16 * t + 4 * lq);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, w0[t].x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, w1[t].x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, w0[t].y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, w1[t].y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, w0[t].z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, w1[t].z, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, w0[t].w, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, w1[t].w, acc1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s_z[(4 * lq + i) * HP + n0] = acc0[i];
            s_z[(4 * lq + i) * HP + n1] = acc1[i];
        }
        return;
    }
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

// =================================================================================================
// The descriptor learner (round 5): one MADDPG update on the replay ring of obs descriptors
// (Rollout(desc_ring=True)) as FOUR launches, the sample drawn inside them.  Layer 1 never runs
// as a GEMM: an obs is the static map (0 road, -1 inactive) plus <= N + 1 patched cells
// (ma_customenv.py:197-209, :303-322), so for every network with obs inputs
//     x . W1 + b1 = c1 + sum over patched cells c of (obs[c] - map[c]) * W1[c, :],
//     c1 = b1 + map . W1   (kept as partial sums over 64-row groups of W1, refreshed in the
//                           launch that changes W1: the Adam step or the soft update),
// and the W1 gradient X^T dZ1 = map (x) colsum(dZ1) + the patched cells' terms.  So the update
// reads 48-byte descriptors instead of 2 x 8 KB dense rows per sample, and needs no layer-1 GEMM,
// no chunk reduction and no gather launch:
//   dcritic_tail   per (agent k, 16 rows), two 4-wave groups: draws the rows (Philox, the
//                  gather's formula), decodes their descriptors, runs the K target actors two at a
//                  time, then the target critic beside the online critic, the TD target and the
//                  critic backward (its 128 x 128 layer on all 8 waves); records the rows for the
//                  launches below
//   dgrads_adam    the critic's parameter gradients (W1 from the patched cells + the column sums
//                  of dZ1), each element's Adam step in the thread that formed its gradient, the
//                  new critic's c1 partials
//   dactor_tail    the actor forward, GumbelSoftmax, the stepped critic on the mixed actions and
//                  both backwards (each 128 x 128 layer on all 8 waves)
//   dgrads_adam    the actor's gradients + Adam, both soft target updates, the c1 partials of the
//                  actor and both targets
// f32 with fixed summation orders (deterministic; graph / recorded replays equal eager launches).
// Against the dense formulation it differs by summation order in layer 1 and in the W1 gradient.
constexpr int NPM = GW_MAX_AGENTS + 1;  // patch slots per (row, agent obs): the apple + N agents
constexpr int CG = 64;                  // W1 input rows per c1 partial / W1-gradient block
constexpr int DT = 512;                 // tail threads: two 4-wave groups
constexpr int NDW = 12;                 // descriptor words (gridenv.hip NDESC)
constexpr uint32_t DF_RESET = 1u;
constexpr int DMAXB = 256;              // rows per update the W1 blocks' LDS lists are sized for

struct DQ {  // the descriptor ring and the env's obs source
    const uint32_t *desc;
    const float *probs;
    const double *reward;
    const uint8_t *term, *done;
    const int64_t *t_dev;
    int64_t S, E;
    const float *base;
    int apples[MAXK];
    int N, K, HW, variant;
};

struct DWs {
    int32_t *idx;      // [B][2] (transition slot, env) of every row
    int32_t *pc;       // [2][K][B][NPM] patched cells of (state | next state, agent obs, row)
    float *pd;         // [2][K][B][NPM] their obs - map deltas (overridden patches dropped)
    int32_t *np;       // [2][K][B]
    float *act;        // [B][9K] stored action probabilities
    float *tact;       // [B][9K] target actions a'
    float *u;          // [2][K][B][9] Gumbel uniforms (0: target actions, 1: the actor's sample)
    float *probs;      // [K][B][9] the actor phase's fresh probabilities
    float *rw, *t1;    // [K][B] f32(reward), 1 - termination
    Saved sv;          // per-row activations and gradients (critic phase, then the actor's)
    float *cpart[4];   // c1 partials: actor [K][NG][128], actor target, critic [K][K NG][128], critic target
    int32_t *snap;     // [4] the Adam step counts of this update (critic, actor)
    float *adsc;       // [4] this update's Adam scalars (step size, sqrt(bias correction 2)): critic, actor
};

inline int64_t rnd4(int64_t n) { return (n + 3) & ~(int64_t)3; }
inline int d_ng(int HW) { return (HW + CG - 1) / CG; }
inline DWs dws_layout(float *w, int K, int B, int HW) {
    DWs d;
    const int NG = d_ng(HW);
    auto take = [&](int64_t n) { float *q = w; w += rnd4(n); return q; };
    d.idx = reinterpret_cast<int32_t *>(take(2LL * B));
    d.pc = reinterpret_cast<int32_t *>(take(2LL * K * B * NPM));
    d.pd = take(2LL * K * B * NPM);
    d.np = reinterpret_cast<int32_t *>(take(2LL * K * B));
    d.act = take((int64_t)B * NA * K);
    d.tact = take((int64_t)B * NA * K);
    d.u = take(2LL * K * B * NA);
    d.probs = take((int64_t)K * B * NA);
    d.rw = take((int64_t)K * B);
    d.t1 = take((int64_t)K * B);
    float **f[8] = {&d.sv.h1, &d.sv.h2, &d.sv.xh1, &d.sv.xh2, &d.sv.gv1, &d.sv.gv2, &d.sv.dz1, &d.sv.dz2};
    for (float **q : f) *q = take((int64_t)K * B * HID);
    d.sv.g3 = take((int64_t)K * B * NA);
    d.sv.aux = take((int64_t)K * B);
    d.cpart[0] = take((int64_t)K * NG * HID);
    d.cpart[1] = take((int64_t)K * NG * HID);
    d.cpart[2] = take((int64_t)K * K * NG * HID);
    d.cpart[3] = take((int64_t)K * K * NG * HID);
    d.snap = reinterpret_cast<int32_t *>(take(4));
    d.adsc = take(4);
    return d;
}
int64_t dws_floats(int K, int B, int HW) {
    float *z = nullptr;
    const DWs d = dws_layout(z, K, B, HW);
    return (int64_t)(d.adsc - z) + 4;
}

// obs value of agent n in RL agent k's observation (the obs writer's rule, gridenv.hip agent_value)
__device__ __forceinline__ float d_agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;
    if (v == k + 1) v = 1;
    return (float)v;
}

// the patched cells of agent k's obs from descriptor words d (wsel 0: the obs, 1: the terminal
// obs, words 8-11), in the obs writer's order (the own apple, then agents 0 .. N-1; a later
// patch of the same cell overrides an earlier one), reduced to the surviving cells, as deltas
// against the map.  Returns the count.
__device__ __forceinline__ int d_patches(const DQ &q, const uint32_t (&d)[NDW], int wsel, int k, float apple_map,
                                         int *oc, float *od) {
    const uint32_t f = d[4];
    const bool reset = wsel == 0 && (f & DF_RESET);
    const uint32_t apples = wsel == 0 ? (f >> 8) & 0xFFu : (f >> 16) & 0xFFu;
    const int ac = ((apples >> k) & 1u) ? q.apples[k] : -1;
    int pc[NPM];
    float pv[NPM];
    int np = 0;
    if (ac >= 0) {
        float av = apple_map + 9.0f;
        if (!reset && av == (float)(k + 1)) av = 1.0f;
        pc[np] = ac;
        pv[np] = av;
        ++np;
    }
    for (int n = 0; n < q.N; ++n) {
        const uint32_t w = wsel == 0 ? d[n >> 1] : d[8 + (n >> 1)];
        const int c = (int)((w >> (16 * (n & 1))) & 0xFFFFu);
        pc[np] = c;
        pv[np] = d_agent_value(reset, n, k, c == ac, q.variant);
        ++np;
    }
    float bv[NPM];
    for (int i = 0; i < np; ++i) bv[i] = q.base[pc[i]];  // the loads in flight together
    int m = 0;
    for (int i = 0; i < np; ++i) {
        bool keep = true;
        for (int j = i + 1; j < np; ++j) keep = keep && pc[j] != pc[i];
        if (keep) {
            oc[m] = pc[i];
            od[m] = pv[i] - bv[i];
            ++m;
        }
    }
    return m;
}

// row b of the sample: transition slot tr and env e (gw_replay_gather_desc's in-kernel draws)
__device__ __forceinline__ void d_draw(const DQ &q, int64_t t, uint64_t seed, uint32_t c, int b, int64_t &tr,
                                       int64_t &e) {
    const uint4 r = gwrng::philox((uint32_t)b, c, gwrng::TAG_SAMPLE, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float ub = gwrng::unit(r.x);
    e = (int64_t)(((uint64_t)r.y * (uint64_t)q.E) >> 32);
    const int64_t n = t < 1 ? 1 : (t > q.S - 1 ? q.S - 1 : t);
    int64_t step = (int64_t)(ub * (float)n);
    if (step > n - 1) step = n - 1;
    tr = (t - 1 - step) % q.S;
    if (tr < 0) tr += q.S;
}

// sum over n partials p[g * HID] in g order (32 loads in flight: one round trip up to n = 32;
// batches past n re-read partial 0 and skip it)
__device__ __forceinline__ float d_sum_parts(const float *p, int n) {
    float acc = 0.0f;
    for (int g = 0; g < n; g += 32) {
        float v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = p[(int64_t)(g + i < n ? g + i : 0) * HID];
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (g + i < n) acc += v[i];
    }
    return acc;
}

// two such sums (p1 over n1 partials, p2 over n2), every load of a 32-partial batch of both in flight
__device__ __forceinline__ void d_sum_parts2(const float *p1, int n1, const float *p2, int n2, float &s1, float &s2) {
    s1 = s2 = 0.0f;
    for (int g = 0; g < max(n1, n2); g += 32) {
        float v1[32], v2[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            v1[i] = p1[(int64_t)(g + i < n1 ? g + i : 0) * HID];
            v2[i] = p2[(int64_t)(g + i < n2 ? g + i : 0) * HID];
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (g + i < n1) s1 += v1[i];
            if (g + i < n2) s2 += v2[i];
        }
    }
}

// Gumbel uniforms of (agent kk, row r) in phase ph: Philox(seed; r, c, 'GUM' + ph, 4 kk + j)
__device__ __forceinline__ void d_gumbel_u(uint64_t seed, uint32_t c, int ph, int kk, int r, float ur[NA]) {
#pragma unroll
    for (int j = 0; j < (NA + 3) / 4; ++j) {
        const uint4 d = gwrng::philox((uint32_t)r, c, gwrng::TAG_GUMBEL + (uint32_t)ph, (uint32_t)(4 * kk + j),
                                      (uint32_t)seed, (uint32_t)(seed >> 32));
        const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * j + i < NA) ur[4 * j + i] = gwrng::unit(w[i]);
    }
}

// GumbelSoftmax (tau 1) of logits with uniforms ur: gw_gumbel_softmax's op order
__device__ __forceinline__ void d_gumbel(const float lg[NA], const float ur[NA], float pr[NA]) {
    float mx = -INFINITY;
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
}

// z (lane g's 8 features) += the patched cells' terms (in list order): W1 rows row0 + cell.  The
// NPM slots' loads are all issued at once (slots past np re-read slot 0's row and are skipped):
// one round trip, not one per slot
__device__ __forceinline__ void d_add_patches(float z[8], const float *w1, int64_t row0, const int16_t *pc,
                                              const float *pd, int np, int g) {
    float4 a[NPM], b[NPM];
    float dv[NPM];
#pragma unroll
    for (int i = 0; i < NPM; ++i) {
        const int ii = i < np ? i : 0;
        dv[i] = pd[ii];
        const float *wr = w1 + (row0 + pc[ii]) * HID + 8 * g;
        a[i] = *reinterpret_cast<const float4 *>(wr);
        b[i] = *reinterpret_cast<const float4 *>(wr + 4);
    }
#pragma unroll
    for (int i = 0; i < NPM; ++i) {
        if (i < np) {
            z[0] = fmaf(dv[i], a[i].x, z[0]); z[1] = fmaf(dv[i], a[i].y, z[1]);
            z[2] = fmaf(dv[i], a[i].z, z[2]); z[3] = fmaf(dv[i], a[i].w, z[3]);
            z[4] = fmaf(dv[i], b[i].x, z[4]); z[5] = fmaf(dv[i], b[i].y, z[5]);
            z[6] = fmaf(dv[i], b[i].z, z[6]); z[7] = fmaf(dv[i], b[i].w, z[7]);
        }
    }
}

// z += a critic's layer-1 input terms of one row, in order: agent kk = 0 .. K - 1's patched cells
// (W1 rows kk HW + cell, the deltas; d_add_patches per agent), then the 9K action inputs (W1 rows
// K HW + a; round 4's d_add_actions): the same fma order, but NB entries' loads in flight per batch, so ~2
// round trips instead of one per agent plus one per 9 actions (entries past the end re-read a
// valid row and are skipped)
// (sa non-null: the 9K action rows are staged in LDS at sa [9K][HID], so the global batches hold
// only the patched cells and the actions follow from LDS, the same order)
template <int NB>
__device__ __forceinline__ void d_add_critic_in(float z[8], const float *w1, int HW, int K, const int16_t (*pc)[NPM],
                                                const float (*pd)[NPM], const int *np, const float *av, int g,
                                                const float *sa = nullptr) {
    const int na = NA * K;
    int tot = sa ? 0 : na;
    for (int kk = 0; kk < K; ++kk) tot += np[kk];
    int kk = 0, i = 0;
    for (int e0 = 0; e0 < tot; e0 += NB) {
        float4 a[NB], b[NB];
        float dv[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            int64_t row;
            if (kk < K) {
                row = (int64_t)kk * HW + pc[kk][i];
                dv[u] = pd[kk][i];
            } else {
                const int ia = min(i, na - 1);
                row = (int64_t)K * HW + ia;
                dv[u] = av[ia];
            }
            const float *wr = w1 + row * HID + 8 * g;
            a[u] = *reinterpret_cast<const float4 *>(wr);
            b[u] = *reinterpret_cast<const float4 *>(wr + 4);
            ++i;
            if (kk < K && i >= np[kk]) {
                ++kk;
                i = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            if (e0 + u < tot) {
                z[0] = fmaf(dv[u], a[u].x, z[0]); z[1] = fmaf(dv[u], a[u].y, z[1]);
                z[2] = fmaf(dv[u], a[u].z, z[2]); z[3] = fmaf(dv[u], a[u].w, z[3]);
                z[4] = fmaf(dv[u], b[u].x, z[4]); z[5] = fmaf(dv[u], b[u].y, z[5]);
                z[6] = fmaf(dv[u], b[u].z, z[6]); z[7] = fmaf(dv[u], b[u].w, z[7]);
            }
        }
    }
    if (sa) {
        for (int a = 0; a < na; ++a) {
            const float4 x = *reinterpret_cast<const float4 *>(sa + a * HID + 8 * g);
            const float4 y = *reinterpret_cast<const float4 *>(sa + a * HID + 8 * g + 4);
            const float dv = av[a];
            z[0] = fmaf(dv, x.x, z[0]); z[1] = fmaf(dv, x.y, z[1]);
            z[2] = fmaf(dv, x.z, z[2]); z[3] = fmaf(dv, x.w, z[3]);
            z[4] = fmaf(dv, y.x, z[4]); z[5] = fmaf(dv, y.y, z[5]);
            z[6] = fmaf(dv, y.z, z[6]); z[7] = fmaf(dv, y.w, z[7]);
        }
    }
}

// the block's 16 rows through a 128 x 128 layer on all 8 waves of a 512-thread block (wave w:
// columns 16 w .. 16 w + 15; each output the k-ordered f32 fma chain over c = 0 .. 127 from 0, the
// same values as gemv16); every thread calls it, s_z [16][HP] receives z
__device__ __forceinline__ void gemv_all(const float *s_h, const float *__restrict__ w, bool transpose, float *s_z) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15, lq = lane >> 4;
    const int n0 = 16 * wave + lr;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    if (transpose) {  // W^T: k-step 4 t + s takes c = 16 t + 4 lq + s (gemv_t4)
        float4 wv[HID / 16];
#pragma unroll
        for (int t = 0; t < HID / 16; ++t) wv[t] = *reinterpret_cast<const float4 *>(w + n0 * HID + 16 * t + 4 * lq);
#pragma unroll
        for (int t = 0; t < HID / 16; ++t) {
            const float4 a = *reinterpret_cast<const float4 *>(s_h + lr * HP + 16 * t + 4 * lq);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wv[t].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wv[t].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wv[t].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wv[t].w, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) s_z[(4 * lq + i) * HP + n0] = acc[i];
        return;
    }
#pragma unroll
    for (int kk = 0; kk < HID / 4; ++kk) {
        const int c = 4 * kk + lq;
        const float a = s_h[lr * HP + c];
        const float b = transpose ? w[n0 * HID + c] : w[c * HID + n0];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) s_z[(4 * lq + i) * HP + n0] = acc[i];
}

// rows_gemv on all 8 waves: the `own` threads (the row layout's owners) write v and read out
__device__ __forceinline__ void rows_gemv_all(bool own, const float v[8], int rl, int g, const float *w, bool transpose,
                                              float *s_in, float *s_out, float out[8]) {
    if (own) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s_in[rl * HP + 8 * g + i] = v[i];
    }
    __syncthreads();
    gemv_all(s_in, w, transpose, s_out);
    __syncthreads();
    if (own) {
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = s_out[rl * HP + 8 * g + i];
    }
}

// after layer 1: LN -> ReLU -> the 128 x 128 layer (this group's 4 waves) -> LN -> ReLU -> nout outputs
__device__ __forceinline__ void d_fwd_rest(float z[8], const Mlp &m, int nout, int rl, int g, float *s_in,
                                           float *s_out, RowFwd &f, float out[NA]) {
    ln_relu(z, m.lw1, m.lb1, g, f.xh1, f.y1, f.rs1);
    rows_gemv(f.y1, rl, g, m.w2, false, s_in, s_out, z);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] += m.b2[8 * g + i];
    ln_relu(z, m.lw2, m.lb2, g, f.xh2, f.y2, f.rs2);
    for (int a = 0; a < nout; ++a) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = fmaf(f.y2[i], m.w3[(8 * g + i) * nout + a], s);
        out[a] = row_sum(s) + m.b3[a];
    }
}

// a network's small parameters staged in LDS (one slot per network of a tail block): ln1 w / b,
// b2, ln2 w / b, W3, b3 -- loaded once at the block's start, under the prologue's descriptor round
// trips, instead of a dependent global round trip at every LayerNorm and head
constexpr int PSLOT = 5 * HID + HID * NA + NA + 3;  // floats per slot (rounded to 16 bytes)
__device__ __forceinline__ int stage_size(int out) { return 5 * HID + HID * out + out; }
__device__ __forceinline__ float stage_src(const Mlp &m, int out, int o) {
    if (o < 5 * HID) {
        const int v = o / HID, j = o % HID;
        const float *src = v == 0 ? m.lw1 : v == 1 ? m.lb1 : v == 2 ? m.b2 : v == 3 ? m.lw2 : m.lb2;
        return src[j];
    }
    o -= 5 * HID;
    return o < HID * out ? m.w3[o] : m.b3[o - HID * out];
}
// m with its small parameters read from slot sp (W1 and W2 stay in global memory)
__device__ __forceinline__ Mlp staged(Mlp m, const float *sp, int out) {
    m.lw1 = sp;
    m.lb1 = sp + HID;
    m.b2 = sp + 2 * HID;
    m.lw2 = sp + 3 * HID;
    m.lb2 = sp + 4 * HID;
    m.w3 = sp + 5 * HID;
    m.b3 = sp + 5 * HID + HID * out;
    return m;
}

// a network's small parameters as segments of 32 float4 (segment s < 5: ln1 w, ln1 b, b2, ln2 w,
// ln2 b; 5 .. 5 + out - 1: W3's 128-float rows of 4-output groups... i.e. W3 in 128-float pieces)
// into its slot at s * 128 (b3 apart: stage_b3).  Every source piece is 16-byte aligned (the flat
// buffer's [K][128] and [K][128][out] views).
__device__ __forceinline__ int stage_segs(int out) { return 5 + out; }
__device__ __forceinline__ const float4 *stage_seg_src(const Mlp &m, int sg, int lane) {
    const float *src = sg == 0 ? m.lw1 : sg == 1 ? m.lb1 : sg == 2 ? m.b2 : sg == 3 ? m.lw2 : sg == 4 ? m.lb2
                                                                              : m.w3 + (sg - 5) * HID;
    return reinterpret_cast<const float4 *>(src) + lane;
}

// GW_LEARN_STAMP=<file> (diagnostics): each block's thread 0 writes wall_clock64() stamps at its
// phase boundaries into slots [block][0..14] (slot 15: the block type); the host appends them to <file>
constexpr int NSTAMP = 16;
#define DSTAMP_T(P, i, T)                                                                              \
    do {                                                                                               \
        if ((P).stamp && threadIdx.x == (T))                                                           \
            (P).stamp[(int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * NSTAMP + (i)] = wall_clock64(); \
    } while (0)
#define DSTAMP(P, i) DSTAMP_T(P, i, 0)

struct DTail {
    unsigned long long *stamp;
    DQ q;
    DWs w;
    gw_mlp_actors at, ct, c, a;  // actor target, critic target, critic, actor
    uint64_t seed;
    const int32_t *ctr;          // the draws' counter: the critic optimizer's step count
    const int32_t *count;        // the optimizer count this phase snapshots (critic / actor)
    double lr, beta1, beta2;     //   and that optimizer's hyper-parameters (its Adam scalars)
    float gamma;
    int K, B, NG;
};

// this update's step count of the phase's optimizer and its Adam scalars in torch's double forms
// (lr / (1 - beta1^s), sqrt(1 - beta2^s)), once per update for every gradient block (one thread
// of a tail block, on a wave the prologue leaves light)
__device__ __forceinline__ void d_snapshot(const DTail &p, int phase) {
    const int32_t s = p.count[0] + 1;
    p.w.snap[phase] = s;
    p.w.adsc[2 * phase] = (float)(p.lr / (1.0 - pow(p.beta1, (double)s)));
    p.w.adsc[2 * phase + 1] = (float)sqrt(1.0 - pow(p.beta2, (double)s));
}

__global__ void __launch_bounds__(DT) dcritic_tail(DTail p) {
    __shared__ __attribute__((aligned(16))) float s_in[2][RB * HP];
    __shared__ __attribute__((aligned(16))) float s_out[2][RB * HP];
    __shared__ int16_t s_pc[2][RB][MAXK][NPM];
    __shared__ float s_pd[2][RB][MAXK][NPM];
    __shared__ int s_np[2][RB][MAXK];
    __shared__ float s_act[RB][NA * MAXK], s_tact[RB][NA * MAXK];
    __shared__ float s_c1[MAXK + 2][HID];
    __shared__ float s_y[RB], s_rw[RB], s_t1[RB];
    __shared__ __attribute__((aligned(16))) float s_par[MAXK + 2][PSLOT];  // target actors, critic target, critic
    const int k = blockIdx.y, tid = threadIdx.x, grp = tid >> 8, lt = tid & 255, rl = lt >> 4, g = lt & 15;
    const int K = p.K, B = p.B, HW = p.q.HW, r0 = blockIdx.x * RB, r = r0 + rl;
    const int64_t E = p.q.E;
    const int in_c = K * HW + NA * K;
    const bool rec = k == 0;  // the k = 0 blocks record the rows for the later launches
    DSTAMP(p, 0);
    // prologue: every independent load first (the ring's step count, this thread's share of the
    // small parameters), then the roles -- waves 0-3 the rows' descriptors, waves 4-7 the stored
    // probabilities, rewards and c1 sums -- whose round trips overlap; the parameters reach LDS last
    const int64_t t_now = p.q.t_dev[0];
    const uint32_t c = (uint32_t)p.ctr[0];
    // the small parameters: float4 units of 32-unit segments (stage_segs), K target actors then
    // the critic target and the critic, by the threads past the descriptor decoders' waves (whose
    // chain is the prologue's longest); loads first, stores at the end of the prologue
    // when they fit in the slots K + 2 .. MAXK + 1 (K <= 3), the two critics' 9K action rows of W1
    // follow as segments too (critic target then critic, [9K][HID] each), so the critics' layer-1
    // sums read only the patched cells from global memory
    const int sa = stage_segs(NA), sc1 = stage_segs(1), nseg_net = K * sa + 2 * sc1;
    const bool arow = 2 * NA * K * HID <= (MAXK - K) * PSLOT;
    const int nseg = nseg_net + (arow ? 2 * NA * K : 0), nunit = 32 * nseg;
    float *const s_arow = &s_par[0][0] + (size_t)(K + 2) * PSLOT;
    auto unit_net = [&](int v, int &net, int &sg) {
        const int g = v >> 5;
        if (g < K * sa) {
            net = g / sa;
            sg = g - net * sa;
        } else {
            net = K + (g - K * sa) / sc1;
            sg = (g - K * sa) - (net - K) * sc1;
        }
    };
    auto unit_src = [&](int v) -> const float4 * {
        const int gs = v >> 5;
        if (gs >= nseg_net) {  // action row a of critic target (ar < 9K) or critic
            const int ar = gs - nseg_net, a = ar % (NA * K);
            const float *w1 = (ar < NA * K ? p.ct : p.c).w1 + ((int64_t)k * in_c + (int64_t)K * HW + a) * HID;
            return reinterpret_cast<const float4 *>(w1) + (v & 31);
        }
        int net, sg;
        unit_net(v, net, sg);
        const Mlp m = net < K ? mlp_k(p.at, net, HW, NA) : mlp_k(net == K ? p.ct : p.c, k, in_c, 1);
        return stage_seg_src(m, sg, v & 31);
    };
    auto unit_dst = [&](int v) -> float4 * {
        const int gs = v >> 5;
        if (gs >= nseg_net) return reinterpret_cast<float4 *>(s_arow + (gs - nseg_net) * HID) + (v & 31);
        int net, sg;
        unit_net(v, net, sg);
        return reinterpret_cast<float4 *>(&s_par[net][sg * HID]) + (v & 31);
    };
    const int nsd = (RB * 2 * K + 63) / 64 * 64, sid = tid - nsd, sstride = DT - nsd;
    constexpr int NSV = 6;
    float4 sv[NSV];
#pragma unroll
    for (int u = 0; u < NSV; ++u) {
        const int v = sid + u * sstride;
        sv[u] = (sid >= 0 && v < nunit) ? *unit_src(v) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    // b3 (out floats per network, not 16-byte aligned): the last threads
    float b3v = 0.0f;
    const int nb3 = K * NA + 2, tb3 = tid - (DT - nb3);
    if (tb3 >= 0) {
        b3v = tb3 < K * NA ? p.at.b3[(tb3 / NA) * NA + tb3 % NA] : (tb3 == K * NA ? p.ct.b3[k] : p.c.b3[k]);
    }
    if (tid < 256) {
        // the rows' descriptors -> patched cells: one thread per (row, state | next state, agent obs)
        if (tid < RB * 2 * K) {
            const int rr = tid / (2 * K), which = (tid / K) & 1, kk = tid % K;
            int64_t tr, e;
            d_draw(p.q, t_now, p.seed, c, r0 + rr, tr, e);
            const int64_t nx = (tr + 1) % p.q.S;
            const bool dn = p.q.done[tr * E + e] != 0;
            const uint4 *d4 = reinterpret_cast<const uint4 *>(p.q.desc + ((which == 0 ? tr : nx) * E + e) * NDW);
            const uint4 a0 = d4[0], a1 = d4[1], a2 = d4[2];
            const uint32_t d[NDW] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a2.z, a2.w};
            const float apple_map = p.q.apples[kk] >= 0 ? p.q.base[p.q.apples[kk]] : 0.0f;
            int oc[NPM];
            float od[NPM];
            const int m = d_patches(p.q, d, which == 0 ? 0 : (dn ? 1 : 0), kk, apple_map, oc, od);
            s_np[which][rr][kk] = m;
            const int64_t ro = ((int64_t)(which * K + kk) * B + r0 + rr);
            for (int i = 0; i < m; ++i) {
                s_pc[which][rr][kk][i] = (int16_t)oc[i];
                s_pd[which][rr][kk][i] = od[i];
                if (rec) {
                    p.w.pc[ro * NPM + i] = oc[i];
                    p.w.pd[ro * NPM + i] = od[i];
                }
            }
            if (rec) {
                p.w.np[ro] = m;
                if (which == 0 && kk == 0) {
                    p.w.idx[2 * (r0 + rr)] = (int32_t)tr;
                    p.w.idx[2 * (r0 + rr) + 1] = (int32_t)e;
                }
            }
        }
        DSTAMP(p, 11);
    } else {
        const int t2 = tid - 256;
        // c1 of the networks this block runs: the K target actors, critic target k, critic k
        // (two sums per pass: both sums' partial loads in flight together)
        auto c1_src = [&](int o, const float *&pp, int &n, float &b) {
            const int net = o / HID, j = o % HID;
            if (net < K) {
                pp = p.w.cpart[1] + (int64_t)net * p.NG * HID + j;
                n = p.NG;
                b = p.at.b1[net * HID + j];
            } else {
                pp = p.w.cpart[net == K ? 3 : 2] + (int64_t)k * K * p.NG * HID + j;
                n = K * p.NG;
                b = (net == K ? p.ct.b1 : p.c.b1)[k * HID + j];
            }
        };
        for (int o = t2; o < (K + 2) * HID; o += 512) {
            const int o2 = o + 256, ok2 = o2 < (K + 2) * HID;
            const float *p1, *p2;
            int n1, n2;
            float b1v, b2v;
            c1_src(o, p1, n1, b1v);
            c1_src(ok2 ? o2 : o, p2, n2, b2v);
            float v1, v2;
            d_sum_parts2(p1, n1, p2, n2, v1, v2);
            s_c1[o / HID][o % HID] = b1v + v1;
            if (ok2) s_c1[o2 / HID][o2 % HID] = b2v + v2;
        }
        DSTAMP_T(p, 12, 256);
        // the stored action probabilities of every agent (the critic's action inputs) and agent k's
        // reward and termination (the TD target): every draw, then every load, then the stores
        constexpr int NPR = (RB * NA * MAXK + 255) / 256;
        const int npr = RB * NA * K;
        float pv[NPR];
#pragma unroll
        for (int u = 0; u < NPR; ++u) {
            const int o = min(t2 + 256 * u, npr - 1), rr = o / (NA * K), a = o % (NA * K);
            int64_t tr, e;
            if (t2 + 256 * u < npr || u == 0) d_draw(p.q, t_now, p.seed, c, r0 + rr, tr, e);
            else tr = e = 0;
            pv[u] = p.q.probs[((tr * K + a / NA) * E + e) * NA + a % NA];
        }
        const int rrw = max(t2 - (256 - RB), 0);
        int64_t trw, ew;
        d_draw(p.q, t_now, p.seed, c, r0 + rrw, trw, ew);
        const float rw = (float)p.q.reward[(trw * E + ew) * K + k];
        const float t1 = 1.0f - (float)p.q.term[(trw * E + ew) * K + k];
#pragma unroll
        for (int u = 0; u < NPR; ++u) {
            const int o = t2 + 256 * u;
            if (o < npr) {
                s_act[o / (NA * K)][o % (NA * K)] = pv[u];
                if (rec) p.w.act[(int64_t)(r0 + o / (NA * K)) * NA * K + o % (NA * K)] = pv[u];
            }
        }
        if (t2 >= 256 - RB) {
            s_rw[rrw] = rw;
            s_t1[rrw] = t1;
            p.w.rw[(int64_t)k * B + r0 + rrw] = rw;
            p.w.t1[(int64_t)k * B + r0 + rrw] = t1;
        }
        DSTAMP_T(p, 13, 256);
    }
#pragma unroll
    for (int u = 0; u < NSV; ++u) {
        const int v = sid + u * sstride;
        if (sid >= 0 && v < nunit) *unit_dst(v) = sv[u];
    }
    if (sid >= 0)
        for (int v = sid + NSV * sstride; v < nunit; v += sstride) *unit_dst(v) = *unit_src(v);
    if (tb3 >= 0) {
        if (tb3 < K * NA)
            s_par[tb3 / NA][5 * HID + HID * NA + tb3 % NA] = b3v;
        else
            s_par[K + (tb3 - K * NA)][5 * HID + HID] = b3v;
    }
    DSTAMP(p, 14);
    if (blockIdx.x == 0 && k == 0 && tid == 255) d_snapshot(p, 0);
    __syncthreads();
    DSTAMP(p, 1);
    // the target actions a'_kk = GumbelSoftmax(actor_target_kk(s'_kk)), two agents at a time (a
    // group without an agent in the last round recomputes agent K - 1 and discards it)
    for (int rd = 0; rd < (K + 1) / 2; ++rd) {
        const int kk = 2 * rd + grp, kx = kk < K ? kk : K - 1;
        const Mlp m = staged(mlp_k(p.at, kx, HW, NA), s_par[kx], NA);
        float z[8], out[NA];
        RowFwd f;
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = s_c1[kx][8 * g + i];
        d_add_patches(z, m.w1, 0, s_pc[1][rl][kx], s_pd[1][rl][kx], s_np[1][rl][kx], g);
        if (rd == 0) DSTAMP(p, 6);
        d_fwd_rest(z, m, NA, rl, g, s_in[grp], s_out[grp], f, out);
        if (rd == 0) DSTAMP(p, 7);
        if (kk < K) {
            float ur[NA], pr[NA];
            d_gumbel_u(p.seed, c, 0, kk, r, ur);
            d_gumbel(out, ur, pr);
            if (rd == 0) DSTAMP(p, 8);
            if (g == 0) {
#pragma unroll
                for (int a = 0; a < NA; ++a) s_tact[rl][NA * kk + a] = pr[a];
                if (rec) {
#pragma unroll
                    for (int a = 0; a < NA; ++a) {
                        p.w.tact[(int64_t)r * NA * K + NA * kk + a] = pr[a];
                        p.w.u[((int64_t)kk * B + r) * NA + a] = ur[a];
                    }
                }
            }
        }
    }
    __syncthreads();
    DSTAMP(p, 2);
    // group 0: the target critic on (s', a'); group 1: the online critic on (s, a)
    RowFwd f;
    float out[NA];
    {
        const bool tgt = grp == 0;
        const Mlp m = staged(mlp_k(tgt ? p.ct : p.c, k, in_c, 1), s_par[tgt ? K : K + 1], 1);
        const int which = tgt ? 1 : 0;
        float z[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = s_c1[tgt ? K : K + 1][8 * g + i];
        d_add_critic_in<16>(z, m.w1, HW, K, s_pc[which][rl], s_pd[which][rl], s_np[which][rl], tgt ? s_tact[rl] : s_act[rl], g,
                            arow ? s_arow + (tgt ? 0 : NA * K * HID) : nullptr);
        DSTAMP(p, 9);
        d_fwd_rest(z, m, 1, rl, g, s_in[grp], s_out[grp], f, out);
        DSTAMP(p, 10);
    }
    // y = f32(r) + ((1 - d) * gamma) * q_next (gw_td_target's op order)
    if (grp == 0 && g == 0) s_y[rl] = s_rw[rl] + (s_t1[rl] * p.gamma) * out[0];
    __syncthreads();
    DSTAMP(p, 3);
    const Mlp m = staged(mlp_k(p.c, k, in_c, 1), s_par[K + 1], 1);
    float gy[8], gv1[8], dz1[8], gv2[8], dz2[8], dq = 0.0f, diff = 0.0f;
    if (grp == 1) {
        diff = out[0] - s_y[rl];
        dq = (1.0f / (float)B) * (2.0f * diff);  // MSELoss backward (gw_mean_loss_bwd's order)
#pragma unroll
        for (int i = 0; i < 8; ++i) gy[i] = dq * m.w3[8 * g + i];
        ln_relu_bwd(gy, f.y2, f.xh2, f.rs2, m.lw2, g, gv2, dz2);
#pragma unroll
        for (int i = 0; i < 8; ++i) s_in[1][rl * HP + 8 * g + i] = dz2[i];
    }
    __syncthreads();
    gemv_all(s_in[1], m.w2, true, s_out[1]);
    __syncthreads();
    DSTAMP(p, 4);
    if (grp == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) gy[i] = s_out[1][rl * HP + 8 * g + i];
        ln_relu_bwd(gy, f.y1, f.xh1, f.rs1, m.lw1, g, gv1, dz1);
        const Saved &sv = p.w.sv;
        put8(sv.h1, K, B, k, r, g, f.y1);
        put8(sv.h2, K, B, k, r, g, f.y2);
        put8(sv.xh1, K, B, k, r, g, f.xh1);
        put8(sv.xh2, K, B, k, r, g, f.xh2);
        put8(sv.gv1, K, B, k, r, g, gv1);
        put8(sv.gv2, K, B, k, r, g, gv2);
        put8(sv.dz1, K, B, k, r, g, dz1);
        put8(sv.dz2, K, B, k, r, g, dz2);
        if (g == 0) {
            sv.g3[(int64_t)k * B + r] = dq;
            sv.aux[(int64_t)k * B + r] = diff * diff;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s_in[1][rl * HP + 8 * g + i] = dz1[i];
    }
    DSTAMP(p, 5);
}

__global__ void __launch_bounds__(DT) dactor_tail(DTail p) {
    __shared__ __attribute__((aligned(16))) float s_in[RB * HP];
    __shared__ __attribute__((aligned(16))) float s_out[RB * HP];
    __shared__ int16_t s_pc[RB][MAXK][NPM];
    __shared__ float s_pd[RB][MAXK][NPM];
    __shared__ int s_np[RB][MAXK];
    __shared__ float s_act[RB][NA * MAXK];
    __shared__ float s_c1[2][HID];
    __shared__ __attribute__((aligned(16))) float s_par[2][PSLOT];  // actor k, critic k
    __shared__ __attribute__((aligned(16))) float s_wa[NA * MAXK][HID];  // critic k's W1 action rows (all agents)
    const int k = blockIdx.y, tid = threadIdx.x, grp = tid >> 8, lt = tid & 255, rl = lt >> 4, g = lt & 15;
    const int K = p.K, B = p.B, HW = p.q.HW, r0 = blockIdx.x * RB, r = r0 + rl;
    const int in_c = K * HW + NA * K;
    const bool own = grp == 0;  // the row layout's owners; group 1 joins the 128 x 128 layers
    DSTAMP(p, 0);
    // prologue: this thread's share of the small parameters (loads issued first), the c1 sums and
    // the recorded rows (their round trips overlap), then the parameters into LDS
    const int na_ = stage_size(NA), nc_ = stage_size(1), tot = na_ + nc_;
    // the 9K action rows (contiguous, 16-byte aligned: HID | 4), as float4s, loads first
    const float4 *wa = reinterpret_cast<const float4 *>(p.c.w1 + ((int64_t)k * in_c + (int64_t)K * HW) * HID);
    const int nwa = NA * K * HID / 4;
    constexpr int NWA = (NA * MAXK * HID / 4 + DT - 1) / DT;
    float4 wv[NWA];
#pragma unroll
    for (int u = 0; u < NWA; ++u) wv[u] = wa[min(tid + u * DT, nwa - 1)];
    auto par_src = [&](int o) -> float {
        return o < na_ ? stage_src(mlp_k(p.a, k, HW, NA), NA, o) : stage_src(mlp_k(p.c, k, in_c, 1), 1, o - na_);
    };
    auto par_dst = [&](int o) -> float * { return o < na_ ? &s_par[0][o] : &s_par[1][o - na_]; };
    constexpr int NSV = 8;
    float sv[NSV];
#pragma unroll
    for (int u = 0; u < NSV; ++u) {
        const int o = tid + u * DT;
        sv[u] = o < tot ? par_src(o) : 0.0f;
    }
    const uint32_t c = (uint32_t)p.ctr[0];  // the critic's count, advanced by the critic's step
    if (tid < 2 * HID) {
        const int net = tid / HID, j = tid % HID;
        s_c1[net][j] = net == 0 ? p.a.b1[k * HID + j] + d_sum_parts(p.w.cpart[0] + (int64_t)k * p.NG * HID + j, p.NG)
                                : p.c.b1[k * HID + j] +
                                      d_sum_parts(p.w.cpart[2] + (int64_t)k * K * p.NG * HID + j, K * p.NG);
    } else {
        const int t2 = tid - 2 * HID;
        for (int o = t2; o < RB * K * NPM; o += DT - 2 * HID) {  // the rows' states (recorded by the critic tail)
            const int rr = o / (K * NPM), kk = (o / NPM) % K, i = o % NPM;
            const int64_t ro = (int64_t)kk * B + r0 + rr;
            const int n = p.w.np[ro];
            if (i == 0) s_np[rr][kk] = n;
            if (i < n) {
                s_pc[rr][kk][i] = (int16_t)p.w.pc[ro * NPM + i];
                s_pd[rr][kk][i] = p.w.pd[ro * NPM + i];
            }
        }
        for (int o = t2; o < RB * NA * K; o += DT - 2 * HID)
            s_act[o / (NA * K)][o % (NA * K)] = p.w.act[(int64_t)r0 * NA * K + o];
    }
#pragma unroll
    for (int u = 0; u < NSV; ++u) {
        const int o = tid + u * DT;
        if (o < tot) *par_dst(o) = sv[u];
    }
    for (int o = tid + NSV * DT; o < tot; o += DT) *par_dst(o) = par_src(o);
#pragma unroll
    for (int u = 0; u < NWA; ++u)
        if (tid + u * DT < nwa) reinterpret_cast<float4 *>(&s_wa[0][0])[tid + u * DT] = wv[u];
    if (blockIdx.x == 0 && k == 0 && tid == DT - 1) d_snapshot(p, 1);
    __syncthreads();
    DSTAMP(p, 1);
    const Mlp ma = staged(mlp_k(p.a, k, HW, NA), s_par[0], NA);
    const Mlp mc = staged(mlp_k(p.c, k, in_c, 1), s_par[1], 1);
    RowFwd fa, fc;
    float z[8], pr[NA];
    // the actor's forward and its GumbelSoftmax sample
    if (own) {
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = s_c1[0][8 * g + i];
        d_add_patches(z, ma.w1, 0, s_pc[rl][k], s_pd[rl][k], s_np[rl][k], g);
        ln_relu(z, ma.lw1, ma.lb1, g, fa.xh1, fa.y1, fa.rs1);
    }
    rows_gemv_all(own, fa.y1, rl, g, ma.w2, false, s_in, s_out, z);
    DSTAMP(p, 2);
    if (own) {
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] += ma.b2[8 * g + i];
        ln_relu(z, ma.lw2, ma.lb2, g, fa.xh2, fa.y2, fa.rs2);
        float lg[NA], ur[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            float s = 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) s = fmaf(fa.y2[i], ma.w3[(8 * g + i) * NA + a], s);
            lg[a] = row_sum(s) + ma.b3[a];
        }
        DSTAMP(p, 6);
        d_gumbel_u(p.seed, c, 1, k, r, ur);
        d_gumbel(lg, ur, pr);
        DSTAMP(p, 7);
        if (g == 0) {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                p.w.probs[((int64_t)k * B + r) * NA + a] = pr[a];
                p.w.u[((int64_t)(K + k) * B + r) * NA + a] = ur[a];
                s_act[rl][NA * k + a] = pr[a];  // the row's 16 lanes are one wave: LDS in order
            }
        }
        // the stepped critic k on the mixed actions
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = s_c1[1][8 * g + i];
        DSTAMP(p, 8);
        d_add_critic_in<16>(z, mc.w1, HW, K, s_pc[rl], s_pd[rl], s_np[rl], s_act[rl], g, &s_wa[0][0]);
        DSTAMP(p, 9);
        ln_relu(z, mc.lw1, mc.lb1, g, fc.xh1, fc.y1, fc.rs1);
    }
    rows_gemv_all(own, fc.y1, rl, g, mc.w2, false, s_in, s_out, z);
    DSTAMP(p, 3);
    float q = 0.0f, gy[8], gv1[8], dz1[8], gv2[8], dz2[8];
    const float dq = -(1.0f / (float)B);  // -mean Q backward (gw_mean_loss_bwd mode 1)
    if (own) {
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] += mc.b2[8 * g + i];
        ln_relu(z, mc.lw2, mc.lb2, g, fc.xh2, fc.y2, fc.rs2);
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = fmaf(fc.y2[i], mc.w3[8 * g + i], s);
        q = row_sum(s) + mc.b3[0];
#pragma unroll
        for (int i = 0; i < 8; ++i) gy[i] = dq * mc.w3[8 * g + i];
        ln_relu_bwd(gy, fc.y2, fc.xh2, fc.rs2, mc.lw2, g, gv2, dz2);
    }
    DSTAMP(p, 10);
    rows_gemv_all(own, dz2, rl, g, mc.w2, true, s_in, s_out, gy);
    DSTAMP(p, 11);
    float dl[NA];
    if (own) {
        ln_relu_bwd(gy, fc.y1, fc.xh1, fc.rs1, mc.lw1, g, gv1, dz1);
        // d probs_k = dz1 . W1[the agent's action rows]^T, then the softmax backward (tau 1)
        float dp[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const float *wr = s_wa[NA * k + a] + 8 * g;
            float s = 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) s = fmaf(dz1[i], wr[i], s);
            dp[a] = row_sum(s);
        }
        float dot = 0.0f;
#pragma unroll
        for (int a = 0; a < NA; ++a) dot = fmaf(pr[a], dp[a], dot);
#pragma unroll
        for (int a = 0; a < NA; ++a) dl[a] = pr[a] * (dp[a] - dot);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float s = 0.0f;
#pragma unroll
            for (int a = 0; a < NA; ++a) s = fmaf(dl[a], ma.w3[(8 * g + i) * NA + a], s);
            gy[i] = s;
        }
        ln_relu_bwd(gy, fa.y2, fa.xh2, fa.rs2, ma.lw2, g, gv2, dz2);
    }
    DSTAMP(p, 4);
    rows_gemv_all(own, dz2, rl, g, ma.w2, true, s_in, s_out, gy);
    if (own) {
        ln_relu_bwd(gy, fa.y1, fa.xh1, fa.rs1, ma.lw1, g, gv1, dz1);
        const Saved &sv = p.w.sv;
        put8(sv.h1, K, B, k, r, g, fa.y1);
        put8(sv.h2, K, B, k, r, g, fa.y2);
        put8(sv.xh1, K, B, k, r, g, fa.xh1);
        put8(sv.xh2, K, B, k, r, g, fa.xh2);
        put8(sv.gv1, K, B, k, r, g, gv1);
        put8(sv.gv2, K, B, k, r, g, gv2);
        put8(sv.dz1, K, B, k, r, g, dz1);
        put8(sv.dz2, K, B, k, r, g, dz2);
        if (g == 0) {
#pragma unroll
            for (int a = 0; a < NA; ++a) sv.g3[((int64_t)k * B + r) * NA + a] = dl[a];
            sv.aux[(int64_t)k * B + r] = q;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s_in[rl * HP + 8 * g + i] = dz1[i];
    }
    DSTAMP(p, 5);
}

// ---- the parameter gradients with each element's Adam step ------------------------------------
struct DGrad {
    unsigned long long *stamp;
    DWs w;
    const float *base;
    gw_mlp_actors net;           // the network stepped (critic: phase 0, actor: phase 1)
    float *p0, *g0, *m0, *v0;    // its flat parameter / gradient / exp_avg / exp_avg_sq buffers
    float *t0;                   // phase 1: the actor target's flat buffer (soft update)
    gw_mlp_actors cnet;          // phase 1: the (stepped) critic, for the critic target's soft update
    const float *cp0;
    float *ct0;                  //   its flat buffer and the critic target's
    int64_t cn;                  //   their length
    double lr, beta1, beta2, eps;
    float tau;
    int32_t *count;              // the optimizer's step count (written: this step's)
    float *loss;                 // [K]
    int phase, K, B, HW, NG, nobs, in_dim, out, nrest;
    int start[8];                // first block of each block type (7 types)
    gw_actor_images img;         // phase 1, img.part non-null: the fused actor's workspace parts
};

// ---- the fused actor's workspace parts (actor_ops.hip prep_slices / prep_images layouts) ----------
constexpr int AW2B_U16 = 3 * 8 * 4 * 64 * 8;  // the bf16x3 W2 image per agent, 16-bit halves
constexpr int AW3IMG = 8 * 4 * NA * 4;        // the W3 image per agent (floats)
__device__ __forceinline__ uint32_t a_bf16_bits(float x) {  // round to nearest even (actor_ops bf16_rn_bits)
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
// W2 element (row, col) of agent k: its f32 image entry (w2_slot) and its three bf16x3 halves
// (w2b_slot; the row's place in the K-block order kperm inverted)
__device__ __forceinline__ void a_img_w2(const gw_actor_images &im, int k, int row, int col, float w) {
    const int slot = (((col >> 4) * 8 + (row >> 4)) * 4 + ((row >> 2) & 3)) * 16 + (col & 15);
    im.w2img[(size_t)k * HID * HID + 4 * slot + (row & 3)] = w;
    const int kb = row >> 5, rem = row & 31, qq = (rem & 15) >> 2, j = (rem & 3) + (rem >= 16 ? 4 : 0);
    const int lane = (qq << 4) | (col & 15), m = col >> 4, jp = j >> 1, h = j & 1;
    const uint32_t hi = a_bf16_bits(w);
    float r = w - __uint_as_float(hi << 16);
    const uint32_t mi = a_bf16_bits(r);
    r = r - __uint_as_float(mi << 16);
    const uint32_t lo = a_bf16_bits(r);
    uint16_t *b = static_cast<uint16_t *>(im.w2bimg) + (size_t)k * AW2B_U16;
    const uint32_t bits[3] = {hi, mi, lo};
#pragma unroll
    for (int part = 0; part < 3; ++part) {
        const int wd = jp | (lane << 2) | (kb << 8) | (m << 10) | (part << 13);
        b[2 * wd + h] = (uint16_t)bits[part];
    }
}
// W3 element (j, el) of agent k: its image entry (w3_slot, element j & 3)
__device__ __forceinline__ void a_img_w3(const gw_actor_images &im, int k, int j, int el, float w) {
    im.w3img[(size_t)k * AW3IMG + 4 * (((j >> 4) * 4 + ((j >> 2) & 3)) * NA + el) + (j & 3)] = w;
}

struct AdamSc {
    float step_size, bc2, w1, b2, w2, e;
};

// NB elements' Adam steps with every load issued before the first store (a loop of element-wise
// steps would serialise: its stores may alias the next element's loads).  Every offset must be a
// valid element (callers point unused entries at a used one): the loads are unconditional, only
// the first nv entries are computed into the stores.  soft: also the actor target's soft update at
// the same offsets (ti = the new target values).  adam_load may run well before adam_store (the
// operands do not depend on the gradient).
template <int NB>
struct AdamIn {
    float m[NB], v[NB], p[NB], t[NB];
};
template <int NB>
__device__ __forceinline__ void adam_load(const DGrad &p, const int64_t (&off)[NB], bool soft, AdamIn<NB> &in) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        in.m[i] = p.m0[off[i]];
        in.v[i] = p.v0[off[i]];
        in.p[i] = p.p0[off[i]];
        in.t[i] = soft ? p.t0[off[i]] : 0.0f;
    }
}
template <int NB>
__device__ __forceinline__ void adam_store_m(const DGrad &p, const AdamSc &a, const int64_t (&off)[NB], const float (&gi)[NB],
                                             uint32_t valid, bool soft, const AdamIn<NB> &in, float (&pi)[NB], float (&ti)[NB]) {
    float *__restrict__ P = p.p0;
    float *__restrict__ G = p.g0;
    float *__restrict__ M = p.m0;
    float *__restrict__ V = p.v0;
    float *__restrict__ T = p.t0;
    float mo[NB], vo[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        mo[i] = __fmaf_rn(a.w1, gi[i] - in.m[i], in.m[i]);
        vo[i] = __fmaf_rn(a.w2 * gi[i], gi[i], in.v[i] * a.b2);
        const float denom = sqrtf(vo[i]) / a.bc2 + a.e;
        pi[i] = __fmaf_rn(-a.step_size, mo[i] / denom, in.p[i]);
        ti[i] = soft ? p.tau * pi[i] + (1.0f - p.tau) * in.t[i] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        if ((valid >> i) & 1u) {
            G[off[i]] = gi[i];
            M[off[i]] = mo[i];
            V[off[i]] = vo[i];
            P[off[i]] = pi[i];
            if (soft) T[off[i]] = ti[i];
        }
    }
}
// the first nv entries valid
template <int NB>
__device__ __forceinline__ void adam_store(const DGrad &p, const AdamSc &a, const int64_t (&off)[NB], const float (&gi)[NB],
                                           int nv, bool soft, const AdamIn<NB> &in, float (&pi)[NB], float (&ti)[NB]) {
    adam_store_m(p, a, off, gi, nv >= 32 ? 0xFFFFFFFFu : (1u << nv) - 1u, soft, in, pi, ti);
}
template <int NB>
__device__ __forceinline__ void adam_n(const DGrad &p, const AdamSc &a, const int64_t (&off)[NB], const float (&gi)[NB],
                                       int nv, bool soft, float (&pi)[NB], float (&ti)[NB]) {
    AdamIn<NB> in;
    adam_load(p, off, soft, in);
    adam_store(p, a, off, gi, nv, soft, in, pi, ti);
}

// n4 (<= 16 x 256) float4 of global HID-float rows into LDS rows of HID + 4 floats (bank-spread
// row starts): every load in flight before the first store (d_stage_load may run well before
// d_stage_store)
__device__ __forceinline__ void d_stage_load(float4 (&v)[16], const float *src, int n4) {
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int i = threadIdx.x + u * 256;
        v[u] = s4[i < n4 ? i : 0];  // a clamped index, not a predicated load: v stays in registers
    }
}
__device__ __forceinline__ void d_stage_store(float *dst, const float4 (&v)[16], int n4) {
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    constexpr int R4 = HID / 4;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int i = threadIdx.x + u * 256;
        if (i < n4) d4[(i / R4) * (R4 + 1) + i % R4] = v[u];
    }
}
__device__ __forceinline__ void d_stage_rows(float *dst, const float *src, int n4) {
    float4 v[16];
    d_stage_load(v, src, n4);
    d_stage_store(dst, v, n4);
}

__device__ __forceinline__ void dgrads_body(const DGrad &p) {
    __shared__ float s_base[CG], s_pp[2][4][HID];
    __shared__ __attribute__((aligned(16))) float smem[GRG * HID * NA + GRG * (NA + 1) > RB * (TILE_R + 4) + TILE_R * HID
                                                        ? GRG * HID * NA + GRG * (NA + 1)
                                                        : RB * (TILE_R + 4) + TILE_R * HID];
    // the W1 and action-row blocks: dZ1 of the agent in chunks of DZR rows [DZR][DZP] (the W1
    // blocks' G [CG][HID] replaces it), X [B][XP] / the stored actions [B][9K] in the shared buffer
    constexpr int DZR = 128, XP = CG + 4, DZP = HID + 4;
    __shared__ __attribute__((aligned(16))) float s_dzr[DZR * DZP];
    static_assert(DMAXB * XP <= sizeof(smem) / sizeof(float), "X fits the shared buffer");
    const int tid = threadIdx.x, K = p.K, B = p.B, HW = p.HW, NG = p.NG;
    int b = blockIdx.x, type = 0;
    while (type < 6 && b >= p.start[type + 1]) ++type;
    b -= p.start[type];
    if (p.stamp && tid == 0) p.stamp[(int64_t)blockIdx.x * NSTAMP + NSTAMP - 1] = (unsigned long long)type;
    // this step's Adam scalars and count, as the tail snapshotted them (d_snapshot)
    const float sc_step = p.w.adsc[2 * p.phase], sc_bc2 = p.w.adsc[2 * p.phase + 1];
    if (blockIdx.x == 0 && tid == 0) p.count[0] = p.w.snap[p.phase];
    auto get_sc = [&]() {
        AdamSc sc;
        sc.step_size = sc_step;
        sc.bc2 = sc_bc2;
        sc.w1 = (float)(1.0 - p.beta1);
        sc.b2 = (float)p.beta2;
        sc.w2 = (float)(1.0 - p.beta2);
        sc.e = (float)p.eps;
        return sc;
    };
    const bool soft = p.phase == 1;
    const bool img = p.phase == 1 && p.img.part != nullptr;  // (the actor's workspace parts)
    if (type == 0 || type == 5) {
        // W1 rows of one 64-cell group of one agent obs: type 0 the stepped network (gradient +
        // Adam [+ the actor target's soft update]) for one half of the features (blocks (group,
        // half)), type 5 the critic target's soft update; both leave the group's c1 partials, the
        // cells in four chains (cells q, q + 4, ..) summed in q order (dprime's order)
        const int nob = type == 0 ? p.nobs : K;
        const int jh = type == 0 ? (b & 1) : 0;
        if (type == 0) b >>= 1;
        const int k = b / (nob * NG), ob = (b / NG) % nob, grp = b % NG;
        const int c0 = grp * CG, ncell = min(CG, HW - c0);
        const bool critic = type == 5 || p.phase == 0;
        const int in_dim = type == 5 ? K * HW + NA * K : p.in_dim;
        const int64_t row0 = critic ? (int64_t)ob * HW + c0 : c0;  // W1 input row of cell c0
        if (tid < ncell) s_base[tid] = p.base[c0 + tid];
        // chain q's cells q + 4 u (u < 16): the first ncq(q) exist, the others are clamped to the
        // group's last cell (their loads valid, their results unused)
        auto ncq = [&](int q) { return ncell > q ? (ncell - q + 3) / 4 : 0; };
        auto cell = [&](int q, int u) { return min(q + 4 * u, ncell - 1); };
        auto cpart_out = [&](int which, int64_t gi, int j0, int nj, int v) {
            if (tid < nj)
                p.w.cpart[which][gi * HID + j0 + tid] =
                    ((s_pp[v][0][j0 + tid] + s_pp[v][1][j0 + tid]) + s_pp[v][2][j0 + tid]) + s_pp[v][3][j0 + tid];
        };
        if (type == 5) {  // thread (h, j): chains h and h + 2
            const int j = tid & (HID - 1), h = tid >> 7;
            const float *cw = p.cnet.w1 + ((int64_t)k * in_dim + row0) * HID + j;
            const float *__restrict__ CP = p.cp0;
            float *__restrict__ CT = p.ct0;
            float pv[2][16], tv[2][16];  // both chains' loads in flight, then the stores
#pragma unroll
            for (int ps = 0; ps < 2; ++ps)
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t off = (cw + (int64_t)cell(h + 2 * ps, u) * HID) - p.cp0;
                    pv[ps][u] = CP[off];
                    tv[ps][u] = CT[off];
                }
            __syncthreads();  // s_base
#pragma unroll
            for (int ps = 0; ps < 2; ++ps) {
                const int q = h + 2 * ps, nq = ncq(q);
                float tp = 0.0f;
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int cc = cell(q, u);
                    const float ti = p.tau * pv[ps][u] + (1.0f - p.tau) * tv[ps][u];
                    if (u < nq) {
                        CT[(cw + (int64_t)cc * HID) - p.cp0] = ti;
                        tp = fmaf(s_base[cc], ti, tp);
                    }
                }
                s_pp[1][q][j] = tp;
            }
            __syncthreads();
            cpart_out(3, (int64_t)k * K * NG + ob * NG + grp, 0, HID, 1);
            return;
        }
        // X [B][XP]: the rows' obs values of the group's cells -- the map, then the patched cells
        // (a row's patched cells are distinct: d_patches) -- and G [CG][64] = X^T dZ1 over the rows
        // in order on v_mfma_f32_16x16x4_f32 for this block's 64 features (dZ1 in 128-row chunks
        // through LDS): dense and balanced whatever the cells' patch counts (a cell every row
        // patches -- the own apple, the spawn cells -- walks all B rows like any other).  Issued
        // first, their round trips overlapping: the Adam operands, the rows' patch lists, dZ1.
        const int jl = tid & 63, q = tid >> 6, j = 64 * jh + jl;  // thread: feature j, chain q
        const int nq = ncq(q);
        const float *wk = p.net.w1 + ((int64_t)k * in_dim + row0) * HID + j;
        int64_t off[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) off[u] = (wk + (int64_t)cell(q, u) * HID) - p.p0;
        const int obk = p.phase == 0 ? ob : k;
        const int NE = B * NPM;
        constexpr int PI = (DMAXB * NPM + 255) / 256;  // this thread's items t = tid + 256 i
        int npv[PI], pcv[PI];
        float dv[PI];
#pragma unroll
        for (int i = 0; i < PI; ++i) {
            const int t = min(tid + 256 * i, NE - 1);
            const int64_t ro = (int64_t)obk * B + t / NPM;
            npv[i] = pcv[i] = 0;
            dv[i] = 0.0f;
            if (tid + 256 * i < NE) {  // (block-uniform but for the last pass: no wasted loads)
                npv[i] = p.w.np[ro];
                pcv[i] = p.w.pc[ro * NPM + t % NPM];
                dv[i] = p.w.pd[ro * NPM + t % NPM];
            }
        }
        d_stage_rows(s_dzr, p.w.sv.dz1 + (int64_t)k * B * HID, min(B, DZR) * HID / 4);
        DSTAMP(p, 5);
        AdamIn<16> ain;  // in flight under the X build and the MFMA
        adam_load(p, off, soft, ain);
        float *s_X = smem;
        __syncthreads();  // s_base
        DSTAMP(p, 6);
        {
            const int c = tid % CG;  // 256 = 4 x CG: a thread's map column is fixed
            const float v = c < ncell ? s_base[c] : 0.0f;
            for (int r = tid / CG; r < B; r += 256 / CG) s_X[r * XP + c] = v;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PI; ++i) {
            const int t = tid + 256 * i, c = pcv[i] - c0;
            if (t < NE && t % NPM < npv[i] && c >= 0 && c < ncell) s_X[(t / NPM) * XP + c] = s_base[c] + dv[i];
        }
        DSTAMP(p, 3);
        const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
        f32x4 acc[4];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (int rc = 0; rc < B; rc += DZR) {
            const int nr = min(DZR, B - rc);
            __syncthreads();  // X written / the previous chunk read
            if (rc > 0) {
                d_stage_rows(s_dzr, p.w.sv.dz1 + ((int64_t)k * B + rc) * HID, nr * HID / 4);
                __syncthreads();
            }
            const float *xa = s_X + (int64_t)rc * XP + lr, *zb = s_dzr + 64 * jh + 16 * wave + lr;
            for (int k0 = 0; k0 < nr / 4; k0 += 4)  // nr: a multiple of 16
#pragma unroll
            for (int kk = k0; kk < k0 + 4; ++kk) {
                const int r = 4 * kk + lq;
                const float bv = zb[r * DZP];
#pragma unroll
                for (int ct = 0; ct < 4; ++ct)
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[r * XP + 16 * ct], bv, acc[ct], 0, 0, 0);
            }
        }
        __syncthreads();  // dZ1 read: G replaces it
        float *s_G = s_dzr;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
            for (int i = 0; i < 4; ++i) s_G[(16 * ct + 4 * lq + i) * HID + 64 * jh + 16 * wave + lr] = acc[ct][i];
        __syncthreads();
        DSTAMP(p, 1);
        // Adam over the chain's W1 rows; the c1 partials from the new values
        {
            float gv[16], pv[16], tv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) gv[u] = s_G[cell(q, u) * HID + j];
            adam_store(p, get_sc(), off, gv, nq, soft, ain, pv, tv);
            float pp = 0.0f, tp = 0.0f;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const float bs = s_base[cell(q, u)];
                if (u < nq) {
                    pp = fmaf(bs, pv[u], pp);
                    if (soft) tp = fmaf(bs, tv[u], tp);
                }
            }
            s_pp[0][q][j] = pp;
            s_pp[1][q][j] = tp;
            if (img) {  // the new rows, for the actor workspace's row slices below
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (u < nq) s_G[cell(q, u) * HID + j] = pv[u];
            }
        }
        __syncthreads();
        const int64_t gi = p.phase == 0 ? ((int64_t)k * K * NG + ob * NG + grp) : ((int64_t)k * NG + grp);
        cpart_out(p.phase == 0 ? 2 : 0, gi, 64 * jh, 64, 0);
        if (soft) cpart_out(1, gi, 64 * jh, 64, 1);
        if (img && tid < 128) {  // slices 2 grp, 2 grp + 1: prep_slices' fma chain in row order
            const int sl = tid >> 6, j2 = 64 * jh + (tid & 63);
            if (32 * sl < ncell) {
                float acc = 0.0f;
                for (int i = 0; i < 32; ++i) {
                    const int c = 32 * sl + i;
                    if (c < ncell) acc = fmaf(s_base[c], s_G[c * HID + j2], acc);
                }
                p.img.part[((int64_t)k * p.img.nslices + 2 * grp + sl) * HID + j2] = acc;
            }
        }
        return;
    }
    if (type == 1) {  // the critic's action rows: blocks (agent, 8 rows); sum over the batch rows in order
        const int na = NA * K, QB = (na + 7) / 8, k = b / QB, q = b % QB;
        const int j = tid & (HID - 1), h = tid >> 7;
        const int a0 = 8 * q + h;  // this thread's rows a0, a0 + 2, a0 + 4, a0 + 6 (< na; others clamped)
        int ar[4];
        int64_t off[4];
        int nv = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            ar[u] = min(a0 + 2 * u, na - 1);
            off[u] = (p.net.w1 + ((int64_t)k * p.in_dim + (int64_t)K * HW + ar[u]) * HID + j) - p.p0;
            nv += a0 + 2 * u < na ? 1 : 0;
        }
        float4 zst[16];
        const int n4 = min(B, DZR) * HID / 4;
        d_stage_load(zst, p.w.sv.dz1 + (int64_t)k * B * HID, n4);
        float *s_a = smem;  // the rows' stored actions [B][9K] (<= 256 x 72 floats)
        for (int i0 = 0; i0 < B * na; i0 += 8 * 256) {  // 8 loads in flight, then the stores
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * 256 + tid;
                v[u] = p.w.act[i < B * na ? i : 0];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * 256 + tid;
                if (i < B * na) s_a[i] = v[u];
            }
        }
        d_stage_store(s_dzr, zst, n4);
        DSTAMP(p, 3);
        AdamIn<4> ain;  // in flight under the row loop
        adam_load(p, off, false, ain);
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int rc = 0; rc < B; rc += DZR) {
            const int nr = min(DZR, B - rc);
            if (rc > 0) {
                __syncthreads();  // the previous chunk read
                d_stage_rows(s_dzr, p.w.sv.dz1 + ((int64_t)k * B + rc) * HID, nr * HID / 4);
            }
            __syncthreads();
            DSTAMP(p, 4);
            const float *dz = s_dzr + j;
            for (int r0 = 0; r0 < nr; r0 += 8)
#pragma unroll
            for (int rr = r0; rr < r0 + 8; ++rr) {
                const float d = dz[rr * DZP];
                const float *av = s_a + (rc + rr) * na;
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] = fmaf(av[ar[u]], d, acc[u]);
            }
        }
        DSTAMP(p, 5);
        float pv[4], tv[4];
        adam_store(p, get_sc(), off, acc, nv, false, ain, pv, tv);
        return;
    }
    if (type == 2) {  // W2 = h1^T dz2 (v_mfma_f32_16x16x4_f32, rows in order), 16 inputs per block
        const int k = b / (HID / RB), d0 = (b % (HID / RB)) * RB;
        float (*s_x)[TILE_R + 4] = reinterpret_cast<float (*)[TILE_R + 4]>(smem);      // [input][row]
        float (*s_dz)[HID] = reinterpret_cast<float (*)[HID]>(smem + RB * (TILE_R + 4));  // [row][feature]
        const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
        f32x4 acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
        const int n0 = 32 * wave + lr, n1 = n0 + 16;
        const float *w2 = p.net.w2 + (int64_t)k * HID * HID;
        int64_t off[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = d0 + 4 * lq + i;
            off[2 * i] = (w2 + (int64_t)d * HID + n0) - p.p0;
            off[2 * i + 1] = (w2 + (int64_t)d * HID + n1) - p.p0;
        }
        AdamIn<8> ain;  // the Adam operands' round trip under the tiles' staging
        adam_load(p, off, soft, ain);
        for (int r0 = 0; r0 < B; r0 += TILE_R) {
            const int nr = min(TILE_R, B - r0);
            __syncthreads();
            constexpr int XN = RB * TILE_R / 256, ZN = TILE_R * HID / 4 / 256;
            float xv[XN];
            float4 zv[ZN];
#pragma unroll
            for (int t = 0; t < XN; ++t) {
                const int i = tid + 256 * t, rr = i / RB, d = i % RB;
                xv[t] = rr < nr ? p.w.sv.h1[((int64_t)k * B + r0 + rr) * HID + d0 + d] : 0.0f;
            }
#pragma unroll
            for (int t = 0; t < ZN; ++t) {
                const int i = tid + 256 * t, rr = i / (HID / 4), cq = i % (HID / 4);
                zv[t] = rr < nr ? reinterpret_cast<const float4 *>(p.w.sv.dz2 + ((int64_t)k * B + r0 + rr) * HID)[cq]
                                : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
#pragma unroll
            for (int t = 0; t < XN; ++t) {
                const int i = tid + 256 * t;
                if (i / RB < nr) s_x[i % RB][i / RB] = xv[t];
            }
#pragma unroll
            for (int t = 0; t < ZN; ++t) {
                const int i = tid + 256 * t;
                if (i / (HID / 4) < nr) *reinterpret_cast<float4 *>(&s_dz[i / (HID / 4)][4 * (i % (HID / 4))]) = zv[t];
            }
            __syncthreads();
            for (int kk = 0; kk < nr / 4; ++kk) {
                const int rr = 4 * kk + lq;
                const float a = s_x[lr][rr];
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s_dz[rr][n0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s_dz[rr][n1], acc1, 0, 0, 0);
            }
        }
        float gv[8], pv[8], tv[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            gv[2 * i] = acc0[i];
            gv[2 * i + 1] = acc1[i];
        }
        adam_store(p, get_sc(), off, gv, 8, soft, ain, pv, tv);
        if (img) {
#pragma unroll
            for (int i = 0; i < 8; ++i) a_img_w2(p.img, k, d0 + 4 * lq + (i >> 1), (i & 1) ? n1 : n0, pv[i]);
        }
        return;
    }
    const int rg = tid >> 4, g = tid & 15;
    if (type == 3) {  // b1, ln1 affine, b2, ln2 affine: 16 row groups, combined in group order
        const int k = b;
        const int64_t base = (int64_t)k * B * HID;
        const float *dst[6] = {p.net.b1, p.net.ln1_w, p.net.ln1_b, p.net.b2, p.net.ln2_w, p.net.ln2_b};
        int64_t off[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {  // 6 * 128 = 3 * 256 elements
            const int t = tid + 256 * u;
            off[u] = (dst[t / HID] + k * HID + t % HID) - p.p0;
        }
        AdamIn<3> ain;
        adam_load(p, off, soft, ain);
        float acc[6][8];
#pragma unroll
        for (int v = 0; v < 6; ++v)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[v][i] = 0.0f;
#pragma unroll 2
        for (int r = rg; r < B; r += GRG) {
            const int64_t o = base + (int64_t)r * HID + 8 * g;
            const float *src[6] = {p.w.sv.dz1 + o, p.w.sv.gv1 + o, p.w.sv.xh1 + o, p.w.sv.dz2 + o, p.w.sv.gv2 + o,
                                   p.w.sv.xh2 + o};
            float4 q[6][2];
#pragma unroll
            for (int v = 0; v < 6; ++v) {
                q[v][0] = *reinterpret_cast<const float4 *>(src[v]);
                q[v][1] = *reinterpret_cast<const float4 *>(src[v] + 4);
            }
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int o2 = 3 * hh;
                const float dzv[8] = {q[o2][0].x, q[o2][0].y, q[o2][0].z, q[o2][0].w,
                                      q[o2][1].x, q[o2][1].y, q[o2][1].z, q[o2][1].w};
                const float gvv[8] = {q[o2 + 1][0].x, q[o2 + 1][0].y, q[o2 + 1][0].z, q[o2 + 1][0].w,
                                      q[o2 + 1][1].x, q[o2 + 1][1].y, q[o2 + 1][1].z, q[o2 + 1][1].w};
                const float xhv[8] = {q[o2 + 2][0].x, q[o2 + 2][0].y, q[o2 + 2][0].z, q[o2 + 2][0].w,
                                      q[o2 + 2][1].x, q[o2 + 2][1].y, q[o2 + 2][1].z, q[o2 + 2][1].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    acc[o2][i] += dzv[i];
                    acc[o2 + 1][i] = fmaf(gvv[i], xhv[i], acc[o2 + 1][i]);
                    acc[o2 + 2][i] += gvv[i];
                }
            }
        }
        float (*part)[6][HID] = reinterpret_cast<float (*)[6][HID]>(smem);
#pragma unroll
        for (int v = 0; v < 6; ++v)
#pragma unroll
            for (int i = 0; i < 8; ++i) part[rg][v][8 * g + i] = acc[v][i];
        __syncthreads();
        float gv[3], pv[3], tv[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int t = tid + 256 * u, v = t / HID, j = t % HID;
            float sum = 0.0f;
#pragma unroll
            for (int qq = 0; qq < GRG; ++qq) sum += part[qq][v][j];
            gv[u] = sum;
        }
        adam_store(p, get_sc(), off, gv, 3, soft, ain, pv, tv);
        return;
    }
    if (type == 4) {  // W3 = h2^T g3, b3, the loss
        const int k = b, out = p.out;
        const int64_t base = (int64_t)k * B * HID;
        // slot u < NW3 - 1: W3 element tid + 256 u (when < HID * out); the last slot: b3[tid] (tid < out);
        // unused slots point at b3[0] of agent k
        constexpr int NW3 = (HID * NA + 255) / 256 + 1;
        int64_t off[NW3];
        uint32_t valid = 0;
#pragma unroll
        for (int u = 0; u < NW3; ++u) {
            const int t = tid + 256 * u;
            off[u] = (p.net.b3 + k * out) - p.p0;
            if (u < NW3 - 1 && t < HID * out) {
                off[u] = (p.net.w3 + ((int64_t)k * HID + t / out) * out + t % out) - p.p0;
                valid |= 1u << u;
            }
        }
        if (tid < out) {
            off[NW3 - 1] = (p.net.b3 + k * out + tid) - p.p0;
            valid |= 1u << (NW3 - 1);
        }
        AdamIn<NW3> ain;
        adam_load(p, off, soft, ain);
        float acc[8][NA];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int a = 0; a < NA; ++a) acc[i][a] = 0.0f;
        float bacc[NA], lacc = 0.0f;
#pragma unroll
        for (int a = 0; a < NA; ++a) bacc[a] = 0.0f;
#pragma unroll 4
        for (int r = rg; r < B; r += GRG) {
            const float *hs = p.w.sv.h2 + base + (int64_t)r * HID + 8 * g;
            const float4 h0 = *reinterpret_cast<const float4 *>(hs), h1 = *reinterpret_cast<const float4 *>(hs + 4);
            const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
            const float *gs = p.w.sv.g3 + ((int64_t)k * B + r) * out;
            float gv[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const float x = gs[a < out ? a : 0];  // clamped, not predicated: the loads batch
                gv[a] = a < out ? x : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int a = 0; a < NA; ++a) acc[i][a] = fmaf(hv[i], gv[a], acc[i][a]);
#pragma unroll
            for (int a = 0; a < NA; ++a) bacc[a] += gv[a];
            lacc += p.w.sv.aux[(int64_t)k * B + r];
        }
        float (*part)[HID][NA] = reinterpret_cast<float (*)[HID][NA]>(smem);
        float (*pb)[NA + 1] = reinterpret_cast<float (*)[NA + 1]>(smem + GRG * HID * NA);
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
        {
            float gv[NW3], pv[NW3], tv[NW3];
#pragma unroll
            for (int u = 0; u < NW3 - 1; ++u) {
                const int t = min(tid + 256 * u, HID * out - 1);
                float sum = 0.0f;
#pragma unroll
                for (int qq = 0; qq < GRG; ++qq) sum += part[qq][t / out][t % out];
                gv[u] = sum;
            }
            {
                float sum = 0.0f;
#pragma unroll
                for (int qq = 0; qq < GRG; ++qq) sum += pb[qq][min(tid, out - 1)];
                gv[NW3 - 1] = sum;
            }
            adam_store_m(p, get_sc(), off, gv, valid, soft, ain, pv, tv);
            if (img) {
#pragma unroll
                for (int u = 0; u < NW3 - 1; ++u) {
                    const int t = tid + 256 * u;
                    if (t < HID * out) a_img_w3(p.img, k, t / out, t % out, pv[u]);
                }
            }
        }
        if (tid == 64) {
            float sum = 0.0f;
            for (int qq = 0; qq < GRG; ++qq) sum += pb[qq][NA];
            p.loss[k] = p.phase == 0 ? sum / (float)B : -(sum / (float)B);
        }
        return;
    }
    // type 6: the critic target's soft update outside its W1 state rows (grid-stride)
    const int in_c = K * HW + NA * K;
    const int64_t w1off = p.cnet.w1 - p.cp0;
    const float *__restrict__ CP = p.cp0;
    float *__restrict__ CT = p.ct0;
    const int64_t stride = (int64_t)p.nrest * 256;
    for (int64_t i0 = (int64_t)b * 256 + tid; i0 < p.cn; i0 += 8 * stride) {  // 8 elements' loads in flight
        float pv[8], tv[8];
        bool on[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + u * stride, rel = i - w1off;
            on[u] = i < p.cn && !(rel >= 0 && rel < (int64_t)K * in_c * HID && (rel / HID) % in_c < (int64_t)K * HW);
            if (on[u]) {
                pv[u] = CP[i];
                tv[u] = CT[i];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (on[u]) CT[i0 + u * stride] = p.tau * pv[u] + (1.0f - p.tau) * tv[u];
    }
}

__global__ void __launch_bounds__(256) dgrads_adam(DGrad p) {
    DSTAMP(p, 0);
    dgrads_body(p);
    DSTAMP(p, 2);
}

// the c1 partials of one network from its current W1 (the update's own launches refresh them;
// this primes them, e.g. after a load): blocks (network, agent, obs, 64-cell group)
struct DPrime {
    gw_mlp_actors net[4];  // actor, actor target, critic, critic target
    DWs w;
    const float *base;
    int K, HW, NG;
    int start[5];
};
__global__ void __launch_bounds__(256) dprime(DPrime p) {
    __shared__ float s_base[CG], s_pp[4][HID];
    int b = blockIdx.x, net = 0;
    while (net < 3 && b >= p.start[net + 1]) ++net;
    b -= p.start[net];
    const int K = p.K, HW = p.HW, NG = p.NG, tid = threadIdx.x;
    const bool critic = net >= 2;
    const int nob = critic ? K : 1;
    const int k = b / (nob * NG), ob = (b / NG) % nob, grp = b % NG;
    const int c0 = grp * CG, ncell = min(CG, HW - c0), j = tid & (HID - 1), h = tid >> 7;
    const int in_dim = critic ? K * HW + NA * K : HW;
    if (tid < ncell) s_base[tid] = p.base[c0 + tid];
    __syncthreads();
    const float *wk = p.net[net].w1 + ((int64_t)k * in_dim + (int64_t)ob * HW + c0) * HID + j;
    for (int q = h; q < 4; q += 2) {  // chains q: cells q, q + 4, .. (the update's order)
        float pp = 0.0f;
        for (int cc = q; cc < ncell; cc += 4) pp = fmaf(s_base[cc], wk[(int64_t)cc * HID], pp);
        s_pp[q][j] = pp;
    }
    __syncthreads();
    if (tid < HID) {
        const int64_t gi = critic ? ((int64_t)k * K * NG + ob * NG + grp) : ((int64_t)k * NG + grp);
        p.w.cpart[net][gi * HID + tid] = ((s_pp[0][tid] + s_pp[1][tid]) + s_pp[2][tid]) + s_pp[3][tid];
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

// ---- the descriptor learner's entry points ------------------------------------------------------
namespace {

gw_status dnet_ok(const gw_mlp_actors *n, int K, int in_dim, int out, const gw_adam_buf *opt, const char *who) {
    if (!n) return fail(GW_ERR_ARG, std::string(who) + ": null network");
    gw_status st = check_net(*n, K, in_dim, out, who);
    if (st != GW_OK || !opt) return st;
    const float *ps[10] = {n->w1, n->b1, n->ln1_w, n->ln1_b, n->w2, n->b2, n->ln2_w, n->ln2_b, n->w3, n->b3};
    for (const float *q : ps)
        if (q < opt->param || q >= opt->param + opt->n)
            return fail(GW_ERR_ARG, std::string(who) + ": a parameter outside the optimizer's flat buffer");
    if (!opt->grad || !opt->exp_avg || !opt->exp_avg_sq || !opt->step)
        return fail(GW_ERR_ARG, std::string(who) + ": null optimizer buffer");
    return GW_OK;
}

// GW_LEARN_STAMP=<file>: the four launches' block stamps (DSTAMP), appended to <file> after each
// update as records {int32 launch, int32 blocks, blocks x NSTAMP uint64} (a synchronising diagnostic)
constexpr int STAMP_BLOCKS = 8192;
unsigned long long *stamp_buf() {
    static const char *path = GW_MEASURE_ENV("GW_LEARN_STAMP");
    static unsigned long long *buf = nullptr;
    if (path && *path && !buf && hipMalloc(&buf, sizeof(unsigned long long) * 4 * STAMP_BLOCKS * NSTAMP) != hipSuccess)
        buf = nullptr;
    return buf;
}
void stamp_dump(hipStream_t s, const int (&nb)[4]) {
    unsigned long long *buf = stamp_buf();
    if (!buf || hipStreamSynchronize(s) != hipSuccess) return;
    static std::vector<unsigned long long> h(4 * STAMP_BLOCKS * NSTAMP);
    if (hipMemcpy(h.data(), buf, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    FILE *f = std::fopen(GW_MEASURE_ENV("GW_LEARN_STAMP"), "ab");
    if (!f) return;
    for (int l = 0; l < 4; ++l) {
        const int32_t hd[2] = {l, nb[l]};
        std::fwrite(hd, sizeof(hd), 1, f);
        std::fwrite(h.data() + (size_t)l * STAMP_BLOCKS * NSTAMP, sizeof(unsigned long long), (size_t)nb[l] * NSTAMP, f);
    }
    std::fclose(f);
}

gw_status dsrc_ok(const gw_obs_source *src, int B, const float *ws, const char *who) {
    if (!src || !src->base || !ws) return fail(GW_ERR_ARG, std::string(who) + ": null argument");
    if (src->K < 1 || src->K > MAXK || src->N < src->K || src->N > MAXK)
        return fail(GW_ERR_ARG, std::string(who) + ": K / N out of range");
    if ((int64_t)src->H * src->W < 1 || (int64_t)src->H * src->W > 32767)
        return fail(GW_ERR_ARG, std::string(who) + ": grid size out of range");
    if (B < RB || B % RB || B > DMAXB) return fail(GW_ERR_ARG, std::string(who) + ": B must be a multiple of 16 in [16, 256]");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return fail(GW_ERR_ARG, std::string(who) + ": ws must be 16-byte aligned");
    return GW_OK;
}

}  // namespace

extern "C" {

int64_t gw_maddpg_desc_workspace_floats(int32_t K, int32_t B, int32_t H, int32_t W) {
    if (K < 1 || K > MAXK || B < RB || B % RB || H < 1 || W < 1) return -1;
    return dws_floats(K, B, H * W);
}

gw_status gw_maddpg_desc_prime(const gw_obs_source *src, const gw_mlp_actors *actor, const gw_mlp_actors *actor_target,
                               const gw_mlp_actors *critic, const gw_mlp_actors *critic_target, int32_t B, float *ws,
                               void *stream) {
    const char *who = "gw_maddpg_desc_prime";
    gw_status st = dsrc_ok(src, B, ws, who);
    if (st != GW_OK) return st;
    const int K = src->K, HW = src->H * src->W, in_c = K * HW + NA * K;
    if ((st = dnet_ok(actor, K, HW, NA, nullptr, who)) != GW_OK || (st = dnet_ok(actor_target, K, HW, NA, nullptr, who)) != GW_OK ||
        (st = dnet_ok(critic, K, in_c, 1, nullptr, who)) != GW_OK || (st = dnet_ok(critic_target, K, in_c, 1, nullptr, who)) != GW_OK)
        return st;
    DPrime p{};
    p.net[0] = *actor;
    p.net[1] = *actor_target;
    p.net[2] = *critic;
    p.net[3] = *critic_target;
    p.w = dws_layout(ws, K, B, HW);
    p.base = src->base;
    p.K = K;
    p.HW = HW;
    p.NG = d_ng(HW);
    p.start[0] = 0;
    p.start[1] = K * p.NG;
    p.start[2] = 2 * K * p.NG;
    p.start[3] = p.start[2] + K * K * p.NG;
    p.start[4] = p.start[3] + K * K * p.NG;
    hipLaunchKernelGGL(dprime, dim3(p.start[4]), dim3(256), 0, static_cast<hipStream_t>(stream), p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GW_OK : fail(GW_ERR_HIP, std::string(who) + ": " + hipGetErrorString(e));
}

gw_status gw_maddpg_desc_update(const gw_obs_source *src, const gw_desc_ring *ring, const gw_mlp_actors *actor,
                                const gw_mlp_actors *actor_target, const gw_mlp_actors *critic,
                                const gw_mlp_actors *critic_target, const gw_adam_buf *opt_actor,
                                const gw_adam_buf *opt_critic, float *actor_target_flat, float *critic_target_flat,
                                float gamma, float tau, int32_t B, uint64_t seed, float *ws, float *actor_loss,
                                float *critic_loss, void *prof_env, void *stream) {
    return gw_maddpg_desc_update_img(src, ring, actor, actor_target, critic, critic_target, opt_actor, opt_critic,
                                     actor_target_flat, critic_target_flat, gamma, tau, B, seed, ws, actor_loss,
                                     critic_loss, nullptr, prof_env, stream);
}

gw_status gw_maddpg_desc_update_img(const gw_obs_source *src, const gw_desc_ring *ring, const gw_mlp_actors *actor,
                                    const gw_mlp_actors *actor_target, const gw_mlp_actors *critic,
                                    const gw_mlp_actors *critic_target, const gw_adam_buf *opt_actor,
                                    const gw_adam_buf *opt_critic, float *actor_target_flat, float *critic_target_flat,
                                    float gamma, float tau, int32_t B, uint64_t seed, float *ws, float *actor_loss,
                                    float *critic_loss, const gw_actor_images *img, void *prof_env, void *stream) {
    const char *who = "gw_maddpg_desc_update";
    if (img && (!img->part || !img->w2img || !img->w2bimg || !img->w3img || img->nslices != (src ? (src->H * src->W + 31) / 32 : -1) ||
                (reinterpret_cast<uintptr_t>(img->w2bimg) & 3u)))
        return fail(GW_ERR_ARG, std::string(who) + ": actor images do not match the source's grid");
    gw_status st = dsrc_ok(src, B, ws, who);
    if (st != GW_OK) return st;
    if (!ring || !ring->desc || !ring->probs || !ring->reward || !ring->term || !ring->done || !ring->t_dev ||
        ring->S < 2 || !opt_actor || !opt_critic || !actor_target_flat || !critic_target_flat || !actor_loss ||
        !critic_loss || src->E < 1)
        return fail(GW_ERR_ARG, std::string(who) + ": null argument");
    const int K = src->K, HW = src->H * src->W, in_c = K * HW + NA * K, NG = d_ng(HW);
    if ((st = dnet_ok(actor, K, HW, NA, opt_actor, who)) != GW_OK || (st = dnet_ok(actor_target, K, HW, NA, nullptr, who)) != GW_OK ||
        (st = dnet_ok(critic, K, in_c, 1, opt_critic, who)) != GW_OK ||
        (st = dnet_ok(critic_target, K, in_c, 1, nullptr, who)) != GW_OK)
        return st;
    if (actor_target->w1 - actor_target_flat != actor->w1 - opt_actor->param ||
        critic_target->w1 - critic_target_flat != critic->w1 - opt_critic->param)
        return fail(GW_ERR_ARG, std::string(who) + ": target flat buffers must share the online layout");
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the four launches are one GW_SPAN_LEARN span of prof_env's gw_profile (when it profiles)
    gwprof::Span span(prof_env, GW_SPAN_LEARN);
    DQ q{};
    q.desc = ring->desc;
    q.probs = ring->probs;
    q.reward = ring->reward;
    q.term = ring->term;
    q.done = ring->done;
    q.t_dev = ring->t_dev;
    q.S = ring->S;
    q.E = src->E;
    q.base = src->base;
    for (int k = 0; k < MAXK; ++k) q.apples[k] = src->apples[k];
    q.N = src->N;
    q.K = K;
    q.HW = HW;
    q.variant = src->variant;
    DTail t{};
    t.q = q;
    t.w = dws_layout(ws, K, B, HW);
    t.at = *actor_target;
    t.ct = *critic_target;
    t.c = *critic;
    t.a = *actor;
    t.seed = seed;
    t.ctr = opt_critic->step;
    t.count = opt_critic->step;
    t.lr = opt_critic->lr;
    t.beta1 = opt_critic->beta1;
    t.beta2 = opt_critic->beta2;
    t.gamma = gamma;
    t.K = K;
    t.B = B;
    t.NG = NG;
    unsigned long long *const sb = stamp_buf();
    t.stamp = sb;
    gwprof::launch(dcritic_tail, dim3(B / RB, K), dim3(DT), 0, s, t);
    DGrad g{};
    g.w = t.w;
    g.base = src->base;
    g.net = *critic;
    g.p0 = opt_critic->param;
    g.g0 = opt_critic->grad;
    g.m0 = opt_critic->exp_avg;
    g.v0 = opt_critic->exp_avg_sq;
    g.lr = opt_critic->lr;
    g.beta1 = opt_critic->beta1;
    g.beta2 = opt_critic->beta2;
    g.eps = opt_critic->eps;
    g.tau = tau;
    g.count = opt_critic->step;
    g.loss = critic_loss;
    g.phase = 0;
    g.K = K;
    g.B = B;
    g.HW = HW;
    g.NG = NG;
    g.nobs = K;
    g.in_dim = in_c;
    g.out = 1;
    g.stamp = sb ? sb + STAMP_BLOCKS * NSTAMP : nullptr;
    {
        const int n[7] = {2 * K * K * NG, K * ((NA * K + 7) / 8), K * (HID / RB), K, K, 0, 0};
        g.start[0] = 0;
        for (int i = 0; i < 7; ++i) g.start[i + 1] = g.start[i] + n[i];
    }
    gwprof::launch(dgrads_adam, dim3(g.start[7]), dim3(256), 0, s, g);
    t.count = opt_actor->step;
    t.lr = opt_actor->lr;
    t.beta1 = opt_actor->beta1;
    t.beta2 = opt_actor->beta2;
    t.stamp = sb ? sb + 2 * STAMP_BLOCKS * NSTAMP : nullptr;
    gwprof::launch(dactor_tail, dim3(B / RB, K), dim3(DT), 0, s, t);
    g.net = *actor;
    g.p0 = opt_actor->param;
    g.g0 = opt_actor->grad;
    g.m0 = opt_actor->exp_avg;
    g.v0 = opt_actor->exp_avg_sq;
    g.lr = opt_actor->lr;
    g.beta1 = opt_actor->beta1;
    g.beta2 = opt_actor->beta2;
    g.eps = opt_actor->eps;
    g.t0 = actor_target_flat;
    g.cnet = *critic;
    g.cp0 = opt_critic->param;
    g.ct0 = critic_target_flat;
    g.cn = opt_critic->n;
    g.count = opt_actor->step;
    g.loss = actor_loss;
    g.phase = 1;
    g.nobs = 1;
    g.in_dim = HW;
    g.out = NA;
    g.nrest = 256;
    if (img) g.img = *img;
    g.stamp = sb ? sb + 3 * STAMP_BLOCKS * NSTAMP : nullptr;
    const int g0blocks = g.start[7];
    {
        const int n[7] = {2 * K * NG, 0, K * (HID / RB), K, K, K * K * NG, g.nrest};
        g.start[0] = 0;
        for (int i = 0; i < 7; ++i) g.start[i + 1] = g.start[i] + n[i];
    }
    gwprof::launch(dgrads_adam, dim3(g.start[7]), dim3(256), 0, s, g);
    if (sb) stamp_dump(s, {B / RB * K, g0blocks, B / RB * K, g.start[7]});
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GW_OK : fail(GW_ERR_HIP, std::string(who) + ": " + hipGetErrorString(e));
}

}  // extern "C"
