// actor_ops.hip — the MADDPG actors' get_action for every env of a grid-env handle in one
// MI355X kernel (include/actor_ops.h).  Reference: maddpg/agent.py:109-122 (get_action over the
// flattened obs, argmax), agilerl 1.0.15 MADDPG.get_action with an EvolvableMLP actor
// (Linear-LayerNorm-ReLU x2, Linear, GumbelSoftmax; parity of agilerl itself unpinned).
//
// gw_actor_prepare (once per weight update): c1_k = b1_k + map . W1_k, and the LDS images of the
// layer-2/3 MFMA A operands (W2, W3 permuted so each lane's four consecutive k-steps are one
// float4).  gw_actor_act (every step), block = 16 waves = one RL agent k, one block per CU,
// persistent over 16-env tiles, one tile per wave at a time:
//   layer 1   from the obs descriptors: h1 = c1_k + sum_{patched cells c} delta_c * W1_k[c, :].
//             Lane (env = l & 15, quarter q = l >> 4) accumulates features 16j + 4q + i (j < 8,
//             i < 4) of its env: W1 rows are L2 resident and the four lanes of an env read one
//             contiguous 64-byte piece of the patched row per load instruction; the map
//             value of a cell comes from a road bitmask in LDS; the next tile's descriptor is
//             loaded while this tile computes.
//   LN1/ReLU  in registers; the four quarters of an env meet through two lane shuffles.
//   layer 2   (default) bf16x3 on v_mfma_f32_16x16x32_bf16: A1 and W2 split into bf16 hi + mid + lo,
//             6 of the 9 part products (~2^-24 relative each, f32 accumulation) at 16x the f32
//             MFMA rate per instruction; the K order inside each 32-block follows the lane's
//             layer-1 registers (kperm), so A1 needs no lane movement.  GW_ACT_V=2: exact f32:
//             transposed f32 MFMA: H2^T = W2^T A1^T with v_mfma_f32_16x16x4_f32.  The lane's 32
//             layer-1 registers ARE the B operand (k-step s takes feature 16(s >> 2) + 4q + (s & 3)
//             from quarter q: the same feature order as the layer-2 result),
//             W2 the A operand (ds_read_b128: four k-steps per read); the result has env on the
//             lane and features 16m + 4q + r in the registers, so LN2 needs only the shuffles.
//   layer 3   the same with A = W3^T (9 of 16 rows live), B = the LN2 registers in D order.  Its
//             result row 4q + r is action 4q + r, i.e. the logits are already spread over the
//             env's lanes (q 0: actions 0-3, q 1: 4-7, q 2: 8):
//   epilogue  Gumbel noise (one Philox draw per lane), softmax, mask and argmax as 4-lane
//             reductions.
// ~127 VGPRs per lane so 4 waves share each SIMD and one wave's gathers / LayerNorm / epilogue
// overlap another's MFMA chain (the f32 MFMA rate, 64 FLOP/clk/SIMD, bounds layers 2-3).
// f32 throughout: every product exact, k-ordered f32 sums (MFMA), so the result differs from a
// torch fp32 forward only by summation order (tests/test_actor_ops.py states the tolerance).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

#include "actor_ops.h"
#include "prof.h"
#include "measure.h"
#include "window_rows.h"

namespace {

constexpr int HID = 128, NA = 9, TILE = 16, MAXN = GW_MAX_AGENTS;
constexpr int NDESC = 12;
// CNN head: RS = recomputed conv-2 positions per (env, agent) (<= (N + 1) / 2), L1_WAVES per block
constexpr int L1_WAVES = 8, RS = 4;
constexpr uint32_t D_RESET = 1u;
constexpr float LN_EPS = 1e-5f, G_EPS = 1e-20f;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// workspace layout (floats, per gw_actor_workspace_floats)
constexpr int W2IMG = HID * HID;          // per agent
constexpr int W3IMG = 8 * 4 * NA * 4;     // per agent
constexpr int W2B_U4 = 3 * 8 * 4 * 64;    // per agent: the bf16x3 W2 image in 16-byte units
constexpr int W2BIMG = W2B_U4 * 4;        // (floats)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct Ws {
    float *c1;        // [K][128]
    float4 *w2;       // [K][4096]  (w2_slot)
    float4 *w3;       // [K][288]   (w3_slot)
    u32x4 *w2b;       // [K][6144]  (w2b_slot)
    float *part;      // [K][nslices][128] map . W1 row slices
};
inline Ws ws_layout(float *base, int K) {
    Ws w;
    w.c1 = base;
    w.w2 = reinterpret_cast<float4 *>(base + (size_t)K * HID);
    w.w3 = reinterpret_cast<float4 *>(base + (size_t)K * (HID + W2IMG));
    w.w2b = reinterpret_cast<u32x4 *>(base + (size_t)K * (HID + W2IMG + W3IMG));
    w.part = base + (size_t)K * (HID + W2IMG + W3IMG + W2BIMG);
    return w;
}

// the window-variant workspace: the standard images (c1 / part unused), then [K][HW][128]
inline float *patch_table(float *base, int K) { return base + (size_t)K * (HID + W2IMG + W3IMG + W2BIMG); }

// bf16x3 split of an f32 (x = hi + mid + lo to ~2^-24 relative; round-to-nearest-even bits)
__host__ __device__ inline uint32_t bf16_rn_bits(float x) {
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__host__ __device__ inline float bf16_float(uint32_t b) {
    const uint32_t u = b << 16;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}
__host__ __device__ inline void split3(float x, uint32_t &h, uint32_t &m, uint32_t &l) {
    h = bf16_rn_bits(x);
    float r = x - bf16_float(h);
    m = bf16_rn_bits(r);
    r = r - bf16_float(m);
    l = bf16_rn_bits(r);
}
// bf16x3 W2 image for v_mfma_f32_16x16x32_bf16 (GW_ACT_V=4): [part 3][m 8][kb 4][lane 64] x 8 bf16,
// element j of lane l = part of W2[in = kperm(kb, 8 (l >> 4) + j)][out = 16 m + (l & 15)], where the
// K-block's order kperm follows the layer-1 register order of the B operand (lane quarter q holds
// features 32 kb + 4q + j, j < 4, and 32 kb + 16 + 4q + j - 4)
__host__ __device__ inline int w2b_slot(int part, int m, int kb, int lane) { return ((part * 8 + m) * 4 + kb) * 64 + lane; }
__host__ __device__ inline int kperm(int kb, int k) {
    const int q = k >> 3, j = k & 7;
    return 32 * kb + (j < 4 ? 4 * q + j : 16 + 4 * q + j - 4);
}

// LDS images of the MFMA A operands, one float4 (4 consecutive k-steps) per lane and read:
//   W2: [m 8][s4 8][q 4][el 16] float4, element j = W2[16 s4 + 4q + j][16m + el]
//   W3: [m 8][q 4][el 9]        float4, element r = W3[16m + 4q + r][el]  (lanes el >= 9 read 0)
// A wave's ds_read_b128 of W2 covers 1 KB contiguous; within each 16-lane bank group the 16 env
// lanes are distinct and q steps by 256 B, so the reads are conflict-free.
__host__ __device__ inline int w2_slot(int m, int s4, int q, int el) { return ((m * 8 + s4) * 4 + q) * 16 + el; }
__host__ __device__ inline int w3_slot(int m, int q, int el) { return (m * 4 + q) * NA + el; }

struct PrepParams {
    gw_mlp_actors net;
    Ws ws;
    const float *base;
    int HW, nslices;
};

struct ActParams {
    gw_mlp_actors net;
    const float *c1;          // [K][128]
    const float4 *w2img, *w3img;
    const u32x4 *w2bimg;
    const uint32_t *desc;     // [E][12]
    const float *base;        // [HW]
    const uint16_t *mask;     // [E][K] or null
    const float *uniform;     // [K][E][9] or null
    const float *h1;          // [K][E][128] layer-1 pre-activations (H1 kernels: the CNN head)
    const float *rare_z;      // [K][E][RS][128] further layer-1 terms, rare_n[k][e] of them
    const int *rare_n;
    int32_t *actions;         // [E][K]
    float *probs;             // [K][E][9]
    float *logits;            // [K][E][9] or null
    const float *tbl;         // PW: [K][HW][128] layer-1 map part of the window centred on each cell
    int64_t E, env_offset;
    int N, K, HW, variant, training, tiles;
    int W, P, in_dim;         // grid width; PW: window side P, in_dim = P * P (else in_dim = HW)
    int ab;                   // GW_ACT_AB (measurement only): bit 0 zero the W1 deltas, bit 1 skip
                              // layer 2's MFMAs, bit 2 skip the epilogue, bit 4 gather row 0 only
    float tau;
    uint32_t key0, key1, ctr0, ctr1;
    const int64_t *ctr_dev;   // null, or a device counter added to (ctr1:ctr0) at launch time
    int apples[MAXN];
    int *zero_n;              // null, or counters this launch zeroes (the window CNN's bucket sizes,
    int zero_cnt;             //   read by the rare kernel before it), zero_cnt <= 64 * WAVES
    const float *c1_part;     // non-null: c1 = b1 + these [K][c1_nslices][128] slices in slice order
    int c1_nslices;           //   (prep_images' sum; a learner may leave the slices, not c1)
};

// GW_ACT_AB bit 3 (measurement only): wave 0 of each block stamps s_memtime at its phase
// boundaries (tools/act_ab.py reads them through gw_actor_debug_clocks)
__device__ unsigned long long g_act_clk[1024][16];
#define ACT_STAMP(slot)                                                                  \
    do {                                                                                 \
        if ((GW_AB(p.ab, 8)) && tid == 0 && bid < 1024 && (slot) < 16) g_act_clk[bid][slot] = clock64(); \
    } while (0)

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

// ---- gw_actor_prepare ----------------------------------------------------------------------
// map . W1 in row slices: part[k][sl][j] = sum_{c in rows [32 sl, 32 sl + 32)} map[c] * W1[k][c][j]
__global__ void __launch_bounds__(HID) prep_slices(PrepParams p) {
    const int sl = blockIdx.x, k = blockIdx.y, j = threadIdx.x;
    const float *w1 = p.net.w1 + (size_t)k * p.HW * HID;
    const int c0 = sl * 32, c1 = min(p.HW, c0 + 32);
    // the slice's 64 loads in flight together, then the fmas in row order
    float bv[32], wv[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const int c = c0 + i;
        bv[i] = c < c1 ? p.base[c] : 0.0f;
        wv[i] = c < c1 ? w1[(size_t)c * HID + j] : 0.0f;
    }
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i)
        if (c0 + i < c1) acc = fmaf(bv[i], wv[i], acc);
    p.ws.part[((size_t)k * p.nslices + sl) * HID + j] = acc;
}

// c1 = b1 + the slices in order (block 0 of each agent) and the W2 / W3 images (all blocks)
__global__ void __launch_bounds__(256) prep_images(PrepParams p) {
    const int k = blockIdx.y, tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < HID) {
        float part = 0.0f;
        const float *ps = p.ws.part + (size_t)k * p.nslices * HID + tid;
        int sl = 0;
        for (; sl + 8 <= p.nslices; sl += 8) {  // 8 slices' loads in flight, added in slice order
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = ps[(size_t)(sl + i) * HID];
#pragma unroll
            for (int i = 0; i < 8; ++i) part += v[i];
        }
        for (; sl < p.nslices; ++sl) part += ps[(size_t)sl * HID];
        p.ws.c1[k * HID + tid] = p.net.b1[k * HID + tid] + part;
    }
    const float *w2 = p.net.w2 + (size_t)k * HID * HID;
    float *img2 = reinterpret_cast<float *>(p.ws.w2 + (size_t)k * (W2IMG / 4));
    for (int f = blockIdx.x * 256 + tid; f < HID * HID; f += gridDim.x * 256) {
        const int row = f / HID, col = f % HID;
        img2[4 * w2_slot(col >> 4, row >> 4, (row >> 2) & 3, col & 15) + (row & 3)] = w2[f];
    }
    uint32_t *img2b = reinterpret_cast<uint32_t *>(p.ws.w2b + (size_t)k * W2B_U4);
    for (int wd = blockIdx.x * 256 + tid; wd < W2B_U4 * 4; wd += gridDim.x * 256) {
        const int jp = wd & 3, lane = (wd >> 2) & 63, kb = (wd >> 8) & 3, m = (wd >> 10) & 7, part = wd >> 13;
        uint32_t bits[2];
        for (int h = 0; h < 2; ++h) {
            const int j = 2 * jp + h;
            const float x = w2[kperm(kb, 8 * (lane >> 4) + j) * HID + 16 * m + (lane & 15)];
            uint32_t hi, mi, lo;
            split3(x, hi, mi, lo);
            bits[h] = part == 0 ? hi : part == 1 ? mi : lo;
        }
        img2b[wd] = bits[0] | (bits[1] << 16);
    }
    const float *w3 = p.net.w3 + (size_t)k * HID * NA;
    float *img3 = reinterpret_cast<float *>(p.ws.w3 + (size_t)k * (W3IMG / 4));
    for (int i = blockIdx.x * 256 + tid; i < W3IMG; i += gridDim.x * 256) {
        const int r = i & 3, el = (i >> 2) % NA, q = ((i >> 2) / NA) & 3, m = (i >> 2) / (NA * 4);
        img3[i] = w3[(16 * m + 4 * q + r) * NA + el];
    }
}

// ---- gw_patch_actor_prepare: tbl[k][c][j] = b1[k][j] + sum over window positions o of the map
//      value under o (-1 outside the grid) * W1[k][o][j], for the window centred on cell c ----
struct TblParams {
    const float *w1, *b1, *base;
    float *tbl;
    int H, W, P;
};
__global__ void __launch_bounds__(HID) prep_patch_table(TblParams p) {
    const int c = blockIdx.x, k = blockIdx.y, j = threadIdx.x;
    const int HW = p.H * p.W, PP = p.P * p.P, half = p.P / 2;
    const int cr = c / p.W, cc = c % p.W;
    const float *w1 = p.w1 + (size_t)k * PP * HID;
    float acc = 0.0f;
    for (int o = 0; o < PP; ++o) {
        const int r = cr + o / p.P - half, q = cc + o % p.P - half;
        const float mv = (r >= 0 && r < p.H && q >= 0 && q < p.W) ? p.base[r * p.W + q] : -1.0f;
        if (mv != 0.0f) acc = fmaf(mv, w1[(size_t)o * HID + j], acc);
    }
    p.tbl[((size_t)k * HW + c) * HID + j] = p.b1[k * HID + j] + acc;
}

// ---- gw_actor_act --------------------------------------------------------------------------
__device__ __forceinline__ float quad_sum(float s) {  // over the four lanes of an env
    s += __shfl_xor(s, 16, 64);
    return s + __shfl_xor(s, 32, 64);
}
__device__ __forceinline__ float quad_max(float s) {
    s = fmaxf(s, __shfl_xor(s, 16, 64));
    return fmaxf(s, __shfl_xor(s, 32, 64));
}

struct Desc {
    uint4 cells;     // 16-bit agent cells
    uint32_t flags;
    uint32_t mask;   // action mask of (e, k)
};

__device__ __forceinline__ Desc load_desc(const ActParams &p, int64_t e, int k) {
    Desc d;
    if (e < p.E) {
        d.cells = *reinterpret_cast<const uint4 *>(p.desc + e * NDESC);
        d.flags = p.desc[e * NDESC + 4];
        d.mask = p.mask ? p.mask[e * p.K + k] : 0x1FFu;
    } else {
        d.cells = make_uint4(0, 0, 0, 0);
        d.flags = 0;
        d.mask = 0x1FFu;
    }
    return d;
}

// WAVES per block (16: one block per CU holding ONE copy of the 74 KB W2/W3 image, so other
// kernels' blocks fit beside it; 8: two blocks per CU), 4 waves per SIMD (128 VGPRs).
// BF3: layer 2 as bf16x3 products on v_mfma_f32_16x16x32_bf16 (6 of the 9 part products, f32
// accumulation; ~2^-24 relative per product, 16x the f32 MFMA rate per instruction)
// H1: layer 1 is read from p.h1 (computed by cnn_l1_kernel) instead of the obs descriptors
// PW: the input is the agent's P x P egocentric window (gw_obs_patch's layout): layer 1 starts
//     from the table row of the agent's cell (p.tbl: bias + the window's map part) and a patched
//     cell inside the window adds its delta times the W1 row of its window position
// H1 && PW: the window CNN head (gw_patch_cnn_act): layer 1 = the centre's table row + the
//     recomputed positions' terms (RSX slots per (env, agent))
template <int NP, int WAVES, bool BF3 = false, bool H1 = false, bool PW = false, int RSX = RS>  // NP = patch slots per (env, agent) = N + 1
__device__ __forceinline__ void act_body(const ActParams &p) {
    constexpr int THREADS = 64 * WAVES;
    constexpr int NW2 = BF3 ? W2B_U4 : W2IMG / 4;
    __shared__ float4 s_w2[NW2];             // W2 image (w2_slot, 64 KB; BF3: w2b_slot, 96 KB)
    __shared__ float4 s_w3[W3IMG / 4];       // W3 image (w3_slot), 4.5 KB
    __shared__ __attribute__((aligned(16))) float s_vec[6][HID];  // c1, ln1_w, ln1_b, b2, ln2_w, ln2_b
    __shared__ float s_b3[12];
    __shared__ uint32_t s_road[128];         // bit c: cell c is road (map value 0, else -1)

    const int k = blockIdx.y, tid = threadIdx.x;
    const bool ln = p.net.layer_norm != 0;
    const int wave = tid >> 6, lane = tid & 63, el = lane & 15, q = lane >> 4;
    int tile = blockIdx.x * WAVES + wave;
    if (p.zero_n && blockIdx.x == 0 && k == 0 && tid < p.zero_cnt) p.zero_n[tid] = 0;
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    ACT_STAMP(0);
    Desc dn = load_desc(p, (int64_t)tile * TILE + el, k);  // first tile's descriptor, in flight
    {   // stage this agent's W2 / W3 images and vectors (all loads of a lane issued first)
        const float4 *w2 = BF3 ? reinterpret_cast<const float4 *>(p.w2bimg + (size_t)k * W2B_U4)
                               : p.w2img + (size_t)k * (W2IMG / 4);
        constexpr int R = NW2 / THREADS;
        float4 r[R];
        if (!(GW_AB(p.ab, 32))) {  // GW_ACT_AB bit 5 (measurement only): no W2 staging
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = w2[i * THREADS + tid];
#pragma unroll
        for (int i = 0; i < R; ++i) s_w2[i * THREADS + tid] = r[i];
        }
        for (int i = tid; i < W3IMG / 4; i += THREADS) s_w3[i] = p.w3img[(size_t)k * (W3IMG / 4) + i];
        if (tid < HID) {
            if (p.c1_part && !(GW_AB(p.ab, 64))) {  // prep_images' c1 (GW_ACT_AB bit 6, measurement: skipped): b1 + the slices added in slice order (32 loads in flight)
                float part = 0.0f;
                const float *ps = p.c1_part + (size_t)k * p.c1_nslices * HID + tid;
                for (int s0 = 0; s0 < p.c1_nslices; s0 += 32) {
                    float v[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i) v[i] = ps[(size_t)min(s0 + i, p.c1_nslices - 1) * HID];
#pragma unroll
                    for (int i = 0; i < 32; ++i)
                        if (s0 + i < p.c1_nslices) part += v[i];
                }
                s_vec[0][tid] = p.net.b1[k * HID + tid] + part;
            } else {
                s_vec[0][tid] = p.c1[k * HID + tid];
            }
            s_vec[1][tid] = ln ? p.net.ln1_w[k * HID + tid] : 1.0f;
            s_vec[2][tid] = ln ? p.net.ln1_b[k * HID + tid] : 0.0f;
            s_vec[3][tid] = p.net.b2[k * HID + tid];
            s_vec[4][tid] = ln ? p.net.ln2_w[k * HID + tid] : 1.0f;
            s_vec[5][tid] = ln ? p.net.ln2_b[k * HID + tid] : 0.0f;
        } else if (tid < 2 * HID) {  // road bits of cells 32w .. 32w + 31 (HW % 32 == 0 or masked)
            const int w = tid - HID;
            if (32 * w < p.HW) {
                float mv[32];
#pragma unroll
                for (int j = 0; j < 32; ++j) mv[j] = p.base[min(32 * w + j, p.HW - 1)];
                uint32_t bits = 0;
#pragma unroll
                for (int j = 0; j < 32; ++j) bits |= (32 * w + j < p.HW && mv[j] == 0.0f) ? (1u << j) : 0u;
                s_road[w] = bits;
            }
        }
        if (tid < NA) s_b3[tid] = p.net.b3[k * NA + tid];
    }
    __syncthreads();
    ACT_STAMP(1);
    int it = 0;
    const int stride = gridDim.x * WAVES;

    const float *w1 = p.net.w1 + (size_t)k * p.in_dim * HID;
    const int K = p.K;
    const int ac_k = p.apples[k];
    const int half = p.P / 2;
    // layer-1 register 4j + i and layer-2 register (m = j, r = i) both hold feature 16j + 4q + i
    auto vec4 = [q](const float *v, int j) { return *reinterpret_cast<const float4 *>(v + 16 * j + 4 * q); };

    for (; tile < p.tiles; tile += stride, ++it) {
        const int64_t e = (int64_t)tile * TILE + el;
        const bool valid = e < p.E;
        const Desc d = dn;
        // ---- obs patches of (e, k): slot 0 own apple, slot 1 + n agent n; a later slot on
        //      the same cell overrides an earlier one (the obs writer's order) ----
        int pc[NP];
        float pv[NP];
        {
            const bool reset = (d.flags & D_RESET) != 0;
            const int ac = (valid && ((d.flags >> (8 + k)) & 1u)) ? ac_k : -1;
            const float ac_map = ac >= 0 ? (((s_road[ac >> 5] >> (ac & 31)) & 1u) ? 0.0f : -1.0f) : 0.0f;
            float av = ac_map + 9.0f;
            if (!reset && av == (float)(k + 1)) av = 1.0f;  // relabel of :321 (apple on a wall)
            pc[0] = ac;
            pv[0] = av;
            const uint32_t dw[4] = {d.cells.x, d.cells.y, d.cells.z, d.cells.w};
#pragma unroll
            for (int n = 0; n < NP - 1; ++n) {
                const int c = (int)((dw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                pc[1 + n] = valid ? c : -1;
                pv[1 + n] = agent_value(reset, n, k, c == ac, p.variant);
            }
        }
        // the next tile's descriptor, loaded while this tile computes
        dn = load_desc(p, (int64_t)(tile + gridDim.x * WAVES) * TILE + el, k);
        ACT_STAMP(2 + 5 * it);
        float a[32];
        if (H1) {  // ---- layer 1 from the buffer (features 16j + 4q .. + 3: one float4 each) ----
            const size_t ek = (size_t)k * p.E + (valid ? e : 0);
            // PW: the table row of the window's centre (b + Linear-1 of the base window)
            const int ctr = PW ? ((unsigned)pc[1 + k] < (unsigned)p.HW ? pc[1 + k] : 0) : 0;
            const float4 *h = reinterpret_cast<const float4 *>(PW ? p.tbl + ((size_t)k * p.HW + ctr) * HID
                                                                  : p.h1 + ek * HID);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float4 v = h[4 * j + q];
                a[4 * j] = v.x;
                a[4 * j + 1] = v.y;
                a[4 * j + 2] = v.z;
                a[4 * j + 3] = v.w;
            }
            const int nr = valid ? p.rare_n[ek] : 0;
            for (int r = 0; r < nr; ++r) {  // the recomputed positions' terms, in slot order
                const float4 *z = reinterpret_cast<const float4 *>(p.rare_z + (ek * RSX + r) * HID);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float4 v = z[4 * j + q];
                    a[4 * j] += v.x;
                    a[4 * j + 1] += v.y;
                    a[4 * j + 2] += v.z;
                    a[4 * j + 3] += v.w;
                }
            }
        } else {
        // ---- layer 1: c1 + sum of (value - map) * W1 row over the distinct patched cells ----
        const int ctr = PW ? ((unsigned)pc[1 + k] < (unsigned)p.HW ? pc[1 + k] : 0) : 0;  // PW: the window's centre
        if (PW) {  // the table row of the centre: b1 + the window's map part (L2 resident)
            const float4 *t = reinterpret_cast<const float4 *>(p.tbl + ((size_t)k * p.HW + ctr) * HID);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float4 c = t[4 * j + q];
                a[4 * j] = c.x;
                a[4 * j + 1] = c.y;
                a[4 * j + 2] = c.z;
                a[4 * j + 3] = c.w;
            }
        } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // features 16j + 4q .. + 3: one 16-byte LDS read
            const float4 c = vec4(s_vec[0], j);
            a[4 * j] = c.x;
            a[4 * j + 1] = c.y;
            a[4 * j + 2] = c.z;
            a[4 * j + 3] = c.w;
        }
        }
        // unconditional loads (a dead slot reads row 0 with delta 0: fmaf(0, w, a) == a), so
        // the scheduler can keep several slots' row pieces in flight
        int rowc[NP];
        float dlt[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int c = pc[i];
            bool last = (unsigned)c < (unsigned)p.HW;
#pragma unroll
            for (int r = i + 1; r < NP; ++r) last = last && pc[r] != c;
            const int cc = last ? c : 0;
            const float map = ((s_road[cc >> 5] >> (cc & 31)) & 1u) ? 0.0f : -1.0f;
            int row = cc;
            if (PW) {  // window position of the cell (rows / cols -P/2 .. P-1-P/2 around the centre)
                const int wr = cc / p.W - ctr / p.W + half, wc = cc % p.W - ctr % p.W + half;
                const bool in = (unsigned)wr < (unsigned)p.P && (unsigned)wc < (unsigned)p.P;
                last = last && in;
                row = in ? wr * p.P + wc : 0;
            }
            dlt[i] = (last && !(GW_AB(p.ab, 1))) ? pv[i] - map : 0.0f;
            rowc[i] = (GW_AB(p.ab, 16)) ? q : row * (HID / 4) + q;  // float4 index of features 4q .. 4q + 3 of row
        }
        const float4 *w1v = reinterpret_cast<const float4 *>(w1);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            float4 wr[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) wr[j] = w1v[rowc[i] + 4 * j];  // features 16j + 4q .. + 3
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[4 * j + 0] = fmaf(dlt[i], wr[j].x, a[4 * j + 0]);
                a[4 * j + 1] = fmaf(dlt[i], wr[j].y, a[4 * j + 1]);
                a[4 * j + 2] = fmaf(dlt[i], wr[j].z, a[4 * j + 2]);
                a[4 * j + 3] = fmaf(dlt[i], wr[j].w, a[4 * j + 3]);
            }
            __builtin_amdgcn_sched_barrier(0);  // one slot's row pieces (32 VGPRs) in flight at a time
        }
        }  // !H1
        // ---- LN1 + ReLU (nn.LayerNorm(128), eps 1e-5, biased variance) ----
        if (ln) {
            float sm = 0.0f;
#pragma unroll
            for (int i = 0; i < 32; ++i) sm += a[i];
            const float mean = quad_sum(sm) * (1.0f / HID);
            float v = 0.0f;
#pragma unroll
            for (int i = 0; i < 32; ++i) v = fmaf(a[i] - mean, a[i] - mean, v);
            const float rstd = rsqrtf(quad_sum(v) * (1.0f / HID) + LN_EPS);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float4 g = vec4(s_vec[1], j), b = vec4(s_vec[2], j);
                const float gv[4] = {g.x, g.y, g.z, g.w}, bv4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    a[4 * j + i] = fmaxf(fmaf((a[4 * j + i] - mean) * rstd, gv[i], bv4[i]), 0.0f);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) a[i] = fmaxf(a[i], 0.0f);
        }
        ACT_STAMP(4 + 5 * it);
        // ---- layer 2: D[m] (16 features x 16 envs) = W2^T[16m.., k] . A1^T ----
        f32x4 acc[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if (BF3 && !(GW_AB(p.ab, 2))) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                // B fragments: registers 8kb .. 8kb + 7 = features 32kb + 4q + j (j < 4) and
                // 32kb + 16 + 4q + j - 4 (the image's kperm), split into bf16 hi / mid / lo
                u32x4 bh, bm, bl;
#pragma unroll
                for (int jp = 0; jp < 4; ++jp) {
                    uint32_t h0, m0, l0, h1, m1, l1;
                    split3(a[8 * kb + 2 * jp], h0, m0, l0);
                    split3(a[8 * kb + 2 * jp + 1], h1, m1, l1);
                    bh[jp] = h0 | (h1 << 16);
                    bm[jp] = m0 | (m1 << 16);
                    bl[jp] = l0 | (l1 << 16);
                }
                const bf16x8 Bh = __builtin_bit_cast(bf16x8, bh), Bm = __builtin_bit_cast(bf16x8, bm),
                             Bl = __builtin_bit_cast(bf16x8, bl);
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const bf16x8 Ah = __builtin_bit_cast(bf16x8, s_w2[w2b_slot(0, m, kb, lane)]);
                    const bf16x8 Am = __builtin_bit_cast(bf16x8, s_w2[w2b_slot(1, m, kb, lane)]);
                    const bf16x8 Al = __builtin_bit_cast(bf16x8, s_w2[w2b_slot(2, m, kb, lane)]);
                    // small terms first
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Al, Bh, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bl, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Am, Bm, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Am, Bh, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bm, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bh, acc[m], 0, 0, 0);
                }
            }
        } else if (!(GW_AB(p.ab, 2))) {
#pragma unroll
            for (int s4 = 0; s4 < 8; ++s4) {
#pragma unroll
                for (int mh = 0; mh < 8; mh += 4) {
                    float4 w[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) w[m] = s_w2[w2_slot(mh + m, s4, q, el)];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            const float wa = j == 0 ? w[m].x : j == 1 ? w[m].y : j == 2 ? w[m].z : w[m].w;
                            acc[mh + m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa, a[4 * s4 + j], acc[mh + m], 0, 0, 0);
                        }
                }
            }
        }
        ACT_STAMP(5 + 5 * it);
        // register r of tile m holds feature 16m + 4q + r of env el
        float s2 = 0.0f;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const float4 b = vec4(s_vec[3], m);
            acc[m] += f32x4{b.x, b.y, b.z, b.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) s2 += acc[m][r];
        }
        if (ln) {
            const float mean = quad_sum(s2) * (1.0f / HID);
            float v = 0.0f;
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) v = fmaf(acc[m][r] - mean, acc[m][r] - mean, v);
            const float rstd = rsqrtf(quad_sum(v) * (1.0f / HID) + LN_EPS);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const float4 g = vec4(s_vec[4], m), b = vec4(s_vec[5], m);
                const float gv[4] = {g.x, g.y, g.z, g.w}, bv4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[m][r] = fmaxf(fmaf((acc[m][r] - mean) * rstd, gv[r], bv4[r]), 0.0f);
            }
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[m][r] = fmaxf(acc[m][r], 0.0f);
        }
        // ---- layer 3: D3 (16 action rows, 9 live x 16 envs) = W3^T . A2^T; k-step (m, r) pairs
        //      feature 16m + 4q + r of the four quarters; two independent chains ----
        f32x4 o3[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const float4 w3 = el < NA ? s_w3[w3_slot(m, q, el)] : float4{0.0f, 0.0f, 0.0f, 0.0f};
            const float wv[4] = {w3.x, w3.y, w3.z, w3.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) o3[m & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[r], acc[m][r], o3[m & 1], 0, 0, 0);
        }
        const f32x4 out = o3[0] + o3[1];
        if (GW_AB(p.ab, 4)) {
            ACT_STAMP(6 + 5 * it);
            continue;
        }
        // ---- epilogue: D3 row 4q + r = action 4q + r (q 0: 0-3, q 1: 4-7, q 2: 8) ----
        const size_t o = ((size_t)k * p.E + (valid ? e : 0)) * NA;
        float lg[4];
        bool live[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            live[r] = 4 * q + r < NA;
            lg[r] = live[r] ? out[r] + s_b3[4 * q + r] : 0.0f;
        }
        if (p.logits && valid) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (live[r]) p.logits[o + 4 * q + r] = lg[r];
        }
        if (p.training) {  // agilerl GumbelSoftmax: logits - log(-log(u + eps) + eps)
            float u[4];
            if (p.uniform) {
#pragma unroll
                for (int r = 0; r < 4; ++r) u[r] = (live[r] && valid) ? p.uniform[o + 4 * q + r] : 0.5f;
            } else {  // draw q of (env, counter, k): actions 4q .. 4q + 3
                uint64_t ctr = ((uint64_t)p.ctr1 << 32) | p.ctr0;
                if (p.ctr_dev) ctr += (uint64_t)*p.ctr_dev;
                const uint4 x = philox((uint32_t)(p.env_offset + e), (uint32_t)ctr,
                                       (uint32_t)k | ((uint32_t)q << 8) | (0xA7u << 24), (uint32_t)(ctr >> 32),
                                       p.key0, p.key1);
                u[0] = (float)(x.x >> 8) * (1.0f / 16777216.0f);
                u[1] = (float)(x.y >> 8) * (1.0f / 16777216.0f);
                u[2] = (float)(x.z >> 8) * (1.0f / 16777216.0f);
                u[3] = (float)(x.w >> 8) * (1.0f / 16777216.0f);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (live[r]) lg[r] = lg[r] - logf(-logf(u[r] + G_EPS) + G_EPS);
        }
        float z[4], mx = -INFINITY;  // softmax(logits / tau) over the env's four lanes
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            z[r] = lg[r] / p.tau;
            if (live[r]) mx = fmaxf(mx, z[r]);
        }
        mx = quad_max(mx);
        float ex[4], sm = 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ex[r] = live[r] ? expf(z[r] - mx) : 0.0f;
            sm += ex[r];
        }
        sm = quad_sum(sm);
        const uint32_t mk = d.mask;
        float bv = -1.0f;
        int best = 64;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float pr = ex[r] / sm;
            if (live[r] && valid) p.probs[o + 4 * q + r] = pr;
            const float pm = ((mk >> (4 * q + r)) & 1u) ? pr : 0.0f;
            if (live[r] && pm > bv) {  // first maximum within the lane
                bv = pm;
                best = 4 * q + r;
            }
        }
        // argmax across the quarters: larger value wins, ties go to the lower action
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {
            const float ov = __shfl_xor(bv, off, 64);
            const int ob = __shfl_xor(best, off, 64);
            if (ov > bv || (ov == bv && ob < best)) {
                bv = ov;
                best = ob;
            }
        }
        if (q == 0 && valid) p.actions[e * K + k] = best;
        ACT_STAMP(6 + 5 * it);
    }
}


template <int NP, int WAVES, bool BF3 = false, bool H1 = false, bool PW = false, int RSX = RS>
__global__ void __launch_bounds__(64 * WAVES, 4) act_kernel(ActParams p) {
    act_body<NP, WAVES, BF3, H1, PW, RSX>(p);
}

// GW_ACT_WAVES=12|8 (A/B, result-neutral): 12- or 8-wave blocks held to the 16-wave block's 128
// VGPRs per lane, so that a quarter or half of each SIMD's register file stays free for the
// kernels beside the actor (the rollout's obs writer).  Left to itself the compiler spends the
// smaller block's whole budget (8 waves: 243 VGPRs): its LDS allows one block per CU, so it
// ignores waves-per-EU requests; declaring the 16-wave block size (launched with fewer threads)
// is what holds the allocation to 128
template <int NP, int WAVES>
__global__ void __launch_bounds__(1024) act_kernel_lean(ActParams p) {
    act_body<NP, WAVES, true>(p);
}

// ---- the configs/cnn.yaml head (gw_cnn_prepare / gw_cnn_act; include/actor_ops.h) -------------
// Geometry: conv-2 position P = (Y, X) (P = Y (W/4) + X) sees obs cells (4Y + ry, 4X + rx); the
// region's cell t = 4 ry + rx lies in conv-1 window d = 2 (ry >> 1) + (rx >> 1) at tap
// 2 (ry & 1) + (rx & 1), and conv-2 tap d.  Linear-1 feature of (channel o, position P) is o P_n + P.
constexpr int C1 = 32, C2 = 64, NV = 19;  // NV: obs values of a patched cell (cnn_value_index)
struct CnnWs {
    Ws mlp;           // layer-2/3 MFMA images (and an unused c1)
    float *wlt;       // [K][P][64][128]  Linear-1 weight, transposed per position
    float *wlj;       // [K][P][128][64]  (windows) the same per position, feature-major: staged as float4
    float *a2map;     // [K][P][64]       conv-2 activations of the static map
    float *pre2map;   // [K][P][64]       ... before the ReLU
    float *a1map;     // [K][P][4][32]    conv-1 activations of the map, per window
    float *zpart;     // [K][P][128]
    float *zmap;      // [K][128]         b + Wl . a2(map)
    float *table;     // [K][P][16][NV][128]  Wl[:, P] . (a2(P with cell t := value v) - a2map(P))
    float *w2t;       // [K][4][64][32]   conv-2 weight, window-major
    uint32_t *road;   // [128]            road bitmask of the map (bit c: cell c is road)
    float *h1;        // [K][E][128]      z_map + table rows
    float *rare_z;    // [K][E][RS][128]  their Linear-1 contributions
    int *rare_n;      // [K][E]           recomputed positions per (env, agent)
    int *bucket_n;    // [K][P]           items per position (bucket_scan)
    int *bucket;      // [K][P][E]        items (e RS + slot) per position
    int *unit_off;    // [K P + 1]        (unused since the rare kernels plan their units in LDS)
};
inline int64_t cnn_mlp_floats(int K) { return (int64_t)K * (HID + W2IMG + W3IMG + W2BIMG); }
inline CnnWs cnn_ws_layout(float *base, int K, int P, int64_t E) {
    CnnWs w;
    w.mlp = ws_layout(base, K);
    float *f = base + cnn_mlp_floats(K);
    w.wlt = f;        f += (int64_t)K * P * C2 * HID;
    w.a2map = f;      f += (int64_t)K * P * C2;
    w.pre2map = f;    f += (int64_t)K * P * C2;
    w.a1map = f;      f += (int64_t)K * P * 4 * C1;
    w.zpart = f;      f += (int64_t)K * P * HID;
    w.zmap = f;       f += (int64_t)K * HID;
    w.table = f;      f += (int64_t)K * P * 16 * NV * HID;
    w.w2t = f;        f += (int64_t)K * 4 * C2 * C1;
    w.road = reinterpret_cast<uint32_t *>(f);  f += 128;
    w.h1 = f;         f += (int64_t)K * E * HID;
    w.rare_z = f;     f += (int64_t)K * E * RS * HID;
    w.rare_n = reinterpret_cast<int *>(f);    f += (int64_t)K * E;
    w.bucket_n = reinterpret_cast<int *>(f);  f += (int64_t)K * P;
    w.bucket = reinterpret_cast<int *>(f);    f += (int64_t)K * P * E;
    w.unit_off = reinterpret_cast<int *>(f);  f += (int64_t)K * P + 1;
    return w;
}
// The layer-1 kernels' outputs for filling the buckets without global atomics (after unit_off):
//   item [K][E]      the (env, agent)'s positions to recompute (grid: up to RS position bytes in
//                    slot order; windows: a position mask, slot = rank in the mask)
//   cnt / off [nb][nblk]  items per (bucket, layer-1 block) and their offsets in the bucket
// bucket_scan turns the counts into offsets and bucket sizes, the scatter kernels fill the buckets.
// ctr: unused (zeroed by the prepare calls)
struct Lists {
    int *item, *cnt, *off, *ctr;
    int nblk;
};
inline Lists lists_at(int *unit_off, int nb, int K, int64_t E, int per_block) {
    Lists l;
    l.nblk = (int)((E + per_block - 1) / per_block);
    l.item = unit_off + nb + 1;
    l.cnt = l.item + (int64_t)K * E;
    l.off = l.cnt + (int64_t)nb * l.nblk;
    l.ctr = l.off + (int64_t)nb * l.nblk;
    return l;
}
inline int64_t lists_floats(int nb, int K, int64_t E, int per_block) {
    return (int64_t)K * E + 2 * (int64_t)nb * ((E + per_block - 1) / per_block) + 4;
}
constexpr int L1_ENVS = TILE * L1_WAVES;  // envs per cnn_l1_kernel block
inline int64_t cnn_ws_floats(int K, int P, int64_t E) {
    return (int64_t)(cnn_ws_layout(nullptr, K, P, E).unit_off - (int *)nullptr) + (int64_t)K * P + 1 +
           lists_floats(K * P, K, E, L1_ENVS);
}
// value of a patched obs cell -> table column: 0.5 (reset agent), 9.5 (reset agent on its apple),
// 1 .. 17 (agents, relabelled or raw, apples, agents on apples); -1 = not tabulated
__host__ __device__ inline int cnn_value_index(float v) {
    if (v == 0.5f) return 0;
    if (v == 9.5f) return 1;
    const int i = (int)v;
    return ((float)i == v && i >= 1 && i <= NV - 2) ? i + 1 : -1;
}
__host__ __device__ inline float cnn_index_value(int vi) { return vi == 0 ? 0.5f : vi == 1 ? 9.5f : (float)(vi - 1); }

struct CnnParams {
    gw_cnn_actors net;
    CnnWs ws;
    const float *base;        // [HW] map obs values (0 road, -1 inactive)
    const uint32_t *desc;     // [E][12]
    int64_t E;
    int N, K, H, W, P, Wq, HW, variant;
    int PW;                   // window side (gw_patch_cnn_*: P = (PW / 4)^2 positions), 0 = the whole grid
    int ab;                   // GW_CNN_AB (measurement only): bit 0 skip the recomputed positions,
                              // bit 1 skip the table rows; windows: bit 2 list no positions
    int apples[MAXN];
    unsigned long long *stamp = nullptr;  // GW_RARE_STAMP (diagnostics): per block [8] wall clocks
};
#define RSTAMP(P, i)                                                                               \
    do {                                                                                           \
        if ((P).stamp && threadIdx.x == 0) (P).stamp[(int64_t)blockIdx.x * 8 + (i)] = wall_clock64(); \
    } while (0)

// Linear-1 weight, transposed: wlt[k][P][o][j] = lin1_w[k][j][o P_n + P]
__global__ void __launch_bounds__(256) cnn_prep_wlt(CnnParams p) {
    const int64_t F = (int64_t)C2 * p.P, n = (int64_t)p.K * F * HID;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int j = (int)(i % HID);
        const int64_t r = i / HID;
        const int o = (int)(r % C2), P = (int)((r / C2) % p.P), k = (int)(r / (C2 * (int64_t)p.P));
        p.ws.wlt[i] = p.net.lin1_w[((int64_t)k * HID + j) * F + (int64_t)o * p.P + P];
    }
}

// (windows) wlj[k][Q][j][o] = lin1_w[k][j][o P_n + Q]
__global__ void __launch_bounds__(256) wcnn_prep_wlj(CnnParams p) {
    const int64_t F = (int64_t)C2 * p.P, n = (int64_t)p.K * F * HID;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int o = (int)(i % C2);
        const int64_t r = i / C2;
        const int j = (int)(r % HID), Q = (int)((r / HID) % p.P), k = (int)(r / (HID * (int64_t)p.P));
        p.ws.wlj[i] = p.net.lin1_w[((int64_t)k * HID + j) * F + (int64_t)o * p.P + Q];
    }
}

// map activations of position P (block (P, k), 128 threads)
__global__ void __launch_bounds__(128) cnn_prep_map(CnnParams p) {
    const int P = blockIdx.x, k = blockIdx.y, t = threadIdx.x;
    __shared__ float s_a1[4][C1];
    if (P == 0) {  // this agent's window-major conv-2 weight; (agent 0) the road bitmask
        for (int i = t; i < 4 * C2 * C1; i += 128) {
            const int d = i / (C2 * C1), o = (i / C1) % C2, c = i % C1;
            p.ws.w2t[(size_t)k * 4 * C2 * C1 + i] = p.net.conv2_w[((k * C2 + o) * C1 + c) * 4 + d];
        }
        if (k == 0) {
            uint32_t bits = 0;
            for (int j = 0; j < 32; ++j) bits |= (32 * t + j < p.HW && p.base[min(32 * t + j, p.HW - 1)] == 0.0f) ? (1u << j) : 0u;
            p.ws.road[t] = bits;
        }
    }
    const int Y = P / p.Wq, X = P % p.Wq;
    {   // conv 1: window d = t >> 5, channel c = t & 31
        const int d = t >> 5, c = t & 31;
        float acc = p.net.conv1_b[k * C1 + c];
        for (int tap = 0; tap < 4; ++tap) {
            const int y = 4 * Y + 2 * (d >> 1) + (tap >> 1), x = 4 * X + 2 * (d & 1) + (tap & 1);
            acc = fmaf(p.net.conv1_w[(k * C1 + c) * 4 + tap], p.base[y * p.W + x], acc);
        }
        const float a1 = fmaxf(acc, 0.0f);
        s_a1[d][c] = a1;
        p.ws.a1map[(((size_t)k * p.P + P) * 4 + d) * C1 + c] = a1;
    }
    __syncthreads();
    if (t < C2) {  // conv 2
        float acc = p.net.conv2_b[k * C2 + t];
        for (int c = 0; c < C1; ++c)
            for (int d = 0; d < 4; ++d) acc = fmaf(p.net.conv2_w[((k * C2 + t) * C1 + c) * 4 + d], s_a1[d][c], acc);
        p.ws.pre2map[((size_t)k * p.P + P) * C2 + t] = acc;
        p.ws.a2map[((size_t)k * p.P + P) * C2 + t] = fmaxf(acc, 0.0f);
    }
}

// zpart[k][P][j] = Wl[:, P] . a2map(P)   (block (P, k), 128 threads)
__global__ void __launch_bounds__(128) cnn_prep_zpart(CnnParams p) {
    const int P = blockIdx.x, k = blockIdx.y, j = threadIdx.x;
    const float *w = p.ws.wlt + ((size_t)k * p.P + P) * C2 * HID;
    const float *a2 = p.ws.a2map + ((size_t)k * p.P + P) * C2;
    float acc = 0.0f;
    for (int o = 0; o < C2; ++o) acc = fmaf(w[o * HID + j], a2[o], acc);
    p.ws.zpart[((size_t)k * p.P + P) * HID + j] = acc;
}

// zmap = b + the positions' parts in order (block k, 128 threads); also c1 := 0 (unused)
__global__ void __launch_bounds__(128) cnn_prep_zmap(CnnParams p) {
    const int k = blockIdx.x, j = threadIdx.x;
    float acc = 0.0f;
    for (int P = 0; P < p.P; ++P) acc += p.ws.zpart[((size_t)k * p.P + P) * HID + j];
    p.ws.zmap[k * HID + j] = p.net.lin1_b[k * HID + j] + acc;
    p.ws.mlp.c1[k * HID + j] = 0.0f;
}

// the delta table of position P (block (P, k), 4 waves; wave w takes items w, w + 4, ... of the
// 16 cells x NV values)
__global__ void __launch_bounds__(256) cnn_prep_table(CnnParams p) {
    const int P = blockIdx.x, k = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    __shared__ float s_wl[C2][HID];        // Wl block of P, 32 KB
    __shared__ float s_w2[C2][C1][4];      // conv-2 weight, 32 KB
    __shared__ float s_map[16], s_a1[4][C1], s_pre2[C2], s_a2[C2];
    __shared__ float s_da1[4][C1], s_dl[4][C2];
    const int Y = P / p.Wq, X = P % p.Wq;
    const float *wl = p.ws.wlt + ((size_t)k * p.P + P) * C2 * HID;
    for (int i = tid; i < C2 * HID; i += 256) (&s_wl[0][0])[i] = wl[i];
    for (int i = tid; i < C2 * C1 * 4; i += 256) (&s_w2[0][0][0])[i] = p.net.conv2_w[(size_t)k * C2 * C1 * 4 + i];
    if (tid < 16) s_map[tid] = p.base[(4 * Y + (tid >> 2)) * p.W + 4 * X + (tid & 3)];
    if (tid < 4 * C1) (&s_a1[0][0])[tid] = p.ws.a1map[((size_t)k * p.P + P) * 4 * C1 + tid];
    if (tid < C2) {
        s_pre2[tid] = p.ws.pre2map[((size_t)k * p.P + P) * C2 + tid];
        s_a2[tid] = p.ws.a2map[((size_t)k * p.P + P) * C2 + tid];
    }
    __syncthreads();
    for (int item = wave; item < 16 * NV; item += 4) {
        const int t = item / NV, vi = item % NV;
        const int ry = t >> 2, rx = t & 3, d = 2 * (ry >> 1) + (rx >> 1), tap = 2 * (ry & 1) + (rx & 1);
        const float v = cnn_index_value(vi);
        if (lane < C1) {  // conv 1 of window d with cell t := v
            const int c = lane;
            float acc = p.net.conv1_b[k * C1 + c];
            for (int u = 0; u < 4; ++u) {
                const int cy = 2 * (d >> 1) + (u >> 1), cx = 2 * (d & 1) + (u & 1);
                acc = fmaf(p.net.conv1_w[(k * C1 + c) * 4 + u], u == tap ? v : s_map[4 * cy + cx], acc);
            }
            s_da1[wave][c] = fmaxf(acc, 0.0f) - s_a1[d][c];
        }
        __syncthreads();  // (every wave runs the same 76 items)
        {   // conv 2, lane = output channel
            float acc = s_pre2[lane];
            for (int c = 0; c < C1; ++c) acc = fmaf(s_w2[lane][c][d], s_da1[wave][c], acc);
            s_dl[wave][lane] = fmaxf(acc, 0.0f) - s_a2[lane];
        }
        __syncthreads();
        float t0 = 0.0f, t1 = 0.0f;
        for (int o = 0; o < C2; ++o) {
            const float dl = s_dl[wave][o];
            t0 = fmaf(s_wl[o][lane], dl, t0);
            t1 = fmaf(s_wl[o][lane + 64], dl, t1);
        }
        float *row = p.ws.table + ((((size_t)k * p.P + P) * 16 + t) * NV + vi) * HID;
        row[lane] = t0;
        row[lane + 64] = t1;
        __syncthreads();
    }
}


// Layer 1 of the CNN head for every (env, agent): h1 = z_map + the changed positions' deltas.
// cnn_l1_kernel sums the table rows of the positions with one patched cell into h1 and lists the
// positions with several (slot order) with per-block counts; bucket_scan / cnn_scatter file them
// as (env, slot) items into per-(agent, position) buckets (no global atomics); bucket_scan cuts
// the buckets into units of up to 16 x RARE_WAVES items; cnn_rare_kernel
// (persistent) takes units with the position's Linear-1 block staged in LDS, recomputes each
// item's position (conv 1, conv 2) and writes its 128-float contribution; act_kernel<H1> adds an
// env's contributions (in slot order) to h1.  Every sum runs in a fixed order, so the result
// does not depend on the order items entered a bucket.
template <int NP>
__global__ void __launch_bounds__(64 * L1_WAVES, 4) cnn_l1_kernel(CnnParams p, Lists lists) {
    __shared__ uint32_t s_road[128];
    __shared__ int s_hist[256];                 // items per position in this block
    __shared__ int s_rows[L1_WAVES][NP][64];   // the lanes' table rows
    const int k = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, el = lane & 15, q = lane >> 4;
    const int64_t e = ((int64_t)blockIdx.x * L1_WAVES + wave) * TILE + el;
    const bool valid = e < p.E;
    uint4 cells = make_uint4(0, 0, 0, 0);
    uint32_t flags = 0;
    if (valid) {
        cells = *reinterpret_cast<const uint4 *>(p.desc + e * NDESC);
        flags = p.desc[e * NDESC + 4];
    }
    if (tid < 128) s_road[tid] = p.ws.road[tid];
    if (tid < 256) s_hist[tid] = 0;
    __syncthreads();
    auto map_at = [&](int c) { return ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f; };
    // ---- the (env, agent)'s patched cells (act_kernel's decoding) ----
    int pc[NP];
    float pv[NP];
    {
        const bool reset = (flags & D_RESET) != 0;
        const int ac = (valid && ((flags >> (8 + k)) & 1u)) ? p.apples[k] : -1;
        float av = (ac >= 0 ? map_at(ac) : 0.0f) + 9.0f;
        if (!reset && av == (float)(k + 1)) av = 1.0f;
        pc[0] = ac;
        pv[0] = av;
        const uint32_t dw[4] = {cells.x, cells.y, cells.z, cells.w};
#pragma unroll
        for (int n = 0; n < NP - 1; ++n) {
            const int c = (int)((dw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
            pc[1 + n] = valid ? c : -1;
            pv[1 + n] = agent_value(reset, n, k, c == ac, p.variant);
        }
    }
    // distinct cells (a later slot on the same cell wins), their positions, table columns
    int pos[NP], vidx[NP];
    bool live[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int c = pc[i];
        bool l = (unsigned)c < (unsigned)p.HW;
#pragma unroll
        for (int r = i + 1; r < NP; ++r) l = l && pc[r] != c;
        live[i] = l;
        const int cc = l ? c : 0, y = cc / p.W, x = cc % p.W;
        pos[i] = l ? (y >> 2) * p.Wq + (x >> 2) : -1 - i;
        vidx[i] = cnn_value_index(pv[i]);
    }
    // per slot: the table row (float4 index) of a position with exactly one patched cell goes to
    // the lane's row list; `rare` marks the first slot of each position holding several
    unsigned rare = 0;
    int nrow = 0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        int cnt = 0;
        bool leader = live[i];
#pragma unroll
        for (int r = 0; r < NP; ++r) {
            const bool same = live[r] && pos[r] == pos[i];
            cnt += same ? 1 : 0;
            leader = leader && !(r < i && same);
        }
        const bool single = live[i] && cnt == 1 && vidx[i] >= 0;
        rare |= (leader && !single) ? (1u << i) : 0u;
        if (single) {
            const int c = pc[i], y = c / p.W, x = c % p.W;
            s_rows[wave][nrow++][lane] = (((k * p.P + pos[i]) * 16 + 4 * (y & 3) + (x & 3)) * NV + vidx[i]) * (HID / 4);
        }
    }
    if (GW_AB(p.ab, 2)) nrow = 0;
    if (GW_AB(p.ab, 1)) rare = 0;
    {
        float a[32];
        const float4 *z = reinterpret_cast<const float4 *>(p.ws.zmap + k * HID);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 v = z[4 * j + q];
            a[4 * j] = v.x;
            a[4 * j + 1] = v.y;
            a[4 * j + 2] = v.z;
            a[4 * j + 3] = v.w;
        }
        const float4 *tab = reinterpret_cast<const float4 *>(p.ws.table);
#pragma unroll 1
        for (int i = 0; i < nrow; ++i) {  // one row (8 float4 per lane) in flight per wave
            const int r0 = s_rows[wave][i][lane];
            float4 w0[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w0[j] = tab[r0 + 4 * j + q];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[4 * j + 0] += w0[j].x;
                a[4 * j + 1] += w0[j].y;
                a[4 * j + 2] += w0[j].z;
                a[4 * j + 3] += w0[j].w;
            }
        }
        if (valid) {
            float4 *h = reinterpret_cast<float4 *>(p.ws.h1 + ((size_t)k * p.E + e) * HID);
#pragma unroll
            for (int j = 0; j < 8; ++j) h[4 * j + q] = make_float4(a[4 * j], a[4 * j + 1], a[4 * j + 2], a[4 * j + 3]);
        }
    }
    // ---- positions with several patched cells: listed per (env, agent) in slot order and
    //      counted per position (cnn_scatter files them into the buckets, cnn_rare_kernel
    //      computes their contributions) ----
    int ns = 0;
    uint32_t rp = 0;
    while (rare) {
        const int i0 = __builtin_ctz(rare);
        rare &= rare - 1;
        int P = 0;
#pragma unroll
        for (int i = 0; i < NP; ++i)
            if (i == i0) P = pos[i];
        if (q == 0 && valid) atomicAdd(&s_hist[P], 1);   // (LDS)
        rp |= (uint32_t)P << (8 * ns);
        ++ns;
    }
    if (q == 0 && valid) {
        p.ws.rare_n[(size_t)k * p.E + e] = ns;
        lists.item[(size_t)k * p.E + e] = (int)rp;
    }
    __syncthreads();
    for (int i = tid; i < p.P; i += 64 * L1_WAVES)
        lists.cnt[((size_t)k * p.P + i) * lists.nblk + blockIdx.x] = s_hist[i];
}

// files the listed positions into the buckets: block = cnn_l1_kernel's block of envs; the rank
// inside the block's share of a bucket comes from an LDS counter (the order inside a bucket does
// not change any result: every item writes its own slot)
__global__ void __launch_bounds__(L1_ENVS) cnn_scatter(CnnParams p, Lists lists) {
    __shared__ int s_ctr[256];
    const int k = blockIdx.y, tid = threadIdx.x;
    const int64_t e = (int64_t)blockIdx.x * L1_ENVS + tid;
    for (int i = tid; i < 256; i += L1_ENVS) s_ctr[i] = 0;
    __syncthreads();
    if (e >= p.E) return;
    const int ns = p.ws.rare_n[(size_t)k * p.E + e];
    const uint32_t rp = (uint32_t)lists.item[(size_t)k * p.E + e];
    for (int sl = 0; sl < ns; ++sl) {
        const int P = (rp >> (8 * sl)) & 255;
        const int r = atomicAdd(&s_ctr[P], 1);
        const size_t b = (size_t)k * p.P + P;
        p.ws.bucket[b * p.E + lists.off[b * lists.nblk + blockIdx.x] + r] = (int)(e * RS + sl);
    }
}

// Units of work over the buckets: bucket b (= k P_n + P) holds ceil(n_b / RARE_ITEMS) units;
// unit_off[b] = the units before bucket b (block_unit_offsets, in each rare block's LDS).
constexpr int RARE_WAVES = 8, RARE_ITEMS = 16 * RARE_WAVES, RARE_BLOCKS = 256;
constexpr int WR_WAVES_C = 4;  // the window rare kernel's waves per block (WR_WAVES)

// s_uo[b] = the units (RARE_ITEMS items each) before bucket b, s_uo[nb] = all units: a block scan
// of the bucket sizes in bucket order (every rare block computes the same table)
constexpr int RARE_MAX_NB = 2048;  // K x positions (8 agents x 16 x 16 conv-2 positions)
template <int WAVES = RARE_WAVES, int ITEMS = RARE_ITEMS>
__device__ __forceinline__ void block_unit_offsets(const int *bucket_n, int nb, int *s_uo, int *s_wt) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int base = 0;
    for (int c0 = 0; c0 < nb; c0 += 64 * WAVES) {
        const int i = c0 + tid;
        const int n = i < nb ? bucket_n[i] : 0;
        const int u = (n + ITEMS - 1) / ITEMS;
        int incl = u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(incl, d, 64);
            if (lane >= d) incl += o;
        }
        if (lane == 63) s_wt[wave] = incl;
        __syncthreads();
        int before = base, tot = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            before += w < wave ? s_wt[w] : 0;
            tot += s_wt[w];
        }
        if (i < nb) s_uo[i] = before + incl - u;
        __syncthreads();  // s_wt is rewritten by the next chunk
        base += tot;
    }
    if (tid == 0) s_uo[nb] = base;
    __syncthreads();
}

// Persistent: block b takes units b, b + RARE_BLOCKS, ...; per unit the position's conv weights,
// map activations and Linear-1 block are staged in LDS.  Lane (item it = l & 15, quarter q): the
// item's env observation is decoded from its descriptor (act_kernel's rule) and lane q evaluates
// conv-1 window q of the position; conv 2 and the Linear-1 block are f32 MFMAs over the wave's 16
// items (rare_mfma), with the items as the N dimension.
constexpr int W2R = C1 + 4;   // LDS row stride (floats) of the conv-2 image [window][o][c]
constexpr int WLR = C2 + 4;   // LDS row stride (floats) of the Linear-1 block image [j][o]
constexpr int RARE_LDS_W2 = 4 * C2 * W2R, RARE_LDS_WL = HID * WLR;

// stage agent k's conv-2 weight (window-major w2t[k][q][o][c] -> [q][o][W2R]) ...
__device__ __forceinline__ void stage_w2(float *s_w2, const float *w2t, int tid, int nthreads) {
    const float4 *src = reinterpret_cast<const float4 *>(w2t);
    for (int i = tid; i < 4 * C2 * C1 / 4; i += nthreads) {
        const int row = i / (C1 / 4), c4 = i % (C1 / 4);
        *reinterpret_cast<float4 *>(s_w2 + row * W2R + 4 * c4) = src[i];
    }
}
// ... a position's Linear-1 block from its feature-major image (wlj[j][o] -> [j][WLR]): float4
// copies, every load of the thread in flight before its stores
__device__ __forceinline__ void stage_wl4(float *s_wl, const float *wlj, int tid) {
    constexpr int N4 = C2 * HID / 4, PER = N4 / (64 * WR_WAVES_C);
    const float4 *src = reinterpret_cast<const float4 *>(wlj);
    float4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) v[u] = src[tid + u * 64 * WR_WAVES_C];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int i = tid + u * 64 * WR_WAVES_C;
        *reinterpret_cast<float4 *>(s_wl + (i / (C2 / 4)) * WLR + 4 * (i % (C2 / 4))) = v[u];
    }
}
// ... and a position's Linear-1 block (wlt[o][j] -> [j][WLR])
__device__ __forceinline__ void stage_wl(float *s_wl, const float *wlt, int tid, int nthreads) {
    for (int i = tid; i < C2 * HID; i += nthreads) s_wl[(i & (HID - 1)) * WLR + (i >> 7)] = wlt[i];
}

// conv 2 and Linear 1 of one position for the wave's 16 items on v_mfma_f32_16x16x4f32:
//   conv 2:   D[o][it] = sum over k-steps c of W2[o][c][q] (A: lane = (o & 15, window q)) x
//             a1[it][q][c] (B: lane = (window q, item it), the lane's own conv-1 register c);
//             lane (it, q) receives o = 16t + 4q + r (tile t, register r)
//   Linear:   z[j][it] = sum over k-steps (t, r) of Wl[j][16t + 4q + r] (A) x d[it][16t + 4q + r]
//             (B: the lane's own delta), lane (it, q) receives features 16jt + 4q + r: the layout
//             act_kernel sums (one float4 per jt)
// base[4t + r]: the base activation of channel 16t + 4q + r (map / base window).  Products are
// exact in f32, sums in f32 (another order than torch's).
__device__ __forceinline__ void rare_mfma(const float (&a1)[C1], const float *s_w2, const float *s_wl,
                                          const float *s_b2, const float (&base)[16], int lane, float4 (&z)[8]) {
    const int ol = lane & 15, q = lane >> 4;
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int c4 = 0; c4 < C1 / 4; ++c4) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float4 w = *reinterpret_cast<const float4 *>(s_w2 + (q * C2 + 16 * t + ol) * W2R + 4 * c4);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, a1[4 * c4 + 0], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, a1[4 * c4 + 1], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, a1[4 * c4 + 2], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, a1[4 * c4 + 3], acc[t], 0, 0, 0);
        }
    }
    float d[16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) d[4 * t + r] = fmaxf(acc[t][r] + s_b2[16 * t + 4 * q + r], 0.0f) - base[4 * t + r];
    f32x4 zz[8];
#pragma unroll
    for (int jt = 0; jt < 8; ++jt) zz[jt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
            const float4 w = *reinterpret_cast<const float4 *>(s_wl + (16 * jt + ol) * WLR + 16 * t + 4 * q);
            zz[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, d[4 * t + 0], zz[jt], 0, 0, 0);
            zz[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, d[4 * t + 1], zz[jt], 0, 0, 0);
            zz[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, d[4 * t + 2], zz[jt], 0, 0, 0);
            zz[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, d[4 * t + 3], zz[jt], 0, 0, 0);
        }
    }
#pragma unroll
    for (int jt = 0; jt < 8; ++jt) z[jt] = make_float4(zz[jt][0], zz[jt][1], zz[jt][2], zz[jt][3]);
}

template <int NP>
__global__ void __launch_bounds__(64 * RARE_WAVES) cnn_rare_kernel(CnnParams p) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int it = lane & 15, q = lane >> 4;
    const int nb = p.K * p.P;
    __shared__ __attribute__((aligned(16))) float s_w2[RARE_LDS_W2];   // 36 KB
    __shared__ __attribute__((aligned(16))) float s_wl[RARE_LDS_WL];   // 34 KB
    __shared__ float s_w1[C1][4], s_b1[C1], s_b2[C2], s_a2m[C2];
    __shared__ uint32_t s_road[128];
    __shared__ int s_uo[RARE_MAX_NB + 1], s_wt[RARE_WAVES];
    if (tid < 128) s_road[tid] = p.ws.road[tid];
    block_unit_offsets(p.ws.bucket_n, nb, s_uo, s_wt);
    const int nunits = s_uo[nb];
    int staged_k = -1, staged_P = -1;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        int lo = 0, hi = nb;  // the bucket holding unit u: unit_off[lo] <= u < unit_off[lo + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_uo[mid] <= u) lo = mid; else hi = mid;
        }
        const int k = lo / p.P, P = lo % p.P;
        const int n = p.ws.bucket_n[lo];
        const int i_begin = (u - s_uo[lo]) * RARE_ITEMS, i_end = min(n, i_begin + RARE_ITEMS);
        __syncthreads();  // the previous unit is done with the LDS images
        if (k != staged_k) {
            stage_w2(s_w2, p.ws.w2t + (size_t)k * 4 * C2 * C1, tid, 64 * RARE_WAVES);
            if (tid < C1 * 4) (&s_w1[0][0])[tid] = p.net.conv1_w[k * C1 * 4 + tid];
            if (tid < C1) s_b1[tid] = p.net.conv1_b[k * C1 + tid];
            if (tid < C2) s_b2[tid] = p.net.conv2_b[k * C2 + tid];
        }
        if (k != staged_k || P != staged_P) {
            stage_wl(s_wl, p.ws.wlt + ((size_t)k * p.P + P) * C2 * HID, tid, 64 * RARE_WAVES);
            if (tid < C2) s_a2m[tid] = p.ws.a2map[((size_t)k * p.P + P) * C2 + tid];
        }
        staged_k = k;
        staged_P = P;
        __syncthreads();
        auto map_at = [&](int c) { return ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f; };
        const int Y = P / p.Wq, X = P % p.Wq;
        const int b = i_begin + 16 * wave;
        if (b >= i_end) continue;  // (wave-uniform; no barrier until the next unit's)
        const bool ok = b + it < i_end;
        const int item = ok ? p.ws.bucket[(size_t)lo * p.E + b + it] : 0;
        const int64_t e = item / RS;
        // ---- this env's patched cells (act_kernel's decoding), then window q's four cells ----
        const uint4 cells = *reinterpret_cast<const uint4 *>(p.desc + e * NDESC);
        const uint32_t flags = p.desc[e * NDESC + 4];
        const bool reset = (flags & D_RESET) != 0;
        const int ac = ((flags >> (8 + k)) & 1u) ? p.apples[k] : -1;
        float v4[4];
#pragma unroll
        for (int u4 = 0; u4 < 4; ++u4) v4[u4] = map_at((4 * Y + 2 * (q >> 1) + (u4 >> 1)) * p.W + 4 * X + 2 * (q & 1) + (u4 & 1));
        {
            float av = (ac >= 0 ? map_at(ac) : 0.0f) + 9.0f;
            if (!reset && av == (float)(k + 1)) av = 1.0f;
            const uint32_t dw[4] = {cells.x, cells.y, cells.z, cells.w};
#pragma unroll
            for (int sl = 0; sl < NP; ++sl) {  // in slot order: a later slot on the same cell wins
                const int c = sl == 0 ? ac : (int)((dw[(sl - 1) >> 1] >> (16 * ((sl - 1) & 1))) & 0xFFFFu);
                const float v = sl == 0 ? av : agent_value(reset, sl - 1, k, c == ac, p.variant);
                const int y = c / p.W - 4 * Y - 2 * (q >> 1), x = c % p.W - 4 * X - 2 * (q & 1);
                const bool in = c >= 0 && (unsigned)y < 2u && (unsigned)x < 2u;
#pragma unroll
                for (int u4 = 0; u4 < 4; ++u4) v4[u4] = (in && 2 * y + x == u4) ? v : v4[u4];
            }
        }
        float a1[C1];
#pragma unroll
        for (int c = 0; c < C1; ++c) {
            float acc = s_b1[c];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) acc = fmaf(s_w1[c][u4], v4[u4], acc);
            a1[c] = fmaxf(acc, 0.0f);
        }
        float base[16];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) base[4 * t + r] = s_a2m[16 * t + 4 * q + r];
        float4 z[8];
        rare_mfma(a1, s_w2, s_wl, s_b2, base, lane, z);
        if (ok) {
            float4 *zo = reinterpret_cast<float4 *>(p.ws.rare_z + ((size_t)k * p.E * RS + item) * HID);
#pragma unroll
            for (int j = 0; j < 8; ++j) zo[4 * j + q] = z[j];
        }
    }
}

// ---- the CNN head on P x P egocentric windows (gw_patch_cnn_*; include/actor_ops.h) ------------
// The window of agent k centred on cell c differs from its BASE window B_c (the map under the
// window, -1 outside the grid, and the agent's usual own value vo_k at the centre) only at the
// patched cells.  gw_patch_cnn_prepare tabulates, per (agent, centre): a2b = conv-2 activations of
// B_c at every window position Q, and tbl = b + Linear-1(a2b).  Per step, wcnn_l1_kernel lists the
// positions where the actual window differs from B_c (a patched cell inside the window other than
// the centre holding vo_k); bucket_scan / wcnn_scatter file them as items (env, slot) into buckets
// keyed (agent, Q) in env order (a scan of per-block counts: no atomics); the persistent
// wcnn_rare_kernel recomputes each item's position and writes Wl[:, Q] . (a2 - a2b);
// act_kernel<H1, PW> sums tbl[centre] + those terms (slot order) and runs layers 2-3.
constexpr int RSW = MAXN + 1;   // recomputed positions per (env, agent): <= N + 1 patched cells
constexpr int WCG = 8;          // centres per wcnn_prep_base block
constexpr int WNQ = 16;         // positions per window (P <= 16)
inline CnnWs wcnn_ws_layout(float *base, int K, int NQ, int HW, int64_t E) {
    CnnWs w{};
    w.mlp = ws_layout(base, K);
    float *f = base + cnn_mlp_floats(K);
    w.wlt = f;        f += (int64_t)K * NQ * C2 * HID;
    w.wlj = f;        f += (int64_t)K * NQ * C2 * HID;
    w.a2map = f;      f += (int64_t)K * HW * NQ * C2;     // a2b [K][HW][NQ][64]
    w.table = f;      f += (int64_t)K * HW * HID;         // tbl [K][HW][128]
    w.w2t = f;        f += (int64_t)K * 4 * C2 * C1;
    w.road = reinterpret_cast<uint32_t *>(f);  f += 128;
    w.rare_z = f;     f += (int64_t)K * E * RSW * HID;
    w.rare_n = reinterpret_cast<int *>(f);    f += (int64_t)K * E;
    w.bucket_n = reinterpret_cast<int *>(f);  f += (int64_t)K * NQ;
    w.bucket = reinterpret_cast<int *>(f);    f += (int64_t)K * NQ * E;
    w.unit_off = reinterpret_cast<int *>(f);
    return w;
}
inline int64_t wcnn_ws_floats(int K, int NQ, int HW, int64_t E) {
    return (int64_t)(wcnn_ws_layout(nullptr, K, NQ, HW, E).unit_off - (int *)nullptr) + (int64_t)K * NQ + 1 +
           lists_floats(K * NQ, K, E, 256);
}
// the agent's own obs value in a non-reset step off its apple (agent_value(false, k, k, false))
__device__ __forceinline__ float own_value(int k, int variant) { return variant == 1 ? (float)(k + 1) : 1.0f; }

// block (centre group, k), 256 threads: a2b and tbl of WCG centres; block (0, k) also writes the
// window-major conv-2 weight and (k = 0) the road bitmask
__global__ void __launch_bounds__(256) wcnn_prep_base(CnnParams p) {
    const int k = blockIdx.y, tid = threadIdx.x, c0 = blockIdx.x * WCG;
    const int half = p.PW / 2, NF = p.P * C2;
    __shared__ float s_w2[C2 * C1 * 4];          // conv2_w [o][c][d], 32 KB
    __shared__ float s_w1[C1 * 4], s_b1[C1], s_b2[C2];
    __shared__ float s_a1[WNQ][4][C1];           // 8 KB
    __shared__ float s_a2[WCG][WNQ * C2];        // 32 KB
    for (int i = tid; i < C2 * C1 * 4; i += 256) s_w2[i] = p.net.conv2_w[(size_t)k * C2 * C1 * 4 + i];
    if (tid < C1 * 4) s_w1[tid] = p.net.conv1_w[k * C1 * 4 + tid];
    if (tid < C1) s_b1[tid] = p.net.conv1_b[k * C1 + tid];
    if (tid < C2) s_b2[tid] = p.net.conv2_b[k * C2 + tid];
    if (blockIdx.x == 0) {
        for (int i = tid; i < 4 * C2 * C1; i += 256) {
            const int d = i / (C2 * C1), o = (i / C1) % C2, c = i % C1;
            p.ws.w2t[(size_t)k * 4 * C2 * C1 + i] = p.net.conv2_w[((k * C2 + o) * C1 + c) * 4 + d];
        }
        if (k == 0 && tid < 128) {
            uint32_t bits = 0;
            for (int j = 0; j < 32; ++j) bits |= (32 * tid + j < p.HW && p.base[min(32 * tid + j, p.HW - 1)] == 0.0f) ? (1u << j) : 0u;
            p.ws.road[tid] = bits;
        }
    }
    const float vo = own_value(k, p.variant);
    __syncthreads();
    for (int ci = 0; ci < WCG; ++ci) {
        const int c = min(c0 + ci, p.HW - 1);   // (a trailing group repeats its last centre)
        const int cr = c / p.W, cc = c % p.W;
        for (int i = tid; i < p.P * 4 * C1; i += 256) {   // conv 1: (position, window d, channel)
            const int Q = i >> 7, d = (i >> 5) & 3, ch = i & 31, Y = Q / p.Wq, X = Q % p.Wq;
            float acc = s_b1[ch];
            for (int tap = 0; tap < 4; ++tap) {
                const int wr = 4 * Y + 2 * (d >> 1) + (tap >> 1), wc = 4 * X + 2 * (d & 1) + (tap & 1);
                const int r = cr - half + wr, col = cc - half + wc;
                const float v = (wr == half && wc == half) ? vo
                              : (r >= 0 && r < p.H && col >= 0 && col < p.W) ? p.base[r * p.W + col] : -1.0f;
                acc = fmaf(s_w1[ch * 4 + tap], v, acc);
            }
            s_a1[Q][d][ch] = fmaxf(acc, 0.0f);
        }
        __syncthreads();
        for (int i = tid; i < NF; i += 256) {              // conv 2: (position, channel o)
            const int Q = i >> 6, o = i & 63;
            float acc = s_b2[o];
            for (int ch = 0; ch < C1; ++ch)
#pragma unroll
                for (int d = 0; d < 4; ++d) acc = fmaf(s_w2[(o * C1 + ch) * 4 + d], s_a1[Q][d][ch], acc);
            const float a2 = fmaxf(acc, 0.0f);
            s_a2[ci][i] = a2;
            if (c0 + ci < p.HW) p.ws.a2map[((size_t)k * p.HW + c) * NF + i] = a2;
        }
        __syncthreads();
    }
    {   // tbl = b + Wl . a2b: thread (half h, feature j) takes centres 4h .. 4h + 3
        const int j = tid & (HID - 1), h = tid >> 7;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        const float *wl = p.ws.wlt + (size_t)k * NF * HID + j;
        for (int f = 0; f < NF; ++f) {
            const float w = wl[(size_t)f * HID];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = fmaf(w, s_a2[4 * h + i][f], acc[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = c0 + 4 * h + i;
            if (c < p.HW) p.ws.table[((size_t)k * p.HW + c) * HID + j] = p.net.lin1_b[k * HID + j] + acc[i];
        }
    }
}

// one thread per (env, agent): the positions where the window differs from its base window as a
// mask (slot = rank of the position in it; rare_n = their count) and the items per (position,
// block); bucket_scan scans the counts, wcnn_scatter fills the buckets
template <int NP>
__global__ void __launch_bounds__(256) wcnn_l1_kernel(CnnParams p, Lists lists) {
    __shared__ uint32_t s_road[128];
    __shared__ int s_cnt[4][WNQ];
    const int k = blockIdx.y, tid = threadIdx.x;
    const int64_t e = (int64_t)blockIdx.x * 256 + tid;
    const bool valid = e < p.E;
    if (tid < 128) s_road[tid] = p.ws.road[tid];
    __syncthreads();
    auto map_at = [&](int c) { return ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f; };
    const uint4 cells = valid ? *reinterpret_cast<const uint4 *>(p.desc + e * NDESC) : make_uint4(0, 0, 0, 0);
    const uint32_t flags = valid ? p.desc[e * NDESC + 4] : 0u;
    int pc[NP];
    float pv[NP];
    {
        const bool reset = (flags & D_RESET) != 0;
        const int ac = ((flags >> (8 + k)) & 1u) ? p.apples[k] : -1;
        float av = (ac >= 0 ? map_at(ac) : 0.0f) + 9.0f;
        if (!reset && av == (float)(k + 1)) av = 1.0f;
        pc[0] = ac;
        pv[0] = av;
        const uint32_t dw[4] = {cells.x, cells.y, cells.z, cells.w};
#pragma unroll
        for (int n = 0; n < NP - 1; ++n) {
            const int c = (int)((dw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
            pc[1 + n] = c;
            pv[1 + n] = agent_value(reset, n, k, c == ac, p.variant);
        }
    }
    const int ctr = (unsigned)pc[1 + k] < (unsigned)p.HW ? pc[1 + k] : 0;
    const int cr = ctr / p.W, cc = ctr % p.W, half = p.PW / 2;
    const float vo = own_value(k, p.variant);
    uint32_t qmask = 0;
    bool ctr_set = false;   // a patched cell on the centre (else the centre shows its map value)
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int c = pc[i];
        bool live = (unsigned)c < (unsigned)p.HW;
#pragma unroll
        for (int r = i + 1; r < NP; ++r) live = live && pc[r] != c;   // a later slot wins
        if (!live) continue;
        const int wr = c / p.W - cr + half, wc = c % p.W - cc + half;
        if ((unsigned)wr >= (unsigned)p.PW || (unsigned)wc >= (unsigned)p.PW) continue;
        const bool centre = c == ctr;
        ctr_set = ctr_set || centre;
        if (centre && pv[i] == vo) continue;
        qmask |= 1u << ((wr >> 2) * p.Wq + (wc >> 2));
    }
    if (!ctr_set && map_at(ctr) != vo) qmask |= 1u << ((half >> 2) * p.Wq + (half >> 2));
    if (!valid || (GW_AB(p.ab, 4))) qmask = 0;  // (bit 2, measurement only: decode, list nothing)
    if (valid) {
        p.ws.rare_n[(size_t)k * p.E + e] = __popc(qmask);
        lists.item[(size_t)k * p.E + e] = (int)qmask;
    }
    // items per (position, block): the waves' ballot counts summed in LDS (no global atomics:
    // nearly every item shares the centre's position, and same-address atomics serialise)
    const int wave = tid >> 6, lane = tid & 63;
    for (int Q = 0; Q < p.P; ++Q) {
        const uint64_t b = __ballot((qmask >> Q) & 1u);
        if (lane == 0) s_cnt[wave][Q] = __popcll(b);
    }
    __syncthreads();
    if (tid < p.P)
        lists.cnt[((size_t)k * p.P + tid) * lists.nblk + blockIdx.x] = s_cnt[0][tid] + s_cnt[1][tid] + s_cnt[2][tid] + s_cnt[3][tid];
}

// wcnn_l1_kernel with the listing folded in (round 5): a block of 256 threads takes LR_ENVS envs
// (LR_ENVS / 256 per thread), counts its items per position in LDS, claims each position's range
// of its bucket with ONE atomic add on the bucket's counter (64 per bucket and agent at 65,536
// envs instead of one per wave: same-address atomics serialise), and writes its items there.  An
// item's place inside its bucket then depends on the blocks' arrival order, but no result does:
// the rare kernel computes each item on its own and writes it to the item's (env, slot) row, which
// act_kernel sums in slot order.  The counters are zeroed by the act_kernel launch that follows
// (p.zero_n), after the rare kernel has read them.
// (512 envs per block: 8.2 us per launch at c4patch; 1024: 11.8, 256: 8.6 -- fewer envs per thread
// shorten the decode chain until the blocks' same-address bucket claims take over)
constexpr int LR_ENVS = 512;
template <int NP>
__device__ __forceinline__ void list_block(const CnnParams &p, int bx, int k) {
    constexpr int PER = LR_ENVS / 256;
    __shared__ uint32_t s_road[128];
    __shared__ int s_cnt[WNQ], s_base[WNQ];
    const int tid = threadIdx.x;
    if (tid < 128) s_road[tid] = p.ws.road[tid];
    if (tid < WNQ) s_cnt[tid] = 0;
    int64_t ev[PER];
    uint4 cells[PER];
    uint32_t flags[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {  // every descriptor load of the thread in flight together
        ev[r] = (int64_t)bx * LR_ENVS + r * 256 + tid;
        const bool valid = ev[r] < p.E;
        cells[r] = valid ? *reinterpret_cast<const uint4 *>(p.desc + ev[r] * NDESC) : make_uint4(0, 0, 0, 0);
        flags[r] = valid ? p.desc[ev[r] * NDESC + 4] : 0u;
    }
    __syncthreads();
    auto map_at = [&](int c) { return ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f; };
    const int half = p.PW / 2;
    const float vo = own_value(k, p.variant);
    uint32_t qm[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        int pc[NP];
        float pv[NP];
        {
            const bool reset = (flags[r] & D_RESET) != 0;
            const int ac = ((flags[r] >> (8 + k)) & 1u) ? p.apples[k] : -1;
            float av = (ac >= 0 ? map_at(ac) : 0.0f) + 9.0f;
            if (!reset && av == (float)(k + 1)) av = 1.0f;
            pc[0] = ac;
            pv[0] = av;
            const uint32_t dw[4] = {cells[r].x, cells[r].y, cells[r].z, cells[r].w};
#pragma unroll
            for (int n = 0; n < NP - 1; ++n) {
                const int c = (int)((dw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                pc[1 + n] = c;
                pv[1 + n] = agent_value(reset, n, k, c == ac, p.variant);
            }
        }
        const int ctr = (unsigned)pc[1 + k] < (unsigned)p.HW ? pc[1 + k] : 0;
        const int cr = ctr / p.W, cc = ctr % p.W;
        uint32_t qmask = 0;
        bool ctr_set = false;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int c = pc[i];
            bool live = (unsigned)c < (unsigned)p.HW;
#pragma unroll
            for (int q = i + 1; q < NP; ++q) live = live && pc[q] != c;  // a later slot wins
            if (!live) continue;
            const int wr = c / p.W - cr + half, wc = c % p.W - cc + half;
            if ((unsigned)wr >= (unsigned)p.PW || (unsigned)wc >= (unsigned)p.PW) continue;
            const bool centre = c == ctr;
            ctr_set = ctr_set || centre;
            if (centre && pv[i] == vo) continue;
            qmask |= 1u << ((wr >> 2) * p.Wq + (wc >> 2));
        }
        if (!ctr_set && map_at(ctr) != vo) qmask |= 1u << ((half >> 2) * p.Wq + (half >> 2));
        const bool valid = ev[r] < p.E;
        if (!valid || (GW_AB(p.ab, 4))) qmask = 0;
        if (valid) p.ws.rare_n[(size_t)k * p.E + ev[r]] = __popc(qmask);
        qm[r] = qmask;
        for (uint32_t m = qmask; m; m &= m - 1) atomicAdd(&s_cnt[__ffs(m) - 1], 1);  // LDS
    }
    __syncthreads();
    if (tid < p.P && s_cnt[tid]) s_base[tid] = atomicAdd(&p.ws.bucket_n[k * p.P + tid], s_cnt[tid]);
    if (tid < WNQ) s_cnt[tid] = 0;  // reused as the block's fill counts
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        for (uint32_t m = qm[r]; m; m &= m - 1) {
            const int Q = __ffs(m) - 1;
            const int pos = s_base[Q] + atomicAdd(&s_cnt[Q], 1);
            p.ws.bucket[((size_t)k * p.P + Q) * p.E + pos] = (int)(ev[r] * RSW + __popc(qm[r] & ((1u << Q) - 1u)));
        }
    }
}
template <int NP>
__global__ void __launch_bounds__(256) wcnn_list_kernel(CnnParams p) {
    list_block<NP>(p, blockIdx.x, blockIdx.y);
}

// gw_patch_cnn_write_list: the step's windows (the row writer's blocks, window_rows.h) and the
// listing of the next act's recomputed positions in ONE launch -- both read only the step's
// descriptors; the listing's blocks first (a short chain), the writer's HBM stream beside them
template <int NP, int MAXW>
__global__ void __launch_bounds__(256, 4) rows_list_kernel(gw::PatchArgs a, CnnParams p, uint32_t nlist) {
    __shared__ __attribute__((aligned(16))) float4 s_rows[4][64 * (MAXW / 4)];
    if (blockIdx.x < nlist) {
        list_block<NP>(p, blockIdx.x, blockIdx.y);
        return;
    }
    gwrows::rows_block<NP, MAXW, 2>(a, blockIdx.x - nlist, blockIdx.y, s_rows);
}

// one 64-thread block per bucket: the offsets of the layer-1 blocks' items in the bucket (a wave
// scan over the blocks in order) and the bucket's size.  All of a lane's counts are loaded before
// the scan (one memory round trip: beside a concurrent window writer every load waits behind its
// stores).  The rare kernels cut the buckets into units themselves (block_unit_offsets): no
// cross-block step here, so no arrival counter and no device-scope fence (an L2 writeback per
// block on gfx950).  One-wave blocks find a CU slot beside the window writer (a 1024-thread block
// waits for 16 free wave slots on one CU).
constexpr int SCAN_PRE = 8;  // counts per lane loaded up front (nblk <= 512; more: a second pass)
__global__ void __launch_bounds__(64) bucket_scan(CnnParams p, Lists lists) {
    const int lane = threadIdx.x, b = blockIdx.x;
    const int *cnt = lists.cnt + (size_t)b * lists.nblk;
    int *off = lists.off + (size_t)b * lists.nblk;
    int run = 0;
    for (int c0 = 0; c0 < lists.nblk; c0 += 64 * SCAN_PRE) {
        int v[SCAN_PRE];
#pragma unroll
        for (int j = 0; j < SCAN_PRE; ++j) {
            const int i = c0 + 64 * j + lane;
            v[j] = i < lists.nblk ? cnt[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < SCAN_PRE; ++j) {
            const int i = c0 + 64 * j + lane;
            int incl = v[j];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int o = __shfl_up(incl, d, 64);
                if (lane >= d) incl += o;
            }
            if (i < lists.nblk) off[i] = run + incl - v[j];
            run += __shfl(incl, 63, 64);
        }
    }
    if (lane == 0) p.ws.bucket_n[b] = run;
}


// fills the buckets in (block, wave, lane) order: item (e RSW + slot), slot = the position's rank
// in the (env, agent)'s mask
__global__ void __launch_bounds__(256) wcnn_scatter(CnnParams p, Lists lists) {
    __shared__ int s_cnt[4][WNQ];
    const int k = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t e = (int64_t)blockIdx.x * 256 + tid;
    const uint32_t qmask = e < p.E ? (uint32_t)lists.item[(size_t)k * p.E + e] : 0u;
    const uint64_t below = (1ull << lane) - 1;
    for (int Q = 0; Q < p.P; ++Q) {
        const uint64_t b = __ballot((qmask >> Q) & 1u);
        if (lane == 0) s_cnt[wave][Q] = __popcll(b);
    }
    __syncthreads();
    for (int Q = 0; Q < p.P; ++Q) {
        const bool has = (qmask >> Q) & 1u;
        const uint64_t b = __ballot(has);
        if (!has) continue;
        int pos = lists.off[((size_t)k * p.P + Q) * lists.nblk + blockIdx.x] + __popcll(b & below);
        for (int w = 0; w < wave; ++w) pos += s_cnt[w][Q];
        p.ws.bucket[((size_t)k * p.P + Q) * p.E + pos] = (int)(e * RSW + __popc(qmask & ((1u << Q) - 1u)));
    }
}

// cnn_rare_kernel over window positions: per unit (agent k, position Q) the Linear-1 block in LDS;
// lane (item it, quarter q) rebuilds conv-1 window q of Q from the item's descriptor (map under
// the window, -1 outside, the patched cells); rare_mfma against the base window's activations a2b.
// (round 5) units of 64 items on 4-wave blocks, two blocks per CU: ~500 units at c4patch's ~33k
// items for 512 resident blocks, where 128-item units on 256 eight-wave blocks left ~10 % of the
// blocks two units (the kernel's span: two units' staging + compute)
constexpr int WR_WAVES = WR_WAVES_C, WR_ITEMS = 16 * WR_WAVES, WR_BLOCKS = 512;
// buckets (agent, window position): K <= 8 x P <= 16.  The unit table sized for these (not the
// full-grid kernel's 2,048) keeps a block at ~73 KB of LDS: two blocks per CU (at 81 KB only one
// fitted, and half the grid waited for the first half: block starts p50 6.7 us, p75 14 us)
constexpr int WR_MAX_NB = GW_MAX_AGENTS * 16;
template <int NP>
__global__ void __launch_bounds__(64 * WR_WAVES, 2) wcnn_rare_kernel(CnnParams p) {  // (<= 256 VGPRs: two blocks per CU)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int it = lane & 15, q = lane >> 4;
    const int nb = p.K * p.P, half = p.PW / 2;
    __shared__ __attribute__((aligned(16))) float s_w2[RARE_LDS_W2];   // 36 KB
    __shared__ __attribute__((aligned(16))) float s_wl[RARE_LDS_WL];   // 34 KB
    __shared__ float s_w1[C1][4], s_b1[C1], s_b2[C2];
    __shared__ uint32_t s_road[128];
    __shared__ int s_uo[WR_MAX_NB + 1], s_wt[WR_WAVES];
    RSTAMP(p, 0);
    if (tid < 128) s_road[tid] = p.ws.road[tid];
    block_unit_offsets<WR_WAVES, WR_ITEMS>(p.ws.bucket_n, nb, s_uo, s_wt);
    const int nunits = s_uo[nb];
    RSTAMP(p, 1);
    int nu = 0;
    int staged_k = -1, staged_Q = -1;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x, ++nu) {
        int lo = 0, hi = nb;  // the bucket holding unit u: unit_off[lo] <= u < unit_off[lo + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_uo[mid] <= u) lo = mid; else hi = mid;
        }
        const int k = lo / p.P, Q = lo % p.P;
        const int n = p.ws.bucket_n[lo];
        const int i_begin = (u - s_uo[lo]) * WR_ITEMS, i_end = min(n, i_begin + WR_ITEMS);
        __syncthreads();  // the previous unit is done with the LDS images
        if (k != staged_k) {
            stage_w2(s_w2, p.ws.w2t + (size_t)k * 4 * C2 * C1, tid, 64 * WR_WAVES);
            if (tid < C1 * 4) (&s_w1[0][0])[tid] = p.net.conv1_w[k * C1 * 4 + tid];
            if (tid < C1) s_b1[tid] = p.net.conv1_b[k * C1 + tid];
            if (tid < C2) s_b2[tid] = p.net.conv2_b[k * C2 + tid];
        }
        if (k != staged_k || Q != staged_Q) stage_wl4(s_wl, p.ws.wlj + ((size_t)k * p.P + Q) * C2 * HID, tid);
        staged_k = k;
        staged_Q = Q;
        __syncthreads();
        if (nu == 0) RSTAMP(p, 2);
        auto map_at = [&](int c) { return ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f; };
        const int Y = Q / p.Wq, X = Q % p.Wq;
        const int b = i_begin + 16 * wave;
        if (b >= i_end) continue;  // (wave-uniform; no barrier until the next unit's)
        const bool ok = b + it < i_end;
        const int item = ok ? p.ws.bucket[(size_t)lo * p.E + b + it] : 0;
        const int64_t e = item / RSW;
        const uint4 cells = *reinterpret_cast<const uint4 *>(p.desc + e * NDESC);
        const uint32_t flags = p.desc[e * NDESC + 4];
        const bool reset = (flags & D_RESET) != 0;
        const int ac = ((flags >> (8 + k)) & 1u) ? p.apples[k] : -1;
        const uint32_t dw[4] = {cells.x, cells.y, cells.z, cells.w};
        const int own = (int)((dw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        const int ctr = (unsigned)own < (unsigned)p.HW ? own : 0;
        // the base window's activations of channels 16t + 4q + r (in flight during conv 1)
        const float4 *ab = reinterpret_cast<const float4 *>(p.ws.a2map + (((size_t)k * p.HW + ctr) * p.P + Q) * C2 + 4 * q);
        float4 bq[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) bq[t] = ab[4 * t];
        // grid row / col of window q's top-left cell
        const int r0 = ctr / p.W - half + 4 * Y + 2 * (q >> 1), c0 = ctr % p.W - half + 4 * X + 2 * (q & 1);
        float v4[4];
#pragma unroll
        for (int u4 = 0; u4 < 4; ++u4) {
            const int r = r0 + (u4 >> 1), c = c0 + (u4 & 1);
            v4[u4] = (r >= 0 && r < p.H && c >= 0 && c < p.W) ? map_at(r * p.W + c) : -1.0f;
        }
        {
            float av = (ac >= 0 ? map_at(ac) : 0.0f) + 9.0f;
            if (!reset && av == (float)(k + 1)) av = 1.0f;
#pragma unroll
            for (int sl = 0; sl < NP; ++sl) {  // in slot order: a later slot on the same cell wins
                const int c = sl == 0 ? ac : (int)((dw[(sl - 1) >> 1] >> (16 * ((sl - 1) & 1))) & 0xFFFFu);
                const float v = sl == 0 ? av : agent_value(reset, sl - 1, k, c == ac, p.variant);
                const bool on = (unsigned)c < (unsigned)p.HW;
                const int y = (on ? c / p.W : -8) - r0, x = (on ? c % p.W : -8) - c0;
                const bool in = on && (unsigned)y < 2u && (unsigned)x < 2u;
#pragma unroll
                for (int u4 = 0; u4 < 4; ++u4) v4[u4] = (in && 2 * y + x == u4) ? v : v4[u4];
            }
        }
        float a1[C1];
#pragma unroll
        for (int c = 0; c < C1; ++c) {
            float acc = s_b1[c];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) acc = fmaf(s_w1[c][u4], v4[u4], acc);
            a1[c] = fmaxf(acc, 0.0f);
        }
        float base[16];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            base[4 * t + 0] = bq[t].x;
            base[4 * t + 1] = bq[t].y;
            base[4 * t + 2] = bq[t].z;
            base[4 * t + 3] = bq[t].w;
        }
        if (nu == 0) RSTAMP(p, 3);
        float4 z[8];
        rare_mfma(a1, s_w2, s_wl, s_b2, base, lane, z);
        if (nu == 0) RSTAMP(p, 4);
        if (ok) {
            float4 *zo = reinterpret_cast<float4 *>(p.ws.rare_z + ((size_t)k * p.E * RSW + item) * HID);
#pragma unroll
            for (int j = 0; j < 8; ++j) zo[4 * j + q] = z[j];
        }
    }
    if (p.stamp && tid == 0) p.stamp[(int64_t)blockIdx.x * 8 + 6] = (unsigned long long)nu;
    RSTAMP(p, 5);
}

gw_status err(gw_status s, const std::string &msg) {
    gw_set_last_error(msg.c_str());
    return s;
}

gw_status check_net(const gw_obs_source &src, const gw_mlp_actors *net, const char *who, int P = 0) {
    const std::string w(who);
    if (net->K != src.K) return err(GW_ERR_ARG, w + ": net K != env K");
    if (P > 0 && (P > 129 || net->in_dim != P * P)) return err(GW_ERR_ARG, w + ": need 1 <= P <= 129 and in_dim == P*P");
    if (P <= 0 && net->in_dim != src.H * src.W) return err(GW_ERR_ARG, w + ": in_dim != H*W");
    if (src.H * src.W > 128 * 32) return err(GW_ERR_ARG, w + ": H*W must be <= 4096");
    if (net->hidden != HID || net->n_actions != NA) return err(GW_ERR_ARG, w + ": only hidden 128 and 9 actions are fused");
    if (!net->w1 || !net->b1 || !net->w2 || !net->b2 || !net->w3 || !net->b3 ||
        (net->layer_norm && (!net->ln1_w || !net->ln1_b || !net->ln2_w || !net->ln2_b)))
        return err(GW_ERR_ARG, w + ": null parameter");
    if (reinterpret_cast<uintptr_t>(net->w1) & 15u) return err(GW_ERR_ARG, w + ": w1 must be 16-byte aligned");
    return GW_OK;
}


gw_status check_cnn(const gw_obs_source &src, const gw_cnn_actors *net, const char *who) {
    const std::string w(who);
    if (net->K != src.K) return err(GW_ERR_ARG, w + ": net K != env K");
    if (net->H != src.H || net->W != src.W) return err(GW_ERR_ARG, w + ": net H, W != env H, W");
    if (net->H % 4 || net->W % 4 || net->H * net->W > 128 * 32)
        return err(GW_ERR_ARG, w + ": H and W must be multiples of 4, H*W <= 4096");
    if (net->c1 != C1 || net->c2 != C2 || net->hidden != HID || net->n_actions != NA)
        return err(GW_ERR_ARG, w + ": only channels 32-64, hidden 128 and 9 actions are fused");
    if (!net->conv1_w || !net->conv1_b || !net->conv2_w || !net->conv2_b || !net->lin1_w || !net->lin1_b ||
        !net->w2 || !net->b2 || !net->w3 || !net->b3)
        return err(GW_ERR_ARG, w + ": null parameter");
    return GW_OK;
}

CnnParams cnn_params(const gw_obs_source &src, const gw_cnn_actors *net, float *ws) {
    CnnParams p;
    p.net = *net;
    p.H = src.H;
    p.W = src.W;
    p.HW = src.H * src.W;
    p.Wq = src.W / 4;
    p.P = (src.H / 4) * p.Wq;
    p.ws = cnn_ws_layout(ws, src.K, p.P, src.E);
    p.base = src.base;
    p.desc = src.desc;
    p.E = src.E;
    p.N = src.N;
    p.K = src.K;
    p.variant = src.variant;
    p.PW = 0;
    for (int k = 0; k < MAXN; ++k) p.apples[k] = src.apples[k];
    const char *ab = GW_MEASURE_ENV("GW_CNN_AB");
    p.ab = ab ? std::atoi(ab) : 0;
    return p;
}

gw_mlp_actors cnn_tail(const gw_cnn_actors *net) {  // layers 2-3 as act_kernel's net (no LayerNorm)
    gw_mlp_actors m{};
    m.K = net->K;
    m.in_dim = net->H * net->W;
    m.hidden = HID;
    m.n_actions = NA;
    m.layer_norm = 0;
    m.w1 = net->lin1_w;
    m.b1 = net->lin1_b;
    m.w2 = net->w2;
    m.b2 = net->b2;
    m.w3 = net->w3;
    m.b3 = net->b3;
    return m;
}

}  // namespace

extern "C" {

// measurement only (not part of the ABI): the stamps of the last GW_ACT_AB & 8 launch
int gw_actor_debug_clocks(unsigned long long *out, int nblocks) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_act_clk), sizeof(unsigned long long) * 16 * std::min(nblocks, 1024)) ==
                   hipSuccess ? 0 : -1;
}

int64_t gw_actor_workspace_floats(int32_t in_dim, int32_t K) {
    return (int64_t)K * (HID + W2IMG + W3IMG + W2BIMG + (int64_t)((in_dim + 31) / 32) * HID);
}

gw_status gw_actor_prepare(void *env, const gw_mlp_actors *net, float *ws, void *stream) {
    if (!env || !net || !ws) return err(GW_ERR_ARG, "gw_actor_prepare: null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, "gw_actor_prepare: ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_net(src, net, "gw_actor_prepare")) != GW_OK) return st;
    PrepParams p;
    p.net = *net;
    p.HW = src.H * src.W;
    p.nslices = (p.HW + 31) / 32;
    p.ws = ws_layout(ws, src.K);
    p.base = src.base;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(prep_slices, dim3(p.nslices, src.K), dim3(HID), 0, s, p);
    hipLaunchKernelGGL(prep_images, dim3(64, src.K), dim3(256), 0, s, p);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_actor_prepare: ") + hipGetErrorString(e));
    return GW_OK;
}

gw_status gw_actor_images_view(float *ws, int32_t in_dim, int32_t K, gw_actor_images *out) {
    if (!ws || !out || in_dim < 1 || K < 1 || K > MAXN) return err(GW_ERR_ARG, "gw_actor_images_view: bad argument");
    const Ws wl = ws_layout(ws, K);
    out->part = wl.part;
    out->nslices = (in_dim + 31) / 32;
    out->w2img = reinterpret_cast<float *>(wl.w2);
    out->w2bimg = reinterpret_cast<void *>(wl.w2b);
    out->w3img = reinterpret_cast<float *>(wl.w3);
    return GW_OK;
}

}  // extern "C"

namespace {
// gw_actor_act (P = 0) and gw_patch_actor_act (P > 0: the P x P window variant)
gw_status actor_act(const char *who, void *env, int32_t P, const gw_mlp_actors *net, const float *ws, int training,
                    float tau, uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                    const uint16_t *mask,
                    int32_t *actions, float *probs, float *logits, void *stream) {
    const std::string w(who);
    if (!env || !net || !ws || !actions || !probs) return err(GW_ERR_ARG, w + ": null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, w + ": ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_net(src, net, who, P)) != GW_OK) return st;
    if (!(tau > 0.0f)) return err(GW_ERR_ARG, w + ": tau must be > 0");
    ActParams p{};
    p.net = *net;
    const Ws wl = ws_layout(const_cast<float *>(ws), src.K);
    p.c1 = wl.c1;
    p.w2img = wl.w2;
    p.w3img = wl.w3;
    p.w2bimg = wl.w2b;
    if (P == 0) {  // c1 from the row slices (gw_actor_prepare's or a learner's: gw_actor_images)
        p.c1_part = wl.part;
        p.c1_nslices = (src.H * src.W + 31) / 32;
    }
    p.desc = src.desc;
    p.base = src.base;
    p.mask = mask;
    p.uniform = uniform;
    p.h1 = nullptr;
    p.rare_z = nullptr;
    p.rare_n = nullptr;
    p.actions = actions;
    p.probs = probs;
    p.logits = logits;
    p.E = src.E;
    p.env_offset = src.env_offset;
    p.N = src.N;
    p.K = src.K;
    p.HW = src.H * src.W;
    p.W = src.W;
    p.P = P;
    p.in_dim = P > 0 ? P * P : p.HW;
    p.tbl = P > 0 ? patch_table(const_cast<float *>(ws), src.K) : nullptr;
    p.variant = src.variant;
    p.training = training ? 1 : 0;
    p.tau = tau;
    p.key0 = (uint32_t)seed;
    p.key1 = (uint32_t)(seed >> 32);
    p.ctr0 = (uint32_t)counter;
    p.ctr1 = (uint32_t)(counter >> 32);
    p.ctr_dev = counter_dev;
    for (int k = 0; k < MAXN; ++k) p.apples[k] = src.apples[k];
    const char *ab = GW_MEASURE_ENV("GW_ACT_AB");
    p.ab = ab ? std::atoi(ab) : 0;
    const int64_t tiles = (src.E + TILE - 1) / TILE;
    p.tiles = (int)tiles;
    // GW_ACT_V (A/B): 4 (default) = one 16-wave block per CU, layer 2 as bf16x3 MFMA products;
    // 2 = the same with f32 MFMA (exact products); 0 = two 8-wave blocks per CU, f32 MFMA
    const char *av = std::getenv("GW_ACT_V");
    const int v = P > 0 ? 4 : (av ? std::atoi(av) : 4);
    // small env counts (C2: 4,096 envs = 256 tiles per agent): 16-wave blocks would leave most
    // CUs idle with 4 waves per SIMD each doing one tile; 4-wave blocks spread the same tiles over
    // 4x the CUs (one wave per SIMD).  GW_ACT_WAVES=16|12|8|4 forces the block's waves
    // (result-neutral, tests/test_actor_ops.py): 12 / 8 leave a quarter / half of each SIMD's
    // VGPRs to co-resident kernels (the rollout's obs writer)
    const char *aw = std::getenv("GW_ACT_WAVES");
    const int awv = aw ? std::atoi(aw) : 0;
    const bool small = P == 0 && v == 4 && (aw ? awv == 4 : (tiles + 15) / 16 < std::max(1, 256 / src.K) / 2);
    const int waves = v == 0 ? 8 : small ? 4 : (P == 0 && v == 4 && (awv == 12 || awv == 8)) ? awv : 16;
    const int resident = v == 0 ? 512 : 256;
    const int64_t want = (tiles + waves - 1) / waves;
    const int per_agent = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(1, resident / src.K)));
    const dim3 grid(per_agent, src.K), block(64 * waves);
    hipStream_t s = static_cast<hipStream_t>(stream);
    gwprof::Span span(env, GW_SPAN_ACT);
#define ACT_LAUNCH(NP)                                                                   \
    do {                                                                                 \
        if (P > 0)                                                                       \
            gwprof::launch(act_kernel<NP, 16, true, false, true>, grid, block, 0, s, p); \
        else if (v == 0)                                                                 \
            gwprof::launch(act_kernel<NP, 8>, grid, block, 0, s, p);                     \
        else if (v == 4 && small)                                                        \
            gwprof::launch(act_kernel<NP, 4, true>, grid, block, 0, s, p);               \
        else if (v == 4 && waves == 12)                                                  \
            gwprof::launch(act_kernel_lean<NP, 12>, grid, block, 0, s, p);               \
        else if (v == 4 && waves == 8)                                                   \
            gwprof::launch(act_kernel_lean<NP, 8>, grid, block, 0, s, p);                \
        else if (v == 4)                                                                 \
            gwprof::launch(act_kernel<NP, 16, true>, grid, block, 0, s, p);              \
        else                                                                             \
            gwprof::launch(act_kernel<NP, 16>, grid, block, 0, s, p);                    \
    } while (0)
    switch (src.N) {
        case 1: ACT_LAUNCH(2); break;
        case 2: ACT_LAUNCH(3); break;
        case 3: ACT_LAUNCH(4); break;
        case 4: ACT_LAUNCH(5); break;
        case 5: ACT_LAUNCH(6); break;
        case 6: ACT_LAUNCH(7); break;
        case 7: ACT_LAUNCH(8); break;
        case 8: ACT_LAUNCH(9); break;
        default: return err(GW_ERR_ARG, w + ": N out of range");
    }
#undef ACT_LAUNCH
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, w + ": " + hipGetErrorString(e));
    return GW_OK;
}
}  // namespace

extern "C" {

gw_status gw_actor_act(void *env, const gw_mlp_actors *net, const float *ws, int training, float tau, uint64_t seed,
                       uint64_t counter, const int64_t *counter_dev, const float *uniform, const uint16_t *mask,
                       int32_t *actions, float *probs,
                       float *logits, void *stream) {
    return actor_act("gw_actor_act", env, 0, net, ws, training, tau, seed, counter, counter_dev, uniform, mask, actions, probs,
                     logits, stream);
}

int64_t gw_patch_actor_workspace_floats(int32_t P, int32_t H, int32_t W, int32_t K) {
    (void)P;
    return (int64_t)K * (HID + W2IMG + W3IMG + W2BIMG) + (int64_t)K * H * W * HID;
}

gw_status gw_patch_actor_prepare(void *env, int32_t P, const gw_mlp_actors *net, float *ws, void *stream) {
    if (!env || !net || !ws) return err(GW_ERR_ARG, "gw_patch_actor_prepare: null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, "gw_patch_actor_prepare: ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_net(src, net, "gw_patch_actor_prepare", P)) != GW_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    TblParams tp;
    tp.w1 = net->w1;
    tp.b1 = net->b1;
    tp.base = src.base;
    tp.tbl = patch_table(ws, src.K);
    tp.H = src.H;
    tp.W = src.W;
    tp.P = P;
    hipLaunchKernelGGL(prep_patch_table, dim3(src.H * src.W, src.K), dim3(HID), 0, s, tp);
    PrepParams pp;  // the layer-2/3 MFMA images (prep_images; nslices 0: c1 = b1, unused)
    pp.net = *net;
    pp.HW = P * P;
    pp.nslices = 0;
    pp.ws = ws_layout(ws, src.K);
    pp.base = src.base;
    hipLaunchKernelGGL(prep_images, dim3(64, src.K), dim3(256), 0, s, pp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_patch_actor_prepare: ") + hipGetErrorString(e));
    return GW_OK;
}

gw_status gw_patch_actor_act(void *env, int32_t P, const gw_mlp_actors *net, const float *ws, int training, float tau,
                             uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                             const uint16_t *mask,
                             int32_t *actions, float *probs, float *logits, void *stream) {
    if (P < 1) return err(GW_ERR_ARG, "gw_patch_actor_act: P must be >= 1");
    return actor_act("gw_patch_actor_act", env, P, net, ws, training, tau, seed, counter, counter_dev, uniform, mask, actions,
                     probs, logits, stream);
}


int64_t gw_cnn_workspace_floats(int32_t H, int32_t W, int32_t K, int64_t E) {
    return cnn_ws_floats(K, (H / 4) * (W / 4), E);
}

gw_status gw_cnn_prepare(void *env, const gw_cnn_actors *net, float *ws, void *stream) {
    if (!env || !net || !ws) return err(GW_ERR_ARG, "gw_cnn_prepare: null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, "gw_cnn_prepare: ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_cnn(src, net, "gw_cnn_prepare")) != GW_OK) return st;
    const CnnParams p = cnn_params(src, net, ws);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(cnn_prep_wlt, dim3(2048), dim3(256), 0, s, p);
    hipLaunchKernelGGL(cnn_prep_map, dim3(p.P, src.K), dim3(128), 0, s, p);
    hipLaunchKernelGGL(cnn_prep_zpart, dim3(p.P, src.K), dim3(128), 0, s, p);
    hipLaunchKernelGGL(cnn_prep_zmap, dim3(src.K), dim3(128), 0, s, p);
    hipLaunchKernelGGL(cnn_prep_table, dim3(p.P, src.K), dim3(256), 0, s, p);
    {  // (the lists' spare counter word starts at 0)
        const Lists l = lists_at(p.ws.unit_off, src.K * p.P, src.K, src.E, L1_ENVS);
        if (hipMemsetAsync(l.ctr, 0, sizeof(int), s) != hipSuccess) return err(GW_ERR_HIP, "gw_cnn_prepare: memset");
    }
    PrepParams pp;  // the layer-2/3 MFMA images (prep_images; nslices 0: c1 is rewritten below)
    pp.net = cnn_tail(net);
    pp.HW = p.HW;
    pp.nslices = 0;
    pp.ws = p.ws.mlp;
    pp.base = src.base;
    hipLaunchKernelGGL(prep_images, dim3(64, src.K), dim3(256), 0, s, pp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_cnn_prepare: ") + hipGetErrorString(e));
    return GW_OK;
}

gw_status gw_cnn_act(void *env, const gw_cnn_actors *net, const float *ws, int training, float tau, uint64_t seed,
                     uint64_t counter, const int64_t *counter_dev, const float *uniform, const uint16_t *mask,
                     int32_t *actions, float *probs,
                     float *logits, void *stream) {
    if (!env || !net || !ws || !actions || !probs) return err(GW_ERR_ARG, "gw_cnn_act: null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, "gw_cnn_act: ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_cnn(src, net, "gw_cnn_act")) != GW_OK) return st;
    if (!(tau > 0.0f)) return err(GW_ERR_ARG, "gw_cnn_act: tau must be > 0");
    const CnnParams cp = cnn_params(src, net, const_cast<float *>(ws));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t tiles = (src.E + TILE - 1) / TILE;
    const Lists lists = lists_at(cp.ws.unit_off, src.K * cp.P, src.K, src.E, L1_ENVS);
    const dim3 lgrid((unsigned)lists.nblk, src.K);
    {
        gwprof::Span span(env, GW_SPAN_CNN_L1);
        switch (src.N) {
            case 1: gwprof::launch(cnn_l1_kernel<2>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 2: gwprof::launch(cnn_l1_kernel<3>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 3: gwprof::launch(cnn_l1_kernel<4>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 4: gwprof::launch(cnn_l1_kernel<5>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 5: gwprof::launch(cnn_l1_kernel<6>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 6: gwprof::launch(cnn_l1_kernel<7>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 7: gwprof::launch(cnn_l1_kernel<8>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            case 8: gwprof::launch(cnn_l1_kernel<9>, lgrid, dim3(64 * L1_WAVES), 0, s, cp, lists); break;
            default: return err(GW_ERR_ARG, "gw_cnn_act: N out of range");
        }
    }
    if (src.K * cp.P > RARE_MAX_NB) return err(GW_ERR_ARG, "gw_cnn_act: K x conv-2 positions above the rare kernels' table");
    {
        gwprof::Span span(env, GW_SPAN_CNN_LIST);
        gwprof::launch(bucket_scan, dim3(src.K * cp.P), dim3(64), 0, s, cp, lists);
        gwprof::launch(cnn_scatter, lgrid, dim3(L1_ENVS), 0, s, cp, lists);
    }
#define RARE(NP) gwprof::launch(cnn_rare_kernel<NP>, dim3(RARE_BLOCKS), dim3(64 * RARE_WAVES), 0, s, cp)
    {
        gwprof::Span span(env, GW_SPAN_CNN_RARE);
        switch (src.N) {
            case 1: RARE(2); break;
            case 2: RARE(3); break;
            case 3: RARE(4); break;
            case 4: RARE(5); break;
            case 5: RARE(6); break;
            case 6: RARE(7); break;
            case 7: RARE(8); break;
            default: RARE(9); break;
        }
    }
#undef RARE
    ActParams p{};
    p.net = cnn_tail(net);
    p.c1 = cp.ws.mlp.c1;
    p.w2img = cp.ws.mlp.w2;
    p.w3img = cp.ws.mlp.w3;
    p.w2bimg = cp.ws.mlp.w2b;
    p.desc = src.desc;
    p.base = src.base;
    p.mask = mask;
    p.uniform = uniform;
    p.h1 = cp.ws.h1;
    p.rare_z = cp.ws.rare_z;
    p.rare_n = cp.ws.rare_n;
    p.actions = actions;
    p.probs = probs;
    p.logits = logits;
    p.E = src.E;
    p.env_offset = src.env_offset;
    p.N = src.N;
    p.K = src.K;
    p.HW = src.H * src.W;
    p.W = src.W;
    p.P = 0;
    p.in_dim = p.HW;
    p.tbl = nullptr;
    p.variant = src.variant;
    p.training = training ? 1 : 0;
    p.tau = tau;
    p.key0 = (uint32_t)seed;
    p.key1 = (uint32_t)(seed >> 32);
    p.ctr0 = (uint32_t)counter;
    p.ctr1 = (uint32_t)(counter >> 32);
    p.ctr_dev = counter_dev;
    for (int k = 0; k < MAXN; ++k) p.apples[k] = src.apples[k];
    p.ab = 0;
    p.tiles = (int)tiles;
    const int64_t want = (tiles + 15) / 16;
    const int per_agent = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(1, 256 / src.K)));
    {
        gwprof::Span span(env, GW_SPAN_ACT);
        gwprof::launch(act_kernel<2, 16, true, true>, dim3(per_agent, src.K), dim3(1024), 0, s, p);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_cnn_act: ") + hipGetErrorString(e));
    return GW_OK;
}

int64_t gw_patch_cnn_workspace_floats(int32_t P, int32_t H, int32_t W, int32_t K, int64_t E) {
    const int NQ = (P / 4) * (P / 4);
    return wcnn_ws_floats(K, NQ, H * W, E);
}

}  // extern "C"

namespace {
gw_status check_patch_cnn(const gw_obs_source &src, int32_t P, const gw_cnn_actors *net, const char *who) {
    const std::string w(who);
    if (P < 4 || P > 16 || P % 4) return err(GW_ERR_ARG, w + ": P must be 4, 8, 12 or 16");
    if (net->K != src.K) return err(GW_ERR_ARG, w + ": net K != env K");
    if (net->H != P || net->W != P) return err(GW_ERR_ARG, w + ": net H, W != P");
    if (src.H * src.W > 128 * 32) return err(GW_ERR_ARG, w + ": H*W must be <= 4096");
    if (net->c1 != C1 || net->c2 != C2 || net->hidden != HID || net->n_actions != NA)
        return err(GW_ERR_ARG, w + ": only channels 32-64, hidden 128 and 9 actions are fused");
    if (!net->conv1_w || !net->conv1_b || !net->conv2_w || !net->conv2_b || !net->lin1_w || !net->lin1_b ||
        !net->w2 || !net->b2 || !net->w3 || !net->b3)
        return err(GW_ERR_ARG, w + ": null parameter");
    return GW_OK;
}
CnnParams wcnn_params(const gw_obs_source &src, int32_t P, const gw_cnn_actors *net, float *ws) {
    CnnParams p = cnn_params(src, net, ws);   // (its full-grid layout is replaced below)
    p.PW = P;
    p.Wq = P / 4;
    p.P = p.Wq * p.Wq;
    p.ws = wcnn_ws_layout(ws, src.K, p.P, p.HW, src.E);
    return p;
}
}  // namespace

extern "C" {

gw_status gw_patch_cnn_prepare(void *env, int32_t P, const gw_cnn_actors *net, float *ws, void *stream) {
    if (!env || !net || !ws) return err(GW_ERR_ARG, "gw_patch_cnn_prepare: null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, "gw_patch_cnn_prepare: ws must be 16-byte aligned");
    gw_obs_source src;
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_patch_cnn(src, P, net, "gw_patch_cnn_prepare")) != GW_OK) return st;
    const CnnParams p = wcnn_params(src, P, net, ws);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(cnn_prep_wlt, dim3(2048), dim3(256), 0, s, p);
    hipLaunchKernelGGL(wcnn_prep_wlj, dim3(2048), dim3(256), 0, s, p);
    hipLaunchKernelGGL(wcnn_prep_base, dim3((p.HW + WCG - 1) / WCG, src.K), dim3(256), 0, s, p);
    {  // (the lists' spare counter word and the fused listing's bucket counters start at 0)
        const Lists l = lists_at(p.ws.unit_off, src.K * p.P, src.K, src.E, 256);
        if (hipMemsetAsync(l.ctr, 0, sizeof(int), s) != hipSuccess ||
            hipMemsetAsync(p.ws.bucket_n, 0, sizeof(int) * src.K * p.P, s) != hipSuccess)
            return err(GW_ERR_HIP, "gw_patch_cnn_prepare: memset");
    }
    PrepParams pp;  // the layer-2/3 MFMA images (c1 unused)
    pp.net = cnn_tail(net);
    pp.HW = P * P;
    pp.nslices = 0;
    pp.ws = p.ws.mlp;
    pp.base = src.base;
    hipLaunchKernelGGL(prep_images, dim3(64, src.K), dim3(256), 0, s, pp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_patch_cnn_prepare: ") + hipGetErrorString(e));
    return GW_OK;
}

// the positions the act recomputes for the env's current descriptors, listed per (agent, position)
// bucket in ONE launch (round 5; GW_WCNN_LIST=scan: the round-4 chain of layer-1 counts, bucket
// scan and scatter, A/B).  The bucket counters start from zero: the act kernel zeroes them after
// the rare kernel read them, and this call (zero = true) zeroes them itself, so a listing that no
// act consumed (gw_patch_cnn_write_list before an env reset) leaves no counts behind.
static gw_status patch_cnn_list(void *env, const gw_obs_source &src, const CnnParams &cp, hipStream_t s) {
    static const char *list_env = std::getenv("GW_WCNN_LIST");
    const bool fused_list = !(list_env && std::string(list_env) == "scan");
    if (fused_list) {
        gwprof::Span span(env, GW_SPAN_CNN_L1);
        if (hipMemsetAsync(cp.ws.bucket_n, 0, sizeof(int) * src.K * cp.P, s) != hipSuccess)
            return err(GW_ERR_HIP, "gw_patch_cnn_act: memset");
        const dim3 fgrid((unsigned)((src.E + LR_ENVS - 1) / LR_ENVS), src.K);
        switch (src.N) {
            case 1: gwprof::launch(wcnn_list_kernel<2>, fgrid, dim3(256), 0, s, cp); break;
            case 2: gwprof::launch(wcnn_list_kernel<3>, fgrid, dim3(256), 0, s, cp); break;
            case 3: gwprof::launch(wcnn_list_kernel<4>, fgrid, dim3(256), 0, s, cp); break;
            case 4: gwprof::launch(wcnn_list_kernel<5>, fgrid, dim3(256), 0, s, cp); break;
            case 5: gwprof::launch(wcnn_list_kernel<6>, fgrid, dim3(256), 0, s, cp); break;
            case 6: gwprof::launch(wcnn_list_kernel<7>, fgrid, dim3(256), 0, s, cp); break;
            case 7: gwprof::launch(wcnn_list_kernel<8>, fgrid, dim3(256), 0, s, cp); break;
            case 8: gwprof::launch(wcnn_list_kernel<9>, fgrid, dim3(256), 0, s, cp); break;
            default: return err(GW_ERR_ARG, "gw_patch_cnn_act: N out of range");
        }
    } else {
        const Lists lists = lists_at(cp.ws.unit_off, src.K * cp.P, src.K, src.E, 256);
        const dim3 lgrid((unsigned)lists.nblk, src.K);
        {
            gwprof::Span span(env, GW_SPAN_CNN_L1);
            switch (src.N) {
                case 1: gwprof::launch(wcnn_l1_kernel<2>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 2: gwprof::launch(wcnn_l1_kernel<3>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 3: gwprof::launch(wcnn_l1_kernel<4>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 4: gwprof::launch(wcnn_l1_kernel<5>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 5: gwprof::launch(wcnn_l1_kernel<6>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 6: gwprof::launch(wcnn_l1_kernel<7>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 7: gwprof::launch(wcnn_l1_kernel<8>, lgrid, dim3(256), 0, s, cp, lists); break;
                case 8: gwprof::launch(wcnn_l1_kernel<9>, lgrid, dim3(256), 0, s, cp, lists); break;
                default: return err(GW_ERR_ARG, "gw_patch_cnn_act: N out of range");
            }
        }
        gwprof::Span span(env, GW_SPAN_CNN_LIST);
        gwprof::launch(bucket_scan, dim3(src.K * cp.P), dim3(64), 0, s, cp, lists);
        gwprof::launch(wcnn_scatter, lgrid, dim3(256), 0, s, cp, lists);
    }
    return GW_OK;
}

static gw_status patch_cnn_check(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, gw_obs_source &src,
                                 const char *who) {
    const std::string w(who);
    if (!env || !net || !ws) return err(GW_ERR_ARG, w + ": null argument");
    if (reinterpret_cast<uintptr_t>(ws) & 15u) return err(GW_ERR_ARG, w + ": ws must be 16-byte aligned");
    gw_status st = gw_obs_view(env, &src);
    if (st != GW_OK) return st;
    if ((st = check_patch_cnn(src, P, net, who)) != GW_OK) return st;
    if (src.K * (P / 4) * (P / 4) > WR_MAX_NB) return err(GW_ERR_ARG, w + ": K x window positions above the rare kernel's table");
    return GW_OK;
}

// the rare kernel and the actor over the listed positions
static gw_status patch_cnn_rest(void *env, const gw_obs_source &src, const CnnParams &cp, int32_t P,
                                const gw_cnn_actors *net, int training, float tau, uint64_t seed, uint64_t counter,
                                const int64_t *counter_dev, const float *uniform, const uint16_t *mask,
                                int32_t *actions, float *probs, float *logits, hipStream_t s) {
    if (!actions || !probs) return err(GW_ERR_ARG, "gw_patch_cnn_act: null argument");
    if (!(tau > 0.0f)) return err(GW_ERR_ARG, "gw_patch_cnn_act: tau must be > 0");
    static const char *list_env = std::getenv("GW_WCNN_LIST");
    const bool fused_list = !(list_env && std::string(list_env) == "scan");
    static const char *stat_env = GW_MEASURE_ENV("GW_WCNN_STAT");  // diagnostics: the buckets' sizes (synchronises)
    if (stat_env && *stat_env && fused_list) {
        std::vector<int> bn((size_t)src.K * cp.P);
        if (hipStreamSynchronize(s) == hipSuccess &&
            hipMemcpy(bn.data(), cp.ws.bucket_n, sizeof(int) * bn.size(), hipMemcpyDeviceToHost) == hipSuccess) {
            long tot = 0, units = 0;
            int mx = 0;
            for (int v : bn) {
                tot += v;
                units += (v + WR_ITEMS - 1) / WR_ITEMS;
                mx = std::max(mx, v);
            }
            std::fprintf(stderr, "wcnn buckets: %ld items (%.3f per env-agent), %ld units, max bucket %d:", tot,
                         (double)tot / ((double)src.E * src.K), units, mx);
            for (int b = 0; b < (int)bn.size(); ++b) std::fprintf(stderr, " %d", bn[b]);
            std::fprintf(stderr, "\n");
        }
    }
    static const char *rstamp_env = GW_MEASURE_ENV("GW_RARE_STAMP");  // diagnostics: block stamps (synchronises)
    static unsigned long long *rstamp = nullptr;
    if (rstamp_env && *rstamp_env && !rstamp && hipMalloc(&rstamp, sizeof(unsigned long long) * WR_BLOCKS * 8) != hipSuccess)
        rstamp = nullptr;
    CnnParams cps = cp;
    cps.stamp = rstamp;
#define RARE(NP) gwprof::launch(wcnn_rare_kernel<NP>, dim3(WR_BLOCKS), dim3(64 * WR_WAVES), 0, s, cps)
    {
        gwprof::Span span(env, GW_SPAN_CNN_RARE);
        switch (src.N) {
            case 1: RARE(2); break;
            case 2: RARE(3); break;
            case 3: RARE(4); break;
            case 4: RARE(5); break;
            case 5: RARE(6); break;
            case 6: RARE(7); break;
            case 7: RARE(8); break;
            default: RARE(9); break;
        }
    }
#undef RARE
    if (rstamp) {
        std::vector<unsigned long long> h((size_t)WR_BLOCKS * 8);
        if (hipStreamSynchronize(s) == hipSuccess &&
            hipMemcpy(h.data(), rstamp, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE *f = std::fopen(rstamp_env, "ab")) {
                std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                std::fclose(f);
            }
        }
    }
    ActParams p{};
    p.net = cnn_tail(net);
    p.c1 = cp.ws.mlp.c1;
    p.w2img = cp.ws.mlp.w2;
    p.w3img = cp.ws.mlp.w3;
    p.w2bimg = cp.ws.mlp.w2b;
    p.desc = src.desc;
    p.base = src.base;
    p.mask = mask;
    p.uniform = uniform;
    p.h1 = nullptr;
    p.rare_z = cp.ws.rare_z;
    p.rare_n = cp.ws.rare_n;
    p.actions = actions;
    p.probs = probs;
    p.logits = logits;
    p.E = src.E;
    p.env_offset = src.env_offset;
    p.N = src.N;
    p.K = src.K;
    p.HW = src.H * src.W;
    p.W = src.W;
    p.P = P;
    p.in_dim = P * P;
    p.tbl = cp.ws.table;
    p.zero_n = cp.ws.bucket_n;  // the fused listing's bucket counters, read by the rare kernel above
    p.zero_cnt = src.K * cp.P;
    p.variant = src.variant;
    p.training = training ? 1 : 0;
    p.tau = tau;
    p.key0 = (uint32_t)seed;
    p.key1 = (uint32_t)(seed >> 32);
    p.ctr0 = (uint32_t)counter;
    p.ctr1 = (uint32_t)(counter >> 32);
    p.ctr_dev = counter_dev;
    for (int k = 0; k < MAXN; ++k) p.apples[k] = src.apples[k];
    p.ab = 0;
    const int64_t tiles = (src.E + TILE - 1) / TILE;
    p.tiles = (int)tiles;
    const int64_t want = (tiles + 15) / 16;
    const int per_agent = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(1, 256 / src.K)));
#define ACTW(NP) gwprof::launch(act_kernel<NP, 16, true, true, true, RSW>, dim3(per_agent, src.K), dim3(1024), 0, s, p)
    gwprof::Span span(env, GW_SPAN_ACT);
    switch (src.N) {
        case 1: ACTW(2); break;
        case 2: ACTW(3); break;
        case 3: ACTW(4); break;
        case 4: ACTW(5); break;
        case 5: ACTW(6); break;
        case 6: ACTW(7); break;
        case 7: ACTW(8); break;
        default: ACTW(9); break;
    }
#undef ACTW
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_patch_cnn_act: ") + hipGetErrorString(e));
    return GW_OK;
}

gw_status gw_patch_cnn_act(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, int training, float tau,
                           uint64_t seed, uint64_t counter, const int64_t *counter_dev, const float *uniform,
                           const uint16_t *mask,
                           int32_t *actions, float *probs, float *logits, void *stream) {
    gw_obs_source src;
    gw_status st = patch_cnn_check(env, P, net, ws, src, "gw_patch_cnn_act");
    if (st != GW_OK) return st;
    const CnnParams cp = wcnn_params(src, P, net, const_cast<float *>(ws));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if ((st = patch_cnn_list(env, src, cp, s)) != GW_OK) return st;
    return patch_cnn_rest(env, src, cp, P, net, training, tau, seed, counter, counter_dev, uniform, mask, actions,
                          probs, logits, s);
}

gw_status gw_patch_cnn_act_listed(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, int training,
                                  float tau, uint64_t seed, uint64_t counter, const int64_t *counter_dev,
                                  const float *uniform, const uint16_t *mask, int32_t *actions, float *probs,
                                  float *logits, void *stream) {
    gw_obs_source src;
    gw_status st = patch_cnn_check(env, P, net, ws, src, "gw_patch_cnn_act_listed");
    if (st != GW_OK) return st;
    const CnnParams cp = wcnn_params(src, P, net, const_cast<float *>(ws));
    return patch_cnn_rest(env, src, cp, P, net, training, tau, seed, counter, counter_dev, uniform, mask, actions,
                          probs, logits, static_cast<hipStream_t>(stream));
}

gw_status gw_patch_cnn_write_list(void *env, int32_t P, const gw_cnn_actors *net, const float *ws, float *patch,
                                  float *final_patch, void *stream) {
    gw_obs_source src;
    gw_status st = patch_cnn_check(env, P, net, ws, src, "gw_patch_cnn_write_list");
    if (st != GW_OK) return st;
    if (!patch) return err(GW_ERR_ARG, "gw_patch_cnn_write_list: null patch");
    if (src.E % 4 != 0 || (uint64_t)src.E * (uint64_t)P >= (1ull << 32))
        return err(GW_ERR_ARG, "gw_patch_cnn_write_list: needs E % 4 == 0 (the row writer's runs)");
    const CnnParams cp = wcnn_params(src, P, net, const_cast<float *>(ws));
    gw::PatchArgs a;
    a.desc = src.desc;
    a.roadbits = cp.ws.road;  // the workspace's copy of the env's road bits (gw_patch_cnn_prepare)
    a.base = src.base;
    a.patch = patch;
    a.final_patch = final_patch;
    a.E = src.E;
    a.H = src.H;
    a.W = src.W;
    a.N = src.N;
    a.K = src.K;
    a.P = P;
    a.variant = src.variant;
    for (int k = 0; k < GW_MAX_AGENTS; ++k) a.apples[k] = src.apples[k];
    const uint32_t nlist = (uint32_t)((src.E + LR_ENVS - 1) / LR_ENVS);
    const uint32_t nrows = (uint32_t)((src.E * P + 511) / 512);
    const dim3 grid(nlist + nrows, src.K);
    hipStream_t s = static_cast<hipStream_t>(stream);
    gwprof::Span span(env, GW_SPAN_WINDOW);
#define RL(NP)                                                                                      \
    do {                                                                                            \
        if (P <= 8) gwprof::launch(rows_list_kernel<NP, 8>, grid, dim3(256), 0, s, a, cp, nlist);  \
        else if (P <= 12) gwprof::launch(rows_list_kernel<NP, 12>, grid, dim3(256), 0, s, a, cp, nlist); \
        else gwprof::launch(rows_list_kernel<NP, 16>, grid, dim3(256), 0, s, a, cp, nlist);           \
    } while (0)
    switch (src.N) {
        case 1: RL(2); break;
        case 2: RL(3); break;
        case 3: RL(4); break;
        case 4: RL(5); break;
        case 5: RL(6); break;
        case 6: RL(7); break;
        case 7: RL(8); break;
        case 8: RL(9); break;
        default: return err(GW_ERR_ARG, "gw_patch_cnn_write_list: N out of range");
    }
#undef RL
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return err(GW_ERR_HIP, std::string("gw_patch_cnn_write_list: ") + hipGetErrorString(e));
    return GW_OK;
}

}  // extern "C"
