// window_rows.h -- the row window writer's block (gw_obs_patch MODE 6), shared by
// patch_ops.hip (its own launch) and actor_ops.hip (the same blocks in the launch that also lists
// the window CNN head's recomputed positions).  One thread per window ROW of the [K][E][P*P] layout;
// a wave's 64 rows leave as one contiguous run of consecutive nontemporal 16-byte stores.
#ifndef GW_WINDOW_ROWS_H
#define GW_WINDOW_ROWS_H

#include <hip/hip_runtime.h>

#include <cstdint>

#include "patch_ops.h"

namespace gwrows {

constexpr uint32_t D_RESET = 1u, D_WRITE = 2u, D_FINAL = 4u;  // obs descriptor flags (gridenv.hip)
constexpr int NDESC = 12;                                     // u32 words per obs descriptor
typedef float f32x4 __attribute__((ext_vector_type(4)));

// the obs writer's value of agent n's cell in agent k's observation (gridenv.hip obs_block)
__device__ __forceinline__ float agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;
    if (v == k + 1) v = 1;
    return (float)v;
}

// block bx of agent k (grid ((E P + 511) / 512, K), 256 threads); s_rows: the block's LDS,
// [WAVES][64 rows x MAXW / 4 float4]
// (WAVES = 2: the 128-thread blocks of a launch shared with gridenv.hip's FeAR kernel; the grid
// then has (E P + 64 WAVES WR_RUNS - 1) / (64 WAVES WR_RUNS) blocks per agent)
template <int NP, int MAXW, int WR_RUNS = 2, int WAVES = 4>  // MAXW: 8, 12 or 16 >= P (the row's registers)
__device__ __forceinline__ void rows_block(const gw::PatchArgs &a, uint32_t bx, int k,
                                           float4 (*s_rows)[64 * (MAXW / 4)]) {

    const int P = a.P, W = a.W, H = a.H, half = P / 2, P4 = P / 4, N4 = 16 * P;  // N4: the run's float4
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nrows = (uint32_t)(a.E * P);
    const uint32_t m_p = (uint32_t)((0x100000000ull + (uint64_t)P - 1) / (uint64_t)P);
    const uint32_t m_w = (uint32_t)((0x100000000ull + (uint64_t)W - 1) / (uint64_t)W);
    // a wave takes WR_RUNS consecutive runs of 64 rows; every run's descriptor loads are issued
    // before the first run's stores (one round trip per wave, not one per 64 rows)
    const uint32_t run0 = (bx * (uint32_t)WAVES + (uint32_t)wave) * WR_RUNS;
    uint32_t fr[WR_RUNS];
    uint4 wsr[WR_RUNS];  // (the terminal words: loaded by the few waves that need them)
#pragma unroll
    for (int j = 0; j < WR_RUNS; ++j) {
        const uint32_t t = (run0 + j) * 64u + lane, tc = t < nrows ? t : nrows - 1;
        const uint32_t *d = a.desc + (int64_t)__umulhi(tc, m_p) * NDESC;
        fr[j] = d[4];
        wsr[j] = *reinterpret_cast<const uint4 *>(d);
    }
#pragma unroll
    for (int j = 0; j < WR_RUNS; ++j) {
    const uint32_t t0 = (run0 + j) * 64u, t = t0 + lane;  // the run's first row, this lane's row
    if (t0 >= nrows) break;  // wave-uniform
    const bool live = t < nrows;
    const uint32_t tc = live ? t : nrows - 1;
    const uint32_t e = __umulhi(tc, m_p);
    const int wr = (int)(tc - e * (uint32_t)P);
    const uint32_t f = fr[j];
    const bool step = live && (f & D_WRITE) && a.patch, fin = live && (f & D_FINAL) && a.final_patch;
    const uint4 ws = wsr[j];
    const uint32_t *dj = a.desc + (int64_t)e * NDESC;
    auto road = [&](int cell) { return (a.roadbits[cell >> 5] >> (cell & 31)) & 1u; };
    // the wave's 64 rows are one contiguous run of 64 P floats: each lane parks its row's map values
    // in the wave's LDS slice, then stores the patched cells that lie on its row over them (scalar
    // LDS stores in slot order: a later slot overrides), and the run leaves as float4 lane + 64 u
    // (consecutive lanes, consecutive 16 bytes), skipping the float4 of rows not written this step
    // (the row mask from a ballot)
    float4 *sw = s_rows[wave];
    float *swf = reinterpret_cast<float *>(sw) + lane * P;
    auto emit = [&](int which, bool mine, float *dst) {
        const uint64_t mask = __ballot(mine);
        if (!mask) return;  // wave-uniform
        const uint4 w4 = which == 0 ? ws : *reinterpret_cast<const uint4 *>(dj + 8);
        const uint32_t wd[4] = {w4.x, w4.y, w4.z, w4.w};
        const bool reset = which == 0 && (f & D_RESET);
        const uint32_t apples = which == 0 ? (f >> 8) & 0xFFu : (f >> 16) & 0xFFu;
        const int ac = ((apples >> k) & 1u) ? a.apples[k] : -1;
        const int ctr = (int)((wd[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        const int cr = (int)__umulhi((uint32_t)ctr, m_w), cc = ctr - cr * W;
        const int grow = cr - half + wr, gc0 = cc - half;  // this row's grid row, its first column
        {   // the map: road bits of columns gc0 .. gc0 + P - 1 (at most two 32-bit words)
            const bool in_row = (unsigned)grow < (unsigned)H;
            const int cmin = max(gc0, 0), cell = (in_row ? grow : 0) * W + cmin;
            const int nroad1 = (H * W + 31) / 32 - 1, w0 = min(cell >> 5, nroad1);
            const uint64_t bits = (((uint64_t)a.roadbits[min(w0 + 1, nroad1)] << 32) | a.roadbits[w0]) >> (cell & 31);
#pragma unroll
            for (int q = 0; q < MAXW / 4; ++q) {  // four columns at a time: no row array in registers
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int col = gc0 + 4 * q + u;
                    v[u] = (in_row && (unsigned)col < (unsigned)W && ((bits >> (col - cmin)) & 1u)) ? 0.0f : -1.0f;
                }
                if ((P & 3) == 0) {
                    if (q < P4) sw[lane * P4 + q] = make_float4(v[0], v[1], v[2], v[3]);
                } else {  // rows not 16-byte aligned in LDS: scalar stores
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (4 * q + u < P) swf[4 * q + u] = v[u];
                }
            }
        }
        auto patch = [&](int cell, float val) {  // the cell's value, if it lies on this row
            const int pr = (int)__umulhi((uint32_t)cell, m_w), pc = cell - pr * W - gc0;
            if ((unsigned)cell < (unsigned)(H * W) && pr == grow && (unsigned)pc < (unsigned)P) swf[pc] = val;
        };
        if (a.probe != 1) {  // (probe 1, measurement only: the map part alone)
            if (ac >= 0) {
                float av = (road(ac) ? 0.0f : -1.0f) + 9.0f;
                if (!reset && av == (float)(k + 1)) av = 1.0f;
                patch(ac, av);
            }
#pragma unroll
            for (int n = 0; n < NP - 1; ++n) {
                const int c = (int)((wd[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                patch(c, agent_value(reset, n, k, c == ac, a.variant));
            }
        }
        __builtin_amdgcn_wave_barrier();  // (a wave's LDS operations complete in order)
        float *run = dst + ((int64_t)k * a.E * P + t0) * P;  // 16-byte aligned: t0 % 64 == 0, E % 4 == 0
        float4 *o4 = reinterpret_cast<float4 *>(run);
#pragma unroll
        for (int u = 0; u < MAXW / 4; ++u) {
            const int i = lane + 64 * u;
            if (i < N4) {
                // the rows float4 i covers (P % 4 == 0: one); a piece across a written and an
                // unwritten row (or past the last row) goes out as its written floats alone
                const int r0 = (int)__umulhi((uint32_t)(4 * i), m_p), r1 = (int)__umulhi((uint32_t)(4 * i + 3), m_p);
                const bool w0 = (mask >> r0) & 1u, w1 = (mask >> r1) & 1u;
                // nontemporal (streamed past the caches, as the obs writer's): alone 18.5 -> 17.7 us at
                // c5patch's shape, 30.3 -> 28.8 us at c4patch's (tools/gpu_r5_nt.sh)
                if (w0 && w1) {
                    __builtin_nontemporal_store(*reinterpret_cast<const f32x4 *>(&sw[i]), reinterpret_cast<f32x4 *>(&o4[i]));
                } else if (w0 || w1) {
                    const float *src = reinterpret_cast<const float *>(sw) + 4 * i;
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        if ((mask >> __umulhi((uint32_t)(4 * i + c), m_p)) & 1u) __builtin_nontemporal_store(src[c], &run[4 * i + c]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    };
    emit(0, step, a.patch);
    emit(1, fin, a.final_patch);
    }
}

}  // namespace gwrows

#endif
