// patch_ops.hip — gw_obs_patch's writer: each RL agent's P x P egocentric window of its last
// observation (X1; not a reference format: the reference observes the whole relabelled grid,
// custom/ma_customenv.py:303-322).  Rows / cols -P/2 .. P-1-P/2 around the agent's own cell, -1
// outside the grid (the map's inactive value), the same encoding as the full-grid obs writer
// (static map + the <= N + 1 patched cells of the env's descriptor), so a window equals a crop of
// the full obs.  Layout [K][E][P*P]; `patch` gets the step's windows (D_WRITE envs), `final` the
// terminal windows of the envs that ended (D_FINAL, centred on the terminal cell).
//
// Block = PB envs (both agents).  Staging: one thread per (which, env, agent) builds the window's
// patched cells in registers, drops a patch that a later one overrides (the obs writer's order),
// and leaves window positions + values in LDS.  The step's windows, P % 4 == 0: one thread per
// 16-byte piece of a window row (four map bits + the window's <= N + 1 overrides, one aligned
// float4 store); other P <= 16: one wave per window writes the map part into an LDS image of the
// block's run (lanes own fixed window positions, so their (row, col) offsets are computed once),
// then the patched cells as one scattered LDS store; the run leaves as aligned 16-byte stores of
// whole lines.  Terminal windows (few envs per step) go straight to HBM from registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "patch_ops.h"
#include "prof.h"
#include "measure.h"
#include "window_rows.h"

namespace {

constexpr int THREADS = 256, MAXP = GW_MAX_AGENTS + 1, MAXPL = 4;  // MAXPL: P * P <= 256
// PB: envs per block (a template parameter: 32, or 64 where the LDS leaves room for enough blocks)
constexpr uint32_t D_RESET = 1u, D_WRITE = 2u, D_FINAL = 4u;
constexpr int NDESC = 12;

__device__ __forceinline__ float agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;
    if (v == k + 1) v = 1;
    return (float)v;
}

__device__ __forceinline__ float map_value(const uint32_t *road, int H, int W, int r, int q) {
    if (r < 0 || r >= H || q < 0 || q >= W) return -1.0f;
    const int cell = r * W + q;
    return ((road[cell >> 5] >> (cell & 31)) & 1u) ? 0.0f : -1.0f;
}

// MODE 0: P * P <= 256, the windows assembled in LDS (kept for A/B); 1: one thread per element
// (windows too large for the tables below); 2: P % 4 == 0, one thread per 16-byte piece of a
// window row (map bits + overrides in registers, no LDS image: every store is a whole aligned
// float4 of the [K][E][P*P] run); 3: any P, one thread per 16-byte piece of the block's run (a
// byte table of the patched cells in LDS, map values from the road bits)
template <int MODE, int PB>
__global__ void __launch_bounds__(THREADS) window_kernel(gw::PatchArgs a, unsigned long long *dbg) {
    constexpr bool SMALL = MODE == 0;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x, K = a.K, N = a.N, W = a.W, H = a.H, P = a.P;
    const int PP = P * P, half = P / 2, np = N + 1, nroad = (a.H * a.W + 31) / 32;
    // c / W as a multiply-high: exact for cells < 2^16 with ceil(2^32 / W)
    const uint32_t a_wmagic = (uint32_t)((0x100000000ull + (uint64_t)W - 1) / (uint64_t)W);
    uint32_t *s_road = lds;
    uint32_t *s_flag = s_road + nroad;                               // [PB]
    int *s_ctr = reinterpret_cast<int *>(s_flag + PB);               // [2][PB][K]  row << 16 | col
    int *s_pw = s_ctr + 2 * PB * K;                                  // [2][PB][K][np] window positions (-1: none)
    float *s_pv = reinterpret_cast<float *>(s_pw + 2 * PB * K * np);
    float *s_out = s_pv + 2 * PB * K * np;                           // SMALL: one agent's run [nenv * PP]
    // MODE 2: per step window (slot el * K + k) and 4-cell segment q, the surviving patch index + 1
    // of each of the segment's cells, one nibble per cell (0: map value)
    uint16_t *s_seg = reinterpret_cast<uint16_t *>(s_pv + 2 * PB * K * np);
    const int Q4 = PP / 4;
    const int64_t e0 = (int64_t)blockIdx.x * PB;
    const int nenv = (int)min((int64_t)PB, a.E - e0);
    if (dbg && tid == 0) dbg[4 * blockIdx.x + 0] = wall_clock64();
    // the descriptors of this thread's (which, env, agent) items are loaded first, the road
    // bitmask beside them; the apple cell's map value then comes from LDS (no dependent load)
    constexpr int ITEMS = (2 * PB * GW_MAX_AGENTS + THREADS - 1) / THREADS;
    uint32_t fl[ITEMS], wd[ITEMS][4];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int t = tid + it * THREADS;
        const int which = t / (PB * K), el = (t / K) % PB;
        const bool ok = t < 2 * PB * K && el < nenv;
        const uint32_t *d = a.desc + (e0 + (ok ? el : 0)) * NDESC;
        fl[it] = ok ? d[4] : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) wd[it][i] = ok ? d[(which == 0 ? 0 : 8) + i] : 0u;
    }
    for (int w = tid; w < nroad; w += THREADS) s_road[w] = a.roadbits[w];
    __syncthreads();
    int has_write = 1, has_final = 0;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {  // staging: thread = (which, env, agent)
        const int t = tid + it * THREADS;
        if (t >= 2 * PB * K) break;
        const int which = t / (PB * K), el = (t / K) % PB, k = t % K;
        const int slot = (which * PB + el) * K + k;
        if (el < nenv) {
            const uint32_t f = fl[it];
            if (k == 0 && which == 0) s_flag[el] = f;
            if (which == 0) has_write &= (f & D_WRITE) != 0;
            else has_final |= (f & D_FINAL) != 0;
            if (which == 1 && !(f & D_FINAL)) continue;  // no terminal window: nothing to stage
            const bool reset = which == 0 && (f & D_RESET);
            const uint32_t apples = which == 0 ? (f >> 8) & 0xFFu : (f >> 16) & 0xFFu;
            uint32_t words[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) words[i] = wd[it][i];
            const int ac = ((apples >> k) & 1u) ? a.apples[k] : -1;
            const int ctr = (int)((words[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
            const int cr = (int)__umulhi((uint32_t)ctr, a_wmagic), cc = ctr - cr * W;
            s_ctr[slot] = (cr << 16) | cc;
            uint16_t *sg = s_seg + slot * Q4;  // which == 0: slot = el * K + k
            if (MODE == 2 && which == 0)
                for (int q = 0; q < Q4; q += 2) *reinterpret_cast<uint32_t *>(sg + q) = 0u;  // Q4 is even
            int cell[MAXP];
            float val[MAXP];
            int u = 0;
            if (ac >= 0) {
                float av = (((s_road[ac >> 5] >> (ac & 31)) & 1u) ? 0.0f : -1.0f) + 9.0f;
                if (!reset && av == (float)(k + 1)) av = 1.0f;
                cell[0] = ac;
                val[0] = av;
                u = 1;
            }
#pragma unroll
            for (int n = 0; n < GW_MAX_AGENTS; ++n) {
                if (n >= N) break;
                const int c = (int)((words[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                cell[u] = c;
                val[u] = agent_value(reset, n, k, c == ac, a.variant);
                ++u;
            }
            for (int i = 0; i < np; ++i) {
                int pos = -1;
                if (i < u) {
                    const int c = cell[i];
                    const int rr = (int)__umulhi((uint32_t)c, a_wmagic);
                    const int wr = rr - cr + half, wc = c - rr * W - cc + half;
                    bool last = (unsigned)wr < (unsigned)P && (unsigned)wc < (unsigned)P;
                    for (int j = i + 1; j < u; ++j) last = last && cell[j] != c;  // a later patch overrides
                    pos = last ? wr * P + wc : -1;
                }
                s_pw[slot * np + i] = pos;
                s_pv[slot * np + i] = i < u ? val[i] : 0.0f;
                if (MODE == 2 && which == 0 && pos >= 0)  // this thread owns the slot's segments
                    sg[pos >> 2] |= (uint16_t)((i + 1) << (4 * (pos & 3)));
            }
        }
    }
    const bool all_write = __syncthreads_and(has_write) != 0;  // (also the barrier after the staging)
    const bool any_final = __syncthreads_or(has_final) != 0;
    if (dbg && tid == 0) dbg[4 * blockIdx.x + 1] = wall_clock64();
    const int wave = tid >> 6, lane = tid & 63;
    if (SMALL && a.patch) {
        int pr[MAXPL], pc[MAXPL];
#pragma unroll
        for (int t = 0; t < MAXPL; ++t) {
            const int c = lane + 64 * t;
            pr[t] = c / P - half;
            pc[t] = c - (c / P) * P - half;
        }
        const int npl = (PP + 63) / 64;
        const int len = nenv * PP;
        for (int k = 0; k < K; ++k) {  // one agent's contiguous run at a time (LDS: nenv * PP floats)
            if (k > 0) __syncthreads();  // the previous agent's run has been stored
            for (int el = wave; el < nenv; el += THREADS / 64) {
                const int slot = el * K + k;
                const int ctr = s_ctr[slot], cr = ctr >> 16, cc = ctr & 0xFFFF;
                float *o = s_out + el * PP;
#pragma unroll
                for (int t = 0; t < MAXPL; ++t) {
                    if (t >= npl) break;
                    const float m = map_value(s_road, H, W, cr + pr[t], cc + pc[t]);
                    if (lane + 64 * t < PP) o[lane + 64 * t] = m;
                }
                // the patched cells (distinct positions), after this wave's map stores (a wave's
                // LDS operations complete in order)
                if (lane < np) {
                    const int pw = s_pw[slot * np + lane];
                    if (pw >= 0) o[pw] = s_pv[slot * np + lane];
                }
            }
            __syncthreads();
            if (dbg && tid == 0 && k == 0) dbg[4 * blockIdx.x + 2] = wall_clock64();
            const int64_t off = ((int64_t)k * a.E + e0) * PP;
            float *o = a.patch + off;
            if (!all_write) {
                for (int i = tid; i < len; i += THREADS)
                    if (s_flag[i / PP] & D_WRITE) o[i] = s_out[i];
                continue;
            }
            const int lead = (int)((4 - (off & 3)) & 3);
            for (int i = tid; i < min(lead, len); i += THREADS) o[i] = s_out[i];
            const int n4 = (len - lead) / 4;
            float4 *o4 = reinterpret_cast<float4 *>(o + lead);
            for (int j = tid; j < n4; j += THREADS) {
                const int i = lead + 4 * j;
                o4[j] = make_float4(s_out[i], s_out[i + 1], s_out[i + 2], s_out[i + 3]);
            }
            for (int i = lead + 4 * n4 + tid; i < len; i += THREADS) o[i] = s_out[i];
        }
    } else if (MODE == 2 && a.patch) {
        const int P4 = P / 4, per_k = nenv * Q4;
        const int nroad1 = nroad - 1;
        // q / P4 and j / Q4 as multiply-highs (exact for the small numerators here; Q4 >= 4,
        // P4 = 1 is q itself: its magic 2^32 does not fit)
        const uint32_t m_p4 = P4 > 1 ? (uint32_t)((0x100000000ull + (uint64_t)P4 - 1) / (uint64_t)P4) : 0u;
        const uint32_t m_q4 = (uint32_t)((0x100000000ull + (uint64_t)Q4 - 1) / (uint64_t)Q4);
        for (int k = 0; k < K; ++k) {
            float4 *o4 = reinterpret_cast<float4 *>(a.patch + ((int64_t)k * a.E + e0) * PP);
            for (int j = tid; j < per_k; j += THREADS) {
                const int el = (int)__umulhi((uint32_t)j, m_q4), q = j - el * Q4;
                if (!(s_flag[el] & D_WRITE)) continue;
                const int slot = el * K + k;
                const int ctr = s_ctr[slot];
                const int wr = P4 > 1 ? (int)__umulhi((uint32_t)q, m_p4) : q, wc = 4 * (q - wr * P4);
                const int row = (ctr >> 16) - half + wr, col0 = (ctr & 0xFFFF) - half + wc;
                // the four map values from at most two road words: bits of cells cmin .. cmin + 31
                const int cmin = max(col0, 0), cell = row * W + cmin;
                const bool in_row = (unsigned)row < (unsigned)H;
                const int w0 = in_row ? min(cell >> 5, nroad1) : 0;  // (cols past the edge: masked below)
                const uint64_t bits = (((uint64_t)s_road[min(w0 + 1, nroad1)] << 32) | s_road[w0]) >> (cell & 31);
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int col = col0 + u;
                    const bool road = in_row && (unsigned)col < (unsigned)W && ((bits >> (col - cmin)) & 1u);
                    v[u] = road ? 0.0f : -1.0f;
                }
                // the segment's patched cells (the nibble table built at staging)
                const uint32_t sgv = s_seg[slot * Q4 + q];
                if (sgv) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t idx = (sgv >> (4 * u)) & 0xFu;
                        if (idx) v[u] = s_pv[slot * np + (int)idx - 1];
                    }
                }
                o4[j] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    } else if (MODE == 3 && a.patch) {
        // any P: the block's [nenv * PP] run of one agent leaves as aligned float4 stores; a byte
        // table (the surviving patch index + 1 of every window cell, 0 = map value) is built in
        // LDS per agent, so a thread's four cells need one u32 table read, not an override loop
        uint8_t *s_tab = reinterpret_cast<uint8_t *>(s_pv + 2 * PB * K * np);
        const int len = nenv * PP;
        const uint32_t m_pp = (uint32_t)((0x100000000ull + (uint64_t)PP - 1) / (uint64_t)PP);
        const uint32_t m_p = (uint32_t)((0x100000000ull + (uint64_t)P - 1) / (uint64_t)P);
        if ((GW_MEASURE_ON && a.probe == 2)) {  // measurement only: staging, then zeros
            for (int k = 0; k < K; ++k) {
                const int64_t off = ((int64_t)k * a.E + e0) * PP;
                float *o = a.patch + off;
                const int lead = (int)((4 - (off & 3)) & 3);
                for (int i = tid; i < min(lead, len); i += THREADS) o[i] = 0.0f;
                const int n4 = (len - lead) / 4;
                float4 *o4 = reinterpret_cast<float4 *>(o + lead);
                for (int j = tid; j < n4; j += THREADS) o4[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                for (int i = lead + 4 * n4 + tid; i < len; i += THREADS) o[i] = 0.0f;
            }
            return;
        }
        for (int k = 0; k < K; ++k) {
            const int64_t off = ((int64_t)k * a.E + e0) * PP;
            float *o = a.patch + off;
            const int lead = (int)((4 - (off & 3)) & 3);  // floats before the first 16-byte boundary
            const int sh = (4 - lead) & 3;                  // table index = run index + sh: the float4
                                                            // pieces' four entries are one aligned u32
            if (k > 0) __syncthreads();                     // the previous agent's table is read
            for (int w = tid; w < (len + sh + 3) / 4; w += THREADS) reinterpret_cast<uint32_t *>(s_tab)[w] = 0u;
            __syncthreads();
            for (int t = tid; t < nenv * np; t += THREADS) {
                const int el = t / np, i = t - el * np;
                const int pw = s_pw[(el * K + k) * np + i];
                if (pw >= 0) s_tab[el * PP + pw + sh] = (uint8_t)(i + 1);
            }
            __syncthreads();
            if (!all_write) {  // partial resets: only the written envs' windows (rare)
                for (int i = tid; i < len; i += THREADS) {
                    const int el = (int)__umulhi((uint32_t)i, m_pp), c = i - el * PP;
                    if (!(s_flag[el] & D_WRITE)) continue;
                    const int slot = el * K + k, ctr = s_ctr[slot];
                    const int wr = (int)__umulhi((uint32_t)c, m_p);
                    const int idx = s_tab[i + sh];
                    o[i] = idx ? s_pv[slot * np + idx - 1]
                               : map_value(s_road, H, W, (ctr >> 16) + wr - half, (ctr & 0xFFFF) + c - wr * P - half);
                }
                continue;
            }
            for (int i = tid; i < min(lead, len); i += THREADS) {
                const int el = (int)__umulhi((uint32_t)i, m_pp), c = i - el * PP;
                const int slot = el * K + k, ctr = s_ctr[slot];
                const int wr = (int)__umulhi((uint32_t)c, m_p);
                const int idx = s_tab[i + sh];
                o[i] = idx ? s_pv[slot * np + idx - 1]
                           : map_value(s_road, H, W, (ctr >> 16) + wr - half, (ctr & 0xFFFF) + c - wr * P - half);
            }
            const int n4 = (len - lead) / 4;
            float4 *o4 = reinterpret_cast<float4 *>(o + lead);
            for (int j = tid; j < n4; j += THREADS) {
                if ((GW_MEASURE_ON && a.probe == 1)) {  // measurement only: the table was built, zeros stored
                    reinterpret_cast<float4 *>(o + lead)[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    continue;
                }
                const int i0 = lead + 4 * j;
                int el = (int)__umulhi((uint32_t)i0, m_pp), c = i0 - el * PP;
                int wr = (int)__umulhi((uint32_t)c, m_p), wc = c - wr * P;
                int ctr = s_ctr[el * K + k];
                const uint32_t tab = reinterpret_cast<const uint32_t *>(s_tab)[(i0 + sh) >> 2];
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (u > 0) {  // the next cell of the run: next column, row or window
                        if (++wc == P) {
                            wc = 0;
                            if (++wr == P) {
                                wr = 0;
                                ++el;
                                ctr = s_ctr[el * K + k];
                            }
                        }
                    }
                    const uint32_t idx = (tab >> (8 * u)) & 0xFFu;
                    v[u] = idx ? s_pv[(el * K + k) * np + (int)idx - 1]
                               : map_value(s_road, H, W, (ctr >> 16) + wr - half, (ctr & 0xFFFF) + wc - half);
                }
                o4[j] = make_float4(v[0], v[1], v[2], v[3]);
            }
            for (int i = lead + 4 * n4 + tid; i < len; i += THREADS) {
                const int el = (int)__umulhi((uint32_t)i, m_pp), c = i - el * PP;
                const int slot = el * K + k, ctr = s_ctr[slot];
                const int wr = (int)__umulhi((uint32_t)c, m_p);
                const int idx = s_tab[i + sh];
                o[i] = idx ? s_pv[slot * np + idx - 1]
                           : map_value(s_road, H, W, (ctr >> 16) + wr - half, (ctr & 0xFFFF) + c - wr * P - half);
            }
        }
    } else if (MODE == 4 && a.patch) {
        // the map part of every window is a copy of the table row of its centre (one wave per
        // window, 64 consecutive floats per store), then the patched cells are stored over it
        // (staging left each surviving patch's window position, overridden ones at -1)
        // one wave per window: 64 consecutive floats per load and store (batching several windows'
        // loads per lane measured slower: 33.4 vs 28.9 us at c5patch's shape, profiles/r4_window)
        for (int k = 0; k < K; ++k) {
            float *o = a.patch + ((int64_t)k * a.E + e0) * PP;
            for (int el = wave; el < nenv; el += THREADS / 64) {
                if (!(s_flag[el] & D_WRITE)) continue;  // wave-uniform
                const int ctr = s_ctr[el * K + k];
                const float *src = a.tbl + (int64_t)((ctr >> 16) * W + (ctr & 0xFFFF)) * PP;
                float *dst = o + (int64_t)el * PP;
                for (int c = lane; c < PP; c += 64) dst[c] = src[c];
            }
        }
        // the block's map stores complete (vmcnt counts stores on gfx9) before any patch store
        // to the same cells is issued
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        for (int t = tid; t < nenv * K * np; t += THREADS) {
            const int slot = t / np, i = t - slot * np, el = slot / K, k = slot - el * K;
            if (!(s_flag[el] & D_WRITE)) continue;
            const int pw = s_pw[slot * np + i];
            if (pw >= 0) a.patch[((int64_t)k * a.E + e0 + el) * PP + pw] = s_pv[slot * np + i];
        }
    } else if (a.patch) {  // one thread per element (consecutive lanes: consecutive floats), overrides in registers
        // i / PP and c / P as multiply-highs (i < PB * PP; P >= 2)
        const uint32_t m_pp = (uint32_t)((0x100000000ull + (uint64_t)PP - 1) / (uint64_t)PP);
        const uint32_t m_p = (uint32_t)((0x100000000ull + (uint64_t)P - 1) / (uint64_t)P);
        for (int k = 0; k < K; ++k) {
            float *o = a.patch + ((int64_t)k * a.E + e0) * PP;
            for (int i = tid; i < nenv * PP; i += THREADS) {
                const int el = (int)__umulhi((uint32_t)i, m_pp), c = i - el * PP;
                if (!(s_flag[el] & D_WRITE)) continue;
                const int slot = el * K + k;
                const int ctr = s_ctr[slot];
                const int wr = (int)__umulhi((uint32_t)c, m_p);
                float v = map_value(s_road, H, W, (ctr >> 16) + wr - half, (ctr & 0xFFFF) + c - wr * P - half);
                for (int u = 0; u < np; ++u) {
                    const float pv = s_pv[slot * np + u];
                    v = s_pw[slot * np + u] == c ? pv : v;
                }
                o[i] = v;
            }
        }
    }
    if (dbg) {
        __syncthreads();
        if (tid == 0) dbg[4 * blockIdx.x + 3] = wall_clock64();
    }
    if (!a.final_patch || !any_final) return;
    // terminal windows: one wave per (ended env, agent), values in registers, straight to HBM
    for (int wi = wave; wi < nenv * K; wi += THREADS / 64) {
        const int el = wi / K, k = wi - el * K;
        if (!(s_flag[el] & D_FINAL)) continue;  // wave-uniform
        const int slot = (PB + el) * K + k;
        const int ctr = s_ctr[slot], cr = ctr >> 16, cc = ctr & 0xFFFF;
        float *o = a.final_patch + ((int64_t)k * a.E + e0 + el) * PP;
        const float *trow = a.tbl ? a.tbl + (int64_t)(cr * W + cc) * PP : nullptr;  // MODE 4's table
        for (int c = lane; c < PP; c += 64) {
            float v = trow ? trow[c] : map_value(s_road, H, W, cr + c / P - half, cc + c % P - half);
            for (int u = 0; u < np; ++u)
                if (s_pw[slot * np + u] == c) v = s_pv[slot * np + u];
            o[c] = v;
        }
    }
}

// MODE 6 (round 5, any P <= 16, E % 4 == 0): one thread per window ROW, no staging phase and no
// block barrier.  Every thread decodes its env's descriptor itself (the P threads of a window read
// the same 48 bytes: one line), writes its row's map values (two road words: P <= 16 columns) into
// its wave's LDS slice, stores the patched cells that fall on its row over them in slot order (the
// apple, then agents 0 .. N - 1: a later slot overrides an earlier one, as the obs writer does; one
// scalar LDS store each, not a select per column), and the wave's 64 rows -- one contiguous run of
// 64 P floats -- leave as consecutive 16-byte stores.  The block-staged writers (MODES 2 / 4) spent
// ~6 us per block on a dependent staging phase with none of that block's stores in flight, and at
// c4patch ran at ~3 TB/s alone (45 us; the launch shape's store floor, GW_PATCH_MODE=9: 18 us).
// Terminal windows (D_FINAL) take the same path from the descriptor's terminal words.
// WR_RUNS = 2 runs of 64 rows per wave, the row's map written four columns at a time and the
// terminal descriptor words loaded only by waves with a terminal window (80 VGPRs at P <= 12:
// six waves per SIMD).  Alone at c4patch's / c5patch's shapes: 1 run 36.1 / 22.7 us, 2 runs
// 29.9 / 18.4, 4 runs 31.0 / 18.9, 8 runs 38.8 / 21.7 (the preloaded descriptors' registers)
template <int NP, int MAXW, int WR_RUNS = 2>  // MAXW: 8, 12 or 16 >= P (the row's registers)
__global__ void __launch_bounds__(256, 4) window_rows_kernel(gw::PatchArgs a) {
    __shared__ __attribute__((aligned(16))) float4 s_rows[4][64 * (MAXW / 4)];  // per wave: 64 rows
    gwrows::rows_block<NP, MAXW, WR_RUNS>(a, blockIdx.x, blockIdx.y, s_rows);
}

// MODE 4's table: tbl[c][o] = the map value under window position o of the window centred on
// cell c (-1 outside the grid); built once per (env, P)
__global__ void __launch_bounds__(256) window_table_kernel(gw::PatchArgs a, float *tbl) {
    const int PP = a.P * a.P, half = a.P / 2;
    const int64_t n = (int64_t)a.H * a.W * PP;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i / PP), o = (int)(i - (int64_t)c * PP);
        const int cr = c / a.W, cc = c - cr * a.W;
        tbl[i] = map_value(a.roadbits, a.H, a.W, cr + o / a.P - half, cc + o % a.P - half);
    }
}

// measurement only (GW_PATCH_MODE=9): the same grid, block size and run layout as the writers,
// every element of the step's windows stored as 0 with aligned float4 stores and no staging: the
// store floor of this launch shape
template <int PB>
__global__ void __launch_bounds__(THREADS) store_floor_kernel(gw::PatchArgs a) {
    const int PP = a.P * a.P;
    const int64_t e0 = (int64_t)blockIdx.x * PB;
    const int nenv = (int)min((int64_t)PB, a.E - e0);
    const int len = nenv * PP;
    for (int k = 0; k < a.K; ++k) {
        const int64_t off = ((int64_t)k * a.E + e0) * PP;
        float *o = a.patch + off;
        const int lead = (int)((4 - (off & 3)) & 3);
        for (int i = threadIdx.x; i < min(lead, len); i += THREADS) o[i] = 0.0f;
        const int n4 = (len - lead) / 4;
        float4 *o4 = reinterpret_cast<float4 *>(o + lead);
        for (int j = threadIdx.x; j < n4; j += THREADS) o4[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        for (int i = lead + 4 * n4 + threadIdx.x; i < len; i += THREADS) o[i] = 0.0f;
    }
}

}  // namespace

namespace gw {

unsigned long long *g_patch_dbg = nullptr;

template <int MODE, int PB>
hipError_t launch_mode(const PatchArgs &a, size_t lds, hipStream_t s) {
    // above the 64 KB a launch gets by default, the kernel's dynamic-LDS limit is raised once (up
    // to gfx950's 160 KB per workgroup)
    static size_t granted = 64 * 1024;
    if (lds > granted) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&window_kernel<MODE, PB>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        granted = lds;
    }
    const unsigned grid = (unsigned)((a.E + PB - 1) / PB);
    gwprof::launch(window_kernel<MODE, PB>, dim3(grid), dim3(THREADS), lds, s, a, g_patch_dbg);
    return hipGetLastError();
}

hipError_t launch_windows(const PatchArgs &args, hipStream_t s) {
    PatchArgs a = args;
    const int np = a.N + 1, PP = a.P * a.P;
    // envs per block: 32, or 64 (GW_PATCH_PB=64, measurement only for now)
    static const char *probe_env = GW_MEASURE_ENV("GW_PATCH_PROBE");  // (measurement only)
    if (probe_env) a.probe = std::atoi(probe_env);
    static const char *pb_env = GW_MEASURE_ENV("GW_PATCH_PB");
    const int PB = (pb_env && std::atoi(pb_env) == 64) ? 64 : 32;
    // LDS: road bitmask, flags, centres, patch cells + values, and per mode: MODE 0 one agent's
    // window run (PP <= 256), MODE 2 the nibble table (PB * K * P * P / 4 u16, patch indices
    // 1..15), MODE 3 one agent's byte table (PB * P * P + 4 bytes).  Preference: MODE 2 (P % 4 ==
    // 0), else MODE 3, each if its LDS fits gfx950's 160 KB per workgroup (above 64 KB through the
    // dynamic-LDS attribute), else the per-element writer (MODE 1, e.g. windows wider than the
    // byte table allows).
    const size_t base = sizeof(uint32_t) * ((a.H * a.W + 31) / 32 + PB) + sizeof(int) * 2 * PB * a.K +
                        sizeof(uint32_t) * (size_t)2 * 2 * PB * a.K * np;
    const size_t extra[6] = {sizeof(float) * (size_t)PB * PP, 0, sizeof(uint16_t) * (size_t)PB * a.K * (PP / 4),
                             (size_t)PB * PP + 16, 0, 0};
    constexpr size_t LDS_MAX = 160 * 1024;
    // MODE 2 for P % 4 == 0 (c4patch: 171 us per step vs 179 with MODE 4), MODE 4 for the other
    // P <= 16 (c5patch's P = 11: 28.9 us per launch vs MODE 3's 34.2), profiles/r4_window
    int mode = (a.P % 4 == 0 && np < 16 && base + extra[2] <= LDS_MAX) ? 2
               : (a.tbl && PP <= 256) ? 4
               : (np < 256 && base + extra[3] <= LDS_MAX) ? 3 : 1;
    static const char *force = GW_MEASURE_ENV("GW_PATCH_MODE");  // (measurement only: A/B of the writers)
    if (force) {
        const int f = std::atoi(force);
        if (f == 1 || (f == 0 && PP <= 64 * MAXPL && base + extra[0] <= LDS_MAX) ||
            (f == 2 && a.P % 4 == 0 && np < 16 && base + extra[2] <= LDS_MAX) || (f == 3 && base + extra[3] <= LDS_MAX) ||
            (f == 4 && a.tbl && PP <= 256))
            mode = f;
    }
    const bool rows_ok = a.P >= 2 && a.P <= 16 && a.E % 4 == 0 && a.N >= 1 && a.N <= GW_MAX_AGENTS &&
                         a.E * a.P < (1LL << 32);
    if (rows_ok && (!force || std::atoi(force) == 6)) {
        const dim3 grid((unsigned)((a.E * a.P + 512 - 1) / 512), a.K);  // 4 waves x 2 runs of 64 rows
        auto go = [&](auto np_c) {
            constexpr int NPv = decltype(np_c)::value;
            if (a.P <= 8) gwprof::launch(window_rows_kernel<NPv, 8>, grid, dim3(256), 0, s, a);
            else if (a.P <= 12) gwprof::launch(window_rows_kernel<NPv, 12>, grid, dim3(256), 0, s, a);
            else gwprof::launch(window_rows_kernel<NPv, 16>, grid, dim3(256), 0, s, a);
        };
        switch (a.N) {
            case 1: go(std::integral_constant<int, 2>{}); break;
            case 2: go(std::integral_constant<int, 3>{}); break;
            case 3: go(std::integral_constant<int, 4>{}); break;
            case 4: go(std::integral_constant<int, 5>{}); break;
            case 5: go(std::integral_constant<int, 6>{}); break;
            case 6: go(std::integral_constant<int, 7>{}); break;
            case 7: go(std::integral_constant<int, 8>{}); break;
            default: go(std::integral_constant<int, 9>{}); break;
        }
        return hipGetLastError();
    }
    if (force && std::atoi(force) == 9 && a.patch) {  // measurement only: the store floor
        const unsigned grid = (unsigned)((a.E + PB - 1) / PB);
        if (PB == 64)
            gwprof::launch(store_floor_kernel<64>, dim3(grid), dim3(THREADS), 0, s, a);
        else
            gwprof::launch(store_floor_kernel<32>, dim3(grid), dim3(THREADS), 0, s, a);
        return hipGetLastError();
    }
    const size_t lds = base + extra[mode];
    if (PB == 64) {
        switch (mode) {
            case 0: return launch_mode<0, 64>(a, lds, s);
            case 2: return launch_mode<2, 64>(a, lds, s);
            case 3: return launch_mode<3, 64>(a, lds, s);
            case 4: return launch_mode<4, 64>(a, lds, s);
            default: return launch_mode<1, 64>(a, lds, s);
        }
    }
    switch (mode) {
        case 0: return launch_mode<0, 32>(a, lds, s);
        case 2: return launch_mode<2, 32>(a, lds, s);
        case 3: return launch_mode<3, 32>(a, lds, s);
        case 4: return launch_mode<4, 32>(a, lds, s);
        default: return launch_mode<1, 32>(a, lds, s);
    }
}

size_t window_table_bytes(int H, int W, int P) { return sizeof(float) * (size_t)H * W * P * P; }

hipError_t build_window_table(const PatchArgs &a, float *tbl, hipStream_t s) {
    const int64_t n = (int64_t)a.H * a.W * a.P * a.P;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(window_table_kernel, dim3(grid), dim3(256), 0, s, a, tbl);
    return hipGetLastError();
}

}  // namespace gw

// measurement only (tools/patch_probe.py): per-block wall-clock stamps of the next launches
extern "C" void gw_patch_debug_buffer(void *buf) { gw::g_patch_dbg = static_cast<unsigned long long *>(buf); }
