// gridenv.hip — MI355X (gfx950) implementation of the vectorised grid world behind
// include/gridenv.h.
//
// Per gw_step, two launches on the caller's stream:
//   1. step_kernel   — everything that is per env: scripted policy (Philox), RL override,
//                      the FeAR counterfactual sims (custom/Responsibility.py:135-210), the
//                      world update (custom/grid_world.py:424-563), rewards/dones
//                      (custom/ma_customenv.py:258-302), the rollout arithmetic
//                      (maddpg/agent.py:124-173), auto-reset and a 48-byte obs descriptor.
//                      Integer/VALU work; with fear on, one block owns BE envs, turns their
//                      counterfactuals into a de-duplicated task list in LDS and lets all
//                      256 lanes run one sim each (no lane idles on a far agent).
//   2. obs_kernel    — writes the K x H*W float32 observation of every env
//                      (custom/ma_customenv.py:303-322) from the descriptors: a pure HBM
//                      store stream, 16 B per lane, coalesced, static map staged in LDS.
// Everything is exact integer logic; the only floating point is the f64 reward arithmetic,
// compiled with -ffp-contract=off and written with explicit _rn intrinsics in the order
// numpy/Python evaluate it.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <new>
#include <type_traits>
#include <string>
#include <vector>

#include "patch_ops.h"
#include "gridenv.h"
#include "prof.h"
#include "window_rows.h"

namespace gw {

constexpr int NA = GW_N_ACTIONS;
typedef float f32x4 __attribute__((ext_vector_type(4)));

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt(float4 *dst, const float4 &v) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4 *>(dst));
}
constexpr int MAXN = GW_MAX_AGENTS;
constexpr int NDESC = 12;  // u32 words per obs descriptor

// desc[4] flag bits
constexpr uint32_t D_RESET = 1u;      // obs uses the reset encoding (0.5 agents, no relabel)
constexpr uint32_t D_WRITE = 2u;      // write obs for this env
constexpr uint32_t D_FINAL = 4u;      // write final_obs for this env (terminal encoding)

struct Tables {
    const uint8_t *okmask;    // [HW] bit d: unit move d (0 U,1 D,2 L,3 R) allowed
    const uint8_t *policy;    // [HW]
    const double *cdf;        // [P][2][9]
    const uint8_t *mdr;       // [HW]
    const uint16_t *amask;    // [HW]
    const int32_t *free_cells;// [F]
    const float *base;        // [HW] 0 road / -1 inactive
    const double *resp;       // [10][10] clip((vm-va)/(vm+EPS),-1,1)
    const uint32_t *celltab;  // [HW] policy | MdR<<8 | action mask<<12 | unit moves<<21 | road<<25
    const uint32_t *roadbits; // [ceil(HW/32)] bit c: cell c is road
};

struct State {
    int32_t *pos;
    uint32_t *flags;
    int32_t *t;
    uint32_t *episode;
    int32_t *prev;
    double *score;
    double *fscore;
};

struct Params {
    Tables tb;
    State st;
    gw_step_out out;
    uint32_t *desc;           // [E][NDESC]
    const int32_t *rl;        // [E][K] or null
    const int32_t *scripted;  // [E][N-K] or null
    const int32_t *spawn;     // [E][N] or null
    const uint8_t *rmask;     // reset mask or null
    int64_t E, env_offset;
    double fear_weight;
    int H, W, HW, N, K, F;
    int max_steps, auto_reset;
    uint32_t key0, key1;
    uint32_t w_magic;         // ceil(2^32 / W)  (exact /W for cells < 2^16)
    uint32_t hw4_magic;       // ceil(2^32 / (H*W/4))
    uint32_t hw8_magic;       // ceil(2^32 / (H*W/8))
    int lds_cdf, n_cdf, ctab_off, resp_off;  // step_v2 dynamic LDS: [cdf][cell table][Resp 100 f64]
    int obs_be;               // envs per obs_kernel block (<= OBS_BE)
    int obs_bf16;             // obs buffers hold bf16 (the merged step_obs kernel's writer role)
    int64_t e_begin, e_end;   // env range of this launch (step_v2 / obs_kernel chunks)
    uint4 *fwork;             // [E][FearRec<N>::R4] deferred-FeAR records (GW_KERNEL=defer)
    int64_t stats_row0;       // first gw_step_out.stats row this launch writes
    int variant;              // 0 CustomMAEnv, 1 single-agent CustomEnv (custom/customenv.py)
    int apples[MAXN];
    unsigned long long *sims;  // gw_count_sims: FeAR counterfactual world updates run (null: not counted)
};

// ---------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based; every draw is keyed by global env id, episode, step, tag)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one 32x32->64 multiply per product (v_mad_u64_u32) instead of mul_lo + mul_hi
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ int div_w(const Params &p, int cell) {
    return (int)__umulhi((uint32_t)cell, p.w_magic);
}

__device__ __forceinline__ int manhattan(const Params &p, int a, int b) {
    const int ra = div_w(p, a), rb = div_w(p, b);
    const int ca = a - ra * p.W, cb = b - rb * p.W;
    return abs(ra - rb) + abs(ca - cb);
}

// ---------------------------------------------------------------------------------------
// One world update (GWorld.UpdateGWorld, custom/grid_world.py:424-563) in registers.
// Floor/ceil sub-path indices of (s+1)*len/4 and the overhang terms are compile-time per
// (len, s): len 1 -> f {0,0,0,1} c {1,1,1,1}; len 2 -> f {0,1,1,2} c {1,1,2,2}.
// ---------------------------------------------------------------------------------------
template <int S> struct SubStep;
template <> struct SubStep<0> { static constexpr int f1 = 0, c1 = 1, f2 = 0, c2 = 1, ohf1 = 3, ohc1 = 1, ohf2 = 2, ohc2 = 2; };
template <> struct SubStep<1> { static constexpr int f1 = 0, c1 = 1, f2 = 1, c2 = 1, ohf1 = 2, ohc1 = 2, ohf2 = 0, ohc2 = 0; };
template <> struct SubStep<2> { static constexpr int f1 = 0, c1 = 1, f2 = 1, c2 = 2, ohf1 = 1, ohc1 = 3, ohf2 = 2, ohc2 = 2; };
template <> struct SubStep<3> { static constexpr int f1 = 1, c1 = 1, f2 = 2, c2 = 2, ohf1 = 0, ohc1 = 0, ohf2 = 0, ohc2 = 0; };

// unit-move bits seen by the world update: the u32 cell table of step_v2 (bits CT_OK..CT_OK+3)
struct CtabOk {
    const uint32_t *t;
    __device__ __forceinline__ uint32_t operator()(int c) const { return t[c] >> 21; }
};

// LIST (N > 4, the 128-thread step_v2 chain): a collision pass walks this lane's own near pairs
// (a 64-bit mask, bit 8 ii + jj) and reads the two agents' floor / ceiling / start cells from a
// per-lane LDS row (`lw`, N uint2), instead of evaluating all N (N - 1) / 2 pairs under lane masks:
// with 64 envs per wave nearly every pair index has some lane near, so the unrolled form paid the
// whole pair list on every pass.
template <int N, bool LIST = false>
struct World {
    int nal[N][5];
    int loc[N];
    int delta[N];
    uint32_t two, mv, dir0, dir1;   // bit masks: 2-step action, moving action, direction bits
    uint32_t crash, restr;
    uint32_t near;                  // bit pair(ii, jj): start cells within Manhattan 4
    uint64_t near8 = 0;             // LIST: bit 8 ii + jj for the same pairs
    uint2 *lw = nullptr;            // LIST: this lane's LDS row [N] {floor | ceil << 16, start | two << 16}
    // A pair whose start cells are more than 4 apart can never trigger a rule of
    // collision_checks_and_resolution: every sub-path entry stays within 2 of its own start
    // (reverts go back to the start), so equal / crossing cells need distance <= 4.  Such
    // pairs are skipped; with no near pair at all the resolution loop is skipped.

    __device__ __forceinline__ static constexpr int pair_bit(int ii, int jj) {
        return ii * (2 * N - ii - 1) / 2 + (jj - ii - 1);
    }

    __device__ __forceinline__ void init(const int (&l)[N], const int (&a)[N], int W, uint32_t w_magic) {
        two = mv = dir0 = dir1 = crash = restr = near = 0;
        int rr[N], cc[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            rr[i] = (int)__umulhi((uint32_t)l[i], w_magic);
            cc[i] = l[i] - rr[i] * W;
        }
#pragma unroll
        for (int ii = 0; ii < N - 1; ++ii)
#pragma unroll
            for (int jj = ii + 1; jj < N; ++jj)
            {
                const bool nr = abs(rr[ii] - rr[jj]) + abs(cc[ii] - cc[jj]) <= 4;
                near |= (uint32_t)nr << pair_bit(ii, jj);
                if (LIST) near8 |= (uint64_t)nr << (8 * ii + jj);
            }
#pragma unroll
        for (int i = 0; i < N; ++i) {
            loc[i] = l[i];
            nal[i][0] = l[i];
            const int act = a[i];
            const int d = (act - 1) & 3;  // 0 U, 1 D, 2 L, 3 R
            two |= (uint32_t)(act >= 5) << i;
            mv |= (uint32_t)(act != 0) << i;
            dir0 |= (uint32_t)(d & 1) << i;
            dir1 |= (uint32_t)(d >> 1) << i;
            delta[i] = (d == 0) ? -W : (d == 1) ? W : (d == 2) ? -1 : 1;
        }
    }

    __device__ __forceinline__ int dir_of(int i) const {
        return (int)(((dir0 >> i) & 1u) | (((dir1 >> i) & 1u) << 1));
    }

    // values, not a conditional lvalue: a select between two element addresses would keep
    // the sub-paths in scratch instead of registers
    template <int S>
    __device__ __forceinline__ int fl(int i) const {
        const int a2 = nal[i][SubStep<S>::f2], a1 = nal[i][SubStep<S>::f1];
        return ((two >> i) & 1u) ? a2 : a1;
    }
    template <int S>
    __device__ __forceinline__ int ce(int i) const {
        const int a2 = nal[i][SubStep<S>::c2], a1 = nal[i][SubStep<S>::c1];
        return ((two >> i) & 1u) ? a2 : a1;
    }

    template <int S, class OK>
    __device__ __forceinline__ void move(const OK &okm) {  // :462-518
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int old = nal[i][S];
            if (S >= 2) {  // every action has at most 2 sub-moves: (0, 0) from here on
                nal[i][S + 1] = old;
                continue;
            }
            const bool active_sub = (S == 0) || ((two >> i) & 1u);
            const bool moving = active_sub && ((mv >> i) & 1u) && !((crash >> i) & 1u);
            int nw = old;
            if (moving) {
                const bool ok = (okm(old) >> dir_of(i)) & 1u;  // clip + WorldState[new] >= 0
                nw = ok ? old + delta[i] : old;
                restr |= (uint32_t)(!ok) << i;
            }
            nal[i][S + 1] = nw;
        }
    }

    template <int S>
    __device__ __forceinline__ void resolve_list() {  // LIST form of resolve<S>
        if (near == 0) return;
#pragma unroll
        for (int i = 0; i < N; ++i) lw[i].y = (uint32_t)loc[i] | (((two >> i) & 1u) << 16);
        for (int pass = 0; pass < 2 * N; ++pass) {
#pragma unroll
            for (int i = 0; i < N; ++i) lw[i].x = (uint32_t)fl<S>(i) | ((uint32_t)ce<S>(i) << 16);
            uint32_t hit = 0;
            uint64_t m = near8;
            while (m) {  // this lane's near pairs, in ascending (ii, jj) order
                const int pb = (int)__builtin_ctzll(m);
                m &= m - 1;
                const int ii = pb >> 3, jj = pb & 7;
                const uint2 a = lw[ii], b = lw[jj];
                const int Af = (int)(a.x & 0xFFFFu), Ac = (int)(a.x >> 16), Li = (int)(a.y & 0xFFFFu);
                const int Bf = (int)(b.x & 0xFFFFu), Bc = (int)(b.x >> 16), Lj = (int)(b.y & 0xFFFFu);
                const bool t_i = (a.y >> 16) & 1u, t_j = (b.y >> 16) & 1u;
                const int ohf_i = t_i ? SubStep<S>::ohf2 : SubStep<S>::ohf1;
                const int ohc_i = t_i ? SubStep<S>::ohc2 : SubStep<S>::ohc1;
                const int ohf_j = t_j ? SubStep<S>::ohf2 : SubStep<S>::ohf1;
                const int ohc_j = t_j ? SubStep<S>::ohc2 : SubStep<S>::ohc1;
                const bool same_dir = (Ac - Af) == (Bc - Bf);
                // the elif chain of :276-378 as selects (the N <= 4 form of resolve)
                const bool x1 = Af == Bc, x2 = Ac == Bf;
                const bool cross = ((Af == Lj) | (Ac == Lj)) & ((Li == Bf) | (Li == Bc));
                const bool tail = x1 ? !((ohf_i + ohc_j) <= 4 && same_dir)
                                     : (x2 ? !((ohf_j + ohc_i) <= 4 && same_dir) : cross);
                const bool coll = (Af == Bf) | (Ac == Bc) | (x1 & x2) | tail;
                hit |= coll ? ((1u << ii) | (1u << jj)) : 0u;
            }
            crash |= hit;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if ((crash >> i) & 1u) {
                    const int f = ((two >> i) & 1u) ? SubStep<S>::f2 : SubStep<S>::f1;
#pragma unroll
                    for (int k = 0; k <= S + 1; ++k)
                        if (k >= f) nal[i][k] = loc[i];
                }
            }
            if (hit == 0) break;
        }
    }

    template <int S>
    __device__ __forceinline__ void resolve() {  // collision_checks_and_resolution :233-405
        if constexpr (LIST) {
            resolve_list<S>();
            return;
        }
        if (near == 0) return;  // no pair can collide: every pass counts 0 (crash stays 0)
        for (int pass = 0; pass < 2 * N; ++pass) {
            uint32_t hit = 0;
#pragma unroll
            for (int ii = 0; ii < N - 1; ++ii) {
                const int Af = fl<S>(ii), Ac = ce<S>(ii);
                const bool t_i = (two >> ii) & 1u;
                const int ohf_i = t_i ? SubStep<S>::ohf2 : SubStep<S>::ohf1;
                const int ohc_i = t_i ? SubStep<S>::ohc2 : SubStep<S>::ohc1;
#pragma unroll
                for (int jj = ii + 1; jj < N; ++jj) {
                    if (!((near >> pair_bit(ii, jj)) & 1u)) continue;
                    const int Bf = fl<S>(jj), Bc = ce<S>(jj);
                    const bool t_j = (two >> jj) & 1u;
                    const int ohf_j = t_j ? SubStep<S>::ohf2 : SubStep<S>::ohf1;
                    const int ohc_j = t_j ? SubStep<S>::ohc2 : SubStep<S>::ohc1;
                    const bool same_dir = (Ac - Af) == (Bc - Bf);
                    bool coll;
                    if constexpr (N <= 4) {  // the same elif chain as selects (few pairs: no VGPR pressure)
                        const bool x1 = Af == Bc, x2 = Ac == Bf;
                        const bool cross = ((Af == loc[jj]) | (Ac == loc[jj])) & ((loc[ii] == Bf) | (loc[ii] == Bc));
                        const bool tail = x1 ? !((ohf_i + ohc_j) <= 4 && same_dir)
                                             : (x2 ? !((ohf_j + ohc_i) <= 4 && same_dir) : cross);
                        coll = (Af == Bf) | (Ac == Bc) | (x1 & x2) | tail;
                    } else if (Af == Bf || Ac == Bc) {
                        coll = true;                                    // :276-278
                    } else if (Af == Bc && Ac == Bf) {
                        coll = true;                                    // :291-294
                    } else if (Af == Bc) {
                        coll = !((ohf_i + ohc_j) <= 4 && same_dir);     // :307-337
                    } else if (Ac == Bf) {
                        coll = !((ohf_j + ohc_i) <= 4 && same_dir);     // :339-368
                    } else {
                        const int Li = loc[ii], Lj = loc[jj];           // :371-378
                        coll = (Af == Lj && Li == Bf) || (Ac == Lj && Li == Bc) ||
                               (Af == Lj && Li == Bc) || (Ac == Lj && Li == Bf);
                    }
                    if (coll) hit |= (1u << ii) | (1u << jj);
                }
            }
            crash |= hit;
            // revertStepsWithCollisions :190-209 (all crashed agents, every pass)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if ((crash >> i) & 1u) {
                    const int f = ((two >> i) & 1u) ? SubStep<S>::f2 : SubStep<S>::f1;
#pragma unroll
                    for (int k = 0; k <= S + 1; ++k)
                        if (k >= f) nal[i][k] = loc[i];
                }
            }
            if (hit == 0) break;  // this pass recorded no collision (CollisionCount == 0)
        }
    }

    template <int S>
    __device__ __forceinline__ int cf(int i) const {  // NewAgentLocations_CurrentFloor
        return (N == 1) ? loc[i] : fl<S>(i);
    }
};

// UpdateGWorld (grid_world.py:424-563).  caught: bits 0-7 = eaters k that stood on apple[k] at
// some sub-step (floor position, :530-545); bits 8+ = the number of (k, apple) entries the
// reference appends to apples_caught (the single-agent env rewards only len == 1).
template <int N, bool APPLES, class OK, bool LIST>
__device__ __forceinline__ void simulate(World<N, LIST> &w, const OK &okm, int K,
                                         const int (&apple)[MAXN], uint32_t &caught, int (&fin)[N]) {
    caught = 0;
    w.template move<0, OK>(okm);
    w.template resolve<0>();
    if (APPLES) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && w.template cf<0>(k) == apple[k]) caught = (caught | (1u << k)) + (1u << 8);
    }
    w.template move<1, OK>(okm);
    w.template resolve<1>();
    if (APPLES) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && w.template cf<1>(k) == apple[k]) caught = (caught | (1u << k)) + (1u << 8);
    }
    w.template move<2, OK>(okm);
    w.template resolve<2>();
    if (APPLES) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && w.template cf<2>(k) == apple[k]) caught = (caught | (1u << k)) + (1u << 8);
    }
    w.template move<3, OK>(okm);
    w.template resolve<3>();
#pragma unroll
    for (int i = 0; i < N; ++i) fin[i] = w.template cf<3>(i);
    if (APPLES) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && fin[k] == apple[k]) caught = (caught | (1u << k)) + (1u << 8);
    }
}

// numpy float64 sum (0.0 + pairwise_sum) of an N*N matrix whose only non-zero row is `row`
// (np.sum(FeAR_vals), custom/ma_customenv.py:252).  Zeros never change a partial sum here
// (no -0.0 can occur), so only the row's terms are accumulated, in numpy's order.
template <int N>
__device__ __forceinline__ double np_sum_row(const double (&v)[N], int row) {
    constexpr int n = N * N;
    if (n < 8) {
        double res = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) res = __dadd_rn(res, v[j]);
        return __dadd_rn(0.0, res);
    } else {
        static_assert(N * N <= 128, "N <= 11");
        double r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = 0.0;
        constexpr int main_end = n - (n % 8);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int idx = row * N + j;
            if (idx < main_end) {
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if ((idx & 7) == q) r[q] = __dadd_rn(r[q], v[j]);
            }
        }
        double res = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                               __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int idx = row * N + j;
            if (idx >= main_end) res = __dadd_rn(res, v[j]);
        }
        return __dadd_rn(0.0, res);
    }
}

// numpy sum of a short 1-D f64 vector (n <= 8): scores += np.sum(rewards) (agent.py:173).
__device__ __forceinline__ double np_sum_small(const double (&a)[MAXN], int n) {
    if (n < 8) {
        double res = 0.0;
#pragma unroll
        for (int i = 0; i < MAXN; ++i)
            if (i < n) res = __dadd_rn(res, a[i]);
        return __dadd_rn(0.0, res);
    }
    double res = __dadd_rn(__dadd_rn(__dadd_rn(a[0], a[1]), __dadd_rn(a[2], a[3])),
                           __dadd_rn(__dadd_rn(a[4], a[5]), __dadd_rn(a[6], a[7])));
    return __dadd_rn(0.0, res);
}

// ---------------------------------------------------------------------------------------
// per-env helpers
// ---------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void spawn_cells(const Params &p, int64_t e, uint32_t episode, int (&pos)[N]) {
    if (p.spawn) {
#pragma unroll
        for (int n = 0; n < N; ++n) pos[n] = p.spawn[e * N + n];
        return;
    }
    // Floyd's uniform N-subset of the road cells, then sorted (ma_customenv.py:373-380).
    const uint32_t gid = (uint32_t)(p.env_offset + e);
    int S[N];
    uint4 r = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int d = 0; d < N; ++d) {
        if ((d & 3) == 0) r = philox(gid, episode, 0xFFFFFFFFu, (3u << 24) | (uint32_t)(d >> 2), p.key0, p.key1);
        const uint32_t word = ((d & 3) == 0) ? r.x : ((d & 3) == 1) ? r.y : ((d & 3) == 2) ? r.z : r.w;
        const uint32_t j = (uint32_t)(p.F - N + d);
        const int cand = (int)(((uint64_t)word * (uint64_t)(j + 1)) >> 32);
        bool dup = false;
#pragma unroll
        for (int q = 0; q < d; ++q) dup |= (S[q] == cand);
        S[d] = dup ? (int)j : cand;
    }
    // sorting network (insertion, unrolled)
#pragma unroll
    for (int a = 1; a < N; ++a) {
#pragma unroll
        for (int b = a; b > 0; --b) {
            const int x = S[b - 1], y = S[b];
            S[b - 1] = min(x, y);
            S[b] = max(x, y);
        }
    }
#pragma unroll
    for (int n = 0; n < N; ++n) pos[n] = p.tb.free_cells[S[n]];
}

__device__ __forceinline__ uint32_t all_bits(int K) { return (K >= 32) ? 0xFFFFFFFFu : ((1u << K) - 1u); }

template <int N>
__device__ __forceinline__ void write_desc_pos(uint32_t *d, const int (&pos)[N]) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int n = 0; n < N; ++n) w[n >> 1] |= ((uint32_t)pos[n] & 0xFFFFu) << (16 * (n & 1));
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = w[q];
}

template <int N, bool ZERO_SCORE = true>
__device__ __forceinline__ void reset_env(const Params &p, int64_t e, uint32_t episode, int (&pos)[N]) {
    spawn_cells<N>(p, e, episode, pos);
#pragma unroll
    for (int n = 0; n < N; ++n) p.st.pos[(int64_t)n * p.E + e] = pos[n];
    p.st.flags[e] = all_bits(p.K);
    p.st.t[e] = 0;
    p.st.episode[e] = episode;
    for (int k = 0; k < p.K; ++k)  // None (ma_customenv.py:213); customenv.py:342-345 sets it at reset
        p.st.prev[(int64_t)k * p.E + e] = p.variant == 1 ? manhattan(p, pos[k], p.apples[k]) : -1;
    if (ZERO_SCORE) {  // with deferred FeAR the fear kernel owns score / fear_score
        p.st.score[e] = 0.0;
        p.st.fscore[e] = 0.0;
    }
}

// Deferred-FeAR record of one env step (GW_KERNEL=defer): what fear_v2 needs to finish the
// step after step_v2 has moved the world on.  R4 uint4 words per env, AoS for 16-byte
// coalesced access:  u16 pre-step cells [N] | u8 actions [N] (bit 7 of byte 0 = done, bit 6 of
// byte k = the single-agent env's +0.1 distance reward of agent k) | i8 integer env rewards [K].
// N <= 4: words 0-1 | 2 | 3;  N <= 8: words 0-3 | 4-5 | 6-7.
template <int N>
struct FearRec {
    static constexpr int R4 = N <= 4 ? 1 : 2, PW = 2 * R4, AW = PW, RW = PW + R4;
    uint32_t w[4 * R4];
};

template <int N>
__device__ __forceinline__ void store_fear_rec(const Params &p, int64_t e, const int (&pos)[N], const int (&act)[N],
                                               const int (&rew)[MAXN], uint32_t bonus, bool done) {
    using R = FearRec<N>;
    R r;
#pragma unroll
    for (int i = 0; i < 4 * R::R4; ++i) r.w[i] = 0u;
#pragma unroll
    for (int n = 0; n < N; ++n) {
        r.w[n >> 1] |= ((uint32_t)pos[n] & 0xFFFFu) << (16 * (n & 1));
        r.w[R::AW + (n >> 2)] |= (((uint32_t)act[n] & 0x3Fu) | (((bonus >> n) & 1u) << 6)) << (8 * (n & 3));
        if (n < p.K) r.w[R::RW + (n >> 2)] |= ((uint32_t)rew[n] & 0xFFu) << (8 * (n & 3));
    }
    r.w[R::AW] |= (uint32_t)done << 7;
    uint4 *dst = p.fwork + e * R::R4;
#pragma unroll
    for (int q = 0; q < R::R4; ++q) dst[q] = make_uint4(r.w[4 * q], r.w[4 * q + 1], r.w[4 * q + 2], r.w[4 * q + 3]);
}

template <int N>
__device__ __forceinline__ void load_fear_rec(const Params &p, int64_t e, int (&pos)[N], int (&act)[N],
                                              int (&rew)[MAXN], uint32_t &bonus, bool &done) {
    using R = FearRec<N>;
    R r;
    const uint4 *src = p.fwork + e * R::R4;
#pragma unroll
    for (int q = 0; q < R::R4; ++q) {
        const uint4 v = src[q];
        r.w[4 * q] = v.x; r.w[4 * q + 1] = v.y; r.w[4 * q + 2] = v.z; r.w[4 * q + 3] = v.w;
    }
    bonus = 0;
#pragma unroll
    for (int n = 0; n < N; ++n) {
        pos[n] = (int)((r.w[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
        const uint32_t byte = (r.w[R::AW + (n >> 2)] >> (8 * (n & 3))) & 0xFFu;
        act[n] = (int)(byte & 0x3Fu);
        bonus |= ((byte >> 6) & 1u) << n;
    }
#pragma unroll
    for (int k = 0; k < MAXN; ++k)
        rew[k] = (k < N) ? (int)(int8_t)((r.w[R::RW + (k >> 2)] >> (8 * (k & 3))) & 0xFFu) : 0;
    done = (r.w[R::AW] >> 7) & 1u;
}

// Rewards, dones, rollout arithmetic, state update, auto-reset, outputs, obs descriptor.
// custom/ma_customenv.py:254-334, maddpg/agent.py:124-173,226-243
struct Contrib {  // this env's share of gw_step_out.stats
    double v[GW_STATS];
};

// one field of a block's stats row: the step's value (stats) and / or its running total.  The
// total is a no-return f64 atomic add (one IEEE add at the L2, as the load + add + store was):
// each row belongs to one block per launch and launches are stream-ordered, so the sum order is
// fixed, and the block's last wave no longer waits a load round trip before it can end.
__device__ __forceinline__ void stats_put(const gw_step_out &o, int64_t idx, double v) {
    if (o.stats) o.stats[idx] = v;
    if (o.stats_acc) __hip_atomic_fetch_add(o.stats_acc + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the step's tick (gw_step_out.tick): one vector atomic by one lane of the step's first block
__device__ __forceinline__ void step_tick(const gw_step_out &o) {
    if (o.tick) __hip_atomic_fetch_add(o.tick, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void contrib_zero(Contrib &c) {
#pragma unroll
    for (int i = 0; i < GW_STATS; ++i) c.v[i] = 0.0;
}

// deterministic wave64 butterfly sum of every field
__device__ __forceinline__ void wave_sum(Contrib &c) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int i = 0; i < GW_STATS; ++i) c.v[i] = __dadd_rn(c.v[i], __shfl_xor(c.v[i], off, 64));
}

// The same butterfly for the fields a kernel can make non-zero only: FM = f64 fields (the same
// order as wave_sum: bit-identical), IM = integer-valued fields (exact counts, summed as int32:
// the same values), every other field 0.0.  Fewer cross-lane moves on the step's latency chain.
template <uint32_t FM, uint32_t IM>
__device__ __forceinline__ void wave_sum_sel(Contrib &c) {
    int iv[GW_STATS];
#pragma unroll
    for (int i = 0; i < GW_STATS; ++i) iv[i] = ((IM >> i) & 1u) ? (int)c.v[i] : 0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int i = 0; i < GW_STATS; ++i) {
            if ((FM >> i) & 1u) c.v[i] = __dadd_rn(c.v[i], __shfl_xor(c.v[i], off, 64));
            else if ((IM >> i) & 1u) iv[i] += __shfl_xor(iv[i], off, 64);
        }
#pragma unroll
    for (int i = 0; i < GW_STATS; ++i)
        if (!((FM >> i) & 1u)) c.v[i] = ((IM >> i) & 1u) ? (double)iv[i] : 0.0;
}

// stats fields: 0 completed-episode return, 2 FeAR, 5 shaped reward (f64); 1 episodes,
// 3 crashes, 4 apples, 6 completed-episode length, 7 env-steps (integer counts)
constexpr uint32_t ST_INT = (1u << 1) | (1u << 3) | (1u << 4) | (1u << 6) | (1u << 7);
constexpr uint32_t ST_F64_FEAR = (1u << 0) | (1u << 2) | (1u << 5);

// One env's state, loaded once (prefetched before the counterfactual phase in step_v2).
template <int N>
struct EnvState {
    int pos[N];
    uint32_t flags, episode;
    int t;
    int prev[N];
    double score, fscore;
};

template <int N>
__device__ __forceinline__ void load_env(const Params &p, int64_t e, EnvState<N> &s) {
#pragma unroll
    for (int n = 0; n < N; ++n) s.pos[n] = p.st.pos[(int64_t)n * p.E + e];
    s.flags = p.st.flags[e];
    s.episode = p.st.episode[e];
    s.t = p.st.t[e];
#pragma unroll
    for (int k = 0; k < N; ++k) s.prev[k] = (k < p.K) ? p.st.prev[(int64_t)k * p.E + e] : -1;
    s.score = p.st.score[e];
    s.fscore = p.st.fscore[e];
}

// What the obs writer needs to know about one env after its step.
template <int N>
struct ObsInfo {
    int pos[N];      // agents of the returned obs (post-step, or the new episode's spawn)
    int fpos[N];     // agents of the terminal obs (valid with D_FINAL)
    uint32_t flags;  // D_RESET | D_WRITE | D_FINAL | apples of obs << 8 | apples of final obs << 16
};

template <int N>
__device__ __forceinline__ void store_desc(const Params &p, int64_t e, const ObsInfo<N> &oi) {
    uint32_t *d = p.desc + e * NDESC;
    write_desc_pos<N>(d, oi.pos);
    d[4] = oi.flags;
    if (oi.flags & D_FINAL) write_desc_pos<N>(d + 8, oi.fpos);
    if (p.out.desc_copy) {  // the second destination (a descriptor replay ring's slot)
        uint32_t *c = p.out.desc_copy + e * NDESC;
        write_desc_pos<N>(c, oi.pos);
        c[4] = oi.flags;
        if (oi.flags & D_FINAL) write_desc_pos<N>(c + 8, oi.fpos);
    }
}

// DEFER (GW_KERNEL=defer, FeAR on): everything FeAR touches -- fear, shaped reward, score,
// fear_score, ep_return / ep_fear and stats fields 0, 2, 5 -- is left to fear_v2, which gets a
// FearRec; the rest (positions, dones, env rewards, auto-reset, obs descriptor) is final here.
template <int N, bool DEFER = false>
__device__ __forceinline__ void finish_env(const Params &p, int64_t e, const EnvState<N> &es,
                                           const int (&act)[N], const int (&mdr)[N],
                                           const double (&fear)[MAXN], uint32_t crash,
                                           uint32_t restr, int (&fin)[N], uint32_t caught,
                                           Contrib &ct, ObsInfo<N> &oi, const uint32_t *ctab = nullptr) {
    const int K = p.K;
    const uint32_t flags = es.flags;
    uint32_t apples = flags & 0xFFu, term = (flags >> 8) & 0xFFu, trunc = (flags >> 16) & 0xFFu;
    const uint32_t allk = all_bits(K);
    int t = es.t + 1;
    int rew[MAXN];
#pragma unroll
    for (int k = 0; k < MAXN; ++k) rew[k] = 0;
    const bool single = p.variant == 1;  // custom/customenv.py:127-160 (K = 1)
    // apples (:258-275): own apple, once; all eaten -> +20 to all, truncation.  Single agent
    // (customenv.py:142-148): rewarded only when apples_caught holds exactly one entry.
    const uint32_t popped = single ? (((caught >> 8) == 1u) ? (caught & apples & 1u) : 0u) : (caught & apples & 0xFFu);
    apples &= ~popped;
    int apple_rewarded = __popc(popped);
#pragma unroll
    for (int k = 0; k < N; ++k)
        if ((popped >> k) & 1u) rew[k] += 20;
    if (popped && apples == 0) {
        if (single) {
            trunc |= 1u;
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (k < K) rew[k] += 20;
            trunc = allk;
        }
    }
    int crash_count = 0;
    uint32_t bonus = 0;  // single agent: +0.1 for moving closer to the apple (customenv.py:155-156)
    double rewd[MAXN];
    double shaped[MAXN];
    double fsum_in[MAXN];
#pragma unroll
    for (int k = 0; k < MAXN; ++k) shaped[k] = fsum_in[k] = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (k >= K) continue;
        if ((crash >> k) & 1u) {  // :281-285 (single agent :138-140: terminated only)
            rew[k] -= 10;
            ++crash_count;
            if (!single) trunc = allk;
            term |= 1u << k;
        }
        const int64_t pi = (int64_t)k * p.E + e;
        const int prev = es.prev[k];
        if (single) {  // distance to the apple cell, eaten or not (apple_loc is read before the pop)
            const int d = manhattan(p, fin[k], p.apples[k]);
            bonus |= (uint32_t)(d < prev) << k;
            p.st.prev[pi] = d;
        } else {
            const int d = ((apples >> k) & 1u) ? manhattan(p, fin[k], p.apples[k]) : -1;  // :287-294
            if (prev >= 0 && d >= 0 && prev > d) rew[k] += 1;  // :296-300
            p.st.prev[pi] = d;
        }
        rewd[k] = ((bonus >> k) & 1u) ? __dadd_rn((double)rew[k], 0.1) : (double)rew[k];
        shaped[k] = __dadd_rn(__dmul_rn(p.fear_weight, fear[k]), rewd[k]);  // agent.py:130
        fsum_in[k] = fear[k];
    }
    const double score = DEFER ? 0.0 : __dadd_rn(es.score, np_sum_small(shaped, K));    // agent.py:173
    const double fscore = DEFER ? 0.0 : __dadd_rn(es.fscore, np_sum_small(fsum_in, K));  // agent.py:141
    const bool done = ((term & allk) == allk) || ((trunc & allk) == allk) ||
                      (p.max_steps > 0 && t >= p.max_steps);                       // agent.py:241-243

    const gw_step_out &o = p.out;
    ct.v[0] = (done && !DEFER) ? score : 0.0;
    ct.v[1] = done ? 1.0 : 0.0;
    ct.v[2] = DEFER ? 0.0 : np_sum_small(fsum_in, K);
    ct.v[3] = (double)crash_count;
    ct.v[4] = (double)apple_rewarded;
    ct.v[5] = DEFER ? 0.0 : np_sum_small(shaped, K);
    ct.v[6] = done ? (double)t : 0.0;
    ct.v[7] = 1.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (k >= K) continue;
        const int64_t ek = e * K + k;
        if (o.reward) o.reward[ek] = rewd[k];
        if (!DEFER && o.fear) o.fear[ek] = fear[k];
        if (!DEFER && o.shaped) o.shaped[ek] = shaped[k];
        if (o.term) o.term[ek] = (uint8_t)((term >> k) & 1u);
        if (o.trunc) o.trunc[ek] = (uint8_t)((trunc >> k) & 1u);
    }
    if (o.done) o.done[e] = done;
    if (o.done_copy) o.done_copy[e] = done;
    if (o.crashes) o.crashes[e] = crash_count;
    if (o.apples) o.apples[e] = apple_rewarded;
    if (!DEFER && o.ep_return) o.ep_return[e] = score;
    if (!DEFER && o.ep_fear) o.ep_fear[e] = fscore;
    if (o.ep_len) o.ep_len[e] = t;
    if (DEFER) store_fear_rec<N>(p, e, es.pos, act, rew, bonus, done);
    if (o.crash_bits) o.crash_bits[e] = (uint8_t)crash;
    if (o.restr_bits) o.restr_bits[e] = (uint8_t)restr;
#pragma unroll
    for (int n = 0; n < N; ++n) {
        if (o.actions) o.actions[e * N + n] = act[n];
        if (o.mdr) o.mdr[e * N + n] = mdr[n];
        if (o.final_pos) o.final_pos[e * N + n] = fin[n];
    }

    if (done && p.auto_reset) {
        // terminal obs -> final_obs, then CustomMAEnv.reset for the next episode
        const uint32_t ep = es.episode + 1;
        int np_[N];
        reset_env<N, !DEFER>(p, e, ep, np_);
#pragma unroll
        for (int n = 0; n < N; ++n) {
            oi.fpos[n] = fin[n];
            oi.pos[n] = np_[n];
        }
        // the terminal descriptor is kept for every done env (writers skip it without a
        // final_obs buffer; gw_obs_patch's terminal windows need no dense obs)
        oi.flags = D_RESET | D_WRITE | D_FINAL | (all_bits(K) << 8) | (apples << 16);
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && o.mask) o.mask[e * K + k] = ctab ? (uint16_t)((ctab[np_[k]] >> 12) & 0x1FFu) : p.tb.amask[np_[k]];
    } else {
#pragma unroll
        for (int n = 0; n < N; ++n) p.st.pos[(int64_t)n * p.E + e] = fin[n];
        p.st.flags[e] = apples | (term << 8) | (trunc << 16);
        p.st.t[e] = t;
        if (!DEFER) {
            p.st.score[e] = score;
            p.st.fscore[e] = fscore;
        }
#pragma unroll
        for (int n = 0; n < N; ++n) oi.pos[n] = oi.fpos[n] = fin[n];
        oi.flags = D_WRITE | (apples << 8);
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k < K && o.mask) o.mask[e * K + k] = ctab ? (uint16_t)((ctab[fin[k]] >> 12) & 0x1FFu) : p.tb.amask[fin[k]];
    }
}

// a plain 16-byte-per-lane copy (gw_obs_desc_copy)
__global__ void __launch_bounds__(256) copy16_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------
// reset kernel (CustomMAEnv.reset for masked envs)
// ---------------------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(256) reset_kernel(Params p) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= p.E) return;
    uint32_t *d = p.desc + e * NDESC;
    if (p.rmask && !p.rmask[e]) {
        d[4] = 0;
        return;
    }
    int pos[N];
    reset_env<N>(p, e, p.st.episode[e] + 1u, pos);
    write_desc_pos<N>(d, pos);
    d[4] = D_RESET | D_WRITE | (all_bits(p.K) << 8);
    if (p.out.mask)
        for (int k = 0; k < p.K; ++k) p.out.mask[e * p.K + k] = p.tb.amask[pos[k]];
}

// ---------------------------------------------------------------------------------------
// obs kernel: obs[k][e][cell] float32 from the descriptors.
//   step obs  (ma_customenv.py:303-322): map, agent n -> n+1, +9 own apple, relabel
//   reset obs (ma_customenv.py:197-209): map, 0.5 at agents, +9 own apple
// Each (env, k) has at most N+1 non-map cells ("patches"), computed once per block in LDS;
// the store loop is then map float4 + <= N+1 compares per 16-byte store.
// ---------------------------------------------------------------------------------------
constexpr int OBS_BE = 16;     // envs per block (max)
constexpr int OBS_THREADS = 256;

__device__ __forceinline__ float agent_value(bool reset, int n, int k, bool on_apple, int variant) {
    if (reset) return on_apple ? 9.5f : 0.5f;
    if (on_apple) return (float)(n + 1 + 9);
    if (variant == 1) return (float)(n + 1);  // customenv.py:163-166: raw WorldState ids
    int v = n + 1;
    if (v >= 1 && v <= 4 && v != k + 1) v = 5;   // other ids -> 5 (all_ids = [1,2,3,4], :314)
    if (v == k + 1) v = 1;                        // my id -> 1 (:321)
    return (float)v;
}

// bf16 bits of an obs value: every value the env writes (-1, 0, 0.5, 1, 5..13, 9.5) is exact in
// bf16, so the compact format is lossless (the low 16 bits of the f32 are zero)
__device__ __forceinline__ uint32_t bf16_bits(float v) { return __float_as_uint(v) >> 16; }

// The f32 writer's patch tables (round 6).  Per (env, agent) the float4s its
// <= N + 1 patches touch are built ONCE in LDS (the map float4 with every patch of that float4
// applied in slot order) and a byte per float4 of the obs names its entry (0 = map only), so a
// 16-byte store costs one byte lookup instead of N + 1 compares and selects.  Used where the byte
// tables fit (obs_tab_bytes <= OBS_TAB_MAX); else the compare loop.  The terminal obs of the few
// envs that ended (final_obs) keep the compare loop: tables for them would double the block's LDS,
// which decides whether the rollout's large-LDS kernels (the learner's tails) fit beside writer blocks.
constexpr int OBS_TAB_MAX = 16384;
__host__ __device__ __forceinline__ int obs_tab_stride(int HW) { return ((HW >> 2) + 15) & ~15; }
__host__ __device__ __forceinline__ int obs_tab_bytes(int HW, int obs_be, int K) {
    return obs_be * K * obs_tab_stride(HW);
}
__host__ __device__ __forceinline__ bool obs_tab_ok(int HW, int obs_be, int K) {
    return HW % 4 == 0 && obs_tab_bytes(HW, obs_be, K) <= OBS_TAB_MAX;
}
// offset (bytes) of the float4 entries in obs_lds: after road bits, flags, patch cells + values
__host__ __device__ __forceinline__ int obs_ent_off(int HW, int obs_be, int K, int npatch) {
    const int words = (HW + 31) / 32 + OBS_BE + 2 * 2 * obs_be * K * npatch;
    return ((words * 4) + 15) & ~15;
}

// The f32 writer's store loop over the patch tables.  J = H*W / 4 / T > 0: each thread owns the
// same J float4 columns of every env, their map values in registers (J is a template parameter,
// so they stay in VGPRs), and the env loop is uniform; J = 0: any shape, one float4 per iteration.
template <int T, int J, bool NT>
__device__ __forceinline__ void obs_store_cols(const Params &p, float *__restrict__ obs, float *__restrict__ final_obs,
                                               int64_t e0, int nenv, int npatch, int tstride, const uint32_t *s_road,
                                               const uint32_t *s_flag, const float4 *s_ent, const uint8_t *s_tab) {
    const int tid = threadIdx.x, HW = p.HW, HW4 = HW >> 2, K = p.K;
    auto map4 = [&](int c4) {
        const int c0 = c4 << 2;
        const uint32_t rb = s_road[c0 >> 5] >> (c0 & 31);
        float4 v;
        v.x = (rb & 1u) ? 0.0f : -1.0f;
        v.y = (rb & 2u) ? 0.0f : -1.0f;
        v.z = (rb & 4u) ? 0.0f : -1.0f;
        v.w = (rb & 8u) ? 0.0f : -1.0f;
        return v;
    };
    if constexpr (J > 0) {
        float4 mapv[J];
#pragma unroll
        for (int j = 0; j < J; ++j) mapv[j] = map4(j * T + tid);
        {
            float *dst = obs;
            if (!dst) return;
            const uint32_t need = D_WRITE;
            for (int k = 0; k < K; ++k) {
                float4 *out4 = reinterpret_cast<float4 *>(dst + ((int64_t)k * p.E + e0) * HW);
                for (int el = 0; el < nenv; ++el) {
                    if (!(s_flag[el] & need)) continue;
                    const int own = el * K + k;
                    const uint8_t *tb = s_tab + own * tstride;
                    const float4 *ent = s_ent + own * npatch - 1;
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                        const int c4 = j * T + tid;
                        const int en = tb[c4];
                        // both operands read, then a value select: a select of the two addresses
                        // would put mapv in scratch behind a flat load (ent[0] is readable LDS:
                        // the previous owner's last entry, or the patch values before s_ent)
                        const float4 ev = ent[en];
                        float4 v;
                        v.x = en ? ev.x : mapv[j].x;
                        v.y = en ? ev.y : mapv[j].y;
                        v.z = en ? ev.z : mapv[j].z;
                        v.w = en ? ev.w : mapv[j].w;
                        if (NT)
                            store_nt(&out4[el * HW4 + c4], v);
                        else
                            out4[el * HW4 + c4] = v;
                    }
                }
            }
        }
    } else {
        const int total4 = nenv * HW4;
        {
            float *dst = obs;
            if (!dst) return;
            const uint32_t need = D_WRITE;
            for (int k = 0; k < K; ++k) {
                float4 *out4 = reinterpret_cast<float4 *>(dst + ((int64_t)k * p.E + e0) * HW);
                for (int i4 = tid; i4 < total4; i4 += T) {
                    const int el = HW4 == 1 ? i4 : (int)__umulhi((uint32_t)i4, p.hw4_magic);
                    if (!(s_flag[el] & need)) continue;
                    const int c4 = i4 - el * HW4;
                    const int own = el * K + k;
                    const int en = s_tab[own * tstride + c4];
                    const float4 ev = s_ent[own * npatch + en - 1], mv = map4(c4);  // value select, as above
                    float4 v;
                    v.x = en ? ev.x : mv.x;
                    v.y = en ? ev.y : mv.y;
                    v.z = en ? ev.z : mv.z;
                    v.w = en ? ev.w : mv.w;
                    if (NT)
                        store_nt(&out4[i4], v);
                    else
                        out4[i4] = v;
                }
            }
        }
    }
}

// One obs block (T threads): the envs [e_begin + bid * obs_be, + obs_be) of the launch.
// obs_lds: road bitmask, flags, then per (which, env, k) N + 1 patch cells and values, sized to
// the launch (640 B at 32x32, N = 4, K = 2, 4 envs), so obs blocks never take the LDS a
// co-resident kernel (the fused actor's 74-104 KB per CU) needs.
template <int T, bool VEC4, bool NT, bool BF16>
__device__ __forceinline__ void obs_block(const Params &p, float *__restrict__ obs, float *__restrict__ final_obs,
                                          int64_t bid, uint32_t *obs_lds) {
    const int tid = threadIdx.x;
    const int HW = p.HW, N = p.N, K = p.K;
    const int npatch = N + 1;
    const int nroad = (HW + 31) / 32;
    uint32_t *s_road = obs_lds;
    uint32_t *s_flag = s_road + nroad;
    int *s_pc = reinterpret_cast<int *>(s_flag + OBS_BE);          // [2][obs_be][K][npatch]
    float *s_pv = reinterpret_cast<float *>(s_pc + 2 * p.obs_be * K * npatch);
    const int64_t e0 = p.e_begin + bid * p.obs_be;
    if (e0 >= p.e_end) return;  // uniform per block
    const int nenv = (int)min((int64_t)p.obs_be, p.e_end - e0);
    for (int w = tid; w < nroad; w += T) s_road[w] = p.tb.roadbits[w];
    // patches: one thread per (which, env, k)
    if (tid < 2 * p.obs_be * K) {
        const int which = tid / (p.obs_be * K), el = (tid / K) % p.obs_be, k = tid % K;
        const int slot = ((which * p.obs_be + el) * K + k) * npatch;
        if (el < nenv) {
            const uint32_t *d = p.desc + (e0 + el) * NDESC;
            const uint32_t f = d[4];
            if (k == 0 && which == 0) s_flag[el] = f;
            const bool reset = (which == 0) && (f & D_RESET);
            const uint32_t apples = which == 0 ? (f >> 8) & 0xFFu : (f >> 16) & 0xFFu;
            const uint32_t *pw = d + (which == 0 ? 0 : 8);
            const int ac = ((apples >> k) & 1u) ? p.apples[k] : -1;
            int np = 0;
            if (ac >= 0) {  // apple first, agents override it
                float av = p.tb.base[ac] + 9.0f;
                if (!reset && av == (float)(k + 1)) av = 1.0f;  // relabel of :321 (apple on a wall, K = 8)
                s_pc[slot + np] = ac;
                s_pv[slot + np] = av;
                ++np;
            }
            for (int n = 0; n < N; ++n) {
                const int c = (int)((pw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu);
                s_pc[slot + np] = c;
                s_pv[slot + np] = agent_value(reset, n, k, c == ac, p.variant);
                ++np;
            }
            for (; np < npatch; ++np) s_pc[slot + np] = -1;
        }
    }
    if (tid < OBS_BE && tid >= nenv) s_flag[tid] = 0;
    const bool tab = VEC4 && !BF16 && obs_tab_ok(HW, p.obs_be, K);
    float4 *s_ent = reinterpret_cast<float4 *>(reinterpret_cast<uint8_t *>(obs_lds) + obs_ent_off(HW, p.obs_be, K, npatch));
    uint8_t *s_tab = reinterpret_cast<uint8_t *>(s_ent + p.obs_be * K * npatch);
    const int tstride = obs_tab_stride(HW);
    if (tab) {  // zero the byte tables (16 B per thread and pass)
        const int n16 = obs_tab_bytes(HW, p.obs_be, K) >> 4;
        for (int i = tid; i < n16; i += T) reinterpret_cast<uint4 *>(s_tab)[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    for (int t = tid; tab && t < p.obs_be * K * npatch; t += T) {
        // one thread per patch slot q of (env, agent) of the step obs: the first slot touching a
        // float4 builds its entry (the map float4 with every slot of that float4 applied in slot
        // order: a later slot overrides, the obs writer's rule) and names it in the byte table
        const int own = t / npatch, q = t - own * npatch;
        const int el = own / K;
        const int slot = own * npatch;  // == ((0 * obs_be + el) * K + k) * npatch: the step obs' slots
        const int c = s_pc[slot + q];
        if (el < nenv && (s_flag[el] & D_WRITE) && c >= 0 && c < HW) {
            bool first = true;
            for (int q2 = 0; q2 < q; ++q2) {
                const int c2 = s_pc[slot + q2];
                first = first && (c2 < 0 || (c2 >> 2) != (c >> 2));
            }
            if (first) {
                const int c0 = c & ~3;
                const uint32_t rb = s_road[c0 >> 5] >> (c0 & 31);
                float4 v;
                v.x = (rb & 1u) ? 0.0f : -1.0f;
                v.y = (rb & 2u) ? 0.0f : -1.0f;
                v.z = (rb & 4u) ? 0.0f : -1.0f;
                v.w = (rb & 8u) ? 0.0f : -1.0f;
                for (int q2 = q; q2 < npatch; ++q2) {
                    const int dd = s_pc[slot + q2] - c0;
                    if ((unsigned)dd < 4u) {
                        const float pv = s_pv[slot + q2];
                        v.x = dd == 0 ? pv : v.x;
                        v.y = dd == 1 ? pv : v.y;
                        v.z = dd == 2 ? pv : v.z;
                        v.w = dd == 3 ? pv : v.w;
                    }
                }
                s_ent[slot + q] = v;
                s_tab[own * tstride + (c >> 2)] = (uint8_t)(q + 1);
            }
        }
    }
    if (tab) {
        __syncthreads();
        const int HW4 = HW >> 2;
        const int J = HW4 % T == 0 ? HW4 / T : 0;
        if (J == 1)
            obs_store_cols<T, 1, NT>(p, obs, final_obs, e0, nenv, npatch, tstride, s_road, s_flag, s_ent, s_tab);
        else if (J == 2)
            obs_store_cols<T, 2, NT>(p, obs, final_obs, e0, nenv, npatch, tstride, s_road, s_flag, s_ent, s_tab);
        else if (J == 4)
            obs_store_cols<T, 4, NT>(p, obs, final_obs, e0, nenv, npatch, tstride, s_road, s_flag, s_ent, s_tab);
        else
            obs_store_cols<T, 0, NT>(p, obs, final_obs, e0, nenv, npatch, tstride, s_road, s_flag, s_ent, s_tab);
    }

    // the terminal obs with the tables (the step obs without them, every obs of the bf16 / odd-HW
    // formats): per float4 the N + 1 patch compares
    for (int which = tab ? 1 : 0; which < 2; ++which) {
        float *dst = which == 0 ? obs : final_obs;
        if (!dst) continue;
        const uint32_t need = which == 0 ? D_WRITE : D_FINAL;
        if constexpr (BF16) {  // 8 cells = one 16-byte store per thread (HW % 8 == 0)
            const int HW8 = HW >> 3;
            const int total8 = nenv * HW8;
            for (int k = 0; k < K; ++k) {
                uint4 *out8 = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(dst) + ((int64_t)k * p.E + e0) * HW);
                for (int i8 = tid; i8 < total8; i8 += T) {
                    const int el = HW8 == 1 ? i8 : (int)__umulhi((uint32_t)i8, p.hw8_magic);
                    if (!(s_flag[el] & need)) continue;
                    const int c0 = (i8 - el * HW8) << 3;
                    const uint32_t rb = s_road[c0 >> 5] >> (c0 & 31);  // 8 cells share one word
                    // map: road 0.0 (bits 0x0000), inactive -1.0 (0xBF80), two cells per word
                    u32x4 w;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        w[j] = (((rb >> (2 * j)) & 1u) ? 0u : 0xBF80u) | (((rb >> (2 * j + 1)) & 1u) ? 0u : 0xBF800000u);
                    const int slot = ((which * p.obs_be + el) * K + k) * npatch;
                    for (int q = 0; q < npatch; ++q) {  // later patches override earlier ones
                        const int dd = s_pc[slot + q] - c0;
                        if ((unsigned)dd < 8u) {
                            const uint32_t sh = 16u * (dd & 1), b = bf16_bits(s_pv[slot + q]) << sh;
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                w[j] = (dd >> 1) == j ? ((w[j] & ~(0xFFFFu << sh)) | b) : w[j];
                        }
                    }
                    if (NT)
                        __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(&out8[i8]));
                    else
                        *reinterpret_cast<u32x4 *>(&out8[i8]) = w;
                }
            }
        } else if (VEC4) {
            const int HW4 = HW >> 2;
            const int total4 = nenv * HW4;
            for (int k = 0; k < K; ++k) {
                float4 *out4 = reinterpret_cast<float4 *>(dst + ((int64_t)k * p.E + e0) * HW);
                for (int i4 = tid; i4 < total4; i4 += T) {
                    const int el = HW4 == 1 ? i4 : (int)__umulhi((uint32_t)i4, p.hw4_magic);
                    if (!(s_flag[el] & need)) continue;
                    const int c0 = (i4 - el * HW4) << 2;
                    const uint32_t rb = s_road[c0 >> 5] >> (c0 & 31);  // 4 cells share one word
                    float4 v;
                    v.x = (rb & 1u) ? 0.0f : -1.0f;
                    v.y = (rb & 2u) ? 0.0f : -1.0f;
                    v.z = (rb & 4u) ? 0.0f : -1.0f;
                    v.w = (rb & 8u) ? 0.0f : -1.0f;
                    const int slot = ((which * p.obs_be + el) * K + k) * npatch;
                    for (int q = 0; q < npatch; ++q) {
                        const int dd = s_pc[slot + q] - c0;
                        if ((unsigned)dd < 4u) {
                            const float pv = s_pv[slot + q];
                            v.x = dd == 0 ? pv : v.x;
                            v.y = dd == 1 ? pv : v.y;
                            v.z = dd == 2 ? pv : v.z;
                            v.w = dd == 3 ? pv : v.w;
                        }
                    }
                    if (NT)
                        store_nt(&out4[i4], v);
                    else
                        out4[i4] = v;
                }
            }
        } else {
            const int total = nenv * HW;
            for (int k = 0; k < K; ++k) {
                float *o = dst + ((int64_t)k * p.E + e0) * HW;
                for (int i = tid; i < total; i += T) {
                    const int el = i / HW;
                    if (!(s_flag[el] & need)) continue;
                    const int c = i - el * HW;
                    float v = ((s_road[c >> 5] >> (c & 31)) & 1u) ? 0.0f : -1.0f;
                    const int slot = ((which * p.obs_be + el) * K + k) * npatch;
                    for (int q = 0; q < npatch; ++q)
                        if (s_pc[slot + q] == c) v = s_pv[slot + q];
                    o[i] = v;
                }
            }
        }
    }
}

template <bool VEC4, bool NT, bool BF16 = false>
__global__ void __launch_bounds__(OBS_THREADS) obs_kernel(Params p, float *__restrict__ obs,
                                                          float *__restrict__ final_obs) {
    extern __shared__ uint32_t obs_lds[];
    obs_block<OBS_THREADS, VEC4, NT, BF16>(p, obs, final_obs, blockIdx.x, obs_lds);
}

// ---------------------------------------------------------------------------------------
// step_v2 (default): CustomMAEnv.step of BE envs per 128-thread block.
//   A  per env (tid < BE): state loaded once into registers, scripted policy + RL override,
//      MdR, close sets, and the de-duplicated FeAR task list (see FeAR note above)
//   B  every lane: one world update per task (the env's real update = the first BE slots)
//   C  per env: FeAR sums in numpy order, rewards, dones, state, outputs, obs descriptor
// All per-cell tables live in one u32 LDS table (policy | MdR | action mask | unit moves |
// road), the policy CDFs in LDS too, so no lane walks a dependent chain of global loads.
// Small blocks (2 waves) keep ~9 blocks per CU resident so their latency-bound phases overlap.
// ---------------------------------------------------------------------------------------
// cell table bits
constexpr uint32_t CT_POL = 0, CT_MDR = 8, CT_AMASK = 12, CT_OK = 21, CT_ROAD = 25;

#ifndef GW_LIST_MIN_N  // the FeAR-off chain's world update walks per-lane near-pair lists from this N on
#define GW_LIST_MIN_N 5
#endif
#ifndef GW_NOFEAR_BE  // envs per block of the FeAR-off step_v2 with N <= 4 (measurement builds: 16)
#define GW_NOFEAR_BE 32
#endif
// DEF: the deferred-FeAR world-update kernel (step_v2<.., DEFER>, GW_KERNEL=defer with FeAR on):
// one env per thread in 128-env blocks (it runs beside the large obs writer, where per-block
// table fills and barriers cost more than the lane-parallel draws save)
template <int N, int KMAX, bool FEAR, bool WIDE = false, bool DEF = false> struct V2Cfg {
    static constexpr int THREADS = 128;
    // WIDE (fear_v2, GW_FEAR_BE=wide): twice the envs per block, half the resident waves
    static constexpr int BE = (WIDE ? 2 : 1) *
        (FEAR ? (KMAX <= 2 ? (N <= 4 ? 32 : 16) : (N <= 4 ? 16 : 4))
              : (KMAX <= 2 && (N > 4 || DEF) ? 128 : GW_NOFEAR_BE));
    // FeAR off with 32 envs per block: the 128 threads draw the (env, agent) actions in parallel
    // before one thread per env runs the rest (step_v2_block); with 128 envs per block (N > 4,
    // large batches) each env thread draws its own
    static constexpr bool XDRAW = !FEAR && BE <= 32 && N <= 4;
    static_assert(!FEAR || BE <= 64, "task encoding holds 6 env bits");
    // task list: [env sims (step_v2 only: BE)][base sims: 2 per actor k with act != MdR] then
    // groups of 16 counterfactuals (one entry per (actor k, close j), expanded on the fly)
    static constexpr int MAXB = FEAR ? BE * (1 + 2 * KMAX) : 1;
    static constexpr int MAXG = FEAR ? BE * KMAX * (N > 1 ? N - 1 : 1) : 1;
    using Task = typename std::conditional<(KMAX <= 2), uint16_t, uint32_t>::type;
    // task bits: env 0-5 | b 6-9 (15 = base sim) | var 10 | j 11-13 | k 14+
    static __device__ __forceinline__ Task enc(int el, int k, int j, int var, int b) {
        return (Task)((uint32_t)el | ((uint32_t)b << 6) | ((uint32_t)var << 10) | ((uint32_t)j << 11) |
                      ((uint32_t)k << 14));
    }
};

template <int N, int KMAX, bool FEAR, bool WIDE = false, bool DEF = false>
struct alignas(16) V2Shared {
    using Cfg = V2Cfg<N, KMAX, FEAR, WIDE, DEF>;
    static constexpr int BE = Cfg::BE, FB = FEAR ? BE : 1;
    double red[Cfg::THREADS / 64][GW_STATS];
    typename Cfg::Task tasks[Cfg::MAXB];
    typename Cfg::Task groups[Cfg::MAXG];
    int pos[FB][N];
    int fin[FB][N];
    int apple[FB][KMAX];
    uint32_t bits[FB];
    int8_t act[FB][N];
    int8_t mdr[FB][N];
    uint8_t close[FB][KMAX];
    uint8_t base[FB][KMAX][2];
    uint8_t cj[FB][KMAX][FEAR ? N : 1][2][NA];
    uint2 wl[(N >= GW_LIST_MIN_N) ? Cfg::THREADS * N : 1];  // World<N, true> rows (one per thread)
    int8_t xact[Cfg::XDRAW ? BE : 1][N];   // FeAR off: the (env, agent) threads' action draws and MdRs
    int8_t xmdr[Cfg::XDRAW ? BE : 1][N];
    int nbase, ngroup;  // base-sim entries after the env sims; counterfactual groups
};

// setup_step (ma_customenv.py:432-452) + RL override (:239-242) from the LDS tables: agent n
__device__ __forceinline__ int draw_action(const Params &p, int64_t e, int n, uint32_t episode, int t, int pos,
                                           const uint32_t *ctab, const double *cdf_s) {
    const uint32_t gid = (uint32_t)(p.env_offset + e);
    int a;
    if (n < p.K) {
        if (p.rl) {
            a = p.rl[e * p.K + n];
        } else {
            const uint4 r = philox(gid, episode, (uint32_t)t, (2u << 24) | (uint32_t)n, p.key0, p.key1);
            a = (int)(((uint64_t)r.x * 9u) >> 32);
        }
    } else if (p.scripted) {
        a = p.scripted[e * (p.N - p.K) + (n - p.K)];
    } else {
        const uint4 r = philox(gid, episode, (uint32_t)t, (1u << 24) | (uint32_t)n, p.key0, p.key1);
        const int uni = r.x < 0x40000000u;  // random.random() < 0.25 (:441)
        const double u = ((double)(r.y >> 5) * 67108864.0 + (double)(r.z >> 6)) * (1.0 / 9007199254740992.0);
        const int pid = (int)((ctab[pos] >> CT_POL) & 0xFFu);
        const double *cdf = (cdf_s ? cdf_s : p.tb.cdf) + (pid * 2 + uni) * NA;
        a = NA - 1;
#pragma unroll
        for (int q = NA - 2; q >= 0; --q)
            if (u < cdf[q]) a = q;  // searchsorted(cdf, u, 'right')
    }
    return ((unsigned)a < (unsigned)NA) ? a : 0;
}

template <int N>
__device__ __forceinline__ void select_actions_v2(const Params &p, int64_t e, const EnvState<N> &es,
                                                  const uint32_t *ctab, const double *cdf_s, int (&act)[N]) {
#pragma unroll
    for (int n = 0; n < N; ++n) act[n] = draw_action(p, e, n, es.episode, es.t, es.pos[n], ctab, cdf_s);
}

// Copy n 32-bit words global -> LDS with 16-byte accesses, all loads of a lane issued before
// its stores (a plain element loop serialises one L2 round trip per iteration).
template <int T>
__device__ __forceinline__ void lds_fill(uint32_t *dst, const uint32_t *__restrict__ src, int n, int tid) {
    const int n4 = n >> 2;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    constexpr int U = 4;
    for (int base = 0; n4 > 0 && base < n4; base += U * T) {
        uint4 v0, v1, v2, v3;  // named registers: loads clamped in range, stores predicated
        const int i0 = base + tid, i1 = i0 + T, i2 = i1 + T, i3 = i2 + T;
        v0 = s4[min(i0, n4 - 1)];
        v1 = s4[min(i1, n4 - 1)];
        v2 = s4[min(i2, n4 - 1)];
        v3 = s4[min(i3, n4 - 1)];
        if (i0 < n4) d4[i0] = v0;
        if (i1 < n4) d4[i1] = v1;
        if (i2 < n4) d4[i2] = v2;
        if (i3 < n4) d4[i3] = v3;
    }
    for (int i = (n4 << 2) + tid; i < n; i += T) dst[i] = src[i];
}

// FeAR phase A of one env (custom/ma_customenv.py:247-251, Responsibility.py:135-210): close sets
// (:456-464) into sh.close and the de-duplicated counterfactual task list appended to sh.tasks.
// Expects sh.pos / sh.act / sh.mdr of the env filled.
template <int N, int KMAX, class Sh>
__device__ __forceinline__ void fear_plan(const Params &p, Sh &sh, int el, const int (&pos)[N], const int (&act)[N],
                                          int off0) {
    using Cfg = typename Sh::Cfg;
    const int K = p.K;
    int nb = 0, ng = 0;
    uint32_t close[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        close[k] = 0;
        if (k >= K) continue;
#pragma unroll
        for (int n = 0; n < N; ++n)
            if (n == k || manhattan(p, pos[k], pos[n]) <= 5) close[k] |= 1u << n;
        sh.close[el][k] = (uint8_t)close[k];
        if (act[k] != (int)sh.mdr[el][k]) {
            nb += 2;
            ng += __popc(close[k]) - 1;
        }
    }
    if (!nb) return;
    int sb = off0 + atomicAdd(&sh.nbase, nb);
    int sg = ng ? atomicAdd(&sh.ngroup, ng) : 0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k >= K || act[k] == (int)sh.mdr[el][k]) continue;
        sh.tasks[sb++] = Cfg::enc(el, k, 0, 0, 15);
        sh.tasks[sb++] = Cfg::enc(el, k, 0, 1, 15);
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j != k && ((close[k] >> j) & 1u)) sh.groups[sg++] = Cfg::enc(el, k, j, 0, 0);
    }
}

// Task ti of phase B: entries [0, nb_end) are stored; past them, group g = (ti - nb_end) / 16
// expands to var = bit 3 and the 8 alternatives b != act[j] of agent j.
template <class Sh>
__device__ __forceinline__ uint32_t fear_task_at(const Sh &sh, int ti, int nb_end) {
    if (ti < nb_end) return sh.tasks[ti];
    const int g = (ti - nb_end) >> 4, s = (ti - nb_end) & 15;
    const uint32_t tk = sh.groups[g];
    const int el = tk & 63, j = (tk >> 11) & 7;
    const int bi = s & 7;
    const int b = bi + (bi >= (int)sh.act[el][j]);
    return tk | ((uint32_t)b << 6) | ((uint32_t)(s >> 3) << 10);
}

// FeAR phase B, one counterfactual world update (task bits: see V2Cfg::enc): the joint action
// with actor k's action (var 0: MdR, var 1: its own) and agent j's alternative b (15 = none);
// agents outside k's close set stay.  Records which agents end valid (no crash, no restriction).
template <int N, int KMAX, class Sh, class OK>
__device__ __forceinline__ void fear_task(const Params &p, Sh &sh, uint32_t tk, const OK &okv) {
    const int el = tk & 63, b = (tk >> 6) & 15, var = (tk >> 10) & 1, j = (tk >> 11) & 7, k = (int)(tk >> 14);
    int pos[N], joint[N], fin[N];
    const uint32_t cl = sh.close[el][k];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        pos[n] = sh.pos[el][n];
        joint[n] = ((cl >> n) & 1u) ? (int)sh.act[el][n] : 0;
        if (n == k && var == 0) joint[n] = sh.mdr[el][n];
        if (n == j && b != 15) joint[n] = b;
    }
    int apple[MAXN];
#pragma unroll
    for (int q = 0; q < MAXN; ++q) apple[q] = -1;
    constexpr bool LIST = N >= GW_LIST_MIN_N;  // a wave's sims belong to different envs
    World<N, LIST> w;
    w.init(pos, joint, p.W, p.w_magic);
    if constexpr (LIST) w.lw = &sh.wl[threadIdx.x * N];
    uint32_t caught;
    simulate<N, true>(w, okv, 0, apple, caught, fin);
    const uint32_t valid = ~(w.crash | w.restr) & ((1u << N) - 1u);
    if (b == 15)
        sh.base[el][k][var] = (uint8_t)valid;
    else
        sh.cj[el][k][j][var][b] = (uint8_t)((valid >> j) & 1u);
}

// FeAR phase C of one env: V counts -> Resp table -> np.sum of the Resp row in numpy's order.
template <int N, int KMAX, class Sh>
__device__ __forceinline__ void fear_values(const Params &p, const Sh &sh, int el, const int (&act)[N],
                                            const int (&mdr)[N], const double *resp_s, double (&fear)[MAXN]) {
#pragma unroll
    for (int k = 0; k < MAXN; ++k) fear[k] = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k >= p.K || act[k] == mdr[k]) continue;
        const uint32_t cl = sh.close[el][k];
        const uint32_t b0 = sh.base[el][k][0], b1 = sh.base[el][k][1];
        double resp[N];
#pragma unroll
        for (int jj = 0; jj < N; ++jj) {
            resp[jj] = 0.0;
            if (jj == k) continue;
            int vm, va;
            if ((cl >> jj) & 1u) {
                vm = 0;
                va = 0;
                for (int b = 0; b < NA; ++b) {
                    vm += (b == act[jj]) ? (int)((b0 >> jj) & 1u) : (int)sh.cj[el][k][jj][0][b];
                    va += (b == act[jj]) ? (int)((b1 >> jj) & 1u) : (int)sh.cj[el][k][jj][1][b];
                }
            } else {
                vm = 9 * (int)((b0 >> jj) & 1u);
                va = 9 * (int)((b1 >> jj) & 1u);
            }
            resp[jj] = resp_s[vm * 10 + va];
        }
        fear[k] = np_sum_row<N>(resp, k);
    }
}

// Block statistics: deterministic wave butterfly + fixed-order cross-wave sum, one row per block.
template <int T, uint32_t FM = 0xFFu, uint32_t IM = 0u>
__device__ __forceinline__ void block_stats(const Params &p, Contrib &ct, double (&red)[T / 64][GW_STATS], int tid,
                                            int64_t row) {
    const bool want = p.out.stats || p.out.stats_acc;
    if (want) {
        wave_sum_sel<FM, IM>(ct);
        if ((tid & 63) == 0)
#pragma unroll
            for (int i = 0; i < GW_STATS; ++i) red[tid >> 6][i] = ct.v[i];
    }
    __syncthreads();
    if (want && tid < GW_STATS) {
        double acc = red[0][tid];
#pragma unroll
        for (int w = 1; w < T / 64; ++w) acc = __dadd_rn(acc, red[w][tid]);
        stats_put(p.out, row * GW_STATS + tid, acc);
    }
}

#ifdef GW_STEP_CLK  // measurement build only (tools/step_clk.sh): thread 0's phase stamps per block
__device__ unsigned long long g_step_clk[64][16];
#define STEP_STAMP(slot)                                                             \
    do {                                                                             \
        if (tid == 0 && bid < 64) g_step_clk[bid][slot] = clock64();                 \
    } while (0)
#else
#define STEP_STAMP(slot) \
    do {                 \
    } while (0)
#endif

template <int N, int KMAX, bool FEAR, bool DEFER>
__device__ __forceinline__ void step_v2_block(const Params &p, int64_t bid, V2Shared<N, KMAX, FEAR, false, DEFER> &sh,
                                              uint8_t *dyn) {  // dyn: [cdf P*18 f64][cell table HW u32][Resp]
    using Cfg = V2Cfg<N, KMAX, FEAR, false, DEFER>;
    constexpr int BE = Cfg::BE, T = Cfg::THREADS;
    const double *cdf_s = p.lds_cdf ? reinterpret_cast<const double *>(dyn) : nullptr;
    uint32_t *ctab = reinterpret_cast<uint32_t *>(dyn + p.ctab_off);
    double *resp_s = reinterpret_cast<double *>(dyn + p.resp_off);  // [10][10] Resp table
    const uint8_t *okb = nullptr;  // sims read the unit-move bits through ctab (see OkView)
    (void)okb;

    const int tid = threadIdx.x;
    if (p.e_begin + bid * BE >= p.e_end) return;  // uniform per block
    const int64_t e0 = p.e_begin + bid * BE;
    const int nenv = (int)min((int64_t)BE, p.e_end - e0);
    const int K = p.K;
    STEP_STAMP(0);
#ifdef GW_STEP_CLK
    if (tid == 0 && bid < 64) g_step_clk[bid][15] = wall_clock64();
#endif
    if (e0 == 0 && tid == 0) step_tick(p.out);  // once per step: the block of env 0
    Contrib ct;
    contrib_zero(ct);
    EnvState<N> es;
    // XDRAW: the env chains run on the first BE / 2 lanes of each of the two waves (16 envs per
    // wave instead of 32: a wave waits for fewer divergent collision passes and resets)
    constexpr bool XDRAW = Cfg::XDRAW;
    constexpr int CPW = XDRAW ? BE / (T / 64) : 64;  // chain lanes per wave
    const int cel = XDRAW ? (((tid & 63) < CPW) ? (tid >> 6) * CPW + (tid & 63) : BE) : tid;
    // the env's state loads are issued first so that their latency overlaps the table fill
    if (cel < nenv) load_env<N>(p, e0 + cel, es);
    // XDRAW: thread i also draws agent i / BE of env i % BE: its inputs
    constexpr int NPAIR = XDRAW ? (BE * N + T - 1) / T : 1;
    int xpos[NPAIR], xt[NPAIR];
    uint32_t xep[NPAIR];
    if constexpr (XDRAW) {
#pragma unroll
        for (int j = 0; j < NPAIR; ++j) {
            const int i = tid + j * T, el = i % BE, n = i / BE;
            xpos[j] = xt[j] = 0;
            xep[j] = 0;
            if (n < N && el < nenv) {
                const int64_t e = e0 + el;
                xpos[j] = p.st.pos[(int64_t)n * p.E + e];
                xep[j] = p.st.episode[e];
                xt[j] = p.st.t[e];
            }
        }
    }
    lds_fill<T>(ctab, p.tb.celltab, p.HW, tid);
    if (p.lds_cdf)
        lds_fill<T>(reinterpret_cast<uint32_t *>(dyn), reinterpret_cast<const uint32_t *>(p.tb.cdf), 2 * p.n_cdf, tid);
    if (FEAR) lds_fill<T>(reinterpret_cast<uint32_t *>(resp_s), reinterpret_cast<const uint32_t *>(p.tb.resp), 200, tid);
    if (tid == 0) sh.nbase = sh.ngroup = 0;
    __syncthreads();
    STEP_STAMP(1);
    const CtabOk okv{ctab};

    if constexpr (FEAR) {
        // ---- A ----
        if (tid < nenv) {
            const int64_t e = e0 + tid;
            int act[N];
            select_actions_v2<N>(p, e, es, ctab, cdf_s, act);
#pragma unroll
            for (int n = 0; n < N; ++n) {
                sh.pos[tid][n] = es.pos[n];
                sh.act[tid][n] = (int8_t)act[n];
                sh.mdr[tid][n] = (int8_t)((ctab[es.pos[n]] >> CT_MDR) & 0xFu);
            }
#pragma unroll
            for (int k = 0; k < KMAX; ++k) sh.apple[tid][k] = (k < K && ((es.flags >> k) & 1u)) ? p.apples[k] : -1;
            sh.tasks[tid] = Cfg::enc(tid, 0, 0, 0, 0);
            fear_plan<N, KMAX>(p, sh, tid, es.pos, act, BE);
        }
        __syncthreads();
        // ---- B ----
        const int nb_end = BE + sh.nbase, ntask = nb_end + 16 * sh.ngroup;
        if (tid == 0 && p.sims && ntask > BE) atomicAdd(p.sims, (unsigned long long)(ntask - BE));
        for (int ti = tid; ti < ntask; ti += T) {
            if (ti < BE && ti >= nenv) continue;
            const uint32_t tk = fear_task_at(sh, ti, nb_end);
            const int el = tk & 63, b = (tk >> 6) & 15, var = (tk >> 10) & 1, j = (tk >> 11) & 7, k = (int)(tk >> 14);
            int pos[N], joint[N], fin[N];
#pragma unroll
            for (int n = 0; n < N; ++n) pos[n] = sh.pos[el][n];
            int apple[MAXN];
#pragma unroll
            for (int q = 0; q < MAXN; ++q) apple[q] = -1;
            int nk = 0;
            if (ti < BE) {
#pragma unroll
                for (int n = 0; n < N; ++n) joint[n] = sh.act[el][n];
#pragma unroll
                for (int q = 0; q < KMAX; ++q) apple[q] = sh.apple[el][q];
                nk = K;
            } else {
                const uint32_t cl = sh.close[el][k];
#pragma unroll
                for (int n = 0; n < N; ++n) joint[n] = ((cl >> n) & 1u) ? (int)sh.act[el][n] : 0;
#pragma unroll
                for (int n = 0; n < N; ++n)
                    if (n == k && var == 0) joint[n] = sh.mdr[el][n];
                if (b != 15) {
#pragma unroll
                    for (int n = 0; n < N; ++n)
                        if (n == j) joint[n] = b;
                }
            }
            constexpr bool LIST = N >= GW_LIST_MIN_N;
            World<N, LIST> w;
            w.init(pos, joint, p.W, p.w_magic);
            if constexpr (LIST) w.lw = &sh.wl[tid * N];
            uint32_t caught;
            simulate<N, true>(w, okv, nk, apple, caught, fin);
            if (ti < BE) {
#pragma unroll
                for (int n = 0; n < N; ++n) sh.fin[el][n] = fin[n];
                sh.bits[el] = w.crash | (w.restr << 8) | (caught << 16);
            } else {
                const uint32_t valid = ~(w.crash | w.restr) & ((1u << N) - 1u);
                if (b == 15)
                    sh.base[el][k][var] = (uint8_t)valid;
                else
                    sh.cj[el][k][j][var][b] = (uint8_t)((valid >> j) & 1u);
            }
        }
        __syncthreads();
        // ---- C ----
        if (tid < nenv) {
            const int64_t e = e0 + tid;
            int act[N], mdr[N], fin[N];
#pragma unroll
            for (int n = 0; n < N; ++n) {
                act[n] = sh.act[tid][n];
                mdr[n] = sh.mdr[tid][n];
                fin[n] = sh.fin[tid][n];
            }
            double fear[MAXN];
            fear_values<N, KMAX>(p, sh, tid, act, mdr, resp_s, fear);
            const uint32_t bits = sh.bits[tid];
            ObsInfo<N> oi;
            finish_env<N>(p, e, es, act, mdr, fear, bits & 0xFFu, (bits >> 8) & 0xFFu, fin, bits >> 16, ct, oi, ctab);
            store_desc<N>(p, e, oi);
        }
    } else {
        if constexpr (XDRAW) {  // the action draws and MdRs, one thread per (env, agent)
#pragma unroll
            for (int j = 0; j < NPAIR; ++j) {
                const int i = tid + j * T, el = i % BE, n = i / BE;
                if (n < N && el < nenv) {
                    sh.xact[el][n] = (int8_t)draw_action(p, e0 + el, n, xep[j], xt[j], xpos[j], ctab, cdf_s);
                    sh.xmdr[el][n] = (int8_t)((ctab[xpos[j]] >> CT_MDR) & 0xFu);
                }
            }
            __syncthreads();
        }
        if (cel < nenv) {  // the rest of the env on one thread
            const int64_t e = e0 + cel;
            int act[N], mdr[N], fin[N], pos[N];
            if constexpr (XDRAW) {
#pragma unroll
                for (int n = 0; n < N; ++n) {
                    act[n] = sh.xact[cel][n];
                    mdr[n] = sh.xmdr[cel][n];
                    pos[n] = es.pos[n];
                }
            } else {
                select_actions_v2<N>(p, e, es, ctab, cdf_s, act);
#pragma unroll
                for (int n = 0; n < N; ++n) {
                    pos[n] = es.pos[n];
                    mdr[n] = (int)((ctab[pos[n]] >> CT_MDR) & 0xFu);
                }
            }
#ifdef GW_STEP_CLK
            if (bid < 64 && tid == 0) g_step_clk[bid][2] = clock64() + (uint64_t)(act[0] + mdr[N - 1] < -1000);
#endif
            int apple[MAXN];
#pragma unroll
            for (int k = 0; k < MAXN; ++k) apple[k] = (k < K && ((es.flags >> k) & 1u)) ? p.apples[k] : -1;
            constexpr bool LIST = N >= GW_LIST_MIN_N;
            World<N, LIST> w;
            w.init(pos, act, p.W, p.w_magic);
            if constexpr (LIST) w.lw = &sh.wl[tid * N];
            uint32_t caught;
            simulate<N, true>(w, okv, K, apple, caught, fin);
#ifdef GW_STEP_CLK
            if (bid < 64 && tid == 0) g_step_clk[bid][3] = clock64() + (uint64_t)(fin[0] + (int)caught < -1000);
#endif
            double fear[MAXN];
#pragma unroll
            for (int k = 0; k < MAXN; ++k) fear[k] = 0.0;
            ObsInfo<N> oi;
            finish_env<N, DEFER>(p, e, es, act, mdr, fear, w.crash, w.restr, fin, caught, ct, oi, ctab);
            STEP_STAMP(4);
            store_desc<N>(p, e, oi);
        }
    }

    // ---- block statistics (deterministic tree) ----
    // deferred FeAR: the FeAR-owned f64 fields are fear_v2's; without FeAR field 2 stays 0
    constexpr uint32_t FM = DEFER ? 0u : ((1u << 0) | (1u << 5) | (FEAR ? (1u << 2) : 0u));
    STEP_STAMP(5);
    block_stats<T, FM, ST_INT>(p, ct, sh.red, tid, p.stats_row0 + e0 / BE);
    STEP_STAMP(6);
}

template <int N, int KMAX, bool FEAR, bool DEFER = false>
__global__ void __launch_bounds__(128) step_v2(Params p) {
    __shared__ V2Shared<N, KMAX, FEAR, false, DEFER> sh;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    step_v2_block<N, KMAX, FEAR, DEFER>(p, blockIdx.x, sh, dyn);
}

// gw_obs_patch (egocentric P x P windows of the env's last observation, -1 outside the grid,
// the same encoding as obs_block) is written by csrc/patch_ops.hip (launch_windows).

// ---------------------------------------------------------------------------------------
// step_obs (GW_KERNEL=merged with async obs): ONE launch per gw_step on the caller's stream.
// Blocks [0, nstep) are step_v2 (FeAR inline) of step t; blocks [nstep, grid) write the obs of
// step t-1 from its descriptor buffer (q; the step writes the other buffer).  The two roles
// share no data, so the latency-bound world update + FeAR and the HBM-bound store stream
// overlap inside one kernel, with no second queue and no cross-queue events between steps.
// ---------------------------------------------------------------------------------------
template <int N, int KMAX, bool FEAR>
__global__ void __launch_bounds__(128) step_obs(Params p, Params q, float *__restrict__ obs,
                                                float *__restrict__ final_obs, uint32_t nstep) {
    __shared__ V2Shared<N, KMAX, FEAR> sh;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    // the step blocks first: their long latency chains start first
    const bool is_step = blockIdx.x < nstep;
    const uint32_t rb = is_step ? blockIdx.x : blockIdx.x - nstep;
    if (is_step)
        step_v2_block<N, KMAX, FEAR, false>(p, rb, sh, dyn);
    else if (q.obs_bf16)
        obs_block<128, true, true, true>(q, obs, final_obs, rb, reinterpret_cast<uint32_t *>(dyn));
    else
        obs_block<128, true, true, false>(q, obs, final_obs, rb, reinterpret_cast<uint32_t *>(dyn));
}

// ---------------------------------------------------------------------------------------
// fear_v2 (GW_KERNEL=defer, FeAR on): the FeAR half of CustomMAEnv.step + the rollout's reward
// shaping (custom/Responsibility.py:135-210, ma_customenv.py:247-252, maddpg/agent.py:124-173),
// launched after step_v2<.., DEFER> on a second stream so that its integer-VALU-bound world
// updates overlap the HBM-store-bound obs_kernel.  Inputs: the FearRec of each env (pre-step
// cells, joint action, env rewards, done) and score / fear_score; same phases A/B/C as step_v2
// without the env's own update.  Dynamic LDS: [cell table][Resp 100 f64] (no CDFs).
// ---------------------------------------------------------------------------------------
template <int N, int KMAX, bool WIDE>
__device__ __forceinline__ void fear_block(const Params &p, uint32_t bid) {
    using Cfg = V2Cfg<N, KMAX, true, WIDE>;
    using Sh = V2Shared<N, KMAX, true, WIDE>;
    constexpr int BE = Cfg::BE, T = Cfg::THREADS;
    __shared__ Sh sh;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    uint32_t *ctab = reinterpret_cast<uint32_t *>(dyn + p.ctab_off);
    double *resp_s = reinterpret_cast<double *>(dyn + p.resp_off);

    const int tid = threadIdx.x;
    if (p.e_begin + (int64_t)bid * BE >= p.e_end) return;  // uniform per block
    const int64_t e0 = p.e_begin + (int64_t)bid * BE;
    const int nenv = (int)min((int64_t)BE, p.e_end - e0);
    const int K = p.K;
    int pos[N], act[N], rew[MAXN];
    uint32_t bonus = 0;
    bool done = false;
    double score0 = 0.0, fscore0 = 0.0;
    if (tid < nenv) {
        const int64_t e = e0 + tid;
        load_fear_rec<N>(p, e, pos, act, rew, bonus, done);
        score0 = p.st.score[e];
        fscore0 = p.st.fscore[e];
    }
    lds_fill<T>(ctab, p.tb.celltab, p.HW, tid);
    lds_fill<T>(reinterpret_cast<uint32_t *>(resp_s), reinterpret_cast<const uint32_t *>(p.tb.resp), 200, tid);
    if (tid == 0) sh.nbase = sh.ngroup = 0;
    __syncthreads();
    const CtabOk okv{ctab};
    // ---- A ----
    int mdr[N];
    if (tid < nenv) {
#pragma unroll
        for (int n = 0; n < N; ++n) {
            mdr[n] = (int)((ctab[pos[n]] >> CT_MDR) & 0xFu);
            sh.pos[tid][n] = pos[n];
            sh.act[tid][n] = (int8_t)act[n];
            sh.mdr[tid][n] = (int8_t)mdr[n];
        }
        fear_plan<N, KMAX>(p, sh, tid, pos, act, 0);
    }
    __syncthreads();
    // ---- B ----
    const int nb_end = sh.nbase, ntask = nb_end + 16 * sh.ngroup;
    if (tid == 0 && p.sims && ntask) atomicAdd(p.sims, (unsigned long long)ntask);
    for (int ti = tid; ti < ntask; ti += T) fear_task<N, KMAX>(p, sh, fear_task_at(sh, ti, nb_end), okv);
    __syncthreads();
    // ---- C ----
    Contrib ct;
    contrib_zero(ct);
    if (tid < nenv) {
        const int64_t e = e0 + tid;
        double fear[MAXN];
        fear_values<N, KMAX>(p, sh, tid, act, mdr, resp_s, fear);
        double shaped[MAXN], fsum_in[MAXN];
#pragma unroll
        for (int k = 0; k < MAXN; ++k) {
            shaped[k] = fsum_in[k] = 0.0;
            if (k >= K) continue;
            const double r = ((bonus >> k) & 1u) ? __dadd_rn((double)rew[k], 0.1) : (double)rew[k];
            shaped[k] = __dadd_rn(__dmul_rn(p.fear_weight, fear[k]), r);  // agent.py:130
            fsum_in[k] = fear[k];
        }
        const double score = __dadd_rn(score0, np_sum_small(shaped, K));    // agent.py:173
        const double fscore = __dadd_rn(fscore0, np_sum_small(fsum_in, K));  // agent.py:141
        const gw_step_out &o = p.out;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k >= K) continue;
            const int64_t ek = e * K + k;
            if (o.fear) o.fear[ek] = fear[k];
            if (o.shaped) o.shaped[ek] = shaped[k];
        }
        if (o.ep_return) o.ep_return[e] = score;
        if (o.ep_fear) o.ep_fear[e] = fscore;
        const bool fresh = done && p.auto_reset;  // the next episode starts from 0
        p.st.score[e] = fresh ? 0.0 : score;
        p.st.fscore[e] = fresh ? 0.0 : fscore;
        ct.v[0] = done ? score : 0.0;
        ct.v[2] = np_sum_small(fsum_in, K);
        ct.v[5] = np_sum_small(shaped, K);
    }
    block_stats<T, ST_F64_FEAR, 0u>(p, ct, sh.red, tid, p.stats_row0 + e0 / BE);
}

template <int N, int KMAX, bool WIDE>
__global__ void __launch_bounds__(128) fear_v2(Params p) {
    fear_block<N, KMAX, WIDE>(p, blockIdx.x);
}

// fear_v2 and the step's P x P windows (gw_step_patch_next; the row writer of csrc/window_rows.h on
// two waves per block) in ONE launch: both read only the world update's outputs, and the writer's
// HBM stream fills the CU slots the latency-bound FeAR blocks leave
template <int N, int KMAX, bool WIDE>
__global__ void __launch_bounds__(128) fear_rows_kernel(Params p, PatchArgs a, uint32_t nfear, uint32_t nrx) {
    if (blockIdx.x < nfear) {
        fear_block<N, KMAX, WIDE>(p, blockIdx.x);
        return;
    }
    // the rows' LDS slices in the dynamic region the FeAR blocks use for their tables.  One launch
    // has one footprint: the dynamic region is max(FeAR tables, 8 KB of row slices), so on small
    // grids (32x32: ~4.9 KB of tables) the FeAR blocks reserve 8 KB, and the row blocks also
    // reserve fear_block's static shared state; both stay far below the 160 KB per CU
    extern __shared__ __attribute__((aligned(16))) uint8_t dynr[];
    const uint32_t r = blockIdx.x - nfear;
    gwrows::rows_block<N + 1, 16, 2, 2>(a, r % nrx, (int)(r / nrx), reinterpret_cast<float4 (*)[64 * 4]>(dynr));
}

// ---------------------------------------------------------------------------------------
// Responsibility.FeAR (custom/Responsibility.py:57-132, every agent as actor) and FeAL
// (:213-303) for n world snapshots, one 128-thread block per snapshot.  Every world update the
// two need is one task (9 per group):  "act" groups jj = 0..N-1 (the action list unchanged,
// agent jj's 9 actions: ValidMoves_action[.][jj] and FeAL's action count of jj), "MdR" groups
// (ii, jj != ii) (actor ii swapped to its MdR: ValidMoves_moveDeRigueur[ii][jj]) and "FeAL"
// groups ii (every other listed agent swapped to its MdR).  Agents outside the action list
// stay and ignore swaps (SwapActionIDs4Agents, grid_world.py:709-726).  Valid-move bits are
// OR-ed into LDS, counted, and mapped through exact host-computed f64 tables.
// ---------------------------------------------------------------------------------------
struct FmParams {
    const uint32_t *celltab;
    const double *tab;        // [0, 100) Resp(vm, va), [100, 200) FeAL(vm, va)
    int HW, W;
    uint32_t w_magic;
    const int32_t *cells, *acts, *mdr;  // [n][N]; mdr may be null (the cells' MdR)
    const uint8_t *in_list;             // [n] bit a: agent a in ActionID4Agents; null = all
    double *resp;                       // [n][N][N]
    int32_t *vm, *va;                   // [n][N][N] or null
    double *feal;                       // [n][N] or null
    int32_t *feal_vm, *feal_va;         // [n][N] or null
};

template <int N>
__global__ void __launch_bounds__(128) fear_matrix_kernel(FmParams q) {
    constexpr int T = 128, NG = N + N * (N - 1) + N;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    uint32_t *ctab = reinterpret_cast<uint32_t *>(dyn);
    __shared__ int s_loc[N], s_act[N], s_mdr[N];
    __shared__ uint32_t s_bits[NG];  // 9-bit valid masks per group
    __shared__ uint32_t s_in;
    const int tid = threadIdx.x;
    const int64_t e = blockIdx.x;
    lds_fill<T>(ctab, q.celltab, q.HW, tid);
    for (int g = tid; g < NG; g += T) s_bits[g] = 0;
    if (tid < N) {
        const int c = q.cells[e * N + tid];
        const int a = q.acts[e * N + tid];
        s_loc[tid] = ((unsigned)c < (unsigned)q.HW) ? c : 0;
        s_act[tid] = ((unsigned)a < (unsigned)NA) ? a : 0;
    }
    if (tid == 0) s_in = q.in_list ? (uint32_t)q.in_list[e] : 0xFFu;
    __syncthreads();
    if (tid < N) {
        const int m = q.mdr ? q.mdr[e * N + tid] : (int)((ctab[s_loc[tid]] >> CT_MDR) & 0xFu);
        s_mdr[tid] = ((unsigned)m < (unsigned)NA) ? m : 0;
    }
    __syncthreads();
    const uint32_t in = s_in;
    const CtabOk okv{ctab};
    for (int t = tid; t < 9 * NG; t += T) {
        const int g = t / 9, b = t - 9 * (t / 9);
        int joint[N], loc[N], fin[N];
#pragma unroll
        for (int n = 0; n < N; ++n) {
            loc[n] = s_loc[n];
            joint[n] = ((in >> n) & 1u) ? s_act[n] : 0;  // defaultAction 'stay' for the unlisted
        }
        int affected;
        if (g < N) {  // action list unchanged
            affected = g;
        } else if (g < N + N * (N - 1)) {  // actor ii -> MdR
            const int idx = g - N, ii = idx / (N - 1), r = idx - ii * (N - 1);
            affected = r + (r >= ii);
#pragma unroll
            for (int n = 0; n < N; ++n)
                if (n == ii && ((in >> n) & 1u)) joint[n] = s_mdr[n];
        } else {  // everybody but ii -> MdR (FeAL)
            affected = g - N - N * (N - 1);
#pragma unroll
            for (int n = 0; n < N; ++n)
                if (n != affected && ((in >> n) & 1u)) joint[n] = s_mdr[n];
        }
#pragma unroll
        for (int n = 0; n < N; ++n)
            if (n == affected && ((in >> n) & 1u)) joint[n] = b;
        int apple[MAXN];
#pragma unroll
        for (int k = 0; k < MAXN; ++k) apple[k] = -1;
        World<N> w;
        w.init(loc, joint, q.W, q.w_magic);
        uint32_t caught;
        simulate<N, false>(w, okv, 0, apple, caught, fin);
        if (!(((w.crash | w.restr) >> affected) & 1u)) atomicOr(&s_bits[g], 1u << b);
    }
    __syncthreads();
    if (tid < N * N) {
        const int ii = tid / N, jj = tid - ii * N;
        int m = 0, a = 0;
        double r = 0.0;
        if (ii != jj) {
            m = __popc(s_bits[N + ii * (N - 1) + (jj - (jj > ii))]);
            a = __popc(s_bits[jj]);
            r = q.tab[m * 10 + a];
        }
        q.resp[e * N * N + tid] = r;
        if (q.vm) q.vm[e * N * N + tid] = m;
        if (q.va) q.va[e * N * N + tid] = a;
    }
    if (tid < N) {
        const int m = __popc(s_bits[N + N * (N - 1) + tid]), a = __popc(s_bits[tid]);
        if (q.feal) q.feal[e * N + tid] = q.tab[100 + m * 10 + a];
        if (q.feal_vm) q.feal_vm[e * N + tid] = m;
        if (q.feal_va) q.feal_va[e * N + tid] = a;
    }
}

}  // namespace gw

// =========================================================================================
// C ABI
// =========================================================================================
namespace {

thread_local std::string g_err;

gw_status fail(gw_status s, const std::string &msg) {
    g_err = msg;
    return s;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) return fail(GW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define GW_TRY(expr)                   \
    do {                               \
        gw_status _s = (expr);         \
        if (_s != GW_OK) return _s;    \
    } while (0)

struct Env {
    int device = 0;
    int H = 0, W = 0, HW = 0, N = 0, K = 0, F = 0, P = 0;
    int64_t E = 0, env_offset = 0;
    int fear = 0, max_steps = 0, auto_reset = 1, variant = 0;
    double fear_weight = 0.0;
    uint64_t seed = 0;
    int apples[GW_MAX_AGENTS] = {0};
    bool initialized = false;
    int mode = 3;        // kernel path (gw_create picks by batch size; GW_KERNEL=defer|merged forces):
                         // 3 "defer" (FeAR on: step_v2 <DEFER>, then fear_v2 || obs_kernel; FeAR off:
                         // step_v2, then obs_kernel), 4 "merged" (synchronous as defer with FeAR
                         // inline; with async obs one step_obs launch per step)
    int obs_be = 2;      // envs per obs_kernel block (default: see gw_create)
    bool obs_bf16 = false;  // gw_set_obs_dtype(env, GW_OBS_BF16): obs buffers hold bf16 (lossless)
    int obs_be_f32 = 2;         // the float32 writer's default
    uint32_t *celltab = nullptr;
    uint32_t *roadbits = nullptr;
    // fear_v2 with 2x envs per block (default since the obs writers overlap: C3 93.8 -> 92.1 us,
    // C5 175 -> 166, C4f 368 -> 358 per step; the bf16 line loses 2 %: profiles/r2_events);
    // GW_FEAR_BE=narrow: 1x (A/B)
    bool fear_wide = true;
    bool fear_wide_fixed = false;   // GW_FEAR_BE given (else the obs format picks, before any reset)
    hipStream_t aux = nullptr;      // second (high-priority) stream: fear_v2 beside the writer
    std::vector<hipEvent_t> sync_ev;  // fork/chunk/join events (timing disabled)
    // async obs (gw_set_obs_async): obs_kernel of step t runs on obs_stream while the world update
    // of step t+1 runs; the descriptor is double-buffered (desc_buf[dcur] = the latest step's)
    // (launched lazily: at the start of gw_step t+1, behind the caller's work between the steps,
    // e.g. the fused actor, so the writer never competes with it for the CUs; or at a fence)
    bool obs_async = false;
    hipStream_t last_stream = nullptr;            // merged mode: the stream of the last gw_step
    bool obs_lazy = false;                        // gw_set_obs_async(env, 2): launch at the next step
    int obs_chunks = 1;                           // GW_OBS_CHUNKS: the obs writer as this many launches
    // gw_step_patch_next: the next gw_step also writes the step's P x P windows (in the FeAR launch
    // where it can: fear_rows_kernel; else as gw_obs_patch right after the step)
    struct PatchReq {
        bool armed = false, done = false;
        int P = 0;
        float *patch = nullptr, *final_patch = nullptr;
    } patch_req;
    // one obs stream: a second one alternating with the descriptor buffer (so obs_kernel(t+1)
    // could start while obs_kernel(t) drains) measured 2.1x slower at C3 (more streams than the
    // process's hardware queues, GPU_MAX_HW_QUEUES = 4; profiles/r1_async)
    hipStream_t obs_stream = nullptr;
    // a second obs stream, used when consecutive steps write DIFFERENT obs buffers (a replay
    // ring's slots): writer t+1 then needs no order after writer t and starts while it drains,
    // instead of behind the ~10 us kernel boundary + cross-queue wait (GW_OBS_STREAMS=1: off)
    hipStream_t obs_stream2 = nullptr;
    int obs_streams = 2;
    int obs_cur = 0;                              // stream of the last writer (0 / 1)
    const void *obs_last[2] = {nullptr, nullptr}; // obs / final_obs buffers of the last writer
    hipEvent_t obs_done[2] = {nullptr, nullptr};  // obs_kernel that read desc_buf[i] has finished
    bool obs_pending[2] = {false, false};
    hipEvent_t world_ev = nullptr;                // world update of the queued step has finished
    // gw_set_obs_async(env, | 4): the caller's stream joins only the world update; fear_v2 (FeAR,
    // shaped reward, returns, FeAR stats rows) finishes on the aux stream, ordered by gw_fear_fence
    bool fear_async = false;
    bool fear_pending = false;
    hipEvent_t fear_ev = nullptr;
    bool obs_queued = false;                      // an obs_kernel launch waits in qobs
    bool qobs_prof = false;                       // profiling state of the step that queued it
    int qobs_buf = 0;
    gw::Params qobs;
    uint32_t *desc_buf[2] = {nullptr, nullptr};
    int dcur = 0;
    // tables
    uint8_t *okmask = nullptr, *policy = nullptr, *mdr = nullptr;
    double *cdf = nullptr, *resp = nullptr;
    uint16_t *amask = nullptr;
    int32_t *free_cells = nullptr;
    float *base = nullptr;
    // state
    int32_t *pos = nullptr, *t = nullptr, *prev = nullptr;
    uint32_t *flags = nullptr, *episode = nullptr, *desc = nullptr;
    uint4 *fwork = nullptr;  // deferred-FeAR records (mode 3 with FeAR on)
    unsigned long long *sims = nullptr;  // gw_count_sims counter (device), or null
    // gw_obs_patch's per-P tables of the map part of every window centre (patch_ops.hip MODE 4)
    std::vector<std::pair<int, float *>> ptbls;
    double *score = nullptr, *fscore = nullptr;
    std::vector<void *> allocs;
    // per-launch profiling events (gw_profile)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;   // timing events, reused across calls
    size_t ev_used = 0;
    struct Span { size_t b, e; int kind; };  // kind 0 = step kernel(s), 1 = obs kernel(s), 2 = fear_v2
    std::vector<Span> spans;
    int64_t steps_timed = 0;
    // flags of the pipeline's events.  They only order kernels of this device's queues (every
    // kernel already ends with an agent-scope release), so by default they skip the
    // system-scope fence (L2 write-back + invalidate) that a plain event record / wait costs at
    // every use: 5 us per record and 11-18 us between consecutive obs writers at C3 with it.
    unsigned sync_flags = hipEventDisableTiming | hipEventDisableSystemFence;
    unsigned prof_flags = hipEventDisableSystemFence;  // timing events of gw_profile
    // obs_done / world_ev are bound to the kernel launch they follow (hipExtLaunchKernelGGL stop
    // event) instead of a marker packet after it (+0.5 %, profiles/HISTORY.md)
};

// the second stream and n fork/join events (timing disabled), created on first use
// n fork/join events (timing disabled), created on first use
gw_status ensure_events(Env *env, int n) {
    while ((int)env->sync_ev.size() < n) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, env->sync_flags));
        env->sync_ev.push_back(e);
    }
    return GW_OK;
}

// the second stream (high priority: fear_v2's workgroups are dispatched ahead of the writer's)
// and n events.  Streams are created only where a path uses them: a process has few hardware
// queues (GPU_MAX_HW_QUEUES = 4 on the box) and every extra stream competes for them.
gw_status ensure_aux(Env *env, int n) {
    if (!env->aux) {
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&env->aux, hipStreamNonBlocking, hi));
    }
    return ensure_events(env, n);
}

// the async-obs stream and its per-descriptor-buffer completion events, created on first use
gw_status ensure_obs_stream(Env *env) {
    const gw_status st = ensure_events(env, 3);
    if (st != GW_OK) return st;
    if (!env->obs_stream) HIP_TRY(hipStreamCreateWithFlags(&env->obs_stream, hipStreamNonBlocking));
    for (hipEvent_t &e : env->obs_done)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, env->sync_flags));
    if (!env->world_ev) HIP_TRY(hipEventCreateWithFlags(&env->world_ev, env->sync_flags));
    if (!env->fear_ev) HIP_TRY(hipEventCreateWithFlags(&env->fear_ev, env->sync_flags));
    return GW_OK;
}

// gw_profile spans: the span's kernel launches carry its timing events in their dispatch
// (hipExtLaunchKernelGGL start / stop events: the kernel's own begin / end timestamps, no
// marker packets between the kernels of the pipeline).  The span's first launch takes the
// start event, every launch the stop event (the last one's end wins).
// t_bind_stop: a pipeline event (obs_done, world_ev) bound to the launch the same way, instead
// of a marker packet recorded after it (used when no timing span is open).
using gwprof::t_span_start;
using gwprof::t_span_stop;
using gwprof::t_bind_stop;

template <typename F, typename... Args>
void gw_launch(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
    gwprof::launch(kernel, grid, block, lds, s, args...);
}

hipError_t launch_obs(const Env *env, const gw::Params &p, float *obs, float *final_obs, hipStream_t s);
hipEvent_t next_event(Env *env);
gw_status prof_span_begin(Env *env, size_t &idx);
gw_status prof_span_end(Env *env, size_t idx, int kind);
void prof_span_split(Env *env, int kind);

// launch the queued obs_kernel on the obs stream, after its world update and (after != null)
// after the caller's work up to `after`
gw_status flush_obs(Env *env, hipEvent_t after, hipStream_t on = nullptr) {
    if (!env->obs_queued) return GW_OK;
    if (env->mode == 4) {  // merged: the last step's writer alone, on `on` (default: that step's stream)
        const bool prof = env->qobs_prof;
        size_t b = 0;
        if (prof && prof_span_begin(env, b) != GW_OK) return GW_ERR_HIP;
        HIP_TRY(launch_obs(env, env->qobs, env->qobs.out.obs, env->qobs.out.final_obs, on ? on : env->last_stream));
        if (prof) (void)prof_span_end(env, b, 1);
        env->obs_queued = false;
        return GW_OK;
    }
    // writers into the buffers of the last writer stay on its stream (write-after-write order);
    // a writer into other buffers alternates to the other obs stream
    const bool other = env->obs_streams > 1 && env->qobs.out.obs != env->obs_last[0] &&
                       (env->qobs.out.final_obs == nullptr || env->qobs.out.final_obs != env->obs_last[1]);
    if (other && !env->obs_stream2) HIP_TRY(hipStreamCreateWithFlags(&env->obs_stream2, hipStreamNonBlocking));
    if (other) env->obs_cur ^= 1;
    env->obs_last[0] = env->qobs.out.obs;
    env->obs_last[1] = env->qobs.out.final_obs;
    hipStream_t os = env->obs_cur ? env->obs_stream2 : env->obs_stream;
    HIP_TRY(hipStreamWaitEvent(os, env->world_ev, 0));
    if (after) HIP_TRY(hipStreamWaitEvent(os, after, 0));
    const bool prof = env->qobs_prof;  // timed iff the step that queued it was
    size_t b = 0;
    if (prof && prof_span_begin(env, b) != GW_OK) return GW_ERR_HIP;
    const bool bind = !prof;  // obs_done carried by the writer's launch
    if (bind) t_bind_stop = env->obs_done[env->qobs_buf];
    const hipError_t le = launch_obs(env, env->qobs, env->qobs.out.obs, env->qobs.out.final_obs, os);
    t_bind_stop = nullptr;
    HIP_TRY(le);
    if (prof) (void)prof_span_end(env, b, 1);
    if (!bind) HIP_TRY(hipEventRecord(env->obs_done[env->qobs_buf], os));
    env->obs_pending[env->qobs_buf] = true;
    env->obs_queued = false;
    return GW_OK;
}

// make `s` wait for an async fear_v2 still in flight
gw_status wait_fear(Env *env, hipStream_t s) {
    if (env->fear_pending) HIP_TRY(hipStreamWaitEvent(s, env->fear_ev, 0));
    return GW_OK;
}

// launch a queued obs_kernel and make `s` wait for every obs_kernel of the async-obs stream
// (and for an async fear_v2: the callers rewrite state or descriptors in place)
gw_status wait_obs(Env *env, hipStream_t s) {
    {
        const gw_status st = wait_fear(env, s);
        if (st != GW_OK) return st;
    }
    if (env->obs_queued) {
        if (env->mode == 4) {
            // merged: the writer runs on s, after the step that queued it (a graph replay of
            // captured steps runs on s itself; its capture stream holds no work)
            if (env->last_stream != s) {
                GW_TRY(ensure_events(env, 1));
                HIP_TRY(hipEventRecord(env->sync_ev[0], env->last_stream));
                HIP_TRY(hipStreamWaitEvent(s, env->sync_ev[0], 0));
            }
            GW_TRY(flush_obs(env, nullptr, s));
        } else {
            const gw_status st = flush_obs(env, nullptr);
            if (st != GW_OK) return st;
        }
    }
    for (int i = 0; i < 2; ++i)
        if (env->obs_pending[i]) HIP_TRY(hipStreamWaitEvent(s, env->obs_done[i], 0));
    return GW_OK;
}

hipEvent_t next_event(Env *env) {
    if (env->ev_used == env->ev_pool.size()) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, env->prof_flags) != hipSuccess) return nullptr;
        env->ev_pool.push_back(e);
    }
    return env->ev_pool[env->ev_used++];
}

// a profiled span: two timing events handed to the span's kernel launches (gw_launch).  The open
// span's first event index is also kept thread-locally, so a launch sequence can split it
// (prof_span_split: the obs writer's chunks are one span each, as a kernel trace counts them)
thread_local size_t t_span_idx = 0;

gw_status prof_span_begin(Env *env, size_t &idx) {
    idx = env->ev_used;
    hipEvent_t a = next_event(env), b = next_event(env);
    if (!a || !b) return fail(GW_ERR_HIP, "hipEventCreate failed");
    t_span_start = a;
    t_span_stop = b;
    t_span_idx = idx;
    return GW_OK;
}

gw_status prof_span_end(Env *env, size_t idx, int kind) {
    (void)idx;  // the span open now (a split may have replaced the one `idx` began)
    if (t_span_start) {  // no kernel was launched in the span: nothing to time
        env->ev_used = t_span_idx;
    } else {
        env->spans.push_back({t_span_idx, t_span_idx + 1, kind});
    }
    t_span_start = t_span_stop = nullptr;
    return GW_OK;
}

// close the open span after the launches made so far and open the next one (no-op without an
// open span or before its first launch)
void prof_span_split(Env *env, int kind) {
    if (!t_span_stop || t_span_start) return;
    env->spans.push_back({t_span_idx, t_span_idx + 1, kind});
    size_t idx = 0;
    if (prof_span_begin(env, idx) != GW_OK) t_span_start = t_span_stop = nullptr;
}

}  // namespace

namespace gwprof {
thread_local hipEvent_t t_span_start = nullptr, t_span_stop = nullptr, t_bind_stop = nullptr;

bool span_begin(void *handle, size_t *idx) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !env->profiling) return false;
    return prof_span_begin(env, *idx) == GW_OK;
}

void span_end(void *handle, size_t idx, int kind) {
    (void)prof_span_end(static_cast<Env *>(handle), idx, kind);
}
}  // namespace gwprof

namespace {

template <typename T>
gw_status dalloc(Env *env, T **ptr, size_t count) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, sizeof(T) * (count ? count : 1));
    if (e != hipSuccess) return fail(GW_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    env->allocs.push_back(p);
    *ptr = static_cast<T *>(p);
    return GW_OK;
}


gw::Params make_params(const Env *env) {
    gw::Params p;
    std::memset(&p, 0, sizeof(p));
    p.tb.okmask = env->okmask;
    p.tb.policy = env->policy;
    p.tb.cdf = env->cdf;
    p.tb.mdr = env->mdr;
    p.tb.amask = env->amask;
    p.tb.free_cells = env->free_cells;
    p.tb.base = env->base;
    p.tb.resp = env->resp;
    p.tb.celltab = env->celltab;
    p.n_cdf = env->P * 2 * 9;
    p.lds_cdf = env->P <= 64 ? 1 : 0;
    p.ctab_off = p.lds_cdf ? ((p.n_cdf * 8 + 15) / 16) * 16 : 0;
    p.resp_off = p.ctab_off + ((env->HW * 4 + 15) / 16) * 16;
    p.obs_be = env->obs_be;
    p.obs_bf16 = env->obs_bf16 ? 1 : 0;
    p.e_begin = 0;
    p.e_end = env->E;
    p.fwork = env->fwork;
    p.sims = env->sims;
    p.stats_row0 = 0;
    p.variant = env->variant;
    p.tb.roadbits = env->roadbits;
    p.st.pos = env->pos;
    p.st.flags = env->flags;
    p.st.t = env->t;
    p.st.episode = env->episode;
    p.st.prev = env->prev;
    p.st.score = env->score;
    p.st.fscore = env->fscore;
    p.desc = env->desc;
    p.E = env->E;
    p.env_offset = env->env_offset;
    p.fear_weight = env->fear_weight;
    p.H = env->H;
    p.W = env->W;
    p.HW = env->HW;
    p.N = env->N;
    p.K = env->K;
    p.F = env->F;
    p.max_steps = env->max_steps;
    p.auto_reset = env->auto_reset;
    p.key0 = (uint32_t)env->seed;
    p.key1 = (uint32_t)(env->seed >> 32);
    p.w_magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)env->W - 1) / (uint64_t)env->W);
    {
        const uint64_t hw4 = (uint64_t)std::max(1, env->HW / 4);
        p.hw4_magic = (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, (((uint64_t)1 << 32) + hw4 - 1) / hw4);
        const uint64_t hw8 = (uint64_t)std::max(1, env->HW / 8);
        p.hw8_magic = (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, (((uint64_t)1 << 32) + hw8 - 1) / hw8);
    }
    for (int k = 0; k < GW_MAX_AGENTS; ++k) p.apples[k] = env->apples[k];
    return p;
}

template <int N, int KMAX, bool FEAR, bool DEFER = false>
hipError_t launch_v2(const Env *env, const gw::Params &p, hipStream_t s) {
    constexpr int BE = gw::V2Cfg<N, KMAX, FEAR, false, DEFER>::BE;
    const int64_t n = p.e_end - p.e_begin;  // this launch's env range (a pipeline chunk or all)
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + BE - 1) / BE);
    // dynamic LDS [cdf][cell table][Resp (FeAR)].  (Staging the free-cell list there too for the
    // auto-reset's spawn made C2's step kernel slower: 11.4 -> 12.2 us, profiles/r3_c2.)
    const size_t dyn = (size_t)p.resp_off + (FEAR ? 100 * sizeof(double) : 0);
    gw_launch((gw::step_v2<N, KMAX, FEAR, DEFER>), dim3(grid), dim3(gw::V2Cfg<N, KMAX, FEAR, false, DEFER>::THREADS),
              dyn, s, p);
    return hipGetLastError();
}

// stats rows of the deferred world-update kernel; fear_v2's rows follow them
template <int N>
int64_t defer_step_rows(const Env *env) {
    const int be = env->K <= 2 ? gw::V2Cfg<N, 2, false, false, true>::BE : gw::V2Cfg<N, N, false, false, true>::BE;
    return (env->E + be - 1) / be;
}

template <int N, int KMAX, bool WIDE>
hipError_t launch_fear_k(const Env *env, const gw::Params &p0, hipStream_t s) {
    constexpr int BE = gw::V2Cfg<N, KMAX, true, WIDE>::BE;
    gw::Params p = p0;
    p.lds_cdf = 0;  // dynamic LDS [cell table][Resp]
    p.ctab_off = 0;
    p.resp_off = ((env->HW * 4 + 15) / 16) * 16;
    p.stats_row0 = defer_step_rows<N>(env);
    const int64_t n = p.e_end - p.e_begin;
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + BE - 1) / BE);
    const size_t dyn = (size_t)p.resp_off + 100 * sizeof(double);
    gw_launch((gw::fear_v2<N, KMAX, WIDE>), dim3(grid), dim3(gw::V2Cfg<N, KMAX, true, WIDE>::THREADS), dyn, s, p);
    return hipGetLastError();
}

template <int N>
hipError_t launch_fear(const Env *env, const gw::Params &p, hipStream_t s) {
    if (env->fear_wide)
        return env->K <= 2 ? launch_fear_k<N, 2, true>(env, p, s) : launch_fear_k<N, N, true>(env, p, s);
    return env->K <= 2 ? launch_fear_k<N, 2, false>(env, p, s) : launch_fear_k<N, N, false>(env, p, s);
}

template <int N>
int fear_be(const Env *env) {
    if (env->fear_wide) return env->K <= 2 ? gw::V2Cfg<N, 2, true, true>::BE : gw::V2Cfg<N, N, true, true>::BE;
    return env->K <= 2 ? gw::V2Cfg<N, 2, true>::BE : gw::V2Cfg<N, N, true>::BE;
}

// the windows' writer args for the env's current descriptors (gw_obs_patch's, without its table)
gw::PatchArgs patch_args(const Env *env, int P, float *patch, float *final_patch) {
    gw::PatchArgs a;
    a.desc = env->desc;
    a.roadbits = env->roadbits;
    a.base = env->base;
    a.patch = patch;
    a.final_patch = final_patch;
    a.E = env->E;
    a.H = env->H;
    a.W = env->W;
    a.N = env->N;
    a.K = env->K;
    a.P = P;
    a.variant = env->variant;
    for (int k = 0; k < GW_MAX_AGENTS; ++k) a.apples[k] = k < env->K ? env->apples[k] : -1;
    return a;
}

template <int N, int KMAX, bool WIDE>
hipError_t launch_fear_rows_k(const Env *env, const gw::Params &p0, const gw::PatchArgs &a, hipStream_t s) {
    constexpr int BE = gw::V2Cfg<N, KMAX, true, WIDE>::BE;
    gw::Params p = p0;
    p.lds_cdf = 0;
    p.ctab_off = 0;
    p.resp_off = ((env->HW * 4 + 15) / 16) * 16;
    p.stats_row0 = defer_step_rows<N>(env);
    const int64_t n = p.e_end - p.e_begin;
    const unsigned nfear = (unsigned)((n + BE - 1) / BE);
    const unsigned nrx = (unsigned)((a.E * a.P + 255) / 256);  // 2 waves x 2 runs x 64 rows per block
    // one footprint for both roles: the FeAR tables or the row writer's 2 x 64 x 4 float4 slices
    const size_t dyn = std::max((size_t)p.resp_off + 100 * sizeof(double), sizeof(float4) * 2 * 64 * 4);
    gw_launch((gw::fear_rows_kernel<N, KMAX, WIDE>), dim3(nfear + nrx * (unsigned)a.K), dim3(128), dyn, s, p, a,
              nfear, nrx);
    return hipGetLastError();
}

template <int N>
hipError_t launch_fear_rows(const Env *env, const gw::Params &p, const gw::PatchArgs &a, hipStream_t s) {
    if (env->fear_wide)
        return env->K <= 2 ? launch_fear_rows_k<N, 2, true>(env, p, a, s) : launch_fear_rows_k<N, N, true>(env, p, a, s);
    return env->K <= 2 ? launch_fear_rows_k<N, 2, false>(env, p, a, s) : launch_fear_rows_k<N, N, false>(env, p, a, s);
}

hipError_t dispatch_fear_rows(const Env *env, const gw::Params &p, const gw::PatchArgs &a, hipStream_t s) {
    switch (env->N) {
        case 1: return launch_fear_rows<1>(env, p, a, s);
        case 2: return launch_fear_rows<2>(env, p, a, s);
        case 3: return launch_fear_rows<3>(env, p, a, s);
        case 4: return launch_fear_rows<4>(env, p, a, s);
        case 5: return launch_fear_rows<5>(env, p, a, s);
        case 6: return launch_fear_rows<6>(env, p, a, s);
        case 7: return launch_fear_rows<7>(env, p, a, s);
        case 8: return launch_fear_rows<8>(env, p, a, s);
    }
    return hipErrorInvalidValue;
}

hipError_t dispatch_fear(const Env *env, const gw::Params &p, hipStream_t s) {
    switch (env->N) {
        case 1: return launch_fear<1>(env, p, s);
        case 2: return launch_fear<2>(env, p, s);
        case 3: return launch_fear<3>(env, p, s);
        case 4: return launch_fear<4>(env, p, s);
        case 5: return launch_fear<5>(env, p, s);
        case 6: return launch_fear<6>(env, p, s);
        case 7: return launch_fear<7>(env, p, s);
        case 8: return launch_fear<8>(env, p, s);
    }
    return hipErrorInvalidValue;
}

template <int N>
hipError_t launch_step(const Env *env, const gw::Params &p, hipStream_t s) {
    if (env->mode == 3 && env->fear)  // deferred FeAR: the world update only, + FearRec
        return env->K <= 2 ? launch_v2<N, 2, false, true>(env, p, s) : launch_v2<N, N, false, true>(env, p, s);
    if (env->fear)  // FeAR inline (the merged path's step role, its synchronous steps)
        return env->K <= 2 ? launch_v2<N, 2, true>(env, p, s) : launch_v2<N, N, true>(env, p, s);
    return env->K <= 2 ? launch_v2<N, 2, false>(env, p, s) : launch_v2<N, N, false>(env, p, s);
}

template <int N>
hipError_t launch_reset(const Env *env, const gw::Params &p, hipStream_t s) {
    const unsigned grid = (unsigned)((env->E + 255) / 256);
    gw_launch((gw::reset_kernel<N>), dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t dispatch_step(const Env *env, const gw::Params &p, hipStream_t s) {
    switch (env->N) {
        case 1: return launch_step<1>(env, p, s);
        case 2: return launch_step<2>(env, p, s);
        case 3: return launch_step<3>(env, p, s);
        case 4: return launch_step<4>(env, p, s);
        case 5: return launch_step<5>(env, p, s);
        case 6: return launch_step<6>(env, p, s);
        case 7: return launch_step<7>(env, p, s);
        case 8: return launch_step<8>(env, p, s);
    }
    return hipErrorInvalidValue;
}

hipError_t dispatch_reset(const Env *env, const gw::Params &p, hipStream_t s) {
    switch (env->N) {
        case 1: return launch_reset<1>(env, p, s);
        case 2: return launch_reset<2>(env, p, s);
        case 3: return launch_reset<3>(env, p, s);
        case 4: return launch_reset<4>(env, p, s);
        case 5: return launch_reset<5>(env, p, s);
        case 6: return launch_reset<6>(env, p, s);
        case 7: return launch_reset<7>(env, p, s);
        case 8: return launch_reset<8>(env, p, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_obs_range(const Env *env, const gw::Params &p, float *obs, float *final_obs, hipStream_t s);

// obs_kernel's LDS: road bitmask, OBS_BE flags, [2][obs_be][K][N + 1] patch cells + values
// (+ with the f32 patch tables: [2][obs_be][K][N + 1] float4 entries and the byte tables)
size_t obs_lds_bytes(const Env *env) {
    const size_t base = sizeof(uint32_t) * ((env->HW + 31) / 32 + gw::OBS_BE) +
                        (size_t)2 * 2 * env->obs_be * env->K * (env->N + 1) * sizeof(uint32_t);
    if (env->obs_bf16 || !gw::obs_tab_ok(env->HW, env->obs_be, env->K)) return base;
    return (size_t)gw::obs_ent_off(env->HW, env->obs_be, env->K, env->N + 1) +
           (size_t)env->obs_be * env->K * (env->N + 1) * sizeof(float4) +
           (size_t)gw::obs_tab_bytes(env->HW, env->obs_be, env->K);
}

template <int N, int KMAX, bool FEAR>
hipError_t launch_step_obs_k(const Env *env, const gw::Params &p, const gw::Params &q, hipStream_t s) {
    constexpr int BE = gw::V2Cfg<N, KMAX, FEAR>::BE;
    const int64_t n = p.e_end - p.e_begin, nq = q.e_end - q.e_begin;
    const unsigned nstep = (unsigned)((n + BE - 1) / BE);
    const unsigned nobs = (unsigned)((nq + env->obs_be - 1) / env->obs_be);
    const size_t step_dyn = (size_t)p.resp_off + (FEAR ? 100 * sizeof(double) : 0);
    const size_t dyn = std::max(step_dyn, obs_lds_bytes(env));
    gw_launch((gw::step_obs<N, KMAX, FEAR>), dim3(nstep + nobs), dim3(128), dyn, s, p, q, q.out.obs, q.out.final_obs,
              nstep);
    return hipGetLastError();
}

template <int N>
hipError_t launch_step_obs_n(const Env *env, const gw::Params &p, const gw::Params &q, hipStream_t s) {
    if (env->fear)
        return env->K <= 2 ? launch_step_obs_k<N, 2, true>(env, p, q, s) : launch_step_obs_k<N, N, true>(env, p, q, s);
    return env->K <= 2 ? launch_step_obs_k<N, 2, false>(env, p, q, s) : launch_step_obs_k<N, N, false>(env, p, q, s);
}

// merged mode: step t (p) and the obs writer of step t-1 (q) as one step_obs launch
hipError_t launch_step_obs(const Env *env, const gw::Params &p, const gw::Params &q, hipStream_t s) {
    switch (env->N) {
        case 1: return launch_step_obs_n<1>(env, p, q, s);
        case 2: return launch_step_obs_n<2>(env, p, q, s);
        case 3: return launch_step_obs_n<3>(env, p, q, s);
        case 4: return launch_step_obs_n<4>(env, p, q, s);
        case 5: return launch_step_obs_n<5>(env, p, q, s);
        case 6: return launch_step_obs_n<6>(env, p, q, s);
        case 7: return launch_step_obs_n<7>(env, p, q, s);
        case 8: return launch_step_obs_n<8>(env, p, q, s);
    }
    return hipErrorInvalidValue;
}

// GW_OBS_CHUNKS = c > 1: the writer as c launches over consecutive env ranges.  The hardware
// dispatches one kernel's workgroups ahead of a later kernel of another queue, so a single
// long writer holds the CUs until its last workgroup is placed; between chunk launches the
// caller stream's kernels (the next actor) get their turn.
hipError_t launch_obs(const Env *env, const gw::Params &p, float *obs, float *final_obs, hipStream_t s) {
    if (!obs && !final_obs) return hipSuccess;
    const int64_t n = p.e_end - p.e_begin;
    if (n <= 0) return hipSuccess;
    const int64_t blocks = (n + env->obs_be - 1) / env->obs_be;
    const int64_t c = std::max<int64_t>(1, std::min<int64_t>(env->obs_chunks, blocks));
    for (int64_t i = 0; i < c; ++i) {
        if (i > 0) prof_span_split(const_cast<Env *>(env), 1);  // profiled: one span per chunk
        gw::Params q = p;
        q.e_begin = p.e_begin + blocks * i / c * env->obs_be;
        q.e_end = std::min(p.e_end, p.e_begin + blocks * (i + 1) / c * env->obs_be);
        const hipError_t e = launch_obs_range(env, q, obs, final_obs, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_obs_range(const Env *env, const gw::Params &p, float *obs, float *final_obs, hipStream_t s) {
    const int64_t n = p.e_end - p.e_begin;
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + env->obs_be - 1) / env->obs_be);
    const size_t lds = obs_lds_bytes(env);
    if (env->obs_bf16) {  // gw_set_obs_dtype checked HW % 8 == 0
        gw_launch((gw::obs_kernel<true, true, true>), dim3(grid), dim3(gw::OBS_THREADS), lds, s, p, obs, final_obs);
    } else if (env->HW % 4 == 0) {
        gw_launch((gw::obs_kernel<true, true>), dim3(grid), dim3(gw::OBS_THREADS), lds, s, p, obs, final_obs);
    } else {
        gw_launch((gw::obs_kernel<false, false>), dim3(grid), dim3(gw::OBS_THREADS), lds, s, p, obs, final_obs);
    }
    return hipGetLastError();
}

}  // namespace

namespace {
template <int N>
int64_t stats_rows_n(const Env *env) {
    int be;
    if (env->mode == 3 && env->fear) {
        const int bf = fear_be<N>(env);
        return defer_step_rows<N>(env) + (env->E + bf - 1) / bf;
    }
    if (env->fear) be = env->K <= 2 ? gw::V2Cfg<N, 2, true>::BE : gw::V2Cfg<N, N, true>::BE;
    else be = env->K <= 2 ? gw::V2Cfg<N, 2, false>::BE : gw::V2Cfg<N, N, false>::BE;
    return (env->E + be - 1) / be;
}
}  // namespace

namespace {
template <int N>
hipError_t launch_fear_matrix(const Env *env, int64_t n, const gw::FmParams &q, hipStream_t s) {
    const size_t dyn = ((size_t)env->HW * 4 + 15) / 16 * 16;
    gw_launch((gw::fear_matrix_kernel<N>), dim3((unsigned)n), dim3(128), dyn, s, q);
    return hipGetLastError();
}
}  // namespace

extern "C" {

const char *gw_last_error(void) { return g_err.c_str(); }

gw_status gw_create(const gw_scenario *sc, const gw_config *cfg, int device, void **out_env) {
    if (!sc || !cfg || !out_env) return fail(GW_ERR_ARG, "null argument");
    *out_env = nullptr;
    const int H = sc->H, W = sc->W, N = cfg->N, K = cfg->K;
    if (H < 1 || W < 2 || (int64_t)H * W > 4096) return fail(GW_ERR_ARG, "need W >= 2 and H*W <= 4096");
    if (N < 1 || N > GW_MAX_AGENTS || K < 1 || K > N) return fail(GW_ERR_ARG, "need 1 <= K <= N <= 8");
    if (cfg->num_envs < 1) return fail(GW_ERR_ARG, "num_envs must be >= 1");
    if (cfg->variant != 0 && cfg->variant != 1) return fail(GW_ERR_ARG, "variant must be 0 or 1");
    if (cfg->variant == 1 && K != 1) return fail(GW_ERR_ARG, "the single-agent variant needs K == 1");
    if (cfg->env_offset < 0 || cfg->env_offset + cfg->num_envs > ((int64_t)1 << 32))
        return fail(GW_ERR_ARG, "global env ids must fit in 32 bits");
    if (!sc->region || !sc->policy_id || !sc->policy_cdf || !sc->mdr || !sc->apples || sc->n_policies < 1)
        return fail(GW_ERR_ARG, "incomplete scenario tables");
    const int HW = H * W;
    std::vector<uint8_t> ok(HW), mdr(HW), pol(HW);
    std::vector<uint16_t> am(HW);
    std::vector<float> base(HW);
    std::vector<uint32_t> ctab(HW);
    std::vector<uint32_t> rbits((HW + 31) / 32, 0u);
    std::vector<int32_t> freec;
    for (int c = 0; c < HW; ++c) {
        const int r = c / W, q = c % W;
        const auto road = [&](int rr, int cc) { return rr >= 0 && rr < H && cc >= 0 && cc < W && sc->region[rr * W + cc] != 0; };
        ok[c] = (uint8_t)(road(r - 1, q) | (road(r + 1, q) << 1) | (road(r, q - 1) << 2) | (road(r, q + 1) << 3) |
                          ((sc->region[c] != 0) << 4));  // bit 4: the cell itself is road
        // get_action_mask, custom/ma_customenv.py:467-506
        uint16_t m = 0x1FF;
        if (!road(r - 1, q)) m &= ~(1u << 1);
        if (!road(r + 1, q)) m &= ~(1u << 2);
        if (!road(r, q - 1)) m &= ~(1u << 3);
        if (!road(r, q + 1)) m &= ~(1u << 4);
        if (!road(r - 2, q)) m &= ~(1u << 5);
        if (!road(r + 2, q)) m &= ~(1u << 6);
        if (!road(r, q - 2)) m &= ~(1u << 7);
        if (!road(r, q + 2)) m &= ~(1u << 8);
        am[c] = m;
        base[c] = sc->region[c] ? 0.0f : -1.0f;
        if (sc->region[c]) freec.push_back(c);
        if (sc->mdr[c] >= GW_N_ACTIONS) return fail(GW_ERR_ARG, "MdR action out of range");
        if (sc->policy_id[c] >= sc->n_policies) return fail(GW_ERR_ARG, "policy id out of range");
        mdr[c] = sc->mdr[c];
        pol[c] = sc->policy_id[c];
        ctab[c] = (uint32_t)pol[c] | ((uint32_t)mdr[c] << 8) | ((uint32_t)m << 12) | ((uint32_t)(ok[c] & 0xFu) << 21) |
                  ((uint32_t)(sc->region[c] != 0) << 25);
        if (sc->region[c]) rbits[c >> 5] |= 1u << (c & 31);
    }
    if ((int)freec.size() < N) return fail(GW_ERR_ARG, "fewer road cells than agents");
    for (int k = 0; k < K; ++k)
        if (sc->apples[k] < 0 || sc->apples[k] >= HW) return fail(GW_ERR_ARG, "apple outside the grid");
    // Resp table: Responsibility.py:194-198 evaluated in IEEE f64 exactly as numpy does;
    // entries 100-199: FeAL = clip(va / (vm + EPS), -1, 1) (:282-285)
    std::vector<double> resp(200);
    for (int vm = 0; vm < 10; ++vm)
        for (int va = 0; va < 10; ++va) {
            volatile double num = (double)vm - (double)va;
            volatile double den = (double)vm + 0.000001;
            double r = num / den;
            r = r < -1.0 ? -1.0 : (r > 1.0 ? 1.0 : r);
            resp[vm * 10 + va] = r;
            volatile double fnum = (double)va;
            double f = fnum / den;
            f = f < -1.0 ? -1.0 : (f > 1.0 ? 1.0 : f);
            resp[100 + vm * 10 + va] = f;
        }

    Env *env = new (std::nothrow) Env();
    if (!env) return fail(GW_ERR_ALLOC, "host allocation failed");
    env->device = device;
    env->H = H; env->W = W; env->HW = HW; env->N = N; env->K = K;
    env->F = (int)freec.size();
    env->P = sc->n_policies;
    env->E = cfg->num_envs;
    env->env_offset = cfg->env_offset;
    env->fear = cfg->fear ? 1 : 0;
    env->fear_weight = cfg->fear_weight;
    env->max_steps = cfg->max_steps;
    env->auto_reset = cfg->auto_reset ? 1 : 0;
    env->variant = cfg->variant;
    env->seed = cfg->seed;
    for (int k = 0; k < K; ++k) env->apples[k] = sc->apples[k];
    {
        // the kernel path: merged for small batches, defer above GW_MERGE_BYTES of obs per step
        // (crossover at C3's shape with the obs ring's overlapping writers: merged wins up to
        // 16,384 envs = 128 MiB, defer from 24,576 = 192 MiB; profiles/HISTORY.md);
        // GW_KERNEL=defer|merged forces one of the two (result-neutral: both are pinned to the
        // oracle by tests/test_gpu_parity.py)
        const char *kv = std::getenv("GW_KERNEL");
        env->mode = 3;
        if (HW % 4 == 0) {
            const char *mb = std::getenv("GW_MERGE_BYTES");
            const int64_t lim = mb ? std::atoll(mb) : ((int64_t)160 << 20);
            if (cfg->num_envs * (int64_t)K * HW * 4 <= lim) env->mode = 4;
            if (kv && std::strcmp(kv, "merged") == 0) env->mode = 4;
        }
        if (kv && std::strcmp(kv, "defer") == 0) env->mode = 3;
        // fear_v2 block size (result-neutral): wide (default) or narrow (the bf16 obs default)
        const char *fb = std::getenv("GW_FEAR_BE");
        if (fb && std::strcmp(fb, "wide") == 0) env->fear_wide = true;
        if (fb && std::strcmp(fb, "narrow") == 0) env->fear_wide = false;
        env->fear_wide_fixed = fb != nullptr;
        // obs_kernel block size (profiles/HISTORY.md): 4 float4 stores per thread when the writer
        // runs alone (32x32 K=2 -> 2 envs, 64x64 -> 1), 8 while fear_v2 shares the CUs (32x32 ->
        // 4 envs: 2.5 % faster step at C3)
        int be_def = std::max(1, 4096 / std::max(1, K * HW));
        if (env->mode == 3 && env->fear) be_def *= 2;
        env->obs_be = std::max(1, std::min(8, be_def));  // f32 default <= 8 envs per block
        env->obs_be_f32 = env->obs_be;
        // scheduling of the async writer (result-neutral): c launches per step, one or two streams
        const char *oc = std::getenv("GW_OBS_CHUNKS");
        if (oc) env->obs_chunks = std::max(1, std::min(64, std::atoi(oc)));
        const char *osn = std::getenv("GW_OBS_STREAMS");
        if (osn) env->obs_streams = std::atoi(osn) > 1 ? 2 : 1;
    }

    auto cleanup = [&](gw_status s) {
        for (void *p : env->allocs) (void)hipFree(p);
        delete env;
        return s;
    };
    if (hipSetDevice(device) != hipSuccess) return cleanup(fail(GW_ERR_HIP, "hipSetDevice failed"));
    const size_t E = (size_t)env->E;
    gw_status st = GW_OK;
    if ((st = dalloc(env, &env->okmask, HW)) || (st = dalloc(env, &env->policy, HW)) ||
        (st = dalloc(env, &env->mdr, HW)) || (st = dalloc(env, &env->cdf, (size_t)env->P * 2 * 9)) ||
        (st = dalloc(env, &env->resp, 200)) || (st = dalloc(env, &env->amask, HW)) ||
        (st = dalloc(env, &env->free_cells, freec.size())) || (st = dalloc(env, &env->base, HW)) ||
        (st = dalloc(env, &env->pos, (size_t)N * E)) || (st = dalloc(env, &env->t, E)) ||
        (st = dalloc(env, &env->prev, (size_t)K * E)) || (st = dalloc(env, &env->flags, E)) ||
        (st = dalloc(env, &env->episode, E)) || (st = dalloc(env, &env->desc, 2 * E * gw::NDESC)) ||
        (st = dalloc(env, &env->score, E)) || (st = dalloc(env, &env->fscore, E)) ||
        (st = dalloc(env, &env->celltab, HW)) || (st = dalloc(env, &env->roadbits, rbits.size())) ||
        (env->mode == 3 && env->fear && (st = dalloc(env, &env->fwork, E * (N <= 4 ? 1 : 2)))))
        return cleanup(st);
    hipError_t he = hipSuccess;
#define CP(dst, src, n) if (he == hipSuccess) he = hipMemcpy(dst, src, n, hipMemcpyHostToDevice)
    CP(env->okmask, ok.data(), HW);
    CP(env->policy, pol.data(), HW);
    CP(env->mdr, mdr.data(), HW);
    CP(env->cdf, sc->policy_cdf, sizeof(double) * env->P * 2 * 9);
    CP(env->resp, resp.data(), sizeof(double) * 200);
    CP(env->amask, am.data(), sizeof(uint16_t) * HW);
    CP(env->free_cells, freec.data(), sizeof(int32_t) * freec.size());
    CP(env->base, base.data(), sizeof(float) * HW);
    CP(env->celltab, ctab.data(), sizeof(uint32_t) * HW);
    CP(env->roadbits, rbits.data(), sizeof(uint32_t) * rbits.size());
#undef CP
    if (he == hipSuccess) he = hipMemset(env->episode, 0xFF, sizeof(uint32_t) * E);  // first reset -> 0
    if (he == hipSuccess) he = hipMemset(env->desc, 0, sizeof(uint32_t) * 2 * E * gw::NDESC);
    env->desc_buf[0] = env->desc;
    env->desc_buf[1] = env->desc + E * gw::NDESC;
    if (he == hipSuccess) he = hipDeviceSynchronize();
    if (he != hipSuccess) return cleanup(fail(GW_ERR_HIP, std::string("init: ") + hipGetErrorString(he)));
    *out_env = env;
    return GW_OK;
}

gw_status gw_reset(void *handle, const uint8_t *env_mask, const int32_t *spawn_cells, float *obs,
                   uint16_t *mask, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    env->patch_req = Env::PatchReq{};  // a window request armed before the reset is dropped
    gw::Params p = make_params(env);
    p.rmask = env_mask;
    p.spawn = spawn_cells;
    p.out.mask = mask;
    hipStream_t s = static_cast<hipStream_t>(stream);
    GW_TRY(wait_obs(env, s));  // async obs: the descriptors are rewritten in place below
    HIP_TRY(dispatch_reset(env, p, s));
    HIP_TRY(launch_obs(env, p, obs, nullptr, s));
    env->initialized = true;
    return GW_OK;
}

static gw_status obs_patch_launch(Env *env, int32_t P, float *patch, float *final_patch, hipStream_t s);

static gw_status gw_step_body(void *handle, const int32_t *rl_actions, const int32_t *scripted,
                              const int32_t *spawn, const gw_step_out *out, void *stream);

gw_status gw_step(void *handle, const int32_t *rl_actions, const int32_t *scripted,
                  const int32_t *spawn, const gw_step_out *out, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    const gw_status st = gw_step_body(handle, rl_actions, scripted, spawn, out, stream);
    Env::PatchReq rq = env->patch_req;
    env->patch_req = Env::PatchReq{};
    if (st != GW_OK || !rq.armed || rq.done) return st;
    // the requested windows, not written inside the step's launches: as gw_obs_patch right after
    return obs_patch_launch(env, rq.P, rq.patch, rq.final_patch, static_cast<hipStream_t>(stream));
}

gw_status gw_step_patch_next(void *handle, int32_t P, float *patch, float *final_patch) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (P < 1 || P > 129) return fail(GW_ERR_ARG, "gw_step_patch_next: need 1 <= P <= 129");
    env->patch_req = Env::PatchReq{};
    if (!patch && !final_patch) return GW_OK;
    env->patch_req.armed = true;
    env->patch_req.P = P;
    env->patch_req.patch = patch;
    env->patch_req.final_patch = final_patch;
    return GW_OK;
}

static gw_status gw_step_body(void *handle, const int32_t *rl_actions, const int32_t *scripted,
                              const int32_t *spawn, const gw_step_out *out, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (!env->initialized) return fail(GW_ERR_STATE, "gw_step before gw_reset");
    gw::Params p = make_params(env);
    p.rl = rl_actions;
    p.scripted = scripted;
    p.spawn = spawn;
    if (out) p.out = *out;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool want_obs = p.out.obs || p.out.final_obs;
    if (env->profiling) env->steps_timed++;
    auto span_begin = [&](hipStream_t, size_t &idx) -> gw_status {
        idx = 0;
        return env->profiling ? prof_span_begin(env, idx) : GW_OK;
    };
    auto span_end = [&](hipStream_t, size_t b, int kind) -> gw_status {
        return env->profiling ? prof_span_end(env, b, kind) : GW_OK;
    };
    const bool defer = env->mode == 3 && env->fear;
    if (env->obs_async && want_obs && env->mode == 4) {
        // Merged pipeline: ONE launch per step on the caller's stream: this step's world update
        // + FeAR (writing descriptor buffer nb) and the obs writer of the previous step (reading
        // the other buffer) as the two block roles of step_obs (§5.7).  The writer of the last
        // step stays queued until the next step or a fence.
        env->last_stream = s;
        const int nb = env->dcur ^ 1;
        p.desc = env->desc_buf[nb];
        const bool merge = env->obs_queued;
        size_t b;
        GW_TRY(span_begin(s, b));
        if (merge)
            HIP_TRY(launch_step_obs(env, p, env->qobs, s));
        else
            HIP_TRY(dispatch_step(env, p, s));
        GW_TRY(span_end(s, b, merge ? 1 : 0));
        env->qobs = p;
        env->qobs_buf = nb;
        env->qobs_prof = env->profiling;
        env->obs_queued = true;
        env->dcur = nb;
        env->desc = env->desc_buf[nb];
        return GW_OK;
    }
    if (env->obs_async && want_obs && env->mode == 3) {
        // Software pipeline over steps.  The world update (and FeAR) of step t runs on s
        // (rewards, dones, masks, state, stats: stream-ordered as usual).  The obs writer of
        // step t runs on obs_stream right after the world update (eager), or is queued and
        // launched at the start of step t+1 behind the caller's work in between (lazy), and
        // overlaps FeAR and the world update + FeAR of step t+1, which read only the state.
        // The descriptor is double-buffered: step t writes desc_buf[nb]; obs_kernel(t-2) read
        // that buffer, so the world update waits for it.
        GW_TRY(ensure_obs_stream(env));
        // the world update + FeAR chain runs on the caller's stream itself (no fork / join hops
        // between consecutive steps); only with the unjoined FeAR (| 4) does it go to the aux stream
        const bool on_aux = defer && env->fear_async;
        if (on_aux) GW_TRY(ensure_aux(env, 3));
        hipStream_t ws = on_aux ? env->aux : s;
        if (on_aux || env->obs_queued) HIP_TRY(hipEventRecord(env->sync_ev[0], s));  // the caller's prior work
        GW_TRY(flush_obs(env, env->sync_ev[0]));       // lazy: obs_kernel(t-1), behind that work
        const int nb = env->dcur ^ 1;
        p.desc = env->desc_buf[nb];
        size_t b;
        if (on_aux) HIP_TRY(hipStreamWaitEvent(ws, env->sync_ev[0], 0));
        if (env->obs_pending[nb]) HIP_TRY(hipStreamWaitEvent(ws, env->obs_done[nb], 0));
        GW_TRY(span_begin(ws, b));
        const bool bind = !env->profiling;  // world_ev carried by the launch
        if (bind) t_bind_stop = env->world_ev;
        const hipError_t se = dispatch_step(env, p, ws);
        t_bind_stop = nullptr;
        HIP_TRY(se);
        GW_TRY(span_end(ws, b, 0));
        if (!bind) HIP_TRY(hipEventRecord(env->world_ev, ws));
        if (defer && env->fear_async) {
            // s joins the world update only: the caller's next work (the actor reads the
            // descriptors and masks) overlaps fear_v2; FeAR-owned outputs wait for gw_fear_fence
            HIP_TRY(hipStreamWaitEvent(s, env->world_ev, 0));
            GW_TRY(span_begin(ws, b));
            HIP_TRY(dispatch_fear(env, p, ws));
            GW_TRY(span_end(ws, b, 2));
            HIP_TRY(hipEventRecord(env->fear_ev, ws));
            env->fear_pending = true;
        } else {
            if (defer) {
                GW_TRY(span_begin(ws, b));
                HIP_TRY(dispatch_fear(env, p, ws));
                GW_TRY(span_end(ws, b, 2));
            }
            if (on_aux) {
                HIP_TRY(hipEventRecord(env->sync_ev[2], ws));  // join the world update + FeAR
                HIP_TRY(hipStreamWaitEvent(s, env->sync_ev[2], 0));
            }
        }
        env->qobs = p;
        env->qobs_buf = nb;
        env->qobs_prof = env->profiling;
        env->obs_queued = true;
        if (!env->obs_lazy) GW_TRY(flush_obs(env, nullptr));  // eager: right after the world update
        env->dcur = nb;
        env->desc = env->desc_buf[nb];
        return GW_OK;
    }
    // every other path writes the current descriptor buffer in place: an async obs_kernel still
    // reading it (a step without obs outputs, or a non-pipelining kernel path) must finish first
    if (env->obs_async || env->fear_pending) GW_TRY(wait_obs(env, s));
    if (defer) {
        // world update; then fear_v2 on the aux stream || obs_kernel on s; join
        size_t b;
        GW_TRY(span_begin(s, b));
        HIP_TRY(dispatch_step(env, p, s));
        GW_TRY(span_end(s, b, 0));
        if (!want_obs) {
            Env::PatchReq &rq = env->patch_req;
            const int P = rq.P;
            // the requested windows inside the FeAR launch: the row writer's conditions, whole range
            const bool rows = rq.armed && rq.patch && P >= 2 && P <= 16 && env->E % 4 == 0 &&
                              env->N >= 1 && env->N <= 8 && (uint64_t)env->E * (uint64_t)P < (1ull << 32) &&
                              p.e_begin == 0 && p.e_end == env->E;
            GW_TRY(span_begin(s, b));
            if (rows) {
                // (the world update just wrote env->desc: p.desc is that buffer)
                gw::PatchArgs a = patch_args(env, P, rq.patch, rq.final_patch);
                a.desc = p.desc;
                HIP_TRY(dispatch_fear_rows(env, p, a, s));
                rq.done = true;
            } else {
                HIP_TRY(dispatch_fear(env, p, s));
            }
            GW_TRY(span_end(s, b, 2));
            return GW_OK;
        }
        GW_TRY(ensure_aux(env, 2));
        HIP_TRY(hipEventRecord(env->sync_ev[0], s));  // fork after the world update
        HIP_TRY(hipStreamWaitEvent(env->aux, env->sync_ev[0], 0));
        GW_TRY(span_begin(env->aux, b));
        HIP_TRY(dispatch_fear(env, p, env->aux));
        GW_TRY(span_end(env->aux, b, 2));
        GW_TRY(span_begin(s, b));
        HIP_TRY(launch_obs(env, p, p.out.obs, p.out.final_obs, s));
        GW_TRY(span_end(s, b, 1));
        HIP_TRY(hipEventRecord(env->sync_ev[1], env->aux));
        HIP_TRY(hipStreamWaitEvent(s, env->sync_ev[1], 0));
        return GW_OK;
    }
    size_t b;
    GW_TRY(span_begin(s, b));
    HIP_TRY(dispatch_step(env, p, s));
    GW_TRY(span_end(s, b, 0));
    if (want_obs) {
        GW_TRY(span_begin(s, b));
        HIP_TRY(launch_obs(env, p, p.out.obs, p.out.final_obs, s));
        GW_TRY(span_end(s, b, 1));
    }
    return GW_OK;
}

gw_status gw_set_obs_async(void *handle, int enable) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (!enable && env->obs_async && env->mode == 4 && env->obs_queued) {  // merged: drain the queued writer
        hipStream_t ls = env->last_stream;
        GW_TRY(flush_obs(env, nullptr));
        HIP_TRY(hipStreamSynchronize(ls));
    }
    if (!enable && env->obs_async && env->obs_stream) {
        // the synchronous path writes the current descriptor buffer in place: drain the writer
        GW_TRY(flush_obs(env, nullptr));
        HIP_TRY(hipStreamSynchronize(env->obs_stream));
        if (env->obs_stream2) HIP_TRY(hipStreamSynchronize(env->obs_stream2));
        env->obs_pending[0] = env->obs_pending[1] = false;
    }
    if (!(enable & 4) && env->fear_pending) {
        HIP_TRY(hipEventSynchronize(env->fear_ev));
        env->fear_pending = false;
    }
    env->obs_async = enable != 0;
    env->obs_lazy = (enable & 2) != 0;
    env->fear_async = (enable & 4) != 0;
    return GW_OK;
}

gw_status gw_obs_fence(void *handle, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    GW_TRY(wait_obs(env, static_cast<hipStream_t>(stream)));
    return GW_OK;
}

gw_status gw_set_obs_dtype(void *handle, int dtype) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (dtype != GW_OBS_F32 && dtype != GW_OBS_BF16) return fail(GW_ERR_ARG, "gw_set_obs_dtype: unknown dtype");
    if (dtype == GW_OBS_BF16 && env->HW % 8 != 0)
        return fail(GW_ERR_ARG, "gw_set_obs_dtype: bf16 obs needs H*W % 8 == 0");
    const bool bf = dtype == GW_OBS_BF16;
    if (bf != env->obs_bf16 && env->mode == 4 && env->obs_queued) {  // merged: the queued writer
        hipStream_t ls = env->last_stream;
        GW_TRY(flush_obs(env, nullptr));
        HIP_TRY(hipStreamSynchronize(ls));
    }
    if (bf != env->obs_bf16 && env->obs_stream) {
        // an obs_kernel still queued or in flight was sized for the old format: drain it first
        GW_TRY(flush_obs(env, nullptr));
        HIP_TRY(hipStreamSynchronize(env->obs_stream));
        if (env->obs_stream2) HIP_TRY(hipStreamSynchronize(env->obs_stream2));
    }
    // bf16 writer: ~64 KB of obs per block (C3: 16 envs, 4.3 TB/s; 4 envs 3.4, 8 envs 4.2;
    // C4: 4 envs; profiles/r1_bf16); f32: the create-time default
    env->obs_be = bf ? std::max(1, std::min(gw::OBS_BE, 32768 / std::max(1, env->K * env->HW)))
                 : env->obs_be_f32;
    env->obs_bf16 = bf;
    // the bf16 step is bound by the world update + FeAR chain, where 32 envs per fear block is
    // 2 % faster; the stats rows depend on it, so only before the first reset
    if (!env->initialized && !env->fear_wide_fixed) env->fear_wide = !bf;
    return GW_OK;
}

gw_status gw_set_fear_blocks(void *handle, int wide) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (env->initialized) return fail(GW_ERR_STATE, "gw_set_fear_blocks after gw_reset (the stats rows follow it)");
    if (!env->fear_wide_fixed) env->fear_wide = wide != 0;
    return GW_OK;
}

gw_status gw_fear_fence(void *handle, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    GW_TRY(wait_fear(env, static_cast<hipStream_t>(stream)));
    return GW_OK;
}

gw_status gw_profile(void *handle, int enable) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    env->profiling = enable != 0;
    // the timing events are created here, ahead of the profiled steps (enable > 1: at least
    // `enable` of them): hipEventCreate inside a step puts its host cost between the launches
    const size_t want = env->profiling ? env->ev_used + (size_t)std::max(enable, 32) : 0;
    while (env->ev_pool.size() < want) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, env->prof_flags));
        env->ev_pool.push_back(e);
    }
    return GW_OK;
}

#ifdef GW_STEP_CLK
// measurement build only: thread 0's phase stamps of the last step_v2_block of blocks 0-63
int gw_step_debug_clocks(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gw::g_step_clk), sizeof(unsigned long long) * 64 * 16) == hipSuccess
               ? 0 : -1;
}
#endif

gw_status gw_profile_spans(void *handle, double *out, int64_t cap, int64_t *n_spans) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !n_spans || (cap > 0 && !out)) return fail(GW_ERR_ARG, "null argument");
    *n_spans = (int64_t)env->spans.size();
    if (env->spans.empty() || cap <= 0) return GW_OK;
    const hipEvent_t t0 = env->ev_pool[env->spans.front().b];
    for (size_t i = 0; i < env->spans.size() && (int64_t)i < cap; ++i) {
        const Env::Span &sp = env->spans[i];
        HIP_TRY(hipEventSynchronize(env->ev_pool[sp.e]));
        float b = 0.f, e = 0.f;
        HIP_TRY(hipEventElapsedTime(&b, t0, env->ev_pool[sp.b]));
        HIP_TRY(hipEventElapsedTime(&e, t0, env->ev_pool[sp.e]));
        out[3 * i + 0] = (double)sp.kind;
        out[3 * i + 1] = (double)b;
        out[3 * i + 2] = (double)e;
    }
    return GW_OK;
}

gw_status gw_profile_read(void *handle, double out_ms[3], int64_t *n_steps) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !out_ms) return fail(GW_ERR_ARG, "null argument");
    out_ms[0] = out_ms[1] = out_ms[2] = 0.0;
    for (const Env::Span &sp : env->spans) {
        HIP_TRY(hipEventSynchronize(env->ev_pool[sp.e]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, env->ev_pool[sp.b], env->ev_pool[sp.e]));
        if (sp.kind >= 0 && sp.kind < 3) out_ms[sp.kind] += ms;
    }
    if (n_steps) *n_steps = env->steps_timed;
    env->spans.clear();
    env->ev_used = 0;
    env->steps_timed = 0;
    return GW_OK;
}

gw_status gw_state_view(void *handle, gw_state *out) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !out) return fail(GW_ERR_ARG, "null argument");
    out->pos = env->pos;
    out->flags = env->flags;
    out->t = env->t;
    out->episode = env->episode;
    out->prev_dist = env->prev;
    out->score = env->score;
    out->fear_score = env->fscore;
    return GW_OK;
}

gw_status gw_copy_state(void *handle, const gw_state *buf, int to_env, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !buf) return fail(GW_ERR_ARG, "null argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    GW_TRY(wait_fear(env, s));  // async FeAR writes score / fear_score
    const size_t E = (size_t)env->E;
    struct Item { void *mine; void *theirs; size_t bytes; } items[] = {
        {env->pos, buf->pos, sizeof(int32_t) * env->N * E},
        {env->flags, buf->flags, sizeof(uint32_t) * E},
        {env->t, buf->t, sizeof(int32_t) * E},
        {env->episode, buf->episode, sizeof(uint32_t) * E},
        {env->prev, buf->prev_dist, sizeof(int32_t) * env->K * E},
        {env->score, buf->score, sizeof(double) * E},
        {env->fscore, buf->fear_score, sizeof(double) * E},
    };
    for (const Item &it : items) {
        if (!it.theirs) continue;
        if (to_env)
            HIP_TRY(hipMemcpyAsync(it.mine, it.theirs, it.bytes, hipMemcpyDefault, s));
        else
            HIP_TRY(hipMemcpyAsync(it.theirs, it.mine, it.bytes, hipMemcpyDefault, s));
    }
    if (to_env) env->initialized = true;
    return GW_OK;
}


int64_t gw_stats_rows(void *handle) {
    const Env *env = static_cast<const Env *>(handle);
    if (!env) return -1;
    switch (env->N) {
        case 1: return stats_rows_n<1>(env);
        case 2: return stats_rows_n<2>(env);
        case 3: return stats_rows_n<3>(env);
        case 4: return stats_rows_n<4>(env);
        case 5: return stats_rows_n<5>(env);
        case 6: return stats_rows_n<6>(env);
        case 7: return stats_rows_n<7>(env);
        case 8: return stats_rows_n<8>(env);
    }
    return -1;
}

gw_status gw_fear_matrix(void *handle, int64_t n, const int32_t *cells, const int32_t *actions,
                         const int32_t *mdr, const uint8_t *in_list, double *resp, int32_t *vm, int32_t *va,
                         double *feal, int32_t *feal_vm, int32_t *feal_va, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !cells || !actions || !resp) return fail(GW_ERR_ARG, "null argument");
    if (n < 0 || n > 0x7FFFFFFF) return fail(GW_ERR_ARG, "n out of range");
    if (n == 0) return GW_OK;
    gw::FmParams q;
    q.celltab = env->celltab;
    q.tab = env->resp;
    q.HW = env->HW;
    q.W = env->W;
    q.w_magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)env->W - 1) / (uint64_t)env->W);
    q.cells = cells;
    q.acts = actions;
    q.mdr = mdr;
    q.in_list = in_list;
    q.resp = resp;
    q.vm = vm;
    q.va = va;
    q.feal = feal;
    q.feal_vm = feal_vm;
    q.feal_va = feal_va;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipErrorInvalidValue;
    switch (env->N) {
        case 1: return fail(GW_ERR_ARG, "FeAR needs N >= 2");
        case 2: e = launch_fear_matrix<2>(env, n, q, s); break;
        case 3: e = launch_fear_matrix<3>(env, n, q, s); break;
        case 4: e = launch_fear_matrix<4>(env, n, q, s); break;
        case 5: e = launch_fear_matrix<5>(env, n, q, s); break;
        case 6: e = launch_fear_matrix<6>(env, n, q, s); break;
        case 7: e = launch_fear_matrix<7>(env, n, q, s); break;
        case 8: e = launch_fear_matrix<8>(env, n, q, s); break;
    }
    HIP_TRY(e);
    return GW_OK;
}

gw_status gw_obs_patch(void *handle, int32_t P, float *patch, float *final_patch, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (P < 1 || P > 129) return fail(GW_ERR_ARG, "gw_obs_patch: need 1 <= P <= 129");
    if (!patch && !final_patch) return GW_OK;
    return obs_patch_launch(env, P, patch, final_patch, static_cast<hipStream_t>(stream));
}

static gw_status obs_patch_launch(Env *env, int32_t P, float *patch, float *final_patch, hipStream_t s) {
    GW_TRY(wait_fear(env, s));  // async FeAR: the descriptors are written by the world update (joined)
    gw::PatchArgs a;
    a.desc = env->desc;
    a.roadbits = env->roadbits;
    a.base = env->base;
    a.patch = patch;
    a.final_patch = final_patch;
    a.E = env->E;
    a.H = env->H;
    a.W = env->W;
    a.N = env->N;
    a.K = env->K;
    a.P = P;
    a.variant = env->variant;
    for (int k = 0; k < GW_MAX_AGENTS; ++k) a.apples[k] = k < env->K ? env->apples[k] : -1;
    // the map part of each window (P <= 16) comes from a table of every centre's window (built on
    // first use of this P; 0.5 MB at 32 x 32 and P = 11, 4 MB at 64 x 64 and P = 16);
    const size_t tb = gw::window_table_bytes(env->H, env->W, P);
    if (P * P <= 256 && tb <= (size_t)64 << 20) {
        float *t = nullptr;
        for (auto &pt : env->ptbls)
            if (pt.first == P) t = pt.second;
        if (!t) {
            GW_TRY(dalloc(env, &t, tb / sizeof(float)));
            HIP_TRY(gw::build_window_table(a, t, s));
            // once per (env, P): later calls may come on other streams (a rollout's side stream)
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            HIP_TRY(hipStreamIsCapturing(s, &cs));
            if (cs == hipStreamCaptureStatusNone) HIP_TRY(hipStreamSynchronize(s));
            env->ptbls.emplace_back(P, t);
        }
        a.tbl = t;
    }
    gwprof::Span span(env, GW_SPAN_WINDOW);
    HIP_TRY(gw::launch_windows(a, s));
    return GW_OK;
}

gw_status gw_count_sims(void *handle, uint64_t *counter) {
    if (!handle) return fail(GW_ERR_ARG, "gw_count_sims: null env");
    static_cast<Env *>(handle)->sims = reinterpret_cast<unsigned long long *>(counter);
    return GW_OK;
}

gw_status gw_obs_desc_copy(void *handle, uint32_t *dst, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !dst) return fail(GW_ERR_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(dst) & 15u) return fail(GW_ERR_ARG, "gw_obs_desc_copy: dst not 16-byte aligned");
    // the world update that wrote env->desc is ordered before the caller's later work on its
    // stream on every path (the pipelined ones join it); a later step writes the other buffer.
    // A 16-byte-per-lane copy kernel: the runtime's D2D blit took ~18 us for these 3 MB beside
    // the obs writer (C5), this takes a few
    const int64_t n16 = (int64_t)env->E * gw::NDESC / 4;  // NDESC = 12: whole uint4s per env
    const unsigned grid = (unsigned)std::min<int64_t>((n16 + 255) / 256, 2048);
    gw_launch(gw::copy16_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
              reinterpret_cast<const uint4 *>(env->desc), reinterpret_cast<uint4 *>(dst), n16);
    HIP_TRY(hipGetLastError());
    return GW_OK;
}

gw_status gw_obs_view(void *handle, gw_obs_source *out) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !out) return fail(GW_ERR_ARG, "null argument");
    out->desc = env->desc;
    out->base = env->base;
    for (int k = 0; k < GW_MAX_AGENTS; ++k) out->apples[k] = k < env->K ? env->apples[k] : -1;
    out->N = env->N; out->K = env->K; out->H = env->H; out->W = env->W; out->variant = env->variant;
    out->E = env->E; out->env_offset = env->env_offset;
    return GW_OK;
}

void gw_set_last_error(const char *msg) { g_err = msg ? msg : ""; }

gw_status gw_graph_replayed(void *handle, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return fail(GW_ERR_ARG, "null env");
    if (env->mode == 4 && env->obs_async && env->qobs.desc) {
        env->obs_queued = true;  // qobs: the last captured step's writer
        env->qobs_prof = false;
        env->last_stream = static_cast<hipStream_t>(stream);
    }
    return GW_OK;
}

namespace {
// gw_pipeline_save / gw_pipeline_load: the host-side state a merged-path step leaves behind
struct PipeState {
    gw::Params qobs;
    int32_t qobs_buf, dcur, obs_queued, mode;
    uint32_t *desc;
};
}  // namespace

int64_t gw_pipeline_state_bytes(void) { return (int64_t)sizeof(PipeState); }

gw_status gw_pipeline_save(void *handle, void *buf) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !buf) return fail(GW_ERR_ARG, "null argument");
    PipeState st;
    std::memset(&st, 0, sizeof(st));
    st.qobs = env->qobs;
    st.qobs_buf = env->qobs_buf;
    st.dcur = env->dcur;
    st.obs_queued = env->obs_queued ? 1 : 0;
    st.mode = env->mode;
    st.desc = env->desc;
    std::memcpy(buf, &st, sizeof(st));
    return GW_OK;
}

gw_status gw_pipeline_load(void *handle, const void *buf, void *stream) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !buf) return fail(GW_ERR_ARG, "null argument");
    PipeState st;
    std::memcpy(&st, buf, sizeof(st));
    if (st.mode != env->mode) return fail(GW_ERR_ARG, "gw_pipeline_load: state of another kernel path");
    if (env->mode != 4 && (env->obs_async || st.obs_queued))
        return fail(GW_ERR_STATE, "gw_pipeline_load: only the merged path's async pipeline (or synchronous obs)");
    env->qobs = st.qobs;
    env->qobs_buf = st.qobs_buf;
    env->dcur = st.dcur;
    env->desc = st.desc;
    env->obs_queued = st.obs_queued != 0;
    env->qobs_prof = false;
    env->last_stream = static_cast<hipStream_t>(stream);
    return GW_OK;
}

int64_t gw_kernel_path(void *handle) {
    const Env *env = static_cast<const Env *>(handle);
    return env ? env->mode : -1;
}

gw_status gw_dims(void *handle, int64_t out[5]) {
    Env *env = static_cast<Env *>(handle);
    if (!env || !out) return fail(GW_ERR_ARG, "null argument");
    out[0] = env->H; out[1] = env->W; out[2] = env->N; out[3] = env->K; out[4] = env->E;
    return GW_OK;
}

void gw_destroy(void *handle) {
    Env *env = static_cast<Env *>(handle);
    if (!env) return;
    (void)hipSetDevice(env->device);
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : env->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : env->sync_ev) (void)hipEventDestroy(e);
    if (env->aux) (void)hipStreamDestroy(env->aux);
    if (env->obs_stream) (void)hipStreamDestroy(env->obs_stream);
    if (env->obs_stream2) (void)hipStreamDestroy(env->obs_stream2);
    for (hipEvent_t e : env->obs_done)
        if (e) (void)hipEventDestroy(e);
    if (env->world_ev) (void)hipEventDestroy(env->world_ev);
    if (env->fear_ev) (void)hipEventDestroy(env->fear_ev);
    for (void *p : env->allocs) (void)hipFree(p);
    delete env;
}

}  // extern "C"
