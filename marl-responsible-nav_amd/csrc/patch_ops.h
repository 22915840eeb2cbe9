// Internal interface between gridenv.hip (gw_obs_patch) and patch_ops.hip (the window writer).
#ifndef GW_PATCH_OPS_H
#define GW_PATCH_OPS_H

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gridenv.h"

namespace gw {

struct PatchArgs {
    const uint32_t *desc;      // [E][12] obs descriptors of the env's last step
    const uint32_t *roadbits;  // [ceil(H*W / 32)] bit c: cell c is road
    const float *base;         // [H*W] static map values (0 road, -1 inactive)
    float *patch;              // [K][E][P*P] or null
    float *final_patch;        // [K][E][P*P] or null (terminal windows of the envs that ended)
    int64_t E;
    int H, W, N, K, P, variant;
    int apples[GW_MAX_AGENTS];
    const float *tbl = nullptr;  // MODE 4: [H*W][P*P] the map part of the window centred on each cell
    int probe = 0;  // measurement only (GW_PATCH_PROBE): 1 = MODE 3 stores zeros after its table build,
                    // 2 = zeros right after the staging (no table)
};

hipError_t launch_windows(const PatchArgs &a, hipStream_t s);
// MODE 4's table (bytes: H * W * P * P * 4), built from a.roadbits into tbl on stream s
size_t window_table_bytes(int H, int W, int P);
hipError_t build_window_table(const PatchArgs &a, float *tbl, hipStream_t s);

}  // namespace gw

#endif
