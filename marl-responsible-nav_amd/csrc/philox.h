// philox.h — internal: Philox4x32-10 (the generator of gridenv.hip / actor_ops.hip: counter-based,
// graph-safe, keyed draws) for the learner's sampling and Gumbel noise (rollout_ops.hip,
// maddpg_ops.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace gwrng {

__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return make_uint4(c0, c1, c2, c3);
}

// a uniform float in [0, 1) with 24 random bits (torch.rand's resolution)
__device__ __forceinline__ float unit(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// draw tags (counter word 2)
constexpr uint32_t TAG_SAMPLE = 0x53414D50u;  // the replay sample's (transition, env) draws
constexpr uint32_t TAG_GUMBEL = 0x47554D00u;  // + phase: the learner's Gumbel uniforms

}  // namespace gwrng
