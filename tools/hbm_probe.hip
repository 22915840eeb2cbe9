// HBM ceiling probe for the roofline denominator: pure float4 store stream (the obs write
// pattern) and float4 copy, timed with hipEvents.  Usage: hbm_probe [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) store4(float4 *__restrict__ dst, size_t n4, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) store4nt(float4 *__restrict__ dst, size_t n4, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
        __builtin_nontemporal_store(x, reinterpret_cast<f32x4 *>(dst + i));
    }
}
__global__ void __launch_bounds__(256) copy4(float4 *__restrict__ dst, const float4 *__restrict__ src, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char **argv) {
    size_t mb = argc > 1 ? strtoull(argv[1], 0, 10) : 537;
    size_t bytes = mb << 20, n4 = bytes / 16;
    float4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int grids[] = {2048, 8192, 16384, 32768, 65536};
    for (int g : grids) {
        for (int w = 0; w < 3; ++w) store4<<<g, 256>>>(a, n4, 1.f);
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) store4<<<g, 256>>>(a, n4, (float)r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double st = bytes * (double)reps / (ms * 1e-3) / 1e9;
        for (int w = 0; w < 3; ++w) store4nt<<<g, 256>>>(a, n4, 1.f);
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) store4nt<<<g, 256>>>(a, n4, (float)r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double stnt = bytes * (double)reps / (ms * 1e-3) / 1e9;
        for (int w = 0; w < 3; ++w) copy4<<<g, 256>>>(b, a, n4);
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) copy4<<<g, 256>>>(b, a, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double cp = 2.0 * bytes * reps / (ms * 1e-3) / 1e9;
        printf("{\"probe\": \"hbm\", \"MB\": %zu, \"grid\": %d, \"store_GBs\": %.1f, \"store_nt_GBs\": %.1f, \"copy_GBs\": %.1f}\n", mb, g, st, stnt, cp);
    }
    return 0;
}
