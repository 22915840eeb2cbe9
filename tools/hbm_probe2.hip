// Write-ceiling probe: which float4 store stream shape reaches the highest HBM write rate on
// MI355X (the obs writer is a pure store stream).  Usage: hbm_probe2 [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// grid-stride, U stores in flight per iteration
template <int U, bool NT>
__global__ void __launch_bounds__(256) stride_store(f32x4 *__restrict__ dst, size_t n4, float v) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
    for (; i + (U - 1) * step < n4; i += U * step) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(x, dst + i + u * step);
            else dst[i + u * step] = x;
        }
    }
    for (; i < n4; i += step) {
        if (NT) __builtin_nontemporal_store(x, dst + i);
        else dst[i] = x;
    }
}

// each block owns a contiguous chunk of CH float4 (the obs writer's per-env layout)
template <int CH, bool NT>
__global__ void __launch_bounds__(256) chunk_store(f32x4 *__restrict__ dst, size_t n4, float v) {
    const size_t base = (size_t)blockIdx.x * CH;
    const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
#pragma unroll 4
    for (int j = threadIdx.x; j < CH; j += 256) {
        const size_t i = base + j;
        if (i < n4) {
            if (NT) __builtin_nontemporal_store(x, dst + i);
            else dst[i] = x;
        }
    }
}

// read stream: each lane sums U float4 per iteration (one result per lane, so no load is dead)
template <int U>
__global__ void __launch_bounds__(256) stride_read(const f32x4 *__restrict__ src, size_t n4, float *out) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (; i + (U - 1) * step < n4; i += U * step) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc += __builtin_nontemporal_load(src + i + u * step);
    }
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <class F>
double timeit(F launch, size_t bytes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) launch(0.f);
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) launch((float)r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return bytes * (double)reps / (ms * 1e-3) / 1e9;
}

int main(int argc, char **argv) {
    size_t mb = argc > 1 ? strtoull(argv[1], 0, 10) : 513;
    size_t bytes = mb << 20, n4 = bytes / 16;
    f32x4 *a;
    if (hipMalloc(&a, bytes) != hipSuccess) return 1;
    int grids[] = {4096, 16384, 65536};
    for (int g : grids) {
        printf("{\"probe\": \"stride\", \"grid\": %d, \"U1\": %.0f, \"U1nt\": %.0f, \"U4nt\": %.0f, \"U8nt\": %.0f}\n", g,
               timeit([&](float v) { stride_store<1, false><<<g, 256>>>(a, n4, v); }, bytes),
               timeit([&](float v) { stride_store<1, true><<<g, 256>>>(a, n4, v); }, bytes),
               timeit([&](float v) { stride_store<4, true><<<g, 256>>>(a, n4, v); }, bytes),
               timeit([&](float v) { stride_store<8, true><<<g, 256>>>(a, n4, v); }, bytes));
    }
    printf("{\"probe\": \"chunk\", \"ch1k\": %.0f, \"ch1knt\": %.0f, \"ch4knt\": %.0f, \"ch16knt\": %.0f}\n",
           timeit([&](float v) { chunk_store<1024, false><<<(unsigned)((n4 + 1023) / 1024), 256>>>(a, n4, v); }, bytes),
           timeit([&](float v) { chunk_store<1024, true><<<(unsigned)((n4 + 1023) / 1024), 256>>>(a, n4, v); }, bytes),
           timeit([&](float v) { chunk_store<4096, true><<<(unsigned)((n4 + 4095) / 4096), 256>>>(a, n4, v); }, bytes),
           timeit([&](float v) { chunk_store<16384, true><<<(unsigned)((n4 + 16383) / 16384), 256>>>(a, n4, v); }, bytes));
    float *o;
    (void)hipMalloc(&o, 4096);
    for (int g : grids)
        printf("{\"probe\": \"read\", \"grid\": %d, \"U4\": %.0f, \"U8\": %.0f}\n", g,
               timeit([&](float) { stride_read<4><<<g, 256>>>(a, n4, o); }, bytes),
               timeit([&](float) { stride_read<8><<<g, 256>>>(a, n4, o); }, bytes));
    printf("{\"probe\": \"memset\", \"hipMemsetD32Async\": %.0f}\n",
           timeit([&](float v) { (void)hipMemsetD32Async((hipDeviceptr_t)a, (int)v, bytes / 4, 0); }, bytes));
    return 0;
}
