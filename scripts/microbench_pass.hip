// Floor of one streaming pass over a C3-sized array (M = 2^20 8-B records, 8 MB): what
// a kernel that reads and writes the array once costs on MI355X, against which the
// network's passes (bitonic_global, bitonic_tiles) are judged.  One JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/microbench_pass scripts/microbench_pass.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void k_empty(uint64_t *) {}

// one 8-B record per lane in, out (a register pass's memory pattern, R = 1: 2 per lane)
template <int PER, bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint64_t *__restrict__ src,
                                              uint64_t *__restrict__ dst, uint32_t m) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint64_t v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t p = t + (uint32_t)i * gridDim.x * 256;
        v[i] = p < m ? (NT ? __builtin_nontemporal_load(src + p) : src[p]) : 0;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t p = t + (uint32_t)i * gridDim.x * 256;
        if (p < m) dst[p] = v[i] ^ 1u;
    }
}

// in place (the network passes read and write the same array)
template <int PER>
__global__ __launch_bounds__(256) void k_inplace(uint64_t *__restrict__ a, uint32_t m) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint64_t v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t p = t + (uint32_t)i * gridDim.x * 256;
        v[i] = p < m ? a[p] : 0;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t p = t + (uint32_t)i * gridDim.x * 256;
        if (p < m) a[p] = v[i] ^ 1u;
    }
}

template <typename F>
static float time_us(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) launch(i);
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch(i);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms * 1000.0f / reps;
}

int main() {
    const int reps = 200;
    for (uint32_t mlog : {18u, 20u, 22u, 24u}) {
        const uint32_t m = 1u << mlog;
        uint64_t *x, *y;
        if (hipMalloc(&x, (size_t)m * 8) != hipSuccess || hipMalloc(&y, (size_t)m * 8) != hipSuccess) return 1;
        hipMemset(x, 0, (size_t)m * 8);
        hipMemset(y, 0, (size_t)m * 8);
        const double bytes = 16.0 * m;
        auto line = [&](const char *name, float us) {
            printf("{\"m_log\": %u, \"case\": \"%s\", \"us\": %.3f, \"gbs\": %.1f}\n", mlog, name, us,
                   bytes / (us * 1e-6) / 1e9);
        };
        line("empty, m/512 blocks", time_us([&](int) { hipLaunchKernelGGL(k_empty, dim3(m / 512), dim3(256), 0, 0, x); }, reps));
        line("copy 1/lane", time_us([&](int i) { hipLaunchKernelGGL((k_copy<1, false>), dim3(m / 256), dim3(256), 0, 0, i & 1 ? y : x, i & 1 ? x : y, m); }, reps));
        line("copy 2/lane", time_us([&](int i) { hipLaunchKernelGGL((k_copy<2, false>), dim3(m / 512), dim3(256), 0, 0, i & 1 ? y : x, i & 1 ? x : y, m); }, reps));
        line("copy 8/lane", time_us([&](int i) { hipLaunchKernelGGL((k_copy<8, false>), dim3(m / 2048), dim3(256), 0, 0, i & 1 ? y : x, i & 1 ? x : y, m); }, reps));
        line("copy 2/lane nt", time_us([&](int i) { hipLaunchKernelGGL((k_copy<2, true>), dim3(m / 512), dim3(256), 0, 0, i & 1 ? y : x, i & 1 ? x : y, m); }, reps));
        line("in place 2/lane", time_us([&](int) { hipLaunchKernelGGL((k_inplace<2>), dim3(m / 512), dim3(256), 0, 0, x, m); }, reps));
        line("in place 8/lane", time_us([&](int) { hipLaunchKernelGGL((k_inplace<8>), dim3(m / 2048), dim3(256), 0, 0, x, m); }, reps));
        hipFree(x);
        hipFree(y);
    }
    return 0;
}
