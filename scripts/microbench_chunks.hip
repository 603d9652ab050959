// The streaming fold's access pattern without its arithmetic: 64 lanes of a
// wave own 64 chunks of C records each; per stage the wave reads a window of W records
// (W * 8 bytes, contiguous) from every chunk, W/2 lanes per window with 16-B nontemporal
// loads, one stage ahead, and writes it back out to the same place in dst.  A chunk is
// visited every stage, so W sets how many bytes one DRAM page visit brings.  Against it:
// the same bytes copied as one contiguous block per wave.  Prints us and GB/s (read +
// written) per config, C5's fold size (110M records).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int W>
__global__ __launch_bounds__(64) void chunk_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                 long long m, uint32_t C) {
    constexpr int LW = W / 2;         // lanes per window (16 B each)
    constexpr int WPI = 64 / LW;      // windows per load instruction
    constexpr int NI = 64 / WPI;      // load instructions per stage (64 windows)
    const uint32_t l = threadIdx.x;
    const long long wave0 = (long long)blockIdx.x * 64 * C;
    const uint32_t part = (l % LW) * 2;
    u32x4 cur[NI], nxt[NI];
    auto load = [&](u32x4 (&v)[NI], uint32_t s) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const uint32_t w = l / LW + WPI * i;
            const long long g = wave0 + (long long)w * C + (long long)s * W + part;
            v[i] = g < m ? __builtin_nontemporal_load(src + g / 2) : u32x4{0, 0, 0, 0};
        }
    };
    const uint32_t ns = C / W;
    load(cur, 0);
    for (uint32_t s = 0; s < ns; ++s) {
        if (s + 1 < ns) load(nxt, s + 1);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const uint32_t w = l / LW + WPI * i;
            const long long g = wave0 + (long long)w * C + (long long)s * W + part;
            if (g < m) __builtin_nontemporal_store(cur[i] ^ u32x4{1, 1, 1, 1}, dst + g / 2);
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) cur[i] = nxt[i];
    }
}

__global__ __launch_bounds__(256) void block_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                  long long n16) {
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i) ^ u32x4{1, 1, 1, 1}, dst + i);
}

template <int W>
static void run(const u32x4 *src, u32x4 *dst, long long m, uint32_t C) {
    const long long lanes = (m + C - 1) / C;
    const unsigned blocks = (unsigned)((lanes + 63) / 64);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(chunk_copy<W>, dim3(blocks), dim3(64), 0, 0, src, dst, m, C);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(chunk_copy<W>, dim3(blocks), dim3(64), 0, 0, src, dst, m, C);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / reps;
    printf("{\"kind\":\"chunks\",\"W\":%d,\"C\":%u,\"waves\":%u,\"us\":%.1f,\"gbs\":%.0f}\n", W, C, blocks, us,
           16.0 * m / us / 1e3);
}

// W = 16 windows, but B consecutive stages' loads issued together (B x 8 instructions back to
// back, one batch ahead): does issuing adjacent lines together act like a wider window?
template <int B>
__global__ __launch_bounds__(64) void chunk_copy_batched(const u32x4 *__restrict__ src,
                                                         u32x4 *__restrict__ dst, long long m,
                                                         uint32_t C) {
    constexpr int W = 16, LW = 8, WPI = 8, NI = 8;
    const uint32_t l = threadIdx.x;
    const long long wave0 = (long long)blockIdx.x * 64 * C;
    const uint32_t part = (l % LW) * 2;
    u32x4 cur[B][NI], nxt[B][NI];
    auto load = [&](u32x4 (&v)[B][NI], uint32_t sb) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const uint32_t w = l / LW + WPI * i;
                const long long g = wave0 + (long long)w * C + (long long)(sb * B + b) * W + part;
                v[b][i] = g < m ? __builtin_nontemporal_load(src + g / 2) : u32x4{0, 0, 0, 0};
            }
    };
    const uint32_t nb = C / W / B;
    load(cur, 0);
    for (uint32_t sb = 0; sb < nb; ++sb) {
        if (sb + 1 < nb) load(nxt, sb + 1);
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const uint32_t w = l / LW + WPI * i;
                const long long g = wave0 + (long long)w * C + (long long)(sb * B + b) * W + part;
                if (g < m) __builtin_nontemporal_store(cur[b][i] ^ u32x4{1, 1, 1, 1}, dst + g / 2);
            }
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int i = 0; i < NI; ++i) cur[b][i] = nxt[b][i];
    }
}

template <int B>
static void run_batched(const u32x4 *src, u32x4 *dst, long long m, uint32_t C) {
    const long long lanes = (m + C - 1) / C;
    const unsigned blocks = (unsigned)((lanes + 63) / 64);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(chunk_copy_batched<B>, dim3(blocks), dim3(64), 0, 0, src, dst, m, C);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r)
        hipLaunchKernelGGL(chunk_copy_batched<B>, dim3(blocks), dim3(64), 0, 0, src, dst, m, C);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("{\"kind\":\"batched\",\"W\":16,\"B\":%d,\"C\":%u,\"us\":%.1f,\"gbs\":%.0f}\n", B, C,
           ms * 100, 16.0 * m / (ms * 100) / 1e3);
}

int main() {
    const long long m = 110000000;  // C5's fold span (records)
    u32x4 *src, *dst;
    if (hipMalloc(&src, m * 8 + 4096) != hipSuccess || hipMalloc(&dst, m * 8 + 4096) != hipSuccess) return 1;
    (void)hipMemset(src, 1, m * 8);
    for (uint32_t C : {1024u, 2048u, 4096u}) {
        run<16>(src, dst, m, C);
        run<32>(src, dst, m, C);
        run<64>(src, dst, m, C);
    }
    for (uint32_t C : {2048u, 4096u}) {
        run_batched<2>(src, dst, m, C);
        run_batched<4>(src, dst, m, C);
    }
    for (unsigned grid : {2048u, 8192u}) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(block_copy, dim3(grid), dim3(256), 0, 0, src, dst, m / 2);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(block_copy, dim3(grid), dim3(256), 0, 0, src, dst, m / 2);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("{\"kind\":\"contiguous\",\"grid\":%u,\"us\":%.1f,\"gbs\":%.0f}\n", grid, ms * 100,
               16.0 * m / (ms * 100) / 1e3);
    }
    return hipDeviceSynchronize() != hipSuccess;
}
