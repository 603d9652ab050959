// Streaming-read floor on MI355X for the dense configs' input sizes: a kernel that only
// reads B bytes (16-B nontemporal loads, 8 in flight per lane, XOR-folded, one word
// written per block), launched back to back over rotating buffers whose total exceeds
// the 256 MB Infinity Cache (cold HBM, as bench.py's literal-config line).  Prints the
// per-launch time (HIP events around 50 launches) and GB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ p, size_t n16,
                                                   uint32_t *out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads alive
}

int main() {
    const size_t sizes[3] = {12213600, 40712000, 800000000};
    uint32_t *out;
    (void)hipMalloc(&out, 1 << 20);
    for (size_t B : sizes) {
        const int nbuf = (int)((600u << 20) / B) + 2;
        std::vector<u32x4 *> bufs(nbuf);
        for (auto &b : bufs) { (void)hipMalloc(&b, B); (void)hipMemset(b, 1, B); }
        const size_t n16 = B / 16;
        for (unsigned grid : {1024u, 2048u, 4096u, 8192u}) {
            if ((size_t)grid * 256 * 8 > n16 * 4 && grid > 1024) continue;
            for (int w = 0; w < 5; ++w)
                hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, bufs[w % nbuf], n16, out);
            hipEvent_t a, b;
            (void)hipEventCreate(&a); (void)hipEventCreate(&b);
            (void)hipEventRecord(a);
            for (int l = 0; l < 50; ++l)
                hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, bufs[l % nbuf], n16, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / 50;
            printf("{\"bytes\": %zu, \"buffers\": %d, \"grid\": %u, \"us_per_launch\": %.2f, \"gbs\": %.0f}\n",
                   B, nbuf, grid, us, B / us / 1e3);
        }
        for (auto &b : bufs) (void)hipFree(b);
    }
    return 0;
}
