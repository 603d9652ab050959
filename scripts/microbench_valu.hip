// VALU issue-rate microbenchmark (gfx950): 8 independent chains per lane of one op,
// 4096 iterations, 2^20 lanes; prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define K 0x9E3779B1u
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    const uint32_t kv = K ^ seed;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0x10001u + i + seed;
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // inline asm: the compiler may not fold the chains
            if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(kv));
            if (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(kv));
            if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(kv));
            if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(kv));
        }
        asm volatile("" ::: "memory");
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int OP>
float run(uint32_t *d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(4096), dim3(256), 0, 0, d, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<OP>, dim3(4096), dim3(256), 0, 0, d, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    uint32_t *d;
    hipMalloc(&d, 4096 * 256 * 4);
    const char *names[4] = {"v_mul_lo_u32", "v_mul_u32_u24", "v_mul_hi_u32", "v_add_u32"};
    float t[4] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d)};
    // wave-instructions: 4096 blocks * 4 waves * 4096 iters * 8 chains
    const double winst = 4096.0 * 4 * 4096 * 8;
    for (int i = 0; i < 4; ++i)
        printf("{\"op\": \"%s\", \"ms\": %.3f, \"winst_per_cu_per_ns\": %.4f}\n", names[i], t[i],
               winst / 256 / (t[i] * 1e6));
    return 0;
}
