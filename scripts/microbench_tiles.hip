// Memory floor of one LDS tile pass over the C5-sized array (M = 2^27 8-B records, 1 GB)
// per tile shape: the bitonic_tiles memory pattern (persistent 1024-lane blocks, 16
// records per lane, W = 2^wlog consecutive records x 2^(14 - wlog) rows 2^dtile apart,
// the next tile prefetched into registers while the current one goes through LDS) with
// no compare-exchanges.  Against it the tile kernels' own cost per shape is judged and
// the planner's per-shape launch costs are set.  One JSON line per shape.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/microbench_tiles scripts/microbench_tiles.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NT = 1024, E = 16, TLOG = 14;

__device__ __forceinline__ uint32_t lpad(uint32_t e) { return e + (e >> 4); }

__global__ __launch_bounds__(NT) void k_tile_pass(uint64_t *__restrict__ data, uint32_t wlog,
                                                  uint32_t dtile, uint32_t ntiles, uint32_t rounds,
                                                  uint32_t swz) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    const uint32_t t = threadIdx.x;
    const uint32_t mid = dtile - wlog;
    const uint32_t tbits = 31 - __builtin_clz(ntiles);  // ntiles a power of two
    auto base_of = [&](uint32_t tl) {
        // swz: the order in which the blocks walk the tiles (a bijection of the tile index)
        if (swz == 1) tl = ((tl << 8) | (tl >> (tbits - 8))) & (ntiles - 1);   // rotate by 8
        if (swz == 2) tl = (tl * 0x9E3779B1u) & (ntiles - 1);                    // odd multiplier
        if (swz == 3) tl = __builtin_bitreverse32(tl) >> (32 - tbits);            // bit reversal
        return ((tl >> mid) << (dtile + TLOG - wlog)) | ((tl & ((1u << mid) - 1u)) << wlog);
    };
    const uint32_t voff = (t & ((1u << wlog) - 1u)) + ((t >> wlog) << dtile);
    const uint32_t rstride = (uint32_t)NT << mid;
    // swz 4 / 5: a physical layout that XORs 128-B block bits 4..13 with position bits
    // >= 14 (a bijection: bits >= 14 are unchanged), breaking power-of-two row strides
    auto phys = [&](uint32_t p) -> uint32_t {
        const uint32_t h = p >> 14;
        if (swz == 5) return p ^ (((h * 0x9E3779B1u) >> 22) << 4);
        // GF(2)-linear maps (phys(a ^ b) = phys(a) ^ phys(b) for disjoint bit fields)
        if (swz == 6) return p ^ (((h ^ (h >> 10)) & 0x3FFu) << 4);
        if (swz == 7) return p ^ (((h ^ (h << 5) ^ (h >> 5)) & 0x3FFu) << 4);
        if (swz == 8) return p ^ (((h ^ (h << 3) ^ (h << 7) ^ (h >> 7)) & 0x3FFu) << 4);
        if (swz == 9) return p ^ (((h ^ (h << 1) ^ (h << 6) ^ (h >> 4) ^ (h >> 9)) & 0x3FFu) << 4);
        return p;
    };
    uint64_t pf[E];
    {
        const uint32_t b = base_of(tile);
#pragma unroll
        for (int r = 0; r < E; ++r) pf[r] = data[phys(b + voff + r * rstride)];
    }
    for (;;) {
        const uint32_t b = base_of(tile);
#pragma unroll
        for (int r = 0; r < E; ++r) sm[lpad(t + r * NT)] = pf[r];
        __syncthreads();
        const uint32_t next = tile + gridDim.x;
        {
            const uint32_t nb = base_of(next < ntiles ? next : tile);
#pragma unroll
            for (int r = 0; r < E; ++r) pf[r] = data[phys(nb + voff + r * rstride)];
        }
        // `rounds` LDS round trips of the whole tile (the steps' LDS traffic, no compares)
        for (uint32_t q = 0; q < rounds; ++q) {
            const uint32_t u = (t * 17u + q) & (NT - 1);
            uint64_t x[E];
#pragma unroll
            for (int r = 0; r < E; ++r) x[r] = sm[lpad(u + r * NT)];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < E; ++r) sm[lpad(u + r * NT)] = x[r] ^ 1u;
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < E; ++r) data[phys(b + voff + r * rstride)] = sm[lpad(t + r * NT)];
        if (next >= ntiles) break;
        __syncthreads();
        tile = next;
    }
}

int main() {
    const uint32_t mlog = 27, M = 1u << mlog;
    uint64_t *d;
    if (hipMalloc(&d, (size_t)M * 8) != hipSuccess) return 1;
    hipMemset(d, 0, (size_t)M * 8);
    const size_t lds = ((1u << TLOG) + (1u << TLOG) / 16 + 1) * 8;
    hipFuncSetAttribute((const void *)k_tile_pass, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const uint32_t ntiles = M >> TLOG;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t shapes[][2] = {{14, 14}, {4, 4}, {4, 5}, {4, 7}, {4, 10}, {4, 14}, {4, 17}, {4, 20},
                                  {5, 5}, {5, 7}, {5, 14}, {5, 17}, {6, 14}, {7, 7}, {7, 10}, {7, 15},
                                  {7, 20}, {8, 14}, {9, 14}, {10, 14}, {10, 17}};
    for (uint32_t swz : {0u, 5u, 6u, 7u, 8u, 9u})
    for (auto &sh : shapes) {
        const uint32_t wlog = sh[0], dtile = sh[1], rounds = 0;
        if (dtile + TLOG - wlog > mlog) continue;
        for (int w = 0; w < 3; ++w)
            hipLaunchKernelGGL(k_tile_pass, dim3(256), dim3(NT), lds, 0, d, wlog, dtile, ntiles, rounds, swz);
        const int reps = 20;
        hipEventRecord(a, 0);
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(k_tile_pass, dim3(256), dim3(NT), lds, 0, d, wlog, dtile, ntiles, rounds, swz);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        printf("{\"kernel\": \"tile_pass\", \"M\": %u, \"wlog\": %u, \"dtile\": %u, \"us\": %.1f, "
               "\"tbs\": %.2f, \"lds_rounds\": %u, \"swz\": %u}\n",
               M, wlog, dtile, us, 2.0 * M * 8 / (us * 1e-6) / 1e12, rounds, swz);
        fflush(stdout);
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
