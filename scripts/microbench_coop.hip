// C3's launch boundaries against grid barriers: P phases over a
// C3-sized array (M = 2^20 8-B records, 8 MB, resident in the Infinity Cache), each phase
// an LDS tile pass shaped like the network's (a block loads a 4,096-record tile — 512
// lanes x 8 — does three read/modify/write LDS rounds, stores it back; contiguous and
// strided tiles alternate, so every phase's data crosses blocks through L2 as the
// network's do), run (a) as P back-to-back launches and (b) as ONE cooperative launch of
// 256 blocks (one per CU) looping over the P phases with a device-wide barrier between
// them.  One JSON line per case:  us per phase both ways, and the barrier's own cost.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/microbench_coop scripts/microbench_coop.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NT = 512, PER = 8, TILE = NT * PER;  // 4,096 records
constexpr uint32_t M = 1u << 20, NTILES = M / TILE;  // 256 tiles

// tile t, element e -> position: contiguous (phase even) or strided (rows of 16
// consecutive records, 2^12 apart: the network's strided tiles)
__device__ __forceinline__ uint32_t tpos(uint32_t t, uint32_t e, uint32_t phase) {
    if ((phase & 1) == 0) return t * TILE + e;
    return (t & 255u) * 16u + (e & 15u) + (e >> 4) * 4096u;
}

__device__ __forceinline__ void tile_pass(uint64_t *__restrict__ a, uint64_t *sm, uint32_t t,
                                          uint32_t phase) {
    uint64_t v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = a[tpos(t, threadIdx.x + i * NT, phase)];
#pragma unroll
    for (int i = 0; i < PER; ++i) sm[threadIdx.x + i * NT] = v[i];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 3; ++r) {  // three LDS rounds: read a partner, min/max, write
        uint64_t w[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t e = threadIdx.x + i * NT;
            const uint64_t x = sm[e], y = sm[e ^ (1u << (r + 3))];
            w[i] = (e & (1u << (r + 3))) ? (x > y ? x : y) : (x < y ? x : y);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; ++i) sm[threadIdx.x + i * NT] = w[i];
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) a[tpos(t, threadIdx.x + i * NT, phase)] = sm[threadIdx.x + i * NT] + 1u;
}

__global__ __launch_bounds__(NT) void k_phase(uint64_t *a, uint32_t phase) {
    __shared__ uint64_t sm[TILE];
    tile_pass(a, sm, blockIdx.x, phase);
}

// device-wide barrier: one arrival counter and a generation word, vector atomics only; a
// bounded spin (err set, and the block goes on) so a broken co-residency cannot hang
__device__ __forceinline__ void grid_barrier(uint32_t *cnt, uint32_t *gen, uint32_t nb, uint32_t &g,
                                             uint32_t *err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t arrived = atomicAdd(cnt, 1u);
        if (arrived == nb - 1) {
            atomicExch(cnt, 0u);
            __threadfence();
            atomicExch(gen, g + 1u);
        } else {
            uint32_t spins = 0;
            while (atomicAdd(gen, 0u) == g) {
                if (++spins > (1u << 24)) {
                    atomicOr(err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __threadfence();
    }
    ++g;
    __syncthreads();
}

__global__ __launch_bounds__(NT) void k_coop(uint64_t *a, uint32_t phases, uint32_t *cnt,
                                             uint32_t *gen, uint32_t *err) {
    __shared__ uint64_t sm[TILE];
    uint32_t g = 0;
    if (threadIdx.x == 0) g = atomicAdd(gen, 0u);
    // every block read the same generation before anyone can advance it: the first
    // barrier needs all blocks' arrivals
    g = __shfl(g, 0);
    __shared__ uint32_t gs;
    if (threadIdx.x == 0) gs = g;
    __syncthreads();
    g = gs;
    for (uint32_t p = 0; p < phases; ++p) {
        tile_pass(a, sm, blockIdx.x, p);
        if (p + 1 < phases) grid_barrier(cnt, gen, gridDim.x, g, err);
    }
}

// the barrier alone (no phase work): its cost per use
__global__ __launch_bounds__(NT) void k_coop_empty(uint32_t phases, uint32_t *cnt, uint32_t *gen,
                                                   uint32_t *err) {
    __shared__ uint32_t gs;
    if (threadIdx.x == 0) gs = atomicAdd(gen, 0u);
    __syncthreads();
    uint32_t g = gs;
    for (uint32_t p = 0; p + 1 < phases; ++p) grid_barrier(cnt, gen, gridDim.x, g, err);
}

int main() {
    uint64_t *a;
    uint32_t *w;
    hipMalloc(&a, (size_t)M * 8);
    hipMalloc(&w, 64);
    hipMemset(a, 0, (size_t)M * 8);
    hipMemset(w, 0, 64);
    uint32_t *cnt = w, *gen = w + 1, *err = w + 2;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, coop = 0, ncu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    for (uint32_t P : {8u, 16u, 32u}) {
        float best_l = 1e30f, best_c = 1e30f, best_b = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
            // (a) P launches
            hipEventRecord(e0, 0);
            for (uint32_t p = 0; p < P; ++p) hipLaunchKernelGGL(k_phase, dim3(NTILES), dim3(NT), 0, 0, a, p);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) best_l = ms < best_l ? ms : best_l;
            // (b) one cooperative launch
            void *args[] = {&a, &P, &cnt, &gen, &err};
            hipEventRecord(e0, 0);
            hipError_t ce = hipLaunchCooperativeKernel((const void *)k_coop, dim3(NTILES), dim3(NT), args, 0, 0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            if (ce != hipSuccess) {
                std::printf("{\"error\": \"cooperative launch: %s\"}\n", hipGetErrorString(ce));
                return 1;
            }
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) best_c = ms < best_c ? ms : best_c;
            void *args2[] = {&P, &cnt, &gen, &err};
            hipEventRecord(e0, 0);
            hipLaunchCooperativeKernel((const void *)k_coop_empty, dim3(NTILES), dim3(NT), args2, 0, 0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) best_b = ms < best_b ? ms : best_b;
        }
        uint32_t herr = 0;
        hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
        std::printf("{\"phases\": %u, \"blocks\": %u, \"cus\": %d, \"coop_supported\": %d, "
                    "\"launches_us\": %.2f, \"cooperative_us\": %.2f, \"per_phase_launches_us\": %.3f, "
                    "\"per_phase_cooperative_us\": %.3f, \"barrier_only_us_per_barrier\": %.3f, "
                    "\"barrier_timeouts\": %u}\n",
                    P, NTILES, ncu, coop, best_l * 1e3, best_c * 1e3, best_l * 1e3 / P, best_c * 1e3 / P,
                    P > 1 ? best_b * 1e3 / (P - 1) : 0.0, herr);
    }
    return 0;
}
