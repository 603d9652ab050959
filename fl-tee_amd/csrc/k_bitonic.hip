// k_bitonic.hip — oblivious bitonic networks on 8-byte records (gfx950).
//
// The network is EXACTLY the reference's (advanced.rs:147-176): for stage i
// (2..M) and step j (i/2..1), every k < M/2 forms the pair
//     l = ((k & ~(j-1)) << 1) | (k & (j-1)),  m = l + j
// and swaps iff ((l & i) == 0) ^ cond2.  With cond2 = key[l] < key[m] equal
// keys are swapped inside ascending blocks — the permutation of equal-idx
// records (and hence the fold order) is bit-identical to the enclave's.
//   mode 0: cond2 = (u32)idx[l] < (u32)idx[m]            (advanced.rs:166)
//   mode 1: cond2 = u64[l] < u64[m]                      (stable composite keys)
//   mode 2: cond2 = mix32(l ^ stepkey(seed,i,j)) & 1     (nips19.rs:66-105 shape;
//           keyed mixer replaces the running FxHash of heap addresses)
// Every compare-exchange is branch-free (v_cndmask) and every address depends
// only on (i, j, k): the memory trace is data-independent, like the cmov
// network it replaces.
//
// Schedule for M = 2^m records, LDS tile T = 2^t:
//   tile_sort            all stages i <= T inside LDS (one launch)
//   per stage i > T:     steps j >= T in global passes, R <= 4 levels per pass
//                        held in registers (2^R records / lane);
//                        steps j < T in one LDS merge launch.
// HBM traffic per launch = 2 * M * 8 bytes.
#include "common.h"

namespace fltee {

template <int MODE>
__device__ __forceinline__ bool swap_rule(uint64_t a, uint64_t b, uint32_t l, uint32_t imask,
                                          uint32_t key) {
    const bool asc = (l & imask) == 0;
    bool lt;
    if (MODE == 0) lt = (uint32_t)a < (uint32_t)b;
    else if (MODE == 1) lt = a < b;
    else lt = (mix32(l ^ key) & 1u) != 0;
    return asc ^ lt;
}

constexpr int BT_THREADS = 512;

template <int MODE>
__device__ __forceinline__ void lds_step(uint64_t *sm, uint32_t T, uint32_t base, uint32_t ilog,
                                         uint32_t jlog, uint32_t key) {
    const uint32_t j = 1u << jlog, imask = 1u << ilog;
    for (uint32_t k = threadIdx.x; k < (T >> 1); k += BT_THREADS) {
        const uint32_t l = ((k >> jlog) << (jlog + 1)) | (k & (j - 1));
        const uint32_t m = l + j;
        const uint64_t a = sm[l], b = sm[m];
        const bool sw = swap_rule<MODE>(a, b, base + l, imask, key);
        sm[l] = sw ? b : a;
        sm[m] = sw ? a : b;
    }
}

template <int MODE>
__global__ __launch_bounds__(BT_THREADS) void bitonic_tile_sort(uint64_t *__restrict__ data,
                                                                uint32_t tlog, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    const uint32_t T = 1u << tlog;
    const uint32_t base = blockIdx.x << tlog;
    uint4 *g4 = reinterpret_cast<uint4 *>(data + base);
    uint4 *s4 = reinterpret_cast<uint4 *>(sm);
    for (uint32_t e = threadIdx.x; e < T / 2; e += BT_THREADS) s4[e] = g4[e];
    __syncthreads();
    for (uint32_t ilog = 1; ilog <= tlog; ++ilog) {
        for (int jlog = (int)ilog - 1; jlog >= 0; --jlog) {
            const uint32_t key = MODE == 2 ? shuffle_step_key(seed, ilog, (uint32_t)jlog) : 0u;
            lds_step<MODE>(sm, T, base, ilog, (uint32_t)jlog, key);
            __syncthreads();
        }
    }
    for (uint32_t e = threadIdx.x; e < T / 2; e += BT_THREADS) g4[e] = s4[e];
}

template <int MODE>
__global__ __launch_bounds__(BT_THREADS) void bitonic_tile_merge(uint64_t *__restrict__ data,
                                                                 uint32_t tlog, uint32_t ilog,
                                                                 uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    const uint32_t T = 1u << tlog;
    const uint32_t base = blockIdx.x << tlog;
    uint4 *g4 = reinterpret_cast<uint4 *>(data + base);
    uint4 *s4 = reinterpret_cast<uint4 *>(sm);
    for (uint32_t e = threadIdx.x; e < T / 2; e += BT_THREADS) s4[e] = g4[e];
    __syncthreads();
    for (int jlog = (int)tlog - 1; jlog >= 0; --jlog) {
        const uint32_t key = MODE == 2 ? shuffle_step_key(seed, ilog, (uint32_t)jlog) : 0u;
        lds_step<MODE>(sm, T, base, ilog, (uint32_t)jlog, key);
        __syncthreads();
    }
    for (uint32_t e = threadIdx.x; e < T / 2; e += BT_THREADS) g4[e] = s4[e];
}

// R consecutive steps jlog, jlog-1, ..., jlog-R+1 of stage ilog in registers.
// Lane t owns the group {b + q*delta : q < 2^R}, delta = 2^(jlog-R+1).
template <int MODE, int R>
__global__ __launch_bounds__(256) void bitonic_global(uint64_t *__restrict__ data, uint32_t ilog,
                                                      uint32_t jlog, uint32_t seed,
                                                      uint32_t ngroups) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= ngroups) return;
    const uint32_t dlog = jlog - R + 1;
    const uint32_t delta = 1u << dlog;
    const uint32_t b = ((t >> dlog) << (dlog + R)) | (t & (delta - 1));
    const uint32_t imask = 1u << ilog;
    uint64_t v[1 << R];
#pragma unroll
    for (int q = 0; q < (1 << R); ++q) v[q] = data[b + (uint32_t)q * delta];
#pragma unroll
    for (int lv = R - 1; lv >= 0; --lv) {
        const uint32_t key = MODE == 2 ? shuffle_step_key(seed, ilog, dlog + lv) : 0u;
#pragma unroll
        for (int q = 0; q < (1 << R); ++q) {
            if (q & (1 << lv)) continue;
            const int qm = q | (1 << lv);
            const uint64_t a = v[q], c = v[qm];
            const bool sw = swap_rule<MODE>(a, c, b + (uint32_t)q * delta, imask, key);
            v[q] = sw ? c : a;
            v[qm] = sw ? a : c;
        }
    }
#pragma unroll
    for (int q = 0; q < (1 << R); ++q) data[b + (uint32_t)q * delta] = v[q];
}

template <int MODE>
static hipError_t launch_global(uint64_t *data, uint32_t mlog, uint32_t ilog, uint32_t jlog,
                                int R, uint32_t seed, hipStream_t s) {
    const uint32_t ngroups = 1u << (mlog - R);
    const unsigned blocks = (ngroups + 255) / 256;
    switch (R) {
    case 1: hipLaunchKernelGGL((bitonic_global<MODE, 1>), dim3(blocks), dim3(256), 0, s, data, ilog, jlog, seed, ngroups); break;
    case 2: hipLaunchKernelGGL((bitonic_global<MODE, 2>), dim3(blocks), dim3(256), 0, s, data, ilog, jlog, seed, ngroups); break;
    case 3: hipLaunchKernelGGL((bitonic_global<MODE, 3>), dim3(blocks), dim3(256), 0, s, data, ilog, jlog, seed, ngroups); break;
    default: hipLaunchKernelGGL((bitonic_global<MODE, 4>), dim3(blocks), dim3(256), 0, s, data, ilog, jlog, seed, ngroups); break;
    }
    return hipGetLastError();
}

template <int MODE>
static hipError_t sort_impl(uint64_t *data, size_t m, uint32_t seed, hipStream_t s) {
    const uint32_t mlog = log2_pow2(m);
    uint32_t tlog = mlog < 13 ? mlog : 13;
    while (tlog > 10 && (mlog - tlog) < 8) --tlog;  // keep >= 256 tiles when possible
    if (tlog < 1) tlog = 1;
    const unsigned tiles = 1u << (mlog - tlog);
    const size_t lds = ((size_t)1 << tlog) * 8;
    hipLaunchKernelGGL((bitonic_tile_sort<MODE>), dim3(tiles), dim3(BT_THREADS), lds, s, data, tlog,
                       seed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (uint32_t ilog = tlog + 1; ilog <= mlog; ++ilog) {
        int jlog = (int)ilog - 1;
        while (jlog >= (int)tlog) {
            int R = jlog - (int)tlog + 1;
            if (R > 4) R = 4;
            e = launch_global<MODE>(data, mlog, ilog, (uint32_t)jlog, R, seed, s);
            if (e != hipSuccess) return e;
            jlog -= R;
        }
        hipLaunchKernelGGL((bitonic_tile_merge<MODE>), dim3(tiles), dim3(BT_THREADS), lds, s, data,
                           tlog, ilog, seed);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t bitonic_sort(uint64_t *data, size_t m, uint32_t mode, uint32_t seed, hipStream_t s) {
    if (m < 2) return hipSuccess;
    switch (mode) {
    case 0: return sort_impl<0>(data, m, seed, s);
    case 1: return sort_impl<1>(data, m, seed, s);
    default: return sort_impl<2>(data, m, seed, s);
    }
}

}  // namespace fltee
