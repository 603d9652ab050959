// k_nips19.hip — alg 2 (nips19.rs:18-63, common.rs:25-35,77-98,151-197) on gfx950.
//
//   laplace_r      : r_i from one Laplace(b = 2k/eps) draw per parameter, cut at
//                    T = (2k/eps) ln(d/delta), eps = 100, delta = 1/n (f32 math
//                    as in the enclave; the uniform comes from Philox4x32-10
//                    instead of RDRAND-seeded sgx_rand — see DESIGN.md)
//   nips19_build   : records ++ d*floor(T) dummies, entry (i, j) =
//                    ((r_i < j) ? i : u32::MAX, 0.0) (oblivious_pad, branch-free)
//                    ++ (u32::MAX, 0.0) pads to 2^m
//   [bitonic network, mode 2 = keyed shuffle]
//   safe_aggregate : g[idx] += val for idx < d in shuffled order.  Every entry
//                    with idx < d is added (dummies add +0.0), exactly the
//                    access histogram the enclave reveals.  Sums go through
//                    LDS float atomics per (chunk, d-segment) and one global
//                    atomic per slot per chunk, so the per-index summation
//                    order is not the enclave's: parity is within fp32
//                    tolerance (the enclave's own order is random anyway).
#include "common.h"

namespace fltee {

__device__ __forceinline__ uint32_t f32_to_u32_sat(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}

__global__ void laplace_r_kernel(size_t d, float b, float T, uint32_t k0, uint32_t k1,
                                 uint32_t *__restrict__ r) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    uint32_t c[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), 0u, FLTEE_STREAM_LAPLACE};
    philox4x32_10(c, k0, k1);
    const float p = (float)(c[0] >> 8) * (1.0f / 16777216.0f);
    const float noise = p > 0.5f ? -b * logf(2.0f - 2.0f * p) : b * logf(2.0f * p);
    r[i] = fabsf(noise) > T ? f32_to_u32_sat(ceilf(T)) : f32_to_u32_sat(T + ceilf(noise));
}

hipError_t launch_laplace_r(size_t d, size_t k, float T, uint64_t seed, uint32_t *r,
                            hipStream_t s) {
    if (d == 0) return hipSuccess;
    const float b = 2.0f * (float)k / 100.0f;
    hipLaunchKernelGGL(laplace_r_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, d, b,
                       T, (uint32_t)seed, (uint32_t)(seed >> 32), r);
    return hipGetLastError();
}

// dst[x] = entry pbase + x of the padded array; rec[x] is the record at position
// pbase + x (read only where pbase + x < nrec).  pbase = 0: the whole array.
__global__ void nips19_build_kernel(const uint64_t *__restrict__ rec, size_t nrec,
                                    const uint32_t *__restrict__ r, size_t d, size_t tf,
                                    size_t pbase, size_t m, uint64_t *__restrict__ dst) {
    const size_t npad = d * tf;
    for (size_t x = (size_t)blockIdx.x * 256 + threadIdx.x; x < m; x += (size_t)gridDim.x * 256) {
        const size_t p = pbase + x;
        uint64_t v;
        if (p < nrec) {
            v = rec[x];
        } else if (p < nrec + npad) {
            const size_t e = p - nrec;
            const size_t i = e / tf, j = e - i * tf;
            const uint32_t ri = r[i];
            v = ((size_t)ri < j) ? (uint64_t)(uint32_t)i : (uint64_t)0xFFFFFFFFu;  // o_setb/o_mov
        } else {
            v = (uint64_t)0xFFFFFFFFu;
        }
        dst[x] = v;
    }
}

hipError_t launch_nips19_build_range(const void *rec, size_t nrec, const uint32_t *r, size_t d,
                                     size_t tf, size_t pbase, size_t m, uint64_t *dst,
                                     hipStream_t s) {
    if (m == 0) return hipSuccess;
    size_t blocks = (m + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(nips19_build_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint64_t *)rec, nrec, r, d, tf, pbase, m, dst);
    return hipGetLastError();
}

hipError_t launch_nips19_build(const void *rec, size_t nrec, const uint32_t *r, size_t d,
                               size_t tf, size_t m, uint64_t *dst, hipStream_t s) {
    return launch_nips19_build_range(rec, nrec, r, d, tf, 0, m, dst, s);
}

constexpr uint32_t SA_SEG = 32768;      // floats per LDS segment (128 KB)
constexpr uint32_t SA_SEG_MAX = 40960;  // the whole 160 KB of LDS
constexpr uint32_t SA_CHUNKS = 256;

// VEC: src 16-B aligned, chunks read as record pairs, SA_U pair loads in flight per
// lane (one 8-B load per lane at a time left ~8 KB in flight per CU: latency-bound,
// 0.69 ms for C4's 1 GB).
constexpr int SA_U = 4;
typedef unsigned int sa_u32x4 __attribute__((ext_vector_type(4)));
// TAILG: one LDS segment [0, segsz) and the few indices in [segsz, d) go straight to
// global atomics, so the array is read once (C4, d = 44,964: two 32K segments read it
// twice from HBM, both blocks of a chunk running at the same time).
template <bool VEC, bool TAILG>
__global__ __launch_bounds__(1024) void safe_aggregate_kernel(const uint2 *__restrict__ src,
                                                              size_t m, size_t d, uint32_t segsz,
                                                              float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float acc[];
    // 1-D grid, segment fastest: the blocks of every segment of one chunk are dispatched
    // back to back, so all but the first read that chunk from the Infinity Cache
    const uint32_t nseg = TAILG ? 1u : (uint32_t)((d + segsz - 1) / segsz);
    const uint32_t seg = blockIdx.x % nseg, chunk = blockIdx.x / nseg, nchunks = gridDim.x / nseg;
    const size_t seg_lo = (size_t)seg * segsz;
    const uint32_t seg_n = (uint32_t)((d - seg_lo) < segsz ? (d - seg_lo) : segsz);
    for (uint32_t e = threadIdx.x; e < seg_n; e += 1024) acc[e] = 0.0f;
    __syncthreads();
    const size_t per = ((m + nchunks - 1) / nchunks + 1) & ~(size_t)1;  // even: pairs
    const size_t lo = (size_t)chunk * per < m ? (size_t)chunk * per : m;
    const size_t hi = lo + per < m ? lo + per : m;
    auto add = [&](uint32_t idx, uint32_t val) {
        const uint32_t rel = idx - (uint32_t)seg_lo;
        if (idx < d && rel < seg_n) atomicAdd(&acc[rel], __uint_as_float(val));
        else if (TAILG && idx < d) atomicAdd(&out[idx], __uint_as_float(val));
    };
    size_t p = lo + threadIdx.x;
    if (VEC) {
        const sa_u32x4 *s4 = (const sa_u32x4 *)src;
        const size_t plo = lo / 2, phi = hi / 2;
        size_t q = plo + threadIdx.x;
        for (; q + (SA_U - 1) * 1024 < phi; q += SA_U * 1024) {
            sa_u32x4 w[SA_U];
#pragma unroll
            for (int u = 0; u < SA_U; ++u) w[u] = __builtin_nontemporal_load(&s4[q + u * 1024]);
#pragma unroll
            for (int u = 0; u < SA_U; ++u) {
                add(w[u].x, w[u].y);
                add(w[u].z, w[u].w);
            }
        }
        for (; q < phi; q += 1024) {
            const sa_u32x4 w = __builtin_nontemporal_load(&s4[q]);
            add(w.x, w.y);
            add(w.z, w.w);
        }
        p = 2 * phi + threadIdx.x;  // an odd record at the end of the array
    }
    for (; p < hi; p += 1024) {
        const uint2 w = src[p];
        add(w.x, w.y);
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < seg_n; e += 1024) atomicAdd(&out[seg_lo + e], acc[e]);
}

hipError_t launch_safe_aggregate(const uint64_t *src, size_t m, size_t d, float *out,
                                 hipStream_t s) {
    if (d == 0 || m == 0) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        const void *k[4] = {(const void *)safe_aggregate_kernel<true, false>,
                            (const void *)safe_aggregate_kernel<false, false>,
                            (const void *)safe_aggregate_kernel<true, true>,
                            (const void *)safe_aggregate_kernel<false, true>};
        for (const void *f : k)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, SA_SEG_MAX * 4);
        attr = true;
    }
    // d a little above one 32K segment: one 40K segment + global atomics for the rest
    const bool tailg = d > SA_SEG && d <= SA_SEG_MAX + SA_SEG_MAX / 8;
    const uint32_t segsz = tailg ? SA_SEG_MAX : SA_SEG;
    const unsigned segs = tailg ? 1u : (unsigned)((d + segsz - 1) / segsz);
    size_t chunks = (m + 8191) / 8192;
    if (chunks > SA_CHUNKS) chunks = SA_CHUNKS;
    const size_t lds = (d < segsz ? d : segsz) * 4;
    const bool vec = ((uintptr_t)src & 15) == 0;
    const dim3 grid((unsigned)(chunks * segs));
    const uint2 *s2 = (const uint2 *)src;
    if (vec && tailg) hipLaunchKernelGGL((safe_aggregate_kernel<true, true>), grid, dim3(1024), lds, s, s2, m, d, segsz, out);
    else if (vec) hipLaunchKernelGGL((safe_aggregate_kernel<true, false>), grid, dim3(1024), lds, s, s2, m, d, segsz, out);
    else if (tailg) hipLaunchKernelGGL((safe_aggregate_kernel<false, true>), grid, dim3(1024), lds, s, s2, m, d, segsz, out);
    else hipLaunchKernelGGL((safe_aggregate_kernel<false, false>), grid, dim3(1024), lds, s, s2, m, d, segsz, out);
    return hipGetLastError();
}

}  // namespace fltee
