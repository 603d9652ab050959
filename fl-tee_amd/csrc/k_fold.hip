// k_fold.hip — the `advanced` pipeline around the bitonic network (gfx950).
//
// advanced.rs:39-113 on the device:
//   advanced_init  : records ++ (i, 0.0) for i < d (:116-123) ++ (u32::MAX, 0.0)
//                    pads to M = next_pow2 (:133-142)
//   [bitonic sort, mode 0]
//   fold           : the oblivious fold (:66-101), EXACT and oblivious:
//   [bitonic sort, mode 0]
//   extract        : global[i] = v[i].1 (:32-34) * 1f32/n (common.rs:14-19)
//
// The fold.  The enclave walks the sorted array once, carrying (pre_idx,
// pre_val): position p-1 receives (u32::MAX - (p-1), 0.0) if p continues the
// run of p-1, else the run's left-to-right sum.  A parallel scan would
// re-associate that sum.  Instead every lane folds its own chunk of C
// positions sequentially, after re-folding the H positions in front of it
// (the halo): whenever no run is longer than H+1 the carry entering the chunk
// is then bit-identical to the enclave's.  With each client's indices distinct
// (top-k, utils.py:327-354) a run holds at most n+1 records, so H = n.  Every
// lane performs the same H+C LDS reads whatever the data (oblivious); a run
// longer than H+1 is detected (S[q].idx == S[q-H-1].idx) and reported as
// FLTEE_DEV_ERR_FOLD_OVERFLOW so the host can re-run with a larger halo.
// Tile: W = 256*C outputs + H+2 halo records in LDS, padded one slot per C
// records so the 64 lanes' chunk walks hit distinct banks.
#include "common.h"

namespace fltee {

__global__ void advanced_init_kernel(const uint64_t *__restrict__ rec, size_t nrec, size_t d,
                                     size_t m, uint64_t *__restrict__ dst) {
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (size_t)gridDim.x * 256) {
        uint64_t v;
        if (p < nrec) v = rec[p];
        else if (p < nrec + d) v = (uint64_t)(uint32_t)(p - nrec);  // (i, +0.0)
        else v = (uint64_t)0xFFFFFFFFu;                               // (u32::MAX, +0.0)
        dst[p] = v;
    }
}

hipError_t launch_advanced_init(const void *rec, size_t nrec, size_t d, size_t m, uint64_t *dst,
                                hipStream_t s) {
    size_t blocks = (m + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(advanced_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint64_t *)rec, nrec, d, m, dst);
    return hipGetLastError();
}

constexpr int FOLD_C = 16;
constexpr int FOLD_CLOG = 4;
constexpr int FOLD_W = 256 * FOLD_C;

__device__ __forceinline__ uint32_t padi(uint32_t e) { return e + (e >> FOLD_CLOG); }

__global__ __launch_bounds__(256) void fold_kernel(const uint64_t *__restrict__ src,
                                                   uint64_t *__restrict__ dst, size_t m,
                                                   size_t fold_len, uint32_t H,
                                                   uint32_t *status) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    const long long start = (long long)blockIdx.x * FOLD_W;
    const long long lo = start - (long long)H - 1;  // global position of local 0
    const uint32_t nload = FOLD_W + H + 2;
    for (uint32_t e = threadIdx.x; e < nload; e += 256) {
        const long long g = lo + e;
        sm[padi(e)] = (g >= 0 && g < (long long)m) ? src[g] : 0ull;
    }
    __syncthreads();

    const long long a = start + (long long)threadIdx.x * FOLD_C;  // first owned position
    uint64_t res[FOLD_C];
    uint32_t overflow = 0;
    // halo re-fold: positions [a - H, a)
    uint32_t pre_idx = 0;
    float pre_val = 0.0f;
    long long q = a - (long long)H;
    bool started = false;
    for (uint32_t it = 0; it < H + FOLD_C; ++it, ++q) {
        const uint32_t e = (uint32_t)(q - lo);
        const uint64_t cur = sm[padi(e)];
        const uint32_t ci = rec_idx(cur);
        const float cv = rec_val(cur);
        if (q >= 0) {
            const bool eq = started && (ci == pre_idx);
            pre_val = eq ? __fadd_rn(pre_val, cv) : cv;
            pre_idx = ci;
            started = true;
        }
        if (it >= H) {
            const uint32_t r = it - H;
            // output for position q (only meaningful for q < fold_len)
            const uint64_t nxt = sm[padi(e + 1)];
            const bool cont = (q + 1 < (long long)fold_len) && (rec_idx(nxt) == ci);
            const uint64_t folded = cont ? (uint64_t)(0xFFFFFFFFu - (uint32_t)q)  // (MAX-q, +0.0)
                                         : make_rec(ci, pre_val);
            res[r] = (q < (long long)fold_len) ? folded : cur;
            const uint64_t back = sm[padi(e - H - 1)];
            overflow |= (q >= (long long)H + 1 && q < (long long)fold_len &&
                         rec_idx(back) == ci);
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < FOLD_C; ++r) sm[padi((uint32_t)(a + r - lo))] = res[r];
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < FOLD_W; e += 256) {
        const long long g = start + e;
        if (g < (long long)m) dst[g] = sm[padi((uint32_t)(g - lo))];
    }
    if (overflow) atomicOr(status, FLTEE_DEV_ERR_FOLD_OVERFLOW);
}

hipError_t launch_fold(const uint64_t *src, uint64_t *dst, size_t m, size_t fold_len, size_t halo,
                       uint32_t *status, hipStream_t s) {
    const uint32_t H = (uint32_t)halo;
    const size_t nload = FOLD_W + (size_t)H + 2;
    const size_t lds = (nload + nload / FOLD_C + 2) * 8;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        attr = true;
    }
    const unsigned blocks = (unsigned)((m + FOLD_W - 1) / FOLD_W);
    hipLaunchKernelGGL(fold_kernel, dim3(blocks), dim3(256), lds, s, src, dst, m, fold_len, H,
                       status);
    return hipGetLastError();
}

template <bool ACC>
__global__ void extract_kernel(const uint64_t *__restrict__ src, size_t d, float coef,
                               float *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    const float v = rec_val(src[i]);
    out[i] = ACC ? __fadd_rn(out[i], v) : __fmul_rn(v, coef);
}

hipError_t launch_extract(const uint64_t *src, size_t d, float coef, float *out, bool accumulate,
                          hipStream_t s) {
    if (d == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((d + 255) / 256);
    if (accumulate)
        hipLaunchKernelGGL(extract_kernel<true>, dim3(blocks), dim3(256), 0, s, src, d, coef, out);
    else
        hipLaunchKernelGGL(extract_kernel<false>, dim3(blocks), dim3(256), 0, s, src, d, coef, out);
    return hipGetLastError();
}

// ---------------------------------------------- sparse non_oblivious -------
// keys[p] = idx << 32 | p : a mode-1 sort then orders records by (idx, upload
// position) — the stable order in which non_oblivious.rs:11-13 adds them.
__global__ void composite_init_kernel(const uint2 *__restrict__ rec, size_t nrec, size_t d,
                                      size_t m, uint64_t *__restrict__ keys, uint32_t *status) {
    uint32_t bad = 0;
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (size_t)gridDim.x * 256) {
        uint64_t kv = ~0ull;
        if (p < nrec) {
            const uint32_t idx = rec[p].x;
            bad |= idx >= d;
            kv = ((uint64_t)idx << 32) | (uint32_t)p;
        }
        keys[p] = kv;
    }
    if (bad) atomicOr(status, FLTEE_DEV_ERR_INDEX_RANGE);
}

hipError_t launch_composite_init(const void *rec, size_t nrec, size_t d, size_t m, uint64_t *keys,
                                 uint32_t *status, hipStream_t s) {
    size_t blocks = (m + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(composite_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint2 *)rec, nrec, d, m, keys, status);
    return hipGetLastError();
}

// Run heads walk their run in upload order: out[idx] = ((+0 + v1) + v2) ...
template <bool ACC>
__global__ void ordered_fold_kernel(const uint64_t *__restrict__ keys, size_t nrec,
                                    const uint2 *__restrict__ rec, float coef,
                                    float *__restrict__ out, size_t d) {
    const size_t q = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= nrec) return;
    const uint32_t idx = (uint32_t)(keys[q] >> 32);
    if (q > 0 && (uint32_t)(keys[q - 1] >> 32) == idx) return;
    if (idx >= d) return;
    float acc = 0.0f;
    for (size_t r = q; r < nrec; ++r) {
        const uint64_t kv = keys[r];
        if ((uint32_t)(kv >> 32) != idx) break;
        acc = __fadd_rn(acc, __uint_as_float(rec[(uint32_t)kv].y));
    }
    out[idx] = ACC ? __fadd_rn(out[idx], acc) : __fmul_rn(acc, coef);
}

hipError_t launch_ordered_fold(const uint64_t *keys, size_t nrec, const void *rec, float coef,
                               float *out, size_t d, bool accumulate, hipStream_t s) {
    if (nrec == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((nrec + 255) / 256);
    if (accumulate)
        hipLaunchKernelGGL(ordered_fold_kernel<true>, dim3(blocks), dim3(256), 0, s, keys, nrec,
                           (const uint2 *)rec, coef, out, d);
    else
        hipLaunchKernelGGL(ordered_fold_kernel<false>, dim3(blocks), dim3(256), 0, s, keys, nrec,
                           (const uint2 *)rec, coef, out, d);
    return hipGetLastError();
}

}  // namespace fltee
