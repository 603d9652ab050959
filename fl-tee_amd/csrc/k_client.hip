// k_client.hip — the client-side producers of fl_main.py:221-238 on the device
// (SURVEY §8f row 4): top-k by magnitude, serialisation, (L2 clip and AES-CTR
// encryption reuse k_dp.hip / k_aes.hip).  For a GPU-resident client simulator:
// n clients' flattened update vectors in HBM -> the concatenated ciphertext the
// Aggregate request carries, without a host round trip.
//
// zero_except_top_k_weights (utils.py:327-354) sorts (idx, val) by abs(val) with
// Python's stable sort, reverse=True: |val| descending, equal magnitudes in
// ascending index order; the first k form top_k_indices, and serialize_sparse
// (utils.py:193-209) writes (idx, val) in exactly that order.  Here every client
// gets the composite key ((0x7FFFFFFF - |val| bits) << 32) | idx (ascending key ==
// that order; |val| bits of a non-negative float are monotonic) and the keys are
// sorted per client by the library's bitonic network, stages up to the padded
// segment size only (k_bitonic.hip bitonic_sort_segments): segments come out
// ascending / descending alternately, and the extract reads each one in its
// ascending order.  NaN magnitudes sort above +inf (the reference's Python sort is
// not well-defined for NaN).
#include "common.h"

namespace fltee {

__global__ void client_keys_kernel(const float *__restrict__ values, size_t n, size_t d,
                                   uint32_t slog, uint64_t *__restrict__ keys) {
    const size_t total = n << slog, mask = ((size_t)1 << slog) - 1;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total;
         t += (size_t)gridDim.x * 256) {
        const size_t c = t >> slog, i = t & mask;
        uint64_t key = ~0ull;  // pads sort after every real key
        if (i < d) {
            const uint32_t a = __float_as_uint(values[c * d + i]) & 0x7FFFFFFFu;
            key = ((uint64_t)(0x7FFFFFFFu - a) << 32) | (uint32_t)i;
        }
        keys[t] = key;
    }
}

__global__ void client_topk_extract_kernel(const uint64_t *__restrict__ keys,
                                           const float *__restrict__ values, size_t n, size_t d,
                                           size_t k, uint32_t slog, uint64_t *__restrict__ rec) {
    const size_t total = n * k, seg = (size_t)1 << slog;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total;
         t += (size_t)gridDim.x * 256) {
        const size_t c = t / k, j = t - c * k;
        const size_t base = c << slog;
        const size_t p = (c & 1) ? base + seg - 1 - j : base + j;  // odd segments descending
        const uint32_t idx = (uint32_t)keys[p];
        rec[t] = make_rec(idx, values[c * d + idx]);
    }
}

// serialize_dense (utils.py:171-190): (i, v[i]) for i < d, per client
__global__ void client_dense_kernel(const float *__restrict__ values, size_t n, size_t d,
                                    uint64_t *__restrict__ rec) {
    const size_t total = n * d;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total;
         t += (size_t)gridDim.x * 256) {
        const size_t c = t / d, i = t - c * d;
        rec[t] = make_rec((uint32_t)i, values[t]);
    }
}

static unsigned grid_for(size_t total) {
    size_t b = (total + 255) / 256;
    return (unsigned)(b < 65536 ? (b ? b : 1) : 65536);
}

hipError_t launch_client_topk(const float *values, size_t n, size_t d, size_t k, uint64_t *keys,
                              uint64_t *rec, hipStream_t s) {
    const size_t segp = next_pow2_sz(d < 2 ? 2 : d);
    const uint32_t slog = log2_pow2(segp);
    FLTEE_LAUNCH(client_keys_kernel, dim3(grid_for(n * segp)), dim3(256), 0, s, values, n,
                       d, slog, keys);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // n segments padded to a power of two (pad segments of all-pad keys are inert)
    const size_t m = next_pow2_sz(n * segp);
    if (m > n * segp) {
        e = fl_memset_async(keys + n * segp, 0xFF, (m - n * segp) * 8, s);
        if (e != hipSuccess) return e;
    }
    e = bitonic_sort_segments(keys, m, segp, 1, s);
    if (e != hipSuccess) return e;
    FLTEE_LAUNCH(client_topk_extract_kernel, dim3(grid_for(n * k)), dim3(256), 0, s, keys,
                       values, n, d, k, slog, rec);
    return hipGetLastError();
}

size_t client_topk_workspace(size_t n, size_t d) {
    return next_pow2_sz(n * next_pow2_sz(d < 2 ? 2 : d)) * 8;
}

hipError_t launch_client_dense(const float *values, size_t n, size_t d, uint64_t *rec,
                               hipStream_t s) {
    FLTEE_LAUNCH(client_dense_kernel, dim3(grid_for(n * d)), dim3(256), 0, s, values, n, d,
                       rec);
    return hipGetLastError();
}

}  // namespace fltee
