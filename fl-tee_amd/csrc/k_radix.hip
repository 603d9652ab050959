// k_radix.hip — the stable sort by index of an ordered fold's entries (nips19's selected
// list, common.rs:25-35; non_oblivious's sparse fallback, non_oblivious.rs:6-15).
//
// The ordered fold needs the entries grouped by idx, each group in list order: a stable
// sort by idx.  The enclave's own loop `g[idx] += val` (common.rs:25-35) walks the list in
// order and touches g[idx] for every entry, so the sequence of indices in list order is
// what its memory trace already shows; a stable LSD radix sort over the idx bits
// (hipCUB's onesweep) reads and scatters by that same sequence and reveals nothing more.
// (For non_oblivious the reference is not oblivious at all.)  Keys: idx (< d), values:
// list positions; the output is composed into the (idx << 32 | position) keys the
// ordered fold reads (k_fold.hip) — the same order as the stable composite bitonic sort.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace fltee {

__global__ void radix_keys_kernel(const uint2 *__restrict__ rec, size_t n, size_t d,
                                  uint32_t *__restrict__ kin, uint32_t *__restrict__ vin,
                                  uint32_t *status) {
    uint32_t bad = 0;
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (size_t)gridDim.x * 256) {
        const uint32_t idx = rec[p].x;
        bad |= idx >= d;
        kin[p] = idx < d ? idx : (uint32_t)d;  // out of range: after every index (flagged)
        vin[p] = (uint32_t)p;
    }
    if (bad) atomicOr(status, FLTEE_DEV_ERR_INDEX_RANGE);
}

__global__ void radix_compose_kernel(const uint32_t *__restrict__ kout,
                                     const uint32_t *__restrict__ vout, size_t n,
                                     uint64_t *__restrict__ keys) {
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (size_t)gridDim.x * 256)
        keys[p] = ((uint64_t)kout[p] << 32) | vout[p];
}

static uint32_t key_bits(size_t d) {
    uint32_t b = 1;
    while (b < 32 && ((size_t)1 << b) <= d) ++b;  // idx <= d (d: the out-of-range key)
    return b;
}

size_t radix_scratch_bytes(size_t n, size_t d) {
    size_t tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0,
                                             (int)key_bits(d), (hipStream_t)0);
    return 4 * n * 4 + ((tmp + 255) & ~(size_t)255);
}

hipError_t launch_radix_by_idx(const void *rec, size_t n, size_t d, void *scratch, size_t bytes,
                               uint64_t *keys, uint32_t *status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0x7FFFFFFFull) return hipErrorInvalidValue;
    uint32_t *kin = (uint32_t *)scratch, *vin = kin + n, *kout = vin + n, *vout = kout + n;
    void *tmp = (void *)(vout + n);
    const size_t need = radix_scratch_bytes(n, d);
    if (bytes < need) return hipErrorOutOfMemory;
    size_t tb = need - 4 * n * 4;
    size_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(radix_keys_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint2 *)rec, n,
                       d, kin, vin, status);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, (int)n, 0, (int)key_bits(d), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(radix_compose_kernel, dim3((unsigned)blocks), dim3(256), 0, s, kout, vout, n, keys);
    return hipGetLastError();
}

}  // namespace fltee
