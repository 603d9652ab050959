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
//   safe_aggregate : g[idx] += val for idx < d in shuffled order, left to right
//                    per index exactly like the enclave (compaction of the idx < d
//                    entries + stable composite sort + ordered fold, see below):
//                    bit-exact with the oracle's nips19 under the same seed.
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
    // f32 ln as (float)ln((double)x): the same bits as the oracle's host math (and
    // the correctly rounded f32 ln in practice), so the counts match exactly
    const float noise = p > 0.5f ? -b * (float)log((double)(2.0f - 2.0f * p))
                                 : b * (float)log((double)(2.0f * p));
    r[i] = fabsf(noise) > T ? f32_to_u32_sat(ceilf(T)) : f32_to_u32_sat(T + ceilf(noise));
}

hipError_t launch_laplace_r(size_t d, size_t k, float T, uint64_t seed, uint32_t *r,
                            hipStream_t s) {
    if (d == 0) return hipSuccess;
    const float b = 2.0f * (float)k / 100.0f;
    FLTEE_LAUNCH(laplace_r_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, d, b,
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
    FLTEE_LAUNCH(nips19_build_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint64_t *)rec, nrec, r, d, tf, pbase, m, dst);
    return hipGetLastError();
}

hipError_t launch_nips19_build(const void *rec, size_t nrec, const uint32_t *r, size_t d,
                               size_t tf, size_t m, uint64_t *dst, hipStream_t s) {
    return launch_nips19_build_range(rec, nrec, r, d, tf, 0, m, dst, s);
}

// ------------------------------------------------------------ safe_aggregate --
// common.rs:25-35: for w in v { if w.0 < d { g[w.0] += w.1 } } — a left-to-right
// fp32 sum per index in SHUFFLED order.  Reproduced exactly (bit for bit) as:
//   1. select_count / select_write: order-preserving stream compaction of the
//      entries with idx < d (real records and the valid Laplace dummies; the
//      u32::MAX dummies and pads drop out, as in the reference's branch).  Blocks
//      own contiguous tiles of SEL_TILE entries; ranks inside a tile come from wave
//      ballots, tile bases from one exclusive scan of the tile counts.  The selected
//      count Lc is what the enclave's g[] access pattern reveals anyway (the
//      DP-noised histogram total).
//   2. the composite-key stable sort of non_oblivious (k_fold.hip: key = idx << 32 |
//      compacted position, mode-1 bitonic network over next_pow2(Lc)) and the
//      ordered fold: each run head sums its run in shuffled order from +0.0.
constexpr int SEL_NT = 256;
constexpr size_t SEL_TILE = 8192;  // entries per block
constexpr uint32_t SEL_ROUNDS = (uint32_t)(SEL_TILE / (2 * SEL_NT));
typedef unsigned int sel_u32x4 __attribute__((ext_vector_type(4)));

// entries p, p + 1 (p even); u32::MAX beyond m
template <bool VEC>
__device__ __forceinline__ void sel_load(const uint2 *__restrict__ src, size_t m, size_t p, uint2 &a,
                                         uint2 &b) {
    if (VEC && p + 1 < m) {
        const sel_u32x4 w = __builtin_nontemporal_load((const sel_u32x4 *)(src + p));
        a = make_uint2(w.x, w.y);
        b = make_uint2(w.z, w.w);
    } else {
        a = p < m ? src[p] : make_uint2(0xFFFFFFFFu, 0u);
        b = p + 1 < m ? src[p + 1] : make_uint2(0xFFFFFFFFu, 0u);
    }
}

template <bool VEC>
__global__ __launch_bounds__(SEL_NT) void select_count_kernel(const uint2 *__restrict__ src,
                                                              size_t m, uint32_t d,
                                                              uint32_t *__restrict__ cnt) {
    __shared__ uint32_t wsum[SEL_NT / 64];
    const size_t lo = (size_t)blockIdx.x * SEL_TILE;
    uint32_t c = 0;
#pragma unroll 4
    for (uint32_t r = 0; r < SEL_ROUNDS; ++r) {
        uint2 a, b;
        sel_load<VEC>(src, m, lo + 2 * ((size_t)r * SEL_NT + threadIdx.x), a, b);
        c += (a.x < d) + (b.x < d);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < SEL_NT / 64; ++w) t += wsum[w];
        cnt[blockIdx.x] = t;
    }
}

// exclusive scan of nb tile counts in one block; base[nb] = total
__global__ __launch_bounds__(1024) void select_scan_kernel(const uint32_t *__restrict__ cnt,
                                                           uint32_t nb, uint32_t *__restrict__ base) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t lo = threadIdx.x * per < nb ? threadIdx.x * per : nb;
    const uint32_t hi = lo + per < nb ? lo + per : nb;
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = lo; i < hi; ++i) {
        base[i] = run;
        run += cnt[i];
    }
    if (threadIdx.x == 1023) base[nb] = part[1023];
}

template <bool VEC>
__global__ __launch_bounds__(SEL_NT) void select_write_kernel(const uint2 *__restrict__ src,
                                                              size_t m, uint32_t d,
                                                              const uint32_t *__restrict__ base,
                                                              uint2 *__restrict__ dst) {
    __shared__ uint32_t wsum[2][SEL_NT / 64];
    const size_t lo = (size_t)blockIdx.x * SEL_TILE;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t run = base[blockIdx.x];
    for (uint32_t r = 0; r < SEL_ROUNDS; ++r) {
        uint2 a, b;
        sel_load<VEC>(src, m, lo + 2 * ((size_t)r * SEL_NT + threadIdx.x), a, b);
        const uint32_t f0 = a.x < d, f1 = b.x < d;
        const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
        // lane l holds entries 2l, 2l+1 of the wave's span: all of lanes < l come first
        const uint32_t rank = __popcll(b0 & below) + __popcll(b1 & below);
        if (lane == 0) wsum[r & 1][wv] = __popcll(b0) + __popcll(b1);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < SEL_NT / 64; ++w) {
            const uint32_t x = wsum[r & 1][w];
            pre += w < wv ? x : 0u;
            tot += x;
        }
        const uint32_t o = run + pre + rank;
        if (f0) dst[o] = a;
        if (f1) dst[o + f0] = b;
        run += tot;
    }
}

hipError_t launch_select_count(const uint64_t *src, size_t m, size_t d, uint32_t *cnt,
                               uint32_t *base, hipStream_t s) {
    const size_t nb = select_tiles(m);
    net_account((uint64_t)8 * m, "select_count_kernel", s);
    const bool vec = ((uintptr_t)src & 15) == 0;
    const uint32_t dd = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
    if (vec)
        FLTEE_LAUNCH(select_count_kernel<true>, dim3((unsigned)nb), dim3(SEL_NT), 0, s,
                           (const uint2 *)src, m, dd, cnt);
    else
        FLTEE_LAUNCH(select_count_kernel<false>, dim3((unsigned)nb), dim3(SEL_NT), 0, s,
                           (const uint2 *)src, m, dd, cnt);
    FLTEE_LAUNCH(select_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, (uint32_t)nb, base);
    return hipGetLastError();
}

hipError_t launch_select_write(const uint64_t *src, size_t m, size_t d, const uint32_t *base,
                               uint64_t *dst, hipStream_t s) {
    const size_t nb = select_tiles(m);
    net_account((uint64_t)8 * m, "select_write_kernel", s);
    const bool vec = ((uintptr_t)src & 15) == 0;
    const uint32_t dd = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
    if (vec)
        FLTEE_LAUNCH(select_write_kernel<true>, dim3((unsigned)nb), dim3(SEL_NT), 0, s,
                           (const uint2 *)src, m, dd, base, (uint2 *)dst);
    else
        FLTEE_LAUNCH(select_write_kernel<false>, dim3((unsigned)nb), dim3(SEL_NT), 0, s,
                           (const uint2 *)src, m, dd, base, (uint2 *)dst);
    return hipGetLastError();
}

size_t select_tiles(size_t m) { return m ? (m + SEL_TILE - 1) / SEL_TILE : 1; }

// The shuffle's last pass left tile t's selected entries at data[t << tlog, + cnt[t])
// (bitonic_sort_nips19_select): exclusive scan of the counts, then one block per tile
// copies its entries to sel[base[t], ...) — the whole selected list in position order.
__global__ __launch_bounds__(256) void select_gather_kernel(const uint64_t *__restrict__ data,
                                                            uint32_t tlog,
                                                            const uint32_t *__restrict__ cnt,
                                                            const uint32_t *__restrict__ base,
                                                            uint64_t *__restrict__ sel) {
    const uint32_t t = blockIdx.x, c = cnt[t], b = base[t];
    const uint64_t *src = data + ((size_t)t << tlog);
    for (uint32_t i = threadIdx.x; i < c; i += 256) sel[b + i] = src[i];
}

hipError_t launch_select_scan(const uint32_t *cnt, size_t nb, uint32_t *base, hipStream_t s) {
    FLTEE_LAUNCH(select_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, (uint32_t)nb, base);
    return hipGetLastError();
}

hipError_t launch_select_gather(const uint64_t *data, uint32_t tlog, size_t ntiles,
                                const uint32_t *cnt, const uint32_t *base, uint64_t *sel,
                                hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    FLTEE_LAUNCH(select_gather_kernel, dim3((unsigned)ntiles), dim3(256), 0, s, data, tlog,
                       cnt, base, sel);
    return hipGetLastError();
}

}  // namespace fltee
