// common.h — shared device helpers for libfltee_agg (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "fltee_agg.h"

// One record of the wire / HBM layout: parameters.rs:3-10 Weight(u32 idx, f32 val),
// little-endian, 8 bytes.  Kept as a u64 in registers: low word = idx, high = val bits.
__device__ __forceinline__ uint32_t rec_idx(uint64_t r) { return (uint32_t)r; }

// Block-swizzled physical layout of the large record arrays between the passes of a
// network (k_bitonic.hip: the 2^14-tile sorts): logical
// position p lives at phys(p) = p ^ swz_x(p), the 128-B blocks (16 records) of each
// aligned 2^14-record block permuted by the block's position bits >= 14, so that rows at
// power-of-two strides do not land on the same HBM channels.  Bits >= 14 and bits 0..3
// are unchanged; GF(2)-linear: phys(a ^ b) = phys(a) ^ phys(b).
constexpr uint32_t kSwzMask = 0x3FF0u;
__device__ __forceinline__ uint32_t swz_x(uint32_t p) {
    const uint32_t h = p >> 14;
    return ((h ^ (h >> 10)) << 4) & kSwzMask;
}
__device__ __forceinline__ uint32_t phys(uint32_t p) { return p ^ swz_x(p); }
__device__ __forceinline__ float rec_val(uint64_t r) { return __uint_as_float((uint32_t)(r >> 32)); }
__device__ __forceinline__ uint64_t make_rec(uint32_t idx, float val) {
    return ((uint64_t)__float_as_uint(val) << 32) | idx;
}

// Counter-based generators shared with the oracle (oracle/fltee_oracle.c):
// Philox4x32-10 and the lowbias32 mixer.  Same constants, same stream ids.
#define FLTEE_STREAM_DP 0x44504E5Au
#define FLTEE_STREAM_LAPLACE 0x4C41504Cu
#define FLTEE_STREAM_SAMPLE 0x534D504Cu

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint32_t shuffle_step_key(uint32_t seed, uint32_t ilog,
                                                              uint32_t jlog) {
    return mix32(mix32(seed) + ((ilog << 8) | jlog) * 0x9E3779B9u);
}

__host__ __device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

#define FLTEE_CHECK_LAUNCH(st)                                            \
    do {                                                                  \
        if (hipGetLastError() != hipSuccess) return FLTEE_ERROR_UNEXPECTED; \
    } while (0)

static inline size_t next_pow2_sz(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
static inline uint32_t log2_pow2(size_t x) {
    uint32_t l = 0;
    while (((size_t)1 << l) < x) ++l;
    return l;
}

// ---- the launch trace (obliviousness tests) ---------------------------------------
// Every kernel launch, copy, memset and host synchronisation of the library goes through
// these (tests/test_abi.py rejects a raw hipLaunchKernelGGL / hipMemcpy* / hipMemset* /
// hip*Synchronize in csrc/): with fltee_debug_trace(1) each appends one line — what, the
// call site (the kernel expression as written), grid / block / LDS or the byte count — to
// a process-wide log that tests/test_gpu_oblivious.py compares between inputs of the same
// public sizes.  Off (the default), a relaxed load per call.
namespace fltee {
bool trace_on();
void trace_event(const char *what, const char *site, uint64_t a, uint64_t b, uint64_t c);
}  // namespace fltee
#define FLTEE_LAUNCH(K, GRID, BLOCK, LDS, S, ...)                                              \
    do {                                                                                       \
        const dim3 fltee_g_ = dim3(GRID), fltee_b_ = dim3(BLOCK);                              \
        if (::fltee::trace_on())                                                               \
            ::fltee::trace_event("launch", #K, ((uint64_t)fltee_g_.x << 32) | fltee_g_.y,      \
                                 ((uint64_t)fltee_g_.z << 32) | fltee_b_.x, (uint64_t)(LDS));  \
        hipLaunchKernelGGL(K, fltee_g_, fltee_b_, LDS, S, __VA_ARGS__);                        \
    } while (0)
namespace fltee {
inline hipError_t fl_memcpy_async(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t st) {
    if (trace_on()) trace_event("memcpy", "", n, (uint64_t)k, 0);
    return hipMemcpyAsync(d, s, n, k, st);
}
inline hipError_t fl_memcpy2d_async(void *d, size_t dp, const void *s, size_t sp, size_t w, size_t h,
                                    hipMemcpyKind k, hipStream_t st) {
    if (trace_on()) trace_event("memcpy2d", "", w, h, (uint64_t)k);
    return hipMemcpy2DAsync(d, dp, s, sp, w, h, k, st);
}
inline hipError_t fl_memcpy(void *d, const void *s, size_t n, hipMemcpyKind k) {
    if (trace_on()) trace_event("memcpy_sync", "", n, (uint64_t)k, 0);
    return hipMemcpy(d, s, n, k);
}
inline hipError_t fl_memset_async(void *d, int v, size_t n, hipStream_t st) {
    if (trace_on()) trace_event("memset", "", n, (uint64_t)(uint32_t)v, 0);
    return hipMemsetAsync(d, v, n, st);
}
inline hipError_t fl_memset(void *d, int v, size_t n) {
    if (trace_on()) trace_event("memset_sync", "", n, (uint64_t)(uint32_t)v, 0);
    return hipMemset(d, v, n);
}
inline hipError_t fl_stream_sync(hipStream_t st) {
    if (trace_on()) trace_event("sync", "stream", 0, 0, 0);
    return hipStreamSynchronize(st);
}
inline hipError_t fl_device_sync() {
    if (trace_on()) trace_event("sync", "device", 0, 0, 0);
    return hipDeviceSynchronize();
}
}  // namespace fltee

// ---- kernel launchers (implemented in the k_*.hip files) ------------------
namespace fltee {

// Measurement: HBM bytes the streaming passes of the networks move (algorithmic per
// launch: read + write of the live part of the array they sweep — pad-only blocks a
// launch skips are not counted), counted at launch on the host (engine.hip; read by
// bench.py through fltee_debug_net_stats).  Called once per launch, before it, with the
// kernel's name: with fltee_debug_net_timing on, an event recorded there on `s` times
// each launch (the gap to the next accounted launch or the final event).
void net_account(uint64_t bytes, const char *kernel, hipStream_t s);

// k_accumulate.hip
hipError_t launch_dense_accumulate(const void *rec, size_t n, size_t d, float coef, float *out,
                                   const float *client_coef, bool accumulate, uint32_t *status,
                                   hipStream_t s);
// baseline.rs o_update on sparse records: out[j] = the in-order sum over every record with
// idx j (+0.0 selected elsewhere), exact for any upload, fixed cost nrec * d
hipError_t launch_sweep_accumulate(const void *rec, size_t nrec, size_t d, float coef, float *out,
                                   bool accumulate, hipStream_t s);
hipError_t launch_scale(float *out, size_t d, float coef, hipStream_t s);
hipError_t launch_check_range(const void *rec, size_t nrec, uint32_t limit, uint32_t *status,
                              hipStream_t s);

// k_bitonic.hip
// valid: positions >= valid hold identical pad records (0: unknown); the stage blocks
// made of pads alone are skipped (exact, data-independent)
hipError_t bitonic_sort(uint64_t *data, size_t m, uint32_t mode, uint32_t seed, hipStream_t s,
                        size_t valid = 0);
void set_pad_skip(int on);
void set_swizzle(int on);
bool pad_skip_enabled();
size_t debug_plan(uint32_t mlog, uint32_t tlog, uint32_t NT, int rmax, uint32_t *out, size_t cap);
void debug_pad_units(uint32_t mode, uint32_t valid, uint32_t mlog, uint32_t pbase, uint32_t ilog,
                     uint32_t jstep, uint32_t sblog, uint32_t uplog, uint32_t out[3]);
// stages up to log2(seg) only: aligned segments of seg records sorted, alternating
// ascending (even segments) / descending (odd segments)
hipError_t bitonic_sort_segments(uint64_t *data, size_t m, size_t seg, uint32_t mode,
                                 hipStream_t s);
// the sort (mode 0) of advanced's padded array / the keyed shuffle (mode 2) of nips19's,
// with advanced_init / nips19_build fused into the first pass's loads: data[0, m) gets
// the result.  hipErrorNotSupported: not fusable at this m (build, then sort).
hipError_t bitonic_sort_advanced(uint64_t *data, size_t m, const void *rec, size_t nrec, size_t d,
                                 hipStream_t s);
hipError_t bitonic_sort_nips19(uint64_t *data, size_t m, uint32_t seed, const void *rec, size_t nrec,
                               const uint32_t *r, size_t d, size_t tf, hipStream_t s);
// the same shuffle whose last pass keeps only the entries with idx < d: tile t's are
// left at data[t * (m / tiles), + tile_cnt[t]) in position order (the array itself is not
// written out).  bitonic_select_tiles(m): the tile count, 0 when the last pass cannot
// select (then hipErrorNotSupported).
size_t bitonic_select_tiles(size_t m);
hipError_t bitonic_sort_nips19_select(uint64_t *data, size_t m, uint32_t seed, const void *rec,
                                      size_t nrec, const uint32_t *r, size_t d, size_t tf,
                                      uint32_t *tile_cnt, hipStream_t s);
void set_fused_init(int on);
// one range [pbase, pbase + m) of a larger network (pbase a multiple of m): stages
// 1..log2 m; the steps j < m of stage ilog; the step 2^jlog >= m of stage ilog
// between this range and the partner range pos_theirs = pos_mine ^ 2^jlog
// valid (0 = unknown): positions >= valid of this range hold identical pads
hipError_t bitonic_sort_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                              uint32_t pbase, hipStream_t s, uint32_t valid = 0);
hipError_t bitonic_merge_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                               uint32_t ilog, uint32_t pbase, hipStream_t s);
hipError_t bitonic_steps_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                               uint32_t ilog, uint32_t jtop, uint32_t jbot, uint32_t pbase,
                               hipStream_t s);
hipError_t bitonic_exchange(uint64_t *mine, const uint64_t *theirs, size_t m, uint32_t pos_mine,
                            uint32_t pos_theirs, uint32_t mode, uint32_t seed, uint32_t ilog,
                            uint32_t jlog, hipStream_t s);

// k_fold.hip
hipError_t launch_advanced_init(const void *rec, size_t nrec, size_t d, size_t m, uint64_t *dst,
                                hipStream_t s);
hipError_t launch_advanced_init_range(const void *rec, size_t nrec, size_t d, size_t pbase,
                                      size_t m, uint64_t *dst, hipStream_t s);
size_t fold_context(size_t halo);  // records of context the fold re-reads: halo rounded to 16
// The streaming fold's side record per lane (k_fold.hip header: runs of any length) and the
// segmented aggregate of consecutive pieces the patch scans.
constexpr uint32_t kFsPiece = 1u, kFsFull = 2u, kFsCorr = 4u;
struct FoldSide {
    uint32_t F, K;  // keys of the piece's first and last positions
    float Q;        // in-order partial of the run ending the piece, over the piece
    uint32_t fl;    // kFsPiece: the piece holds positions; kFsFull: one key; kFsCorr: below
    uint32_t ck;    // kFsCorr: the key of a run begun before the walk and ended in the chunk
    float S;        // kFsCorr: that run's in-order sum from the walk start to its end
    uint32_t pad[2];
};
struct FoldAgg {
    uint32_t F, K;
    float Q;
    uint32_t fl;
};
// FoldAgg: the segmented aggregate of consecutive pieces — first key, last key, one key
// throughout, and the in-order (within a piece; re-associated across pieces) partial of
// the run ending the range.  combine is associative.
__device__ __forceinline__ FoldAgg fa_combine(const FoldAgg &x, const FoldAgg &y) {
    if (!(x.fl & kFsPiece)) return y;
    if (!(y.fl & kFsPiece)) return x;
    const bool yfull = (y.fl & kFsFull) != 0;
    FoldAgg r;
    r.F = x.F;
    r.K = y.K;
    r.fl = kFsPiece | (((x.fl & kFsFull) && yfull && x.K == y.F) ? kFsFull : 0u);
    r.Q = (yfull && y.F == x.K) ? __fadd_rn(x.Q, y.Q) : y.Q;
    return r;
}

__device__ __forceinline__ FoldAgg fa_of(const FoldSide &sd) {
    FoldAgg a;
    a.F = sd.F;
    a.K = sd.K;
    a.Q = sd.Q;
    a.fl = sd.fl & (kFsPiece | kFsFull);
    return a;
}

__device__ __forceinline__ FoldAgg fa_empty() {
    FoldAgg a;
    a.F = a.K = 0;
    a.Q = 0.0f;
    a.fl = 0;
    return a;
}

// the fold's side buffer: FoldSide per lane (waves x 64 of them), then FoldAgg per wave
__host__ __device__ inline FoldAgg *fold_wave_aggs(FoldSide *side, size_t waves) {
    return reinterpret_cast<FoldAgg *>(side + waves * 64);
}
// lanes of a streaming fold over span positions (0: the one-lane walk: no side records)
size_t fold_lanes(size_t span, size_t fold_len, size_t halo, size_t origin, long long pbase);
size_t fold_side_bytes(size_t span, size_t fold_len, size_t halo, size_t origin, long long pbase);
// cemit_d != 0: emit the compaction's first-pass form instead (run ends with idx < cemit_d
// as (c = p - idx, sum), the rest as cdummy; whole arrays only: origin = pbase = 0).
// side: fold_lanes() records (required unless the one-lane walk); then
// launch_fold_range_patch writes the long runs' records (after the totals of the ranges
// before, prev[0, nprev), for a position-sharded array)
hipError_t launch_fold_range(const uint64_t *src, uint64_t *dst, size_t m, size_t origin,
                             size_t end, long long pbase, size_t fold_len, size_t halo,
                             FoldSide *side, hipStream_t s, size_t cemit_d = 0,
                             uint64_t cdummy = 0);
hipError_t launch_fold_range_total(const FoldSide *side, size_t lanes, FoldAgg *total,
                                   hipStream_t s);
hipError_t launch_fold_range_patch(uint64_t *dst, size_t span, size_t origin, long long pbase,
                                   size_t fold_len, size_t halo, const FoldSide *side,
                                   const FoldAgg *prev, size_t nprev, hipStream_t s,
                                   size_t cemit_d = 0, uint64_t cdummy = 0);
// the whole array: fold + patch (side_ws: >= fold_side_bytes(m, fold_len, halo, 0, 0))
hipError_t launch_fold(const uint64_t *src, uint64_t *dst, size_t m, size_t fold_len, size_t halo,
                       void *side_ws, size_t side_cap, hipStream_t s, size_t cemit_d = 0,
                       uint64_t cdummy = 0);
hipError_t launch_extract(const uint64_t *src, size_t d, float coef, float *out, bool accumulate,
                          hipStream_t s);
// k_compact.hip
// fold (fold_len == L) + compaction from the SORTED array; hipErrorNotSupported: fold apart
// lb: fc_lookback_bytes() of zeroed look-back slots (the tiles' carries), *epoch: the
// device's launch counter for them (at 2^30 - 1 the caller zeroes the slots and resets it)
size_t fc_lookback_bytes(size_t M, size_t L, size_t d, size_t halo);
hipError_t launch_fold_compact_extract(uint64_t *A, uint64_t *B, size_t M, size_t L, size_t d,
                                       size_t halo, float coef, float *out, bool accumulate,
                                       uint32_t *status, hipStream_t s, void *lb, size_t lb_cap,
                                       uint32_t *epoch);
hipError_t launch_compact_extract(uint64_t *src, uint64_t *tmp, size_t L, size_t d, float coef,
                                  float *out, bool accumulate, hipStream_t s);
// the same from launch_fold(..., cemit_d = d, compact_dummy())'s output
uint64_t compact_dummy();
hipError_t launch_compact_extract_converted(uint64_t *src, uint64_t *tmp, size_t L, size_t d,
                                            float coef, float *out, bool accumulate, hipStream_t s);
hipError_t launch_compact_offset(const uint64_t *chunk, size_t c, size_t d, uint64_t *buf,
                                 uint64_t *tmp, float coef, float *out, hipStream_t s);
hipError_t launch_composite_init(const void *rec, size_t nrec, size_t d, size_t m, uint64_t *keys,
                                 uint32_t *status, hipStream_t s);

// k_nips19.hip
hipError_t launch_laplace_r(size_t d, size_t k, float T, uint64_t seed, uint32_t *r,
                            hipStream_t s);
hipError_t launch_nips19_build(const void *rec, size_t nrec, const uint32_t *r, size_t d,
                               size_t tf, size_t m, uint64_t *dst, hipStream_t s);
// safe_aggregate pieces: tile counts + exclusive scan (base[nb] = total selected),
// then the order-preserving write of the idx < d entries (engine.hip drives them)
size_t select_tiles(size_t m);
hipError_t launch_select_count(const uint64_t *src, size_t m, size_t d, uint32_t *cnt,
                               uint32_t *base, hipStream_t s);
hipError_t launch_select_write(const uint64_t *src, size_t m, size_t d, const uint32_t *base,
                               uint64_t *dst, hipStream_t s);
hipError_t launch_select_scan(const uint32_t *cnt, size_t nb, uint32_t *base, hipStream_t s);
hipError_t launch_select_gather(const uint64_t *data, uint32_t tlog, size_t ntiles,
                                const uint32_t *cnt, const uint32_t *base, uint64_t *sel,
                                hipStream_t s);
hipError_t launch_nips19_build_range(const void *rec, size_t nrec, const uint32_t *r, size_t d,
                                     size_t tf, size_t pbase, size_t m, uint64_t *dst,
                                     hipStream_t s);

// k_radix.hip: the stable sort by idx of an ordered fold's n records (hand-written LSD
// counting sort; scratch: radix_scratch_bytes) -> sorted[0, n) (zero[0, nzero) set to +0.0
// on the way, when given), and the ordered fold over sorted records: out[i] for the indices
// i < d with records (accumulate: adds); the others are left as they are
size_t radix_scratch_bytes(size_t n, size_t d);
hipError_t launch_sort_records_by_idx(const void *rec, size_t n, size_t d, void *scratch,
                                      size_t bytes, uint64_t *sorted, uint32_t *status,
                                      float *zero, size_t nzero, hipStream_t s);
hipError_t launch_fold_sorted(const uint64_t *sorted, size_t n, size_t d, float coef, float *out,
                              bool accumulate, hipStream_t s);
hipError_t launch_gather_by_keys(const uint64_t *keys, size_t n, const void *rec, uint64_t *dst,
                                 hipStream_t s);

// k_oram.hip: path_oram as a tree Path ORAM (Z = 4, stash 20, next_pow2(d) <= 2^22
// blocks).  Default: oram.rs's own access sequence (d prepare writes, a read and a write per
// record, d readout reads -> out[i] * coef, or out[i] += with accumulate); lazy: one
// read-modify-write per record, then every tree/stash slot as an 8-B record (idx, value;
// empty slots idx >= next_pow2(d), unique) in records[oram_slots(d)] for the oblivious
// readout (advanced's network, n = 1).  tree: oram_slots(d) * 16 bytes; keys, keys2:
// next_pow2(oram_accesses()) u64 each (the leaf precompute's sorts).
size_t oram_slots(size_t d);
bool oram_supported(size_t d);
size_t oram_accesses(size_t nrec, size_t d, bool lazy);
bool oram_fits(size_t nrec, size_t d, bool lazy);
void set_oram_bucket(int z);
hipError_t launch_oram_tree(const void *rec, size_t nrec, size_t d, bool lazy, void *tree,
                            uint64_t seed, uint64_t *keys, uint64_t *keys2, uint64_t *records,
                            float coef, bool accumulate, float *out, uint32_t *status,
                            hipStream_t s);

// k_dp.hip
hipError_t launch_dp_noise(float *out, size_t d, float sigma, float clipping, size_t n,
                           uint64_t seed, hipStream_t s);
hipError_t launch_client_clip_coef(const void *rec, size_t n, size_t k, float clipping,
                                   float *coef, hipStream_t s);
hipError_t launch_apply_clip(void *rec, size_t n, size_t k, const float *coef, hipStream_t s);

// k_aes.hip
void aes128_expand_key(const uint8_t key[16], uint32_t rk[44]);
// the round keys of the n clients' session keys (constant time, 8 keys per circuit pass)
void aes128_session_round_keys(const uint32_t *ids, size_t n, uint32_t *rk);
// zero_word (optional): a device word the kernel sets to 0 (a status word, without a
// memset launch)
hipError_t launch_aes_ctr(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                          size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                          hipStream_t s, uint32_t *zero_word = nullptr);
// the bytes [16 * block_off, ...) of each client's payload; idx_sub subtracted from each idx
void set_aes_variant(int v);  // 0: by size, 1: quad kernel, 2: byte-per-lane kernel
hipError_t launch_aes_ctr_slice(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                                size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                                uint64_t block_off, uint32_t idx_sub, hipStream_t s,
                                uint32_t *zero_word = nullptr);

}  // namespace fltee
