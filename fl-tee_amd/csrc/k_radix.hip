// k_radix.hip — the stable sort by index of an ordered fold's records (nips19's selected
// list, common.rs:25-35; non_oblivious's sparse fallback, non_oblivious.rs:6-15), and the
// ordered fold that streams the sorted records.
//
// The ordered fold needs the records grouped by idx, each group in list order: a stable
// sort by idx.  The enclave's own loop `g[idx] += val` (common.rs:25-35) walks the list in
// order and touches g[idx] for every entry, so the sequence of indices in list order is
// what its memory trace already shows; a stable LSD counting sort over the idx bits reads
// and scatters by that same sequence and reveals nothing more.  (For non_oblivious the
// reference is not oblivious at all.)
//
// Hand-written LSD counting sort (no library): the key is min(idx, d) (an out-of-range idx
// is flagged and sorts after every index), b = bitlen(d) key bits in P = ceil(b / 8)
// passes of w = ceil(b / P) bits (C4: d = 44,964 -> 2 passes of 8 bits).  The 8-B records
// themselves move, so the fold streams them in sorted order (round 3 gathered each value
// through a position key: 15x its list bytes in HBM traffic).  Per pass, over tiles of
// kCsTile consecutive records (one 256-lane block each):
//   cs_hist     per-tile digit counts, digit-major (pass 0: every pass's, whose row sums
//               cs_rowsum turns into the digit totals — they do not depend on the order —
//               and the idx >= d flag);
//   cs_scan     one block per digit: its base (the totals of the smaller digits) plus the
//               exclusive scan of its per-tile counts -> each tile's first slot per digit;
//   cs_scatter  the tile's stable ranks: per round of 256 records, per wave, the lanes with
//               the same digit found by w ballots (multi-split), their count kept in LDS per
//               (round, wave, digit); one lane per digit scans those groups in position order
//               and the digits' tile totals are scanned; the records are staged in LDS in
//               their sorted order inside the tile, then written out in that order, so the
//               lanes of a wave store runs of one digit to consecutive slots.
#include "common.h"

namespace fltee {

constexpr int kCsNT = 256;                 // lanes per block (4 waves)
constexpr int kCsItems = 8;                // records per lane per tile
constexpr int kCsTile = kCsNT * kCsItems;  // records per tile
constexpr int kCsGroups = kCsItems * (kCsNT / 64);  // (round, wave) groups per tile
constexpr int kCsBins = 256;
// FLTEE_CS_STAGE: cs_scatter stages the tile in LDS and writes it out in sorted order (1) or
// scatters each record straight from its registers (0) — A/B (scripts/ab_build.sh)
#ifndef FLTEE_CS_STAGE
#define FLTEE_CS_STAGE 1
#endif

struct CsPlan {
    uint32_t passes = 0, width = 0;
    size_t tiles = 0;
};

static CsPlan cs_plan(size_t n, size_t d) {
    CsPlan p;
    uint32_t b = 1;
    while (b < 32 && ((size_t)1 << b) <= d) ++b;  // keys 0 .. d (d: out of range)
    p.passes = (b + 7) / 8;
    p.width = (b + p.passes - 1) / p.passes;
    p.tiles = (n + kCsTile - 1) / kCsTile;
    return p;
}

__device__ __forceinline__ uint32_t cs_key(uint64_t r, uint32_t d) {
    const uint32_t idx = rec_idx(r);
    return idx < d ? idx : d;
}

// per-tile digit counts of pass `shift` -> counts[digit][tile]; ALL (pass 0): every pass's
// counts by pass-0 tile, counts + q * kCsBins * ntiles (pass q's only feed its digit totals:
// those do not depend on the order), and the idx >= d flag
template <bool ALL>
__global__ __launch_bounds__(kCsNT) void cs_hist(const uint64_t *__restrict__ src, uint32_t n,
                                                 uint32_t d, uint32_t shift, uint32_t width,
                                                 uint32_t passes, uint32_t ntiles,
                                                 uint32_t *__restrict__ counts, uint32_t *status,
                                                 float *__restrict__ zero, uint32_t nzero) {
    __shared__ uint32_t h[4][kCsBins];  // [pass][digit] (ALL), [0][digit] otherwise
    const uint32_t t = threadIdx.x;
    if constexpr (ALL)  // the fold's output, for the indices without records (+0.0)
        for (uint32_t i = blockIdx.x * kCsNT + t; i < nzero; i += gridDim.x * kCsNT) zero[i] = 0.0f;
    for (uint32_t q = 0; q < 4; ++q) h[q][t] = 0;
    __syncthreads();
    const uint32_t mask = (1u << width) - 1u;
    const uint32_t base = blockIdx.x * (uint32_t)kCsTile;
    uint32_t bad = 0;
#pragma unroll
    for (int r = 0; r < kCsItems; ++r) {
        const uint32_t p = base + (uint32_t)r * kCsNT + t;
        if (p < n) {
            const uint64_t rec = src[p];
            const uint32_t key = cs_key(rec, d);
            if constexpr (ALL) {
                bad |= rec_idx(rec) >= d;
                for (uint32_t q = 0; q < passes; ++q) atomicAdd(&h[q][(key >> (q * width)) & mask], 1u);
            } else {
                atomicAdd(&h[0][(key >> shift) & mask], 1u);
            }
        }
    }
    __syncthreads();
    if (t <= mask) {
        const uint32_t np = ALL ? passes : 1u;
        for (uint32_t q = 0; q < np; ++q)
            counts[((size_t)q * kCsBins + t) * ntiles + blockIdx.x] = h[q][t];
    }
    if constexpr (ALL)
        if (bad) atomicOr(status, FLTEE_DEV_ERR_INDEX_RANGE);
}

// totals[q][digit] = the digit's count over every tile (block (digit, pass))
__global__ __launch_bounds__(kCsNT) void cs_rowsum(const uint32_t *__restrict__ counts,
                                                   uint32_t ntiles, uint32_t *__restrict__ totals) {
    __shared__ uint32_t part[kCsNT / 64];
    const uint32_t dg = blockIdx.x, q = blockIdx.y, t = threadIdx.x;
    const uint32_t *row = counts + ((size_t)q * kCsBins + dg) * ntiles;
    uint32_t x = 0;
    for (uint32_t i = t; i < ntiles; i += kCsNT) x += row[i];
    for (int o = 32; o; o >>= 1) x += __shfl_xor(x, o);
    if ((t & 63) == 0) part[t >> 6] = x;
    __syncthreads();
    if (t == 0) totals[q * kCsBins + dg] = part[0] + part[1] + part[2] + part[3];
}

// block = one digit: offsets[digit][tile] = sum of the smaller digits' totals + exclusive
// prefix over the tiles (in place over counts)
__global__ __launch_bounds__(kCsNT) void cs_scan(uint32_t *__restrict__ counts, uint32_t ntiles,
                                                 const uint32_t *__restrict__ totals) {
    __shared__ uint32_t part[kCsNT / 64];
    __shared__ uint32_t carry_s;
    const uint32_t dg = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    // base: totals of digits < dg
    uint32_t x = t < dg ? totals[t] : 0u;
    for (int o = 32; o; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) part[wv] = x;
    __syncthreads();
    uint32_t carry = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    uint32_t *row = counts + (size_t)dg * ntiles;
    for (uint32_t b0 = 0; b0 < ntiles; b0 += kCsNT) {
        const uint32_t i = b0 + t;
        const uint32_t v = i < ntiles ? row[i] : 0u;
        // inclusive scan inside the wave, then across the 4 waves
        uint32_t inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= (uint32_t)o) inc += y;
        }
        if (lane == 63) part[wv] = inc;
        __syncthreads();
        uint32_t before = carry;
        for (uint32_t w = 0; w < wv; ++w) before += part[w];
        if (i < ntiles) row[i] = before + inc - v;
        if (t == kCsNT - 1) carry_s = before + inc;
        __syncthreads();
        carry = carry_s;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kCsNT) void cs_scatter(const uint64_t *__restrict__ src, uint32_t n,
                                                    uint32_t d, uint32_t shift, uint32_t width,
                                                    uint32_t ntiles,
                                                    const uint32_t *__restrict__ offsets,
                                                    uint64_t *__restrict__ dst) {
    __shared__ uint16_t grp[kCsGroups][kCsBins];  // (round, wave) x digit: count -> offset
    __shared__ uint32_t tile_at[kCsBins];         // the tile's first slot per digit (global)
    __shared__ uint32_t loc_at[kCsBins];          // ... and inside the tile's staged order
    __shared__ uint32_t part[kCsNT / 64];
    __shared__ uint64_t stage[FLTEE_CS_STAGE ? kCsTile : 1];  // the tile's records, sorted
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t mask = (1u << width) - 1u;
    for (int g = 0; g < kCsGroups; ++g) grp[g][t] = 0;
    if (t <= mask) tile_at[t] = offsets[(size_t)t * ntiles + blockIdx.x];
    __syncthreads();
    const uint32_t base = blockIdx.x * (uint32_t)kCsTile;
    const uint32_t live_n = n - base < (uint32_t)kCsTile ? n - base : (uint32_t)kCsTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t rec[kCsItems];
    uint32_t dig[kCsItems], rank[kCsItems];
#pragma unroll
    for (int r = 0; r < kCsItems; ++r) {
        const uint32_t p = base + (uint32_t)r * kCsNT + t;
        const bool live = p < n;
        rec[r] = live ? src[p] : 0ull;
        dig[r] = (cs_key(rec[r], d) >> shift) & mask;
        // the wave's lanes with this lane's digit: one ballot per digit bit
        uint64_t peers = __ballot(live);
        for (uint32_t b = 0; b < width; ++b) {
            const uint64_t m = __ballot((dig[r] >> b) & 1u);
            peers &= ((dig[r] >> b) & 1u) ? m : ~m;
        }
        rank[r] = (uint32_t)__popcll(peers & lt);
        // the lowest peer records the group's count for this digit
        if (live && (peers & lt) == 0) grp[r * (kCsNT / 64) + wv][dig[r]] = (uint16_t)__popcll(peers);
    }
    __syncthreads();
    if constexpr (!FLTEE_CS_STAGE) {  // straight from the registers: global group offsets
        __shared__ uint32_t gofs[kCsGroups][kCsBins];
        uint32_t run = t <= mask ? tile_at[t] : 0u;
#pragma unroll
        for (int g = 0; g < kCsGroups; ++g) {
            gofs[g][t] = run;
            run += grp[g][t];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kCsItems; ++r)
            if (base + (uint32_t)r * kCsNT + t < n)
                dst[gofs[r * (kCsNT / 64) + wv][dig[r]] + rank[r]] = rec[r];
        return;
    }
    // lane t = digit t: exclusive scan of its counts over the groups in position order, then
    // of the digits' tile totals (the staged order: digit by digit, stable within a digit)
    uint32_t tot;
    {
        uint32_t v[kCsGroups];
#pragma unroll
        for (int g = 0; g < kCsGroups; ++g) v[g] = grp[g][t];
        uint32_t run = 0;
#pragma unroll
        for (int g = 0; g < kCsGroups; ++g) {
            const uint32_t c = v[g];
            v[g] = run;
            run += c;
        }
#pragma unroll
        for (int g = 0; g < kCsGroups; ++g) grp[g][t] = (uint16_t)v[g];
        tot = run;
    }
    uint32_t inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) part[wv] = inc;
    __syncthreads();
    uint32_t ex = inc - tot;
    for (uint32_t w = 0; w < wv; ++w) ex += part[w];
    loc_at[t] = ex;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kCsItems; ++r)
        if (base + (uint32_t)r * kCsNT + t < n)
            stage[loc_at[dig[r]] + grp[r * (kCsNT / 64) + wv][dig[r]] + rank[r]] = rec[r];
    __syncthreads();
    // the staged records in order: runs of one digit go to consecutive global slots
#pragma unroll
    for (int r = 0; r < kCsItems; ++r) {
        const uint32_t j = (uint32_t)r * kCsNT + t;
        if (j < live_n) {
            const uint64_t x = stage[j];
            const uint32_t dg = (cs_key(x, d) >> shift) & mask;
            dst[tile_at[dg] + (j - loc_at[dg])] = x;
        }
    }
}

size_t radix_scratch_bytes(size_t n, size_t d) {
    const CsPlan p = cs_plan(n, d);
    const size_t counts = (size_t)p.passes * kCsBins * (p.tiles ? p.tiles : 1) * 4;
    return ((n * 8 + 255) & ~(size_t)255) + ((counts + 255) & ~(size_t)255) + 4 * kCsBins * 4;
}

hipError_t launch_sort_records_by_idx(const void *rec, size_t n, size_t d, void *scratch,
                                      size_t bytes, uint64_t *sorted, uint32_t *status,
                                      float *zero, size_t nzero, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0x7FFFFFFFull || d > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (bytes < radix_scratch_bytes(n, d)) return hipErrorOutOfMemory;
    const CsPlan p = cs_plan(n, d);
    uint64_t *tmp = (uint64_t *)scratch;
    uint32_t *counts = (uint32_t *)((char *)scratch + ((n * 8 + 255) & ~(size_t)255));
    uint32_t *totals = counts + (((size_t)p.passes * kCsBins * p.tiles * 4 + 255) & ~(size_t)255) / 4;
    const uint32_t nt = (uint32_t)p.tiles, nb = 1u << p.width;
    const uint64_t *src = (const uint64_t *)rec;
    FLTEE_LAUNCH(cs_hist<true>, dim3(nt), dim3(kCsNT), 0, s, src, (uint32_t)n, (uint32_t)d, 0u,
                       p.width, p.passes, nt, counts, status, zero, (uint32_t)(zero ? nzero : 0));
    FLTEE_LAUNCH(cs_rowsum, dim3(nb, p.passes), dim3(kCsNT), 0, s, (const uint32_t *)counts, nt,
                       totals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (uint32_t q = 0; q < p.passes; ++q) {
        // the passes alternate between tmp and sorted, ending in sorted
        uint64_t *dst = ((p.passes - 1 - q) & 1) ? tmp : sorted;
        const uint32_t shift = q * p.width;
        if (q > 0)  // this pass's counts by ITS tiles (pass 0's came with the totals)
            FLTEE_LAUNCH(cs_hist<false>, dim3(nt), dim3(kCsNT), 0, s, src, (uint32_t)n,
                               (uint32_t)d, shift, p.width, p.passes, nt, counts, status, nullptr, 0u);
        FLTEE_LAUNCH(cs_scan, dim3(nb), dim3(kCsNT), 0, s, counts, nt, totals + q * kCsBins);
        FLTEE_LAUNCH(cs_scatter, dim3(nt), dim3(kCsNT), 0, s, src, (uint32_t)n, (uint32_t)d,
                           shift, p.width, nt, (const uint32_t *)counts, dst);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        src = dst;
    }
    return hipSuccess;
}

// ----------------------------------------------------- the ordered fold ---
// out[i] = ((+0 + v1) + v2) ... over index i's records in sorted (= list) order, the order
// of non_oblivious.rs:11-13 and common.rs:25-35; x coef, or accumulate: out[i] += sum.
// (Without accumulate the indices without records hold +0.0: cs_hist zero-fills out.)
// One wave per kFoldCh x 64 sorted records, all loaded up front with one chunk more (one
// memory latency per wave): the run heads among them (a record whose predecessor has
// another idx) are folded one after the other, each by the whole wave — 64 records at a
// time added in lane order by readlane (a uniform serial chain: the exact left fold),
// further chunks read only while a run goes on past the preloaded ones.  (Tried: one LANE
// per run, the segment staged in LDS and each run read at known offsets — C4 8.36 vs
// 8.32 ms with this kernel, `profiles/r04/ab/ab4_fold_lane_per_run_c4_rejected.jsonl`.)
constexpr int kFoldCh = 4;

__device__ __forceinline__ float fold_lanes(float acc, int vb, int from, int to) {
    for (int j = from; j < to; ++j) acc = __fadd_rn(acc, __int_as_float(__builtin_amdgcn_readlane(vb, j)));
    return acc;
}

template <bool ACC>
__global__ __launch_bounds__(256) void fold_chunks_kernel(const uint64_t *__restrict__ srt,
                                                          uint32_t n, uint32_t d, float coef,
                                                          float *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (64u * kFoldCh);
    if (w0 >= n) return;  // uniform per wave
    uint64_t r[kFoldCh + 1];
#pragma unroll
    for (int c = 0; c <= kFoldCh; ++c) {
        const uint32_t q = w0 + (uint32_t)c * 64u + lane;
        r[c] = q < n ? srt[q] : 0ull;
    }
    const uint32_t before = w0 == 0 ? 0xFFFFFFFFu : rec_idx(srt[w0 - 1]);
#pragma unroll
    for (int c = 0; c < kFoldCh; ++c) {
        const uint32_t q0 = w0 + (uint32_t)c * 64u;
        if (q0 >= n) break;
        const uint32_t q = q0 + lane;
        const bool live = q < n;
        const uint32_t idx = live ? rec_idx(r[c]) : 0xFFFFFFFFu;
        uint32_t prev = (uint32_t)__shfl_up((int)idx, 1);
        if (lane == 0)
            prev = c == 0 ? before : (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)r[c > 0 ? c - 1 : 0], 63);
        const bool first = q == 0;
        // a head of an in-range run, or the first out-of-range record (ends the gaps)
        const bool head = live && (first || prev != idx) && (idx < d || first || prev < d);
        uint64_t heads = __ballot(head);
        const int vb = (int)(uint32_t)(r[c] >> 32);
        while (heads) {
            const uint32_t h = (uint32_t)__builtin_ctzll(heads);
            heads &= heads - 1;
            const uint32_t i = (uint32_t)__builtin_amdgcn_readlane((int)idx, (int)h);
            const uint32_t pv = (uint32_t)__builtin_amdgcn_readlane((int)prev, (int)h);
            (void)pv;
            if (i >= d) continue;
            // the run's records among these 64 lanes: lanes h .. h + cnt - 1 (contiguous)
            const int cnt = __popcll(__ballot(idx == i));
            float acc = fold_lanes(0.0f, vb, (int)h, (int)h + cnt);
            bool more = (int)h + cnt == 64;  // the run goes on past this chunk
#pragma unroll
            for (int cc = c + 1; cc <= kFoldCh; ++cc) {
                if (more) {
                    const bool same = w0 + (uint32_t)cc * 64u + lane < n && rec_idx(r[cc]) == i;
                    const int k2 = __popcll(__ballot(same));
                    acc = fold_lanes(acc, (int)(uint32_t)(r[cc] >> 32), 0, k2);
                    more = k2 == 64;
                }
            }
            for (uint32_t p = w0 + (uint32_t)(kFoldCh + 1) * 64u; more; p += 64) {
                const uint32_t qq = p + lane;
                const uint64_t rr = qq < n ? srt[qq] : 0ull;
                const int k2 = __popcll(__ballot(qq < n && rec_idx(rr) == i));
                acc = fold_lanes(acc, (int)(uint32_t)(rr >> 32), 0, k2);
                more = k2 == 64;
            }
            if (lane == 0) out[i] = ACC ? __fadd_rn(out[i], acc) : __fmul_rn(acc, coef);
        }
    }
}


hipError_t launch_fold_sorted(const uint64_t *sorted, size_t n, size_t d, float coef, float *out,
                              bool accumulate, hipStream_t s) {
    if (d == 0 || n == 0) return hipSuccess;
    if (n > 0x7FFFFFFFull || d > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((n + 256 * kFoldCh - 1) / (256 * kFoldCh));
    if (accumulate)
        FLTEE_LAUNCH(fold_chunks_kernel<true>, dim3(blocks), dim3(256), 0, s, sorted,
                           (uint32_t)n, (uint32_t)d, coef, out);
    else
        FLTEE_LAUNCH(fold_chunks_kernel<false>, dim3(blocks), dim3(256), 0, s, sorted,
                           (uint32_t)n, (uint32_t)d, coef, out);
    return hipGetLastError();
}

// the composite-key order (fltee_debug_set_radix_order(0)): the records gathered by the
// sorted (idx << 32 | position) keys
__global__ void gather_by_keys_kernel(const uint64_t *__restrict__ keys, size_t n,
                                      const uint64_t *__restrict__ rec, uint64_t *__restrict__ dst) {
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (size_t)gridDim.x * 256)
        dst[p] = rec[(uint32_t)keys[p]];
}

hipError_t launch_gather_by_keys(const uint64_t *keys, size_t n, const void *rec, uint64_t *dst,
                                 hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    FLTEE_LAUNCH(gather_by_keys_kernel, dim3((unsigned)blocks), dim3(256), 0, s, keys, n,
                       (const uint64_t *)rec, dst);
    return hipGetLastError();
}

}  // namespace fltee
