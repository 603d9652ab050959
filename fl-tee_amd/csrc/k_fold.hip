// k_fold.hip — the `advanced` pipeline around the bitonic network (gfx950).
//
// advanced.rs:39-113 on the device:
//   advanced_init  : records ++ (i, 0.0) for i < d (:116-123) ++ (u32::MAX, 0.0)
//                    pads to M = next_pow2 (:133-142)
//   [bitonic sort, mode 0]
//   fold           : the oblivious fold (:66-101), EXACT and oblivious:
//   [second sort -> k_compact.hip, or bitonic sort mode 0 for the k quirk]
//   extract        : global[i] = v[i].1 (:32-34) * 1f32/n (common.rs:14-19)
//
// The fold.  The enclave walks the sorted array once, carrying (pre_idx,
// pre_val): position p-1 receives (u32::MAX - (p-1), 0.0) if p continues the
// run of p-1, else the run's left-to-right sum.  A parallel scan would
// re-associate that sum.  Instead every lane folds its own chunk of C
// positions sequentially, after re-folding the Hr >= H positions in front of
// it (the halo): whenever the run crossing the chunk start began inside the
// halo, the carry entering the chunk is bit-identical to the enclave's.  With
// each client's indices distinct (top-k, utils.py:327-354) a run holds at most
// n+1 records, so H = n.  Every lane performs the same Hr+C+16 steps whatever the
// data (oblivious).
//
// Runs of any length (round 6).  A run that began before a lane's walk start b (a
// client repeated an index: more than Hr + 1 entries) ends in that lane's chunk with a
// sum missing its part before b.  The lane emits a dummy at that run end instead and
// leaves a side record (FoldSide): the run's key and its sum over [b, end], and — for
// every lane — the aggregate of its piece [b, b + C) (first key, last key, one key or
// not, and the in-order partial of the run ending the piece).  The walk starts are C
// apart, so the pieces tile the array.  fold_patch_kernel then scans the pieces
// (segmented: a run's partials add up only while the key goes on) and writes, at every
// lane's first position a (a fixed address, whatever the data), either what the fold
// left there or — for a lane with such a run — (key, carry + sum): a inside that run,
// the one record of its key.  Exact (bit for bit) for every run inside one lane's walk,
// the enclave's sum re-associated at the walk boundaries otherwise (north_star's 1e-6
// relative tolerance for the aggregate).  No run-length limit, no rerun.
//
// Layout: C >= Hr on large arrays (halo work <= 2x; small arrays take shorter
// chunks, down to 16, to keep ~1024 waves in flight), so a lane walks a long chunk; the 64
// lanes of a wave walk 64 chunks in lockstep, 16 records per stage.  A stage's
// 64 windows of 16 records (128 B each) are loaded coalesced (8 lanes per
// window) one stage ahead into registers, transposed through LDS (row stride
// 17 records: conflict-free 8-B reads), folded, and the outputs go back out
// through the same LDS rows as coalesced 128-B stores.  No block barriers:
// every wave works alone.
#include "common.h"

namespace fltee {

// dst[x] = entry pbase + x of the padded array; rec[x] is the record at position
// pbase + x (read only where pbase + x < nrec).  pbase = 0: the whole array.
__global__ void advanced_init_kernel(const uint64_t *__restrict__ rec, size_t nrec, size_t d,
                                     size_t pbase, size_t m, uint64_t *__restrict__ dst) {
    for (size_t x = (size_t)blockIdx.x * 256 + threadIdx.x; x < m; x += (size_t)gridDim.x * 256) {
        const size_t p = pbase + x;
        uint64_t v;
        if (p < nrec) v = rec[x];
        else if (p < nrec + d) v = (uint64_t)(uint32_t)(p - nrec);  // (i, +0.0)
        else v = (uint64_t)0xFFFFFFFFu;                               // (u32::MAX, +0.0)
        dst[x] = v;
    }
}

hipError_t launch_advanced_init_range(const void *rec, size_t nrec, size_t d, size_t pbase,
                                      size_t m, uint64_t *dst, hipStream_t s) {
    if (m == 0) return hipSuccess;
    size_t blocks = (m + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    FLTEE_LAUNCH(advanced_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint64_t *)rec, nrec, d, pbase, m, dst);
    return hipGetLastError();
}

hipError_t launch_advanced_init(const void *rec, size_t nrec, size_t d, size_t m, uint64_t *dst,
                                hipStream_t s) {
    return launch_advanced_init_range(rec, nrec, d, 0, m, dst, s);
}

constexpr uint32_t FS_W = 16;    // records per window (one 128-B line)
constexpr uint32_t FS_ROW = 17;  // LDS row stride in records (conflict-free lane reads)
typedef unsigned int fs_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One wave per block; lane l of wave w owns positions [a, a + C), a = origin + (w*64 + l)*C,
// up to `end`.  Positions are local to src/dst (length m); pbase + position is the
// global position, which decides fold_len and the dummies' idx.  Range mode (one
// GPU's part of a position-sharded array, SURVEY §8e Option B): [0, origin) holds
// >= Hr + 1 records of context from the previous range, and src[end] is the next
// range's first record (or end + pbase >= fold_len).
// CEMIT (round 5): emit what the compaction's first pass would make of the folded array
// — a run's last record as (sum, c = p - idx) when idx < dsel, every other position as the
// compaction's unselected slot `cdummy` — so that pass needs no conversion (and may move
// 16-B slot pairs); positions past fold_len are copied as before.
// side (nullptr: the one-lane walk, which has no boundary): the lane's FoldSide record.
template <int DEPTH, bool CEMIT = false>
__global__ __launch_bounds__(64) void fold_stream_kernel(const uint64_t *__restrict__ src,
                                                         uint64_t *__restrict__ dst, long long m,
                                                         long long origin, long long end,
                                                         long long pbase, long long fold_len,
                                                         uint32_t Hr, uint32_t C,
                                                         FoldSide *__restrict__ side,
                                                         uint32_t dsel = 0, uint64_t cdummy = 0) {
    __shared__ uint64_t win[2][64 * FS_ROW];
    const uint32_t l = threadIdx.x;
    const long long wave0 = origin + (long long)blockIdx.x * 64 * C;  // first position of lane 0
    const long long a = wave0 + (long long)l * C;
    const long long b = a - (long long)Hr;  // the walk's first position (the piece start)
    const uint32_t nstage = (Hr + C + FS_W) / FS_W;
    const uint32_t hw = Hr / FS_W;  // stage s holds window u = s - hw of the chunk

    // the side record's walk-invariant inputs: the key at the walk's first real position
    // (b, or global position 0 for the array's first lanes) and whether the run there began
    // before the walk (the key in front of it)
    uint32_t pf_key = 0;
    bool in_head = false;
    if (side && a < end) {
        long long fp = b + pbase < 0 ? -pbase : b;
        fp = fp < 0 ? 0 : fp;
        if (fp < m) pf_key = rec_idx(src[fp]);
        if (b - 1 >= 0 && b - 1 + pbase >= 0) in_head = rec_idx(src[b - 1]) == pf_key;
    }

    // cooperative window loads: piece p = l + 64 i -> window w = p >> 3, 16-B part p & 7
    const uint32_t part = (l & 7) * 2;
    // prefetch DEPTH stages ahead (pf[s % DEPTH] holds stage s).  Deeper prefetch helps
    // when there are few waves (small m, or long chunks: the load latency sets the time);
    // one is faster at full chip occupancy (C5 at C = 1024: 692 vs 741 us for two).
    fs_u32x4 pf[DEPTH][8];
    auto load_stage = [&](fs_u32x4 (&pf)[8], uint32_t s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t w = (l >> 3) + 8 * i;
            const long long g = wave0 + (long long)w * C - Hr + (long long)s * FS_W + part;
            if (g >= 0 && g < m) {
                pf[i] = __builtin_nontemporal_load((const fs_u32x4 *)(src + g));
            } else {
                pf[i] = fs_u32x4{0u, 0u, 0u, 0u};
            }
        }
    };
#pragma unroll
    for (int q = 0; q < DEPTH; ++q)
        if ((uint32_t)q < nstage) load_stage(pf[q], (uint32_t)q);

    // pre_idx starts as a key no run has before the walk's first real record: an index
    // >= d (0xFFFFFFFE: a client's out-of-range index at worst, whose sums never reach the
    // output) instead of a separate `started` flag
    uint32_t pre_idx = 0xFFFFFFFEu;
    float pre_val = 0.0f;
    uint64_t prev = 0;
    // the side record: the piece [b, b + C) and the head run (the one holding b)
    bool corr = false, piece = false;
    uint32_t pk = 0;
    float pq = 0.0f, cs = 0.0f;
    auto stage = [&](fs_u32x4 (&pf)[8], uint32_t s) {
        uint64_t *cur = win[s & 1], *old = win[(s + 1) & 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t w = (l >> 3) + 8 * i;
            cur[w * FS_ROW + part] = ((uint64_t)pf[i].y << 32) | pf[i].x;
            cur[w * FS_ROW + part + 1] = ((uint64_t)pf[i].w << 32) | pf[i].z;
        }
        if (s + DEPTH < nstage) load_stage(pf, s + DEPTH);
        wave_sync_lds();
        uint64_t r[FS_W];
#pragma unroll
        for (uint32_t t = 0; t < FS_W; ++t) r[t] = cur[l * FS_ROW + t];
        const long long q0 = a - (long long)Hr + (long long)s * FS_W;
        // step t of stage s emits b + 16 s + t - 1, inside the chunk for 16 s + t in
        // [Hr + 1, Hr + C] (Hr and C multiples of 16): stage-uniform flags for t = 0 and t > 0
        const uint32_t cs_end = hw + C / FS_W;
        const bool in1 = s >= hw && s < cs_end, in0 = s > hw && s <= cs_end;
        // the step's position tests as thresholds on t, once a stage (step t reads q = q0 + t,
        // global qg = qg0 + t): copy <=> qg - 1 >= fold_len, live <=> qg < fold_len, valid
        // <=> q >= 0 && qg >= 0 — a 32-bit compare with the step's constant each instead of
        // 64-bit position arithmetic a step
        const long long qg0 = q0 + pbase;
        auto tclamp = [](long long x) -> uint32_t { return x < 0 ? 0u : (x > 17 ? 17u : (uint32_t)x); };
        uint32_t t_copy = tclamp(fold_len + 1 - qg0), t_live = tclamp(fold_len - qg0);
        uint32_t t_valid = tclamp(-q0 > -qg0 ? -q0 : -qg0);
        // (opaque to the optimizer, which otherwise folds each test back into a 64-bit
        // compare of the unclamped difference)
        asm volatile("" : "+v"(t_copy), "+v"(t_live), "+v"(t_valid));
        const uint32_t pe0 = (uint32_t)(qg0 - 1);  // (uint32_t)(qg - 1) = pe0 + t
#pragma unroll
        for (uint32_t t = 0; t < FS_W; ++t) {
            const uint32_t ci = rec_idx(r[t]);
            const bool eq = ci == pre_idx;
            const bool copy = t >= t_copy, dmy = t < t_live && eq;
            // the head run ends at q - 1: inside the chunk (step si in [Hr + 1, Hr + C], a
            // wave-uniform test) it is the one the side record carries (emitted as a dummy
            // here, its record written by fold_patch_kernel)
            const bool inchunk = t == 0 ? in0 : in1;  // emits inside [a, a + C)
            const bool sup = in_head && !copy && !dmy && inchunk;
            uint64_t emit;
            if constexpr (CEMIT) {
                // (the record computed whatever the case, then selected: no EXEC-mask
                // branch around it)
                uint64_t rec = make_rec(pe0 + t - pre_idx, pre_val);  // (c, sum)
                asm volatile("" : "+v"(rec));
                emit = copy ? prev : dmy || sup || pre_idx >= dsel ? cdummy : rec;
            } else {
                emit = copy ? prev
                       : dmy || sup ? (uint64_t)(0xFFFFFFFFu - (pe0 + t))  // (MAX-p, +0.0)
                                    : make_rec(pre_idx, pre_val);
            }
            // (value selects: a store through a selected address would put these flags on
            // the stack)
            cs = sup ? pre_val : cs;
            corr = corr || sup;
            in_head = in_head && (dmy || (t == 0 && s == 0));  // (step 0 emits b - 1)
            if (t == 0) old[l * FS_ROW + FS_W - 1] = emit;
            else cur[l * FS_ROW + t - 1] = emit;
            const bool valid = t >= t_valid;
            // (selects: no EXEC-mask branch a step)
            const float nv = eq ? __fadd_rn(pre_val, rec_val(r[t])) : rec_val(r[t]);
            pre_val = valid ? nv : pre_val;
            pre_idx = valid ? ci : pre_idx;
            // the piece's last position b + C - 1: its run partial
            if (t == FS_W - 1 && s == C / FS_W - 1) {
                piece = valid;
                pk = pre_idx;
                pq = pre_val;
            }
            prev = r[t];
        }
        wave_sync_lds();
        // window u = s - 1 - hw of every chunk is complete in `old`: store it
        const long long u = (long long)s - 1 - hw;
        if (u >= 0 && u < (long long)(C / FS_W)) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t w = (l >> 3) + 8 * i;
                const long long g = wave0 + (long long)w * C + u * FS_W + part;
                if (g < end) {
                    const uint64_t x0 = old[w * FS_ROW + part], x1 = old[w * FS_ROW + part + 1];
                    const fs_u32x4 v = {(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1,
                                        (uint32_t)(x1 >> 32)};
                    __builtin_nontemporal_store(v, (fs_u32x4 *)(dst + g));
                }
            }
        }
        wave_sync_lds();
    };
    for (uint32_t s = 0; s < nstage; s += DEPTH) {
#pragma unroll
        for (int q = 0; q < DEPTH; ++q)
            if (s + (uint32_t)q < nstage) stage(pf[q], s + (uint32_t)q);
    }
    if (side) {
        const bool live = a < end;
        // (sorted: the piece is one key iff its first and last keys are equal)
        const uint32_t fl = live ? ((piece ? kFsPiece : 0u) | (piece && pk == pf_key ? kFsFull : 0u) |
                                    (corr ? kFsCorr : 0u))
                                 : 0u;
        if (live) {
            FoldSide *o = side + (size_t)blockIdx.x * 64 + l;
            o->F = pf_key;
            o->K = pk;
            o->Q = pq;
            o->fl = fl;
            o->ck = pf_key;  // the head run's key
            o->S = cs;
        }
        // the wave's aggregate of its 64 pieces (in lane order), for the patch's carries
        FoldAgg g;
        g.F = pf_key;
        g.K = pk;
        g.Q = pq;
        g.fl = fl & (kFsPiece | kFsFull);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            FoldAgg y;
            y.F = (uint32_t)__shfl_up((int)g.F, o);
            y.K = (uint32_t)__shfl_up((int)g.K, o);
            y.Q = __shfl_up(g.Q, o);
            y.fl = (uint32_t)__shfl_up((int)g.fl, o);
            if (l >= (uint32_t)o) g = fa_combine(y, g);
        }
        if (l == 63) fold_wave_aggs(side, gridDim.x)[blockIdx.x] = g;
    }
}

size_t fold_context(size_t halo) { return (halo + FS_W - 1) / FS_W * FS_W; }

#ifndef FLTEE_FS_DOUBLE_WAVES
#define FLTEE_FS_DOUBLE_WAVES 1024
#endif
// The chunk length of a fold over span positions with this halo (0: the one-lane walk
// over the whole array, origin = pbase = 0 only).
static size_t fold_chunk(size_t span, size_t Hr) {
    size_t C = 64;
    while (C < Hr) C <<= 1;
    // keep >= ~1024 waves: shorter chunks re-read more halo but put more loads in flight
    // (C3, M = 2^20, Hr = 112: C = 16 gives 19.7 us against 25.5 us at C = 64)
    while (C > FS_W && span / (64 * C) < 1024) C >>= 1;
    // one doubling more while >= 1024 waves remain: less halo re-read (C5: 2048 instead
    // of 1024, 620 vs 643 us; 4096: 700 us, 8192: 1220 us — too few waves in flight)
    if (C >= Hr && span / (64 * 2 * C) >= FLTEE_FS_DOUBLE_WAVES) C <<= 1;
    return C;
}

static bool one_lane(size_t span, size_t fold_len, size_t halo, size_t origin, long long pbase) {
    return (halo + 1 >= span || halo + 1 >= fold_len) && origin == 0 && pbase == 0;
}

size_t fold_lanes(size_t span, size_t fold_len, size_t halo, size_t origin, long long pbase) {
    if (one_lane(span, fold_len, halo, origin, pbase)) return 0;
    const size_t C = fold_chunk(span, fold_context(halo));
    return (span + C - 1) / C;
}

hipError_t launch_fold_range(const uint64_t *src, uint64_t *dst, size_t m, size_t origin,
                             size_t end, long long pbase, size_t fold_len, size_t halo,
                             FoldSide *side, hipStream_t s, size_t cemit_d, uint64_t cdummy) {
    const bool cemit = cemit_d != 0;
    if (cemit && (origin != 0 || pbase != 0 || cemit_d > 0xFFFFFFFFull)) return hipErrorInvalidValue;
    if (end > m || origin >= end || (m & 1) || (origin & 1) || (end & 1)) return hipErrorInvalidValue;
    const size_t span = end - origin;
    if (one_lane(span, fold_len, halo, origin, pbase)) {
        // a halo as long as the array (the exact-runs policy: the public worst case n*k + 1
        // entries per run): ONE lane folds the whole array from position 0, the enclave's
        // own sequential walk (advanced.rs:66-101) — exact for any run, span/16 stages
        // whatever the data.  No halo to re-read, no boundary, no side record.
        const size_t C1 = (span + FS_W - 1) / FS_W * FS_W;
        if (C1 > 0x7FFFFFFFull) return hipErrorInvalidValue;
        net_account((uint64_t)16 * span, "fold_stream_kernel", s);
        if (cemit)
            FLTEE_LAUNCH((fold_stream_kernel<2, true>), dim3(1), dim3(64), 0, s, src, dst,
                               (long long)m, 0ll, (long long)end, 0ll, (long long)fold_len, 0u,
                               (uint32_t)C1, (FoldSide *)nullptr, (uint32_t)cemit_d, cdummy);
        else
            FLTEE_LAUNCH(fold_stream_kernel<2>, dim3(1), dim3(64), 0, s, src, dst, (long long)m,
                               0ll, (long long)end, 0ll, (long long)fold_len, 0u, (uint32_t)C1,
                               (FoldSide *)nullptr, 0u, 0ull);
        return hipGetLastError();
    }
    if (!side) return hipErrorInvalidValue;
    const size_t Hr = fold_context(halo);
    if (Hr > ((size_t)1 << 30)) return hipErrorInvalidValue;
    // range mode reads the record in front of the first walk (the context holds Hr + 1)
    if (origin != 0 && origin < Hr + 1) return hipErrorInvalidValue;
    const size_t C = fold_chunk(span, Hr);
    const size_t lanes = (span + C - 1) / C;
    const size_t blocks = (lanes + 63) / 64;
    net_account((uint64_t)16 * span, "fold_stream_kernel", s);
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    // about one wave per CU: latency-bound, prefetch deeper (2 or 4 stages were no faster
    // on the large arrays, profiles/r01/ab/fold_chunk_depth*.jsonl)
    const int depth = blocks <= 256 ? 2 : 1;
#define FS_GO(D_, E_)                                                                              \
    FLTEE_LAUNCH((fold_stream_kernel<D_, E_>), dim3((unsigned)blocks), dim3(64), 0, s, src,  \
                       dst, (long long)m, (long long)origin, (long long)end, pbase,                \
                       (long long)fold_len, (uint32_t)Hr, (uint32_t)C, side, (uint32_t)cemit_d,    \
                       cdummy)
    if (depth == 2) {
        if (cemit) FS_GO(2, true);
        else FS_GO(2, false);
    } else {
        if (cemit) FS_GO(1, true);
        else FS_GO(1, false);
    }
#undef FS_GO
    return hipGetLastError();
}

// ---- the long-run patch (see the header) ----------------------------------------
// The patch: lanes of 1,024 per block (256 threads x 4).  A block's carry = the totals of
// the ranges before (prev[0, nprev), in order) then the wave aggregates of every wave in
// front of its lanes (the fold kernel's, 64 lanes each; read in slices by the block's
// threads, combined in order by a block scan), then its own lanes' exclusive scan.
// PATCH: dst[a_j] for every lane j (read, then written back or replaced: fixed addresses);
// else (one block): *total = the aggregate of all the waves.
constexpr int kFpNT = 256, kFpPer = 4, kFpLanes = kFpNT * kFpPer;

// the inclusive scan of part[0, kFpNT) in LDS (x before y: order kept); returns part[t]
__device__ FoldAgg fp_block_scan(FoldAgg *part, uint32_t t, FoldAgg v) {
    part[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < kFpNT; o <<= 1) {
        const FoldAgg y = part[t];
        const FoldAgg x = t >= o ? part[t - o] : fa_empty();
        __syncthreads();
        part[t] = fa_combine(x, y);
        __syncthreads();
    }
    return part[t];
}

template <bool PATCH, bool CEMIT>
__global__ __launch_bounds__(kFpNT) void fold_patch_kernel(const FoldSide *__restrict__ side,
                                                           uint32_t G, uint32_t W,
                                                           uint64_t *__restrict__ dst,
                                                           long long origin, uint32_t C,
                                                           long long pbase,
                                                           const FoldAgg *__restrict__ prev,
                                                           uint32_t nprev, FoldAgg *total,
                                                           uint32_t dsel, uint64_t cdummy) {
    __shared__ FoldAgg part[kFpNT];
    const uint32_t t = threadIdx.x;
    const FoldAgg *wagg = fold_wave_aggs(const_cast<FoldSide *>(side), W);
    // the waves in front of this block's lanes (all of them for the total)
    const uint32_t wb = PATCH ? blockIdx.x * (kFpLanes / 64) : W;
    FoldAgg acc = fa_empty();
    {
        const uint32_t w0 = (uint32_t)((uint64_t)wb * t / kFpNT);
        const uint32_t w1 = (uint32_t)((uint64_t)wb * (t + 1) / kFpNT);
        for (uint32_t w = w0; w < w1; ++w) acc = fa_combine(acc, wagg[w]);
    }
    const FoldAgg front = fp_block_scan(part, t, acc), allw = part[kFpNT - 1];
    (void)front;
    if constexpr (!PATCH) {
        if (t == 0) *total = allw;
        return;
    } else {
        FoldAgg carry = fa_empty();
        for (uint32_t i = 0; i < nprev; ++i) carry = fa_combine(carry, prev[i]);
        carry = fa_combine(carry, allw);
        __syncthreads();  // part[] is reused
        const uint32_t j0 = blockIdx.x * kFpLanes + t * kFpPer;
        FoldSide sd[kFpPer];
        FoldAgg mine = fa_empty();
#pragma unroll
        for (int i = 0; i < kFpPer; ++i) {
            if (j0 + i < G) {
                sd[i] = side[j0 + i];
                mine = fa_combine(mine, fa_of(sd[i]));
            }
        }
        const FoldAgg inc = fp_block_scan(part, t, mine);
        (void)inc;
        FoldAgg run = fa_combine(carry, t > 0 ? part[t - 1] : fa_empty());
#pragma unroll
        for (int i = 0; i < kFpPer; ++i) {
            const uint32_t j = j0 + i;
            if (j >= G) break;
            const long long aj = origin + (long long)j * C;
            const uint64_t was = dst[aj];
            // a lane with a run begun before its walk: the run's key is the one in front of
            // the walk, the last key of the pieces before (run.K)
            const bool c = (sd[i].fl & kFsCorr) && (run.fl & kFsPiece) && run.K == sd[i].ck;
            const float tot = __fadd_rn(run.Q, sd[i].S);
            uint64_t rec;
            if constexpr (CEMIT)
                rec = sd[i].ck < dsel ? make_rec((uint32_t)(aj + pbase) - sd[i].ck, tot) : cdummy;
            else
                rec = make_rec(sd[i].ck, tot);
            dst[aj] = c ? rec : was;
            run = fa_combine(run, fa_of(sd[i]));
        }
    }
}

size_t fold_side_bytes(size_t span, size_t fold_len, size_t halo, size_t origin, long long pbase) {
    const size_t waves = (fold_lanes(span, fold_len, halo, origin, pbase) + 63) / 64;
    return waves * (64 * sizeof(FoldSide) + sizeof(FoldAgg));
}

hipError_t launch_fold_range_total(const FoldSide *side, size_t lanes, FoldAgg *total,
                                   hipStream_t s) {
    const size_t waves = (lanes + 63) / 64;
    if (waves > 0xFFFFFFFFull) return hipErrorInvalidValue;
    FLTEE_LAUNCH((fold_patch_kernel<false, false>), dim3(1), dim3(kFpNT), 0, s, side,
                       (uint32_t)lanes, (uint32_t)waves, (uint64_t *)nullptr, 0ll, 0u, 0ll,
                       (const FoldAgg *)nullptr, 0u, total, 0u, 0ull);
    return hipGetLastError();
}

hipError_t launch_fold_range_patch(uint64_t *dst, size_t span, size_t origin, long long pbase,
                                   size_t fold_len, size_t halo, const FoldSide *side,
                                   const FoldAgg *prev, size_t nprev, hipStream_t s,
                                   size_t cemit_d, uint64_t cdummy) {
    const size_t lanes = fold_lanes(span, fold_len, halo, origin, pbase);
    if (lanes == 0) return hipSuccess;  // the one-lane walk: nothing to patch
    if (lanes > 0xFFFFFFFFull || nprev > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const size_t C = fold_chunk(span, fold_context(halo));
    const size_t waves = (lanes + 63) / 64;
    const unsigned blocks = (unsigned)((lanes + kFpLanes - 1) / kFpLanes);
    net_account((uint64_t)sizeof(FoldSide) * lanes + 16 * lanes, "fold_patch_kernel", s);
    if (cemit_d)
        FLTEE_LAUNCH((fold_patch_kernel<true, true>), dim3(blocks), dim3(kFpNT), 0, s, side,
                           (uint32_t)lanes, (uint32_t)waves, dst, (long long)origin, (uint32_t)C,
                           pbase, prev, (uint32_t)nprev, (FoldAgg *)nullptr, (uint32_t)cemit_d,
                           cdummy);
    else
        FLTEE_LAUNCH((fold_patch_kernel<true, false>), dim3(blocks), dim3(kFpNT), 0, s, side,
                           (uint32_t)lanes, (uint32_t)waves, dst, (long long)origin, (uint32_t)C,
                           pbase, prev, (uint32_t)nprev, (FoldAgg *)nullptr, 0u, 0ull);
    return hipGetLastError();
}

hipError_t launch_fold(const uint64_t *src, uint64_t *dst, size_t m, size_t fold_len, size_t halo,
                       void *side_ws, size_t side_cap, hipStream_t s, size_t cemit_d,
                       uint64_t cdummy) {
    if (m == 1 && !cemit_d)  // nothing to fold: position 0 receives itself (:102-103)
        return fl_memcpy_async(dst, src, 8, hipMemcpyDeviceToDevice, s);
    if (m == 0 || (m & 1)) return hipErrorInvalidValue;  // m = next_pow2: 16-B windows
    if (side_cap < fold_side_bytes(m, fold_len, halo, 0, 0)) return hipErrorInvalidValue;
    FoldSide *side = (FoldSide *)side_ws;
    hipError_t e = launch_fold_range(src, dst, m, 0, m, 0, fold_len, halo, side, s, cemit_d, cdummy);
    if (e == hipSuccess)
        e = launch_fold_range_patch(dst, m, 0, 0, fold_len, halo, side, nullptr, 0, s, cemit_d, cdummy);
    return e;
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
        FLTEE_LAUNCH(extract_kernel<true>, dim3(blocks), dim3(256), 0, s, src, d, coef, out);
    else
        FLTEE_LAUNCH(extract_kernel<false>, dim3(blocks), dim3(256), 0, s, src, d, coef, out);
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
    FLTEE_LAUNCH(composite_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint2 *)rec, nrec, d, m, keys, status);
    return hipGetLastError();
}

}  // namespace fltee
