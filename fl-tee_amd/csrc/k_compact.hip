// k_compact.hip — the second half of `advanced` (advanced.rs:106-111 + :32-34):
// after the fold, bring the d run representatives to positions 0..d-1.
//
// The enclave re-runs the whole bitonic network (O(M log^2 M) compare-exchanges)
// and reads positions 0..d-1.  When the fold covered every record (fold_len == L,
// i.e. the request's k equals the payload's, the only case the unchanged client
// produces), the folded array holds, in ascending position order, exactly one
// representative per index 0..d-1 (each index has its initial entry,
// advanced.rs:116-123), the run sums; every other position holds a dummy
// (u32::MAX - p, 0.0), a u32::MAX pad, or a representative of an index >= d.  The
// second sort's prefix [0, d) is therefore "the records with idx < d, in position
// order" — which an order-preserving OBLIVIOUS COMPACTION produces too, with the
// same values bit for bit and no arithmetic at all.
//
// Network (LSB first): a selected record at position p with c = p - idx records
// to drop in front of it moves left by 2^j at level j iff bit j of c is set; at
// level j its current position q satisfies q - idx = c with bits < j cleared, so
// the decision is bit j of (q - idx).  Two selected records never meet: for
// a < b, c_b - c_a <= p_b - p_a - 1 and (c_b mod 2^j) - (c_a mod 2^j) <= c_b - c_a.
// Level j: out[q] = moving(e[q + 2^j]) ? e[q + 2^j] : staying(e[q]) ? e[q] : dummy.
// Every level reads and writes fixed positions; only the select is data-dependent
// (oblivious like the network it replaces).  log2(L - d) levels instead of
// log2(M)(log2(M)+1)/2 steps.
//
// Levels j0..j0+G-1 touch only positions congruent mod 2^j0, so one pass runs G
// levels in LDS on a W x (S + H) tile: W consecutive residues (coalesced rows)
// x S rows of stride 2^j0 plus H = 2^G - 1 halo rows on the right (records move
// left by < 2^G rows within the pass).  Pass 0 is the contiguous case (W = 1).
// The last pass writes out[i] = val * 1f32/n (or out[i] += val for alg 6) for
// i < d instead of records.
#include "common.h"

namespace fltee {

// FLTEE_CP_PICK: 1 = compares + selects; 2 = the staying value as bit operations; 3 = bit
// operations only, no compare; 4 (default, round 5) = form 3 with a dummy's val left as it
// was (see cp_pick, cp_out)
// FLTEE_CP_TWO: two levels per LDS round (3 picks, 4 reads and 1 write per slot) or one
// (1 pick, 2 reads, 1 write and one more barrier per level).  Round 5 A/B, bit-identical:
// one level per round is slower though it issues a third fewer picks — C5 12.22 -> 12.26
// ms, C3 0.1317 -> 0.1350 ms (`profiles/r05/ab/ab16_compact_one_level_rounds_rejected.jsonl`)
#ifndef FLTEE_CP_TWO
#define FLTEE_CP_TWO 1
#endif
// FLTEE_CP_NOHALO: a residue group's only band loads and keeps no halo rows (they lie past
// L), so its rows may be twice as wide (compact_pass NH).  Round 5 A/B, bit-identical
// (`profiles/r05/ab/ab18_*`): C5's last two passes (one band each) ~65 us faster, C5 12.11
// -> 12.06 ms; C3 unchanged (its last pass is the output-prefix tail).
#ifndef FLTEE_CP_NOHALO
#define FLTEE_CP_NOHALO 1
#endif
// FLTEE_CP_SKIP_SELF: a block on its last tile prefetches nothing (else it re-reads its own
// tile, a load with no branch around it).  Round 5 A/B, bit-identical (`ab20_*`): C3 0.1315
// -> 0.1297 ms (its tail pass, one tile per block, 16.6 -> 14.5 us), C5 unchanged.
#ifndef FLTEE_CP_SKIP_SELF
#define FLTEE_CP_SKIP_SELF 1
#endif
// FLTEE_CP_PAD_BAND: a one-band pass on rows of 16 padded to the full tile (compact_levels).
// Round 5 A/B, bit-identical (`profiles/r05/ab/ab19_*`): C5 12.03 -> 12.00 ms (its levels
// 19-23 on the compile-time levels); dropping that band's halo instead (compact_pass NH)
// was slower there (488 vs 459 us: a select per level read in a VALU-bound pass), so NH is
// kept for the bands whose rows it widens (C5's last pass: 293 -> 197 us).
#ifndef FLTEE_CP_PAD_BAND
#define FLTEE_CP_PAD_BAND 1
#endif
// FLTEE_CP_CT: the compaction passes of the common tile shapes (C5's first and middle passes,
// the fused kernel's nine levels) with their levels at compile time (cp_levels_ct).  Round 5
// A/B, bit-identical (`profiles/r05/ab/ab17_*`): C5 12.25 -> 12.15 ms (compact_pass 423 ->
// 403 us on average); the fused kernel 12.3 -> 11.7 us at MLP-MNIST n = 30, 10.2 -> 9.5 us
// at n = 3, 19.8 -> 19.7 us at C3.
#ifndef FLTEE_CP_CT
#define FLTEE_CP_CT 1
#endif
#ifndef FLTEE_CP_PICK
#define FLTEE_CP_PICK 4
#endif
// an unselected slot in flight: c = 2^31 (bit j clear at every level j <= 28, so it never
// moves; form 1's u32::MAX carried the same meaning through its top-bit test), +0.0
constexpr uint64_t CP_DUMMY = FLTEE_CP_PICK >= 3 ? 0x80000000ull : 0xFFFFFFFFull;
constexpr uint64_t CP_PAD = 0xFFFFFFFFull;  // a pad record (idx u32::MAX, +0.0) outside the array

// In flight the key is not idx but c = p0 - idx, the record's total left shift
// (p0 = its position after the fold), CP_DUMMY for records that are not selected
// (idx >= d).  Level j moves a record iff bit j of c is set (c < 2^29; a dummy never
// moves, and a slot it occupies stays a dummy).
//
// cp_pick (round 5, `profiles/r05/ab/ab10_*`): form 2 builds the staying value with bit
// operations — the leaving record's slot becomes the dummy by the sign-extended bit j of
// its c (v_bfe_i32) OR-ed into c and AND-NOT-ed out of the value (v_bfi_b32) — and keeps
// one compare for the mover (bit j set, top bit clear); form 3 drops that compare too: with
// the dummy at c = 2^31 the mover is just bit j of c (j <= 28 since L < 2^29), and both
// selects are v_bfi_b32 on sign-extended bits — six VALU per pick, no lane-mask write
// (form 1: two compares, four selects, and the wait states between a compare and its
// select).  All three move the same records: bit-identical outputs.
__device__ __forceinline__ uint64_t cp_pick(uint64_t self, uint64_t right, uint32_t j) {
    const uint32_t cs = (uint32_t)self, cr = (uint32_t)right;
    if constexpr (FLTEE_CP_PICK == 4) {
        // form 4: a dummy's val is left as it was (the final pass writes +0.0 for any dummy
        // it outputs, cp_out), so the staying val needs no select: five VALU per pick.
        // Round 5 A/B (`profiles/r05/ab/ab15_*`, bit-identical): compact_pass 431 -> 420 us
        // at C5 (12.27 -> 12.23 ms), C3 0.1365 -> 0.1355 ms.
        uint32_t lo, hi, e, em;
        const uint32_t dmy = 0x80000000u;
        asm("v_bfe_i32 %2, %4, %8, 1\n\t"        // e = ~0 iff self leaves
            "v_bfe_i32 %3, %6, %8, 1\n\t"        // em = ~0 iff right moves in
            "v_bfi_b32 %0, %2, %9, %4\n\t"       // stay c: the dummy's when self leaves
            "v_bfi_b32 %0, %3, %6, %0\n\t"       // right's c if it moves in
            "v_bfi_b32 %1, %3, %7, %5"             // right's val if it moves in, else self's
            : "=&v"(lo), "=&v"(hi), "=&v"(e), "=&v"(em)
            : "v"(cs), "v"((uint32_t)(self >> 32)), "v"(cr), "v"((uint32_t)(right >> 32)), "s"(j),
              "s"(dmy));
        return ((uint64_t)hi << 32) | lo;
    }
    if constexpr (FLTEE_CP_PICK == 3) {
        uint32_t lo, hi, e, em;
        const uint32_t dmy = 0x80000000u;
        asm("v_bfe_i32 %2, %4, %8, 1\n\t"        // e = ~0 iff self leaves (bit j of its c)
            "v_bfe_i32 %3, %6, %8, 1\n\t"        // em = ~0 iff right moves in
            "v_bfi_b32 %0, %2, %9, %4\n\t"       // stay c: the dummy's when self leaves
            "v_bfi_b32 %1, %2, 0, %5\n\t"        // stay val: +0.0 when self leaves
            "v_bfi_b32 %0, %3, %6, %0\n\t"       // right's c if it moves in
            "v_bfi_b32 %1, %3, %7, %1"             // right's val if it moves in
            : "=&v"(lo), "=&v"(hi), "=&v"(e), "=&v"(em)
            : "v"(cs), "v"((uint32_t)(self >> 32)), "v"(cr), "v"((uint32_t)(right >> 32)), "s"(j),
              "s"(dmy));
        return ((uint64_t)hi << 32) | lo;
    }
    if constexpr (FLTEE_CP_PICK == 2) {
        uint32_t e, shi;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(e) : "v"(cs), "s"(j));
        asm("v_bfi_b32 %0, %1, 0, %2" : "=v"(shi) : "v"(e), "v"((uint32_t)(self >> 32)));
        const uint64_t stay = ((uint64_t)shi << 32) | (cs | e);
        const uint32_t m = 1u << j;
        return (cr & (m | 0x80000000u)) == m ? right : stay;
    }
    const bool mv = ((cr >> j) & ~(cr >> 31)) & 1u;
    const bool st = !((cs >> j) & 1u);
    return mv ? right : (st ? self : CP_DUMMY);
}

// the value a final pass outputs for slot record r: +0.0 for a dummy (form 4 leaves a
// dummy's val as it was; a position-sharded range outputs +0.0 where it holds no index)
__device__ __forceinline__ float cp_out(uint64_t r) {
    if constexpr (FLTEE_CP_PICK == 4) return ((uint32_t)r >> 31) ? 0.0f : rec_val(r);
    return rec_val(r);
}

typedef unsigned int cp_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int cp_u32x4 __attribute__((ext_vector_type(4)));

// The levels of one tile with its shape known at compile time (FLTEE_CP_CT): G levels on rows
// of 2^LW residues, SH = S + H rows in the tile.  The level loop unrolls, so every LDS slot
// of a round is an immediate offset off one per-lane address, and the range test (f < lim)
// is decided at compile time for every slot but those of the last rows: only the picks'
// five VALU per slot remain (the runtime loop adds ~8 address / range VALU per slot and
// round, `make asm`).  The same levels and picks: bit-identical.
template <int NT, int PER, int G, int LW, int SH, int G0 = 0>
__device__ __forceinline__ void cp_levels_ct(uint64_t *sm, uint32_t j0, uint32_t t) {
    if constexpr (G0 < G) {
        constexpr bool two = FLTEE_CP_TWO && G0 + 1 < G;
        constexpr uint32_t stepf = (1u << LW) << G0;
        constexpr uint32_t gl = two ? G0 + 1 : G0;
        constexpr uint32_t lim = ((uint32_t)SH - ((2u << gl) - 1)) << LW;
        const uint32_t j = j0 + (uint32_t)G0;
        uint64_t *const base = sm + t;
        uint64_t nv[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t o = (uint32_t)i * NT;
            if (o + NT <= lim || t + o < lim) {  // the first test is decided at compile time
                if constexpr (two) {
                    const uint64_t y0 = cp_pick(base[o], base[o + stepf], j);
                    const uint64_t y2 = cp_pick(base[o + 2 * stepf], base[o + 3 * stepf], j);
                    nv[i] = cp_pick(y0, y2, j + 1);
                } else {
                    nv[i] = cp_pick(base[o], base[o + stepf], j);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t o = (uint32_t)i * NT;
            if (o + NT <= lim || t + o < lim) base[o] = nv[i];
        }
        __syncthreads();
        cp_levels_ct<NT, PER, G, LW, SH, G0 + (two ? 2 : 1)>(sm, j0, t);
    }
}

// FIRST: src holds folded records (idx, val); else (c, val).
// FINAL: 0 = write (c, val) records, 1 = out[i] = val*coef, 2 = out[i] += val.
// Persistent: block b walks tiles b, b + grid, ...; the next tile's records are
// prefetched into registers (raw buffer loads, out-of-range lanes selected to the
// dummy afterwards: no per-load branch) while the current tile runs its levels.
// V2 (rows of W >= 2 residues, L even): a lane loads and stores two adjacent slots of a
// row (16 B; 8-B accesses run at about half the 16-B rate, MI355X_MICROARCH.md); the
// levels keep the one-slot-per-lane assignment.
// NH (no halo): the tile is its residue group's only band (S = every row), so the rows a
// halo would hold lie past L — dummies that never move: they are neither loaded nor kept in
// LDS, a level reading one gets the dummy (compact_levels; FLTEE_CP_NOHALO).
template <int NT, int PER, bool FIRST, int FINAL, int MINB = 1, bool V2 = false, int CG = 0, int CLW = 0,
          int CSH = 0, bool NH = false>
__global__ __launch_bounds__(NT, MINB) void compact_pass(const uint64_t *__restrict__ src,
                                                   uint64_t *__restrict__ dst, uint32_t L,
                                                   uint32_t d, uint32_t j0, uint32_t G,
                                                   uint32_t logW, uint32_t S, uint32_t rows,
                                                   uint32_t ngroups, float coef,
                                                   float *__restrict__ out, uint32_t ntiles) {
    constexpr uint32_t CAP = (uint32_t)NT * PER;
    __shared__ uint64_t sm[CAP];
    const uint32_t W = 1u << logW, H = (1u << G) - 1;
    // the lane id re-defined where it is used: per-record positions are recomputed (a few
    // VALU) instead of being hoisted out of the tile loop and spilled — a spill's reload
    // waits vmcnt(0), i.e. for the prefetch in flight (k_bitonic.hip lane_tid)
    auto tid = [] {
        uint32_t x = threadIdx.x;
        asm volatile("; compact tid" : "+v"(x));
        return x;
    };
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, (int)(L * 8u), 0x00020000);
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    // global position of tile slot f (64-bit: rows past L may exceed 2^32 at large j0)
    auto pos_of = [&](uint32_t tl, uint32_t f) -> uint64_t {
        const uint32_t band = tl / ngroups, grp = tl - band * ngroups;
        return ((uint64_t)(band * S + (f >> logW)) << j0) + (grp << logW) + (f & (W - 1));
    };
    static_assert(!V2 || (!FIRST && PER % 2 == 0), "V2: strided passes, slot pairs");
    // the tile slot of prefetch register i: tid + i NT, or with V2 slot pair tid + (i/2) NT
    auto slot = [&](uint32_t i) -> uint32_t {
        return V2 ? 2u * (tid() + (i >> 1) * NT) + (i & 1u) : tid() + i * NT;
    };
    uint64_t pf[PER];
    // the tile's rows in use: S + H (a pass over the output prefix only may use fewer than CAP
    // slots); the other slots, and positions past L, load out of the buffer's range — no
    // memory access, the dummy is selected when the tile lands
    const uint32_t used = (NH ? S : S + H) << logW;
    const uint32_t oob = L * 8u;
    // the loads only: the dummy for slots past L is selected when the tile lands (a use of
    // the loaded value here would make the compiler wait for the prefetch right away)
    auto prefetch = [&](uint32_t tl) {
        if constexpr (V2) {
#pragma unroll
            for (uint32_t i = 0; i < PER; i += 2) {
                const uint64_t p = pos_of(tl, slot(i));  // even (W even), and p + 1 < L with p
                const cp_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(
                    rs, (int)(p < L && slot(i) < used ? (uint32_t)p * 8u : oob), 0, 0);
                pf[i] = ((uint64_t)x.y << 32) | x.x;
                pf[i + 1] = ((uint64_t)x.w << 32) | x.z;
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < PER; ++i) {
                const uint64_t p = pos_of(tl, tid() + i * NT);
                const cp_u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(
                    rs, (int)(p < L && tid() + i * NT < used ? (uint32_t)p * 8u : oob), 0, 0);
                pf[i] = ((uint64_t)x.y << 32) | x.x;
            }
        }
    };
    prefetch(tile);
    for (;;) {
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) {
            uint64_t v = pos_of(tile, slot(i)) < L ? pf[i] : CP_DUMMY;
            if (FIRST) {  // key -> shift c = p - idx (u32::MAX when not selected)
                const uint32_t p = (uint32_t)pos_of(tile, tid() + i * NT), idx = (uint32_t)v;
                v = (v & 0xFFFFFFFF00000000ull) | (idx < d ? (uint64_t)(p - idx) : CP_DUMMY);
            }
            sm[slot(i)] = v;
        }
        __syncthreads();
        const uint32_t next = tile + gridDim.x;
        if (!FLTEE_CP_SKIP_SELF || next < ntiles) prefetch(next < ntiles ? next : tile);
        // Levels two per LDS round: z[f] = pick_{g+1}(pick_g(x[f], x[f+s]),
        // pick_g(x[f+2s], x[f+3s])) — 4 reads + 1 write per record per two levels
        // instead of 2 + 1 per level (ds_write_b64 costs ~3x a ds_read_b64), half the
        // barriers.  After level g the rows still needed are S + H - (2^(g+1) - 1).
        // CG: the tile shape at compile time (launch_pass checked G == CG, logW == CLW and
        // S + H == CSH)
        if constexpr (CG != 0) {
            cp_levels_ct<NT, PER, CG, CLW, CSH>(sm, j0, tid());
        } else {
        uint64_t nv[PER];
        // NH: slots at or past `used` are rows past L (dummies); only rows < S are kept
        auto rdl = [&](uint32_t x) -> uint64_t { return (!NH || x < used) ? sm[x] : CP_DUMMY; };
        for (uint32_t g = 0; g < G;) {
            const uint32_t stepf = W << g;
            const uint32_t j = j0 + g;
            const bool two = FLTEE_CP_TWO && g + 1 < G;
            const uint32_t gl = two ? g + 1 : g;
            const uint32_t lim0 = (S + H - ((2u << gl) - 1)) << logW;
            const uint32_t lim = NH && used < lim0 ? used : lim0;
            if (two) {
#pragma unroll
                for (uint32_t i = 0; i < PER; ++i) {
                    const uint32_t f = tid() + i * NT;
                    if (f < lim) {
                        const uint64_t y0 = cp_pick(rdl(f), rdl(f + stepf), j);
                        const uint64_t y2 = cp_pick(rdl(f + 2 * stepf), rdl(f + 3 * stepf), j);
                        nv[i] = cp_pick(y0, y2, j + 1);
                    }
                }
            } else {
#pragma unroll
                for (uint32_t i = 0; i < PER; ++i) {
                    const uint32_t f = tid() + i * NT;
                    if (f < lim) nv[i] = cp_pick(rdl(f), rdl(f + stepf), j);
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t i = 0; i < PER; ++i) {
                const uint32_t f = tid() + i * NT;
                if (f < lim) sm[f] = nv[i];
            }
            __syncthreads();
            g += two ? 2 : 1;
        }
        }
        const uint32_t nout = S << logW;
        if constexpr (V2 && FINAL == 0) {
            // slot pairs as 16-B stores (p even; nout and L even)
            const __amdgpu_buffer_rsrc_t ds =
                __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, (int)(L * 8u), 0x00020000);
#pragma unroll
            for (uint32_t i = 0; i < PER; i += 2) {
                const uint32_t f = slot(i);
                if (f < nout) {
                    const uint64_t p = pos_of(tile, f);
                    const uint64_t a = sm[f], b = sm[f + 1];
                    const cp_u32x4 x = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
                    // p >= L: past the buffer's range, the store is dropped (no branch)
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_raw_buffer_store_b128(x, ds, (int)(p < L ? (uint32_t)p * 8u : L * 8u), 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");  // dwordx4 store data hazard (k_bitonic.hip)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else {
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) {
            const uint32_t f = tid() + i * NT;
            if (f < nout) {
                const uint64_t p = pos_of(tile, f);
                if (FINAL == 0) {
                    if (p < L) dst[p] = sm[f];
                } else if (p < d) {
                    const float v = cp_out(sm[f]);
                    out[p] = FINAL == 2 ? __fadd_rn(out[p], v) : __fmul_rn(v, coef);
                }
            }
        }
        }
        if (next >= ntiles) break;
        __syncthreads();  // this tile's LDS reads retire before the next tile lands
        tile = next;
    }
}

// Resident 512-lane blocks per CU for the passes after the first: 3 (default) asks hipcc
// for 6 waves per SIMD (launch_bounds' 2nd argument = min waves per EU: <= 80 VGPRs).
// A/B at C5: 497 vs 534 us per middle pass, 499 vs 570 us for the last; the first pass
// (more live state) spills at that bound (868 vs 751 us), so it keeps 2.
// Round 3: the kernels no longer spill (54 VGPRs, the lane id re-read where used), so the
// first pass may take as many blocks as the later ones (FLTEE_COMPACT_FIRST_BLOCKS), and 4
// blocks (8 waves per SIMD, <= 64 VGPRs) fit too (FLTEE_COMPACT_BLOCKS; A/B builds).
#ifndef FLTEE_COMPACT_BLOCKS
#define FLTEE_COMPACT_BLOCKS 4
#endif
#ifndef FLTEE_COMPACT_FIRST_BLOCKS
#define FLTEE_COMPACT_FIRST_BLOCKS 4
#endif
constexpr int kCompactBlocks = FLTEE_COMPACT_BLOCKS;
constexpr int kCompactFirstBlocks = FLTEE_COMPACT_FIRST_BLOCKS;
// fltee_debug_set_compact_variant (A/B): 1 = 32 KiB tiles (default), 0 = 64 KiB tiles
// (1024 lanes x 8), 2 = 32 KiB first pass + 64 KiB strided passes (1024 lanes x 8, one
// block per CU: 6 levels per pass, 4 passes instead of 5 at C5; 512 x 16 spills)
static int g_compact_variant = 1;
void set_compact_variant(int v) { g_compact_variant = v; }

#ifndef FLTEE_COMPACT_V2
#define FLTEE_COMPACT_V2 1
#endif
// the last levels as one pass over the output prefix (compact_levels) on arrays of at most
// 2^FLTEE_CP_TAIL_MERGE records (0: never).  Round 5 A/B (`profiles/r05/ab/ab15_*`,
// bit-identical): C3 0.1365 -> 0.1319 ms, MLP-MNIST n = 30 advanced 0.088 -> 0.082 ms (a
// launch less on arrays that stay in the caches); C5 12.27 -> 12.55 ms (the merged pass
// computes 8 levels over 14x the slots it outputs, 1.07 ms against 0.75 for the two passes
// it replaces), so large arrays keep the separate passes.
#ifndef FLTEE_CP_TAIL_MERGE
#define FLTEE_CP_TAIL_MERGE 21
#endif
template <int NT, int PER, int MINB = 1>
static hipError_t launch_pass(bool first, int fin, unsigned grid, hipStream_t s, const uint64_t *src,
                              uint64_t *dst, uint32_t L, uint32_t d, uint32_t j0, uint32_t G,
                              uint32_t logW, uint32_t S, uint32_t rows, uint32_t ngroups,
                              float coef, float *out, uint32_t ntiles, bool nh = false) {
#define CP_GO(F, X, V)                                                                           \
    FLTEE_LAUNCH((compact_pass<NT, PER, F, X, MINB, V>), dim3(grid), dim3(NT), 0, s, src, dst, L, \
                       d, j0, G, logW, S, rows, ngroups, coef, out, ntiles)
#define CP_GO_CT(V, G_, LW_, SH_)                                                                \
    FLTEE_LAUNCH((compact_pass<NT, PER, false, 0, MINB, V, G_, LW_, SH_>), dim3(grid), dim3(NT), 0, s, \
                       src, dst, L, d, j0, G, logW, S, rows, ngroups, coef, out, ntiles)
    // 16-B slot pairs: rows of >= 2 residues (or a contiguous tile of an even S: the
    // converted first pass), L even, both buffers 16-B aligned
    const bool v2 = FLTEE_COMPACT_V2 && !first && (logW >= 1 || S % 2 == 0) && L % 2 == 0 &&
                    (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0;
    // the tile shapes of C5's passes with compile-time levels (FLTEE_CP_CT): the converted
    // first pass (9 levels, contiguous, S + H = 4,095) and the strided middle ones (5 levels
    // on rows of 16, one 256-row band)
    const uint32_t sh = S + (1u << G) - 1;
    if constexpr (FLTEE_CP_CT && NT * PER == 4096) {
        if (!first && v2 && fin == 0) {
            if (G == 9 && logW == 0 && sh == 4095) { CP_GO_CT(true, 9, 0, 4095); return hipGetLastError(); }
            if (G == 5 && logW == 4 && sh == 256) { CP_GO_CT(true, 5, 4, 256); return hipGetLastError(); }
        }
    }
#define CP_GO_NH(X, V)                                                                           \
    FLTEE_LAUNCH((compact_pass<NT, PER, false, X, MINB, V, 0, 0, 0, true>), dim3(grid), dim3(NT), 0, s, \
                       src, dst, L, d, j0, G, logW, S, rows, ngroups, coef, out, ntiles)
    if (FLTEE_CP_NOHALO && nh && !first) {  // one band: no halo rows (compact_pass NH)
        if (v2) {
            if (fin == 0) CP_GO_NH(0, true); else if (fin == 1) CP_GO_NH(1, true); else CP_GO_NH(2, true);
        } else {
            if (fin == 0) CP_GO_NH(0, false); else if (fin == 1) CP_GO_NH(1, false); else CP_GO_NH(2, false);
        }
        return hipGetLastError();
    }
#undef CP_GO_NH
    if (first) {
        if (fin == 0) CP_GO(true, 0, false); else if (fin == 1) CP_GO(true, 1, false); else CP_GO(true, 2, false);
    } else if (v2) {
        if (fin == 0) CP_GO(false, 0, true); else if (fin == 1) CP_GO(false, 1, true); else CP_GO(false, 2, true);
    } else {
        if (fin == 0) CP_GO(false, 0, false); else if (fin == 1) CP_GO(false, 1, false); else CP_GO(false, 2, false);
    }
#undef CP_GO
#undef CP_GO_CT
    return hipGetLastError();
}

static uint32_t bitlen(uint64_t x) {
    uint32_t b = 0;
    while (x) { ++b; x >>= 1; }
    return b;
}

// src holds the folded array (positions [0, L) meaningful); tmp is scratch of L
// records.  Both are clobbered.  max_shift bounds every selected record's shift
// c = p - idx (L - d for a whole folded array: c counts the unselected records in
// front of p); it sets the number of levels, bitlen(max_shift).
static hipError_t compact_levels(uint64_t *src, uint64_t *tmp, size_t L, size_t d,
                                 size_t max_shift, float coef, float *out, bool accumulate,
                                 hipStream_t s, uint32_t j0_start = 0, bool converted = false) {
    if (d == 0) return hipSuccess;
    const uint32_t nlev = bitlen(max_shift);
    if (nlev == 0) return launch_extract(src, d, coef, out, accumulate, s);
    if (L >= ((size_t)1 << 29)) return hipErrorInvalidValue;  // 32-bit byte offsets
    uint64_t *cur = src, *oth = tmp;
    for (uint32_t j0 = j0_start; j0 < nlev;) {
        const bool small = g_compact_variant == 1 || (g_compact_variant == 2 && j0 == 0);
        const uint32_t CAP = small ? 4096 : 8192;
        const uint32_t gmax = j0 == 0 ? (small ? 9 : 10) : (small ? 5 : 6);
        uint32_t G = min(gmax, nlev - j0), H = (1u << G) - 1;
        const uint64_t rows64 = (L + ((uint64_t)1 << j0) - 1) >> j0;
        const uint32_t rows = (uint32_t)rows64;
        uint32_t logW, S;
        bool nohalo = false;
        // The last levels in one pass over the output prefix (FLTEE_CP_TAIL_MERGE): the final
        // pass writes out[p] for p < d only, i.e. rows < ceil(d / 2^j0) of each residue
        // class, and a record reaches row r from rows < r + 2^G.  So one band of those rows +
        // 2^G - 1 halo rows per residue group covers every level left (G up to 10) when it
        // fits a tile: e.g. C3's levels 9-18 (after the fused fold's 0-8) as one pass of 256
        // tiles, 100 output + 1,023 halo rows of 2 residues each, instead of two.
        bool tail = false;
        uint32_t tcap = CAP;
        if (FLTEE_CP_TAIL_MERGE && L <= ((size_t)1 << FLTEE_CP_TAIL_MERGE) && j0 > 0 && nlev - j0 > G &&
            nlev - j0 <= 10) {
            const uint32_t Gt = nlev - j0, Ht = (1u << Gt) - 1;
            const uint64_t so = (d + ((uint64_t)1 << j0) - 1) >> j0;  // output rows
            // the widest rows (<= 16 residues, <= 2^j0) that fit 4,096 slots, or 8,192 (1,024
            // lanes) when that gives 128-B rows on a large array
            auto widest = [&](uint32_t cap) {
                uint32_t lw = 0;
                while (lw < 4 && lw < j0 && ((so + Ht) << (lw + 1)) <= cap) ++lw;
                return ((so + Ht) << lw) <= cap ? (int)lw : -1;
            };
            int lw = widest(4096);
            if (lw >= 0 && lw < 4 && L > ((size_t)1 << 21) && widest(8192) >= 4) {  // (large arrays)
                lw = widest(8192);
                tcap = 8192;
            }
            if (lw >= 0 && so < rows) {
                tail = true;
                G = Gt;
                H = Ht;
                logW = (uint32_t)lw;
                S = (uint32_t)so;
            }
        }
        if (tail) {
        } else if (j0 == 0) {
            logW = 0;
            S = CAP - H;
            if (converted) S &= ~1u;  // even: 16-B slot pairs
        } else {
            logW = 4;  // 16 residues = 128-B row segments
            // One band: widen the rows instead.  Its halo rows lie past L (dummies).  With
            // FLTEE_CP_NOHALO the tile drops them (compact_pass NH: a select per level read)
            // where that widens the rows; else they stay (they load nothing), and a band of
            // 16-residue rows is padded to the full 256-row tile — rows past L again — so
            // the compile-time levels run it (FLTEE_CP_CT; C5's levels 19-23: 488 -> ~400 us).
            const bool nh_ok = FLTEE_CP_NOHALO && kCompactBlocks >= 4;
            const bool fits = rows + H <= CAP >> logW;
            if (fits || (nh_ok && rows <= CAP >> logW)) {
                uint32_t lw = logW, lwn = logW;
                while (lw < j0 && ((rows + H) << (lw + 1)) <= CAP) ++lw;
                while (lwn < j0 && (rows << (lwn + 1)) <= CAP) ++lwn;
                if (nh_ok && (!fits || lwn > lw)) {
                    logW = lwn;
                    S = rows;
                    nohalo = true;
                } else {
                    logW = lw;
                    S = lw == 4 && FLTEE_CP_CT && FLTEE_CP_PAD_BAND ? (CAP >> 4) - H : rows;
                }
            } else {
                S = (CAP >> logW) - H;
            }
            if (logW > j0) logW = j0;
        }
        const uint32_t ngroups = (uint32_t)(((uint64_t)1 << j0) >> logW);
        const uint64_t bands = tail ? 1 : (rows + S - 1) / S;  // tail: band 0 only
        uint64_t ntiles = bands * ngroups;
        if (ntiles == 0 || ntiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
        const bool last = (j0 + G == nlev);
        const int fin = last ? (accumulate ? 2 : 1) : 0;
        // The last pass writes out[p] for p < d only.  With one band and 2^j0 >= d, a tile's
        // output slots lie at p = row * 2^j0 + grp * W + f: rows >= 1 are past d, so the
        // groups with grp * W >= d write nothing — a suffix of the tiles, skipped (public
        // sizes only).  C5's last pass: 39,063 of 65,536 tiles.
        uint64_t live = ntiles;
        if (last && bands == 1 && j0 > 0 && ((uint64_t)1 << j0) >= d) {
            const uint64_t g = (d + ((uint64_t)1 << logW) - 1) >> logW;
            if (g < live) live = g;
        }
        net_account(tail ? (uint64_t)8 * L + 4 * (uint64_t)d : (uint64_t)(last ? 8 : 16) * L * live / ntiles,
                    "compact_pass", s);
        ntiles = live;
        // persistent grid = resident blocks: one 1024-lane block per CU (72-87 VGPRs), or two 512-lane ones
        const int blk = j0 == 0 ? kCompactFirstBlocks : kCompactBlocks;
        const bool wide = tail ? tcap > 4096 : !small;
        const unsigned res = !wide ? 256u * (unsigned)blk : 256u;
        const unsigned grid = (unsigned)(ntiles < res ? ntiles : res);
        const hipError_t e =
            !wide ? (blk >= 4
                         ? launch_pass<512, 8, 8>(j0 == 0 && !converted, fin, grid, s, cur, oth, (uint32_t)L,
                                                  (uint32_t)d, j0, G, logW, S, rows, ngroups, coef,
                                                  out, (uint32_t)ntiles, nohalo)
                     : blk == 3
                         ? launch_pass<512, 8, 6>(j0 == 0 && !converted, fin, grid, s, cur, oth, (uint32_t)L,
                                                  (uint32_t)d, j0, G, logW, S, rows, ngroups, coef,
                                                  out, (uint32_t)ntiles)
                         : launch_pass<512, 8>(j0 == 0 && !converted, fin, grid, s, cur, oth, (uint32_t)L,
                                               (uint32_t)d, j0, G, logW, S, rows, ngroups, coef, out,
                                               (uint32_t)ntiles))
                  : launch_pass<1024, 8>(j0 == 0 && !converted, fin, grid, s, cur, oth, (uint32_t)L, (uint32_t)d, j0,
                                         G, logW, S, rows, ngroups, coef, out, (uint32_t)ntiles);
        if (e != hipSuccess) return e;
        uint64_t *x = cur; cur = oth; oth = x;
        j0 += G;
    }
    return hipSuccess;
}

uint64_t compact_dummy() { return CP_DUMMY; }

hipError_t launch_compact_extract_converted(uint64_t *src, uint64_t *tmp, size_t L, size_t d,
                                            float coef, float *out, bool accumulate, hipStream_t s) {
    return compact_levels(src, tmp, L, d, L > d ? L - d : 0, coef, out, accumulate, s, 0, true);
}

hipError_t launch_compact_extract(uint64_t *src, uint64_t *tmp, size_t L, size_t d, float coef,
                                  float *out, bool accumulate, hipStream_t s) {
    return compact_levels(src, tmp, L, d, L > d ? L - d : 0, coef, out, accumulate, s);
}

// ------------------------------------------ fold fused into the first pass ---
// advanced.rs:66-101 (the fold) and the compaction's first pass in one kernel: a tile
// reads the SORTED array over its window [a - Hr, a + CAP] (Hr = the fold's halo, the
// record after the tile for the run-end test), folds it in LDS and goes straight on
// with the first G compaction levels.  The fold needs, per position p < L, only what
// the compaction reads: whether p is its run's representative (the run's last
// position: idx[p+1] != idx[p], or p = L-1) with idx < d, and then the run's sum —
// v_head, (v_head + v_next), ... left to right, the enclave's order.  Each lane walks
// back lim = halo + 1 slots from its own and forward through them (FLTEE_FC_FIXED_WALK
// below), so every run of <= lim entries gets the enclave's sum bit for bit.  The folded
// array (1 GB at C5) is never written and read back.  Dummies and non-representatives are
// never selected by the compaction, so their contents do not matter.
//
// Runs of any length (round 6; a client repeated an index).  A run that began before a
// lane's walk start is finished with a re-associated sum: every lane folds its own slots
// again (the run partials from its first slot), the block scans the lanes' segmented
// aggregates (FoldAgg: first key, last key, one key throughout, the partial of the run
// ending the range), and the carry from in front of the window comes from the tiles
// before by a decoupled look-back: each tile publishes the aggregate of its piece (window
// slots [0, S) — the pieces of consecutive tiles tile the array) as soon as its walk is
// done, then its inclusive prefix; wave 0 reads 64 predecessors at a time back to the
// nearest inclusive one.  Every tile runs the same steps whatever the data (the waits
// depend on the other tiles' progress only), and the grid never exceeds the blocks that
// fit on the chip at once (a tile only waits for tiles of lower index, already running),
// with a bounded wait that reports FLTEE_DEV_ERR_LAUNCH instead of hanging.
// Resident blocks per CU of the fused first pass, and whether a block prefetches its next
// window during the fold.  Round 3 (A/B in one process, `profiles/r03/ab/ab18_fold_blocks_*`):
// three blocks without the prefetch ran C5's pass fastest then.  Round 6: with the long-run
// steps (three LDS arrays, the look-back) three blocks' 80 VGPRs spill 20-50 registers;
// two blocks (128 VGPRs) do not (`profiles/r06/ab/`).
#ifndef FLTEE_FC_BLOCKS
#define FLTEE_FC_BLOCKS 2
#endif
#ifndef FLTEE_FC_PF
#define FLTEE_FC_PF 0
#endif
// Round 5, measured and not kept: 8,192-record windows (1,024 lanes x 8, one block per CU)
// for the wide-halo arrays — one 1,024-lane block per CU has too few waves to hide the
// window load that three 512-lane blocks hide (`profiles/r05/ab/ab3_fold_window8192_c5_
// rejected.jsonl`: 1,356-1,358 vs 1,097-1,098 us per pass at C5).
// The fold's lane walks have a trip count fixed by the public sizes (round 5): every lane
// walks back lim slots and forward through its own, branch-free, and stores its own slots'
// sums after a barrier.  That walk grows with n, so the fused kernel takes it only up to
// kFixedWalkMax; longer runs go to the streaming fold (fixed Hr + C + 16 steps per lane) +
// the compaction.  (Round 5 A/B, `profiles/r05/ab/ab9_*`, `ab10_*`: C3 (lim 101) 0.147 vs
// 0.135 ms against a data-dependent walk; C5 (lim 1,001) through the streaming fold 12.33
// vs 12.07 ms — the fused fixed walk there took 11.4 ms alone.  Also measured and not kept:
// the walk's dependent chain as rounds of carries between lanes, C3 0.136-0.139 vs 0.136
// ms, `profiles/r05/ab/ab15_*`.)
// The fixed walk's bound: lim <= 128 at any size, <= 320 on arrays of <= 2^20 records,
// where the streaming fold's launch and latency cost more than the longer walk (MLP-MNIST
// n = 300, lim 301: 0.101 vs 0.138 ms, `profiles/r05/ab/ab12_*`); 320 keeps three windows
// + sums per CU in the 160 KiB of LDS.
#ifndef FLTEE_FC_WALK_MAX
#define FLTEE_FC_WALK_MAX 128
#endif
#ifndef FLTEE_FC_WALK_MAX_SMALL
#define FLTEE_FC_WALK_MAX_SMALL 320
#endif
constexpr uint32_t kFixedWalkMax = FLTEE_FC_WALK_MAX;
constexpr uint32_t kFixedWalkMaxSmall = FLTEE_FC_WALK_MAX_SMALL;
#ifndef FLTEE_FC_LB
#define FLTEE_FC_LB 1
#endif
// tiles per CU the per-lane slot count aims for (the fewest slots with at most this many)
#ifndef FLTEE_FC_TILES_PER_CU
#define FLTEE_FC_TILES_PER_CU 1
#endif
// the look-back's first-round words loaded before the compaction levels (1) or after (0).
// Round 6 A/B (`profiles/r06/ab/ab2_*`): 28.9 vs 27.1 us per C3 pass — the 12 VGPRs held
// across the levels cost more than the load latency they hide
#ifndef FLTEE_FC_LBPRE
#define FLTEE_FC_LBPRE 0
#endif
// the bounded look-back wait: polls of ~0.25 us (about a quarter second in all)
constexpr uint32_t kFcSpinMax = 1u << 20;

// One tile's look-back slot: its piece aggregate and its inclusive prefix, each as three
// 64-bit words (F, K, Q) whose high halves carry the launch's epoch << 2 | fl.  Every word
// is written and read with a relaxed agent-scope atomic: a word is valid on its own (its
// epoch), so no release / acquire fence — on gfx950 those write back / invalidate the
// XCD's L2 (a few us per tile, measured) — is needed between the data and a flag.
struct FcLb {
    uint64_t agg[3], inc[3];
};

__device__ __forceinline__ void fc_put(uint64_t *w, const FoldAgg &g, uint32_t epoch) {
    const uint64_t tag = (uint64_t)((epoch << 2) | (g.fl & 3u)) << 32;
    __hip_atomic_store(&w[0], tag | g.F, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&w[1], tag | g.K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&w[2], tag | __float_as_uint(g.Q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ FoldAgg fa_shfl_up(const FoldAgg &x, int o) {
    FoldAgg r;
    r.F = (uint32_t)__shfl_up((int)x.F, o);
    r.K = (uint32_t)__shfl_up((int)x.K, o);
    r.Q = __shfl_up(x.Q, o);
    r.fl = (uint32_t)__shfl_up((int)x.fl, o);
    return r;
}
__device__ __forceinline__ FoldAgg fa_shfl_down(const FoldAgg &x, int o) {
    FoldAgg r;
    r.F = (uint32_t)__shfl_down((int)x.F, o);
    r.K = (uint32_t)__shfl_down((int)x.K, o);
    r.Q = __shfl_down(x.Q, o);
    r.fl = (uint32_t)__shfl_down((int)x.fl, o);
    return r;
}

// tile `tile` (the whole block): the aggregate of every piece before it (decoupled
// look-back).  Each round reads NW * 64 predecessors, wave w the 64 from tile - 1 - 64 w
// back: up to the nearest one with its inclusive prefix published, aggregates in front of
// it; rounds go on further back only when none of them had it.
// the three words of this epoch already loaded (w), or false
__device__ __forceinline__ bool fc_have(const uint64_t *w, uint32_t epoch, FoldAgg &g) {
    g.F = (uint32_t)w[0];
    g.K = (uint32_t)w[1];
    g.Q = __uint_as_float((uint32_t)w[2]);
    g.fl = (uint32_t)(w[2] >> 32) & 3u;
    return (uint32_t)(w[0] >> 34) == epoch && (uint32_t)(w[1] >> 34) == epoch &&
           (uint32_t)(w[2] >> 34) == epoch;
}

// pre: this thread's first-round predecessor (tile - 1 - t) words, loaded ahead (inc[3],
// agg[3]): used when they are already this epoch's, else polled again
template <int NW>
__device__ FoldAgg fc_lookback(FcLb *lb, uint32_t tile, uint32_t epoch, uint32_t t,
                               uint32_t *status, FoldAgg *sh, uint32_t *shf, const uint64_t *pre) {
    const uint32_t lane = t & 63, wave = t >> 6;
    long long base = (long long)tile - 1;
    bool done = tile == 0;
    if (t == 0) sh[NW] = fa_empty();  // the aggregate so far (sh, shf: NW + 1 entries)
    __syncthreads();
    while (!done) {  // block-uniform
        const long long p = base - (long long)(wave * 64 + lane);
        bool isinc = true;  // before position 0: nothing (an empty inclusive prefix)
        FoldAgg v = fa_empty();
        if (p >= 0) {
            FoldAgg g;
            bool ok = false;
            uint32_t it = 0;
            if (base == (long long)tile - 1) {  // the first round: the words loaded ahead
                if (fc_have(pre, epoch, g)) { isinc = true; ok = true; }
                else if (fc_have(pre + 3, epoch, g)) { isinc = false; ok = true; }
            }
#pragma unroll 1
            while (!ok) {  // the inclusive prefix if it is there, else the aggregate
                // (all six words in flight at once: one memory round trip a poll)
                uint64_t w[6];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    w[i] = __hip_atomic_load(&lb[p].inc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    w[3 + i] = __hip_atomic_load(&lb[p].agg[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (fc_have(w, epoch, g)) { isinc = true; ok = true; break; }
                if (fc_have(w + 3, epoch, g)) { isinc = false; ok = true; break; }
                if (++it >= kFcSpinMax) break;
                __builtin_amdgcn_s_sleep(8);
            }
            if (!ok) {
                atomicOr(status, FLTEE_DEV_ERR_LAUNCH);
                g = fa_empty();
                isinc = true;
            }
            v = g;
        }
        const uint64_t incl = __ballot(isinc);
        const uint32_t first = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
        if (lane > first) v = fa_empty();
        // the window's lanes in position order: a higher lane is an older piece
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const FoldAgg older = fa_shfl_down(v, o);
            if ((lane & (2 * o - 1)) == 0) v = fa_combine(older, v);
        }
        if (lane == 0) {
            sh[wave] = v;
            shf[wave] = first < 64;
        }
        __syncthreads();
        // thread 0: the windows from the newest (wave 0) back to the first with an inclusive
        // prefix, in front of what the rounds before found
        if (t == 0) {
            FoldAgg blk = fa_empty();
            uint32_t found = 0;
#pragma unroll 1
            for (int w = 0; w < NW && !found; ++w) {
                blk = fa_combine(sh[w], blk);
                found = shf[w];
            }
            sh[NW] = fa_combine(blk, sh[NW]);
            shf[NW] = found;
        }
        __syncthreads();
        done = shf[NW] != 0;
        base -= 64 * NW;
    }
    const FoldAgg run = sh[NW];
    __syncthreads();  // sh[] is reused by the next tile
    return run;
}

template <int NT, int PER, int FINAL, int XMAX, int BPC = FLTEE_FC_BLOCKS>
__global__ __launch_bounds__(NT, BPC * NT >= 1024 ? BPC * NT / 256 : 1) void fold_compact_first(const uint64_t *__restrict__ A,
                                                            uint64_t *__restrict__ dst, uint32_t L,
                                                            uint32_t M, uint32_t d, uint32_t G,
                                                            uint32_t S, uint32_t Hr,
                                                            uint32_t ntiles, float coef,
                                                            float *__restrict__ out,
                                                            uint32_t lim, FcLb *lb, uint32_t epoch,
                                                            uint32_t *status) {
    constexpr uint32_t CAP = (uint32_t)NT * PER;
    constexpr int NW = NT / 64;
    // XMAX: window slots beyond CAP per lane, ceil((Hr + 1) / NT)
    extern __shared__ __attribute__((aligned(16))) uint64_t win[];  // Hr + CAP + 1, then the sums
    __shared__ FoldAgg wtot[NW];
    __shared__ FoldAgg agg_s;
    __shared__ FoldAgg lb_sh[NW + 1];
    __shared__ uint32_t lb_shf[NW + 1];
    __shared__ uint32_t fix_s, kw0_s;
    const uint32_t H = (1u << G) - 1;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t Wn = Hr + CAP + 1;
    const uint32_t chunk = (Wn + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, (short)0, (int)(M * 8u), 0x00020000);
    // the window of tile tl into registers: lane t holds window slots t + i*NT; slots
    // before position 0 or past M are dummies (clamped address, select after the load:
    // no branch around the loads)
    uint64_t pf[PER + XMAX];
    auto prefetch = [&](uint32_t tl) {
        const long long wlo = (long long)tl * S - (long long)Hr;
#pragma unroll
        for (uint32_t i = 0; i < PER + XMAX; ++i) {
            const long long p = wlo + t + i * NT;
            const bool ok = p >= 0 && p < (long long)M && t + i * NT < Wn;
            const cp_u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(
                rs, (int)(ok ? (uint32_t)p * 8u : 0u), 0, 0);
            pf[i] = ok ? (((uint64_t)x.y << 32) | x.x) : CP_PAD;
        }
    };
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    if (FLTEE_FC_PF) prefetch(tile);
    for (;;) {
        if (!FLTEE_FC_PF) prefetch(tile);
        const long long a = (long long)tile * S, wlo = a - (long long)Hr;
#pragma unroll
        for (uint32_t i = 0; i < PER + XMAX; ++i)
            if (t + i * NT < Wn) win[t + i * NT] = pf[i];
        __syncthreads();
        const uint32_t next = tile + gridDim.x;
        if (FLTEE_FC_PF && (!FLTEE_CP_SKIP_SELF || next < ntiles))
            prefetch(next < ntiles ? next : tile);  // lands while this tile folds and compacts
        // Each lane owns window slots [x0, x0 + chunk) and computes, for each, the
        // in-order sum of its run up to that slot: a walk from x0 - lim (every run of <= lim
        // entries of an owned slot starts after it), lim + chunk steps whatever the data, no
        // branch, the next slot's LDS read issued a step ahead.  The sums go to their own
        // LDS array (sums[], after the window), so no lane overwrites what another still
        // reads; a run's last slot then holds the run's sum — all the compaction reads.
        // Over its own slots the walk also keeps the run partial from x0 (acc2) and the
        // lane's segmented aggregate, for the runs longer than the walk (see above).
        float *sums = reinterpret_cast<float *>(win + Wn);
        const int x0 = (int)(t * chunk), ys = x0 - (int)lim;
        FoldAgg ca = fa_empty();
        float qS = 0.0f;  // acc2 at the tile's last slot S - 1 (its owner lane's)
        {
            const int pw = (int)wlo;  // |positions| < 2^29 (launch guard)
            auto rd = [&](int y) { return win[min((uint32_t)max(y, 0), Wn - 1)]; };
            uint32_t prevk = 0xFFFFFFFFu;
            bool have = false;
            float acc = 0.0f;
            // (bitwise tests: short-circuit ones turned into EXEC-mask juggling)
            auto step = [&](uint64_t r, int y) {
                const uint32_t p = (uint32_t)(pw + y);  // a position < 0 wraps past L
                const bool valid = ((uint32_t)y < Wn) & (p < L);
                const uint32_t ky = (uint32_t)r;
                const bool cont = have & valid & (p != 0u) & (ky == prevk);
                const float v = rec_val(r);
                acc = cont ? __fadd_rn(acc, v) : v;
                prevk = ky;
                have = valid;
            };
            uint64_t rn = rd(ys);
            for (uint32_t q = 0; q < lim; ++q) {  // the same trip count in every lane
                const uint64_t r = rn;
                rn = rd(ys + (int)q + 1);
                step(r, ys + (int)q);
            }
            uint32_t kl = 0;
            float acc2 = 0.0f;
            bool unb = true;
            for (uint32_t i = 0; i < chunk; ++i) {
                const int y = x0 + (int)i;
                const uint64_t r = rn;
                rn = rd(y + 1);
                step(r, y);
                const bool in = y < (int)Wn;
                const uint32_t ky = (uint32_t)r;
                const bool c2 = i > 0 && ky == kl;
                acc2 = in ? (c2 ? __fadd_rn(acc2, rec_val(r)) : rec_val(r)) : acc2;
                qS = y == (int)S - 1 ? acc2 : qS;
                unb = unb && (!in || i == 0 || c2);
                kl = in ? ky : kl;
                if (in) {
                    sums[y] = acc;
                }
            }
            if (x0 < (int)Wn) {
                ca.F = (uint32_t)win[x0];
                ca.K = kl;
                ca.Q = acc2;
                ca.fl = kFsPiece | (unb ? kFsFull : 0u);
            }
        }
        FoldAgg inc = ca;  // the wave's inclusive scan (lane order = position order)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const FoldAgg y = fa_shfl_up(inc, o);
            if (lane >= (uint32_t)o) inc = fa_combine(y, inc);
        }
        FoldAgg wex = fa_shfl_up(inc, 1);
        if (lane == 0) wex = fa_empty();
        if (lane == 63) wtot[wave] = inc;
        __syncthreads();
        // the lane's exclusive aggregate within the window: the run partial in front of x0
        {
            FoldAgg ex = fa_empty();
            for (uint32_t w = 0; w < wave; ++w) ex = fa_combine(ex, wtot[w]);
            ex = fa_combine(ex, wex);
            const uint32_t k0 = x0 < (int)Wn ? (uint32_t)win[x0] : 0u;
            const bool exf = (ex.fl & kFsPiece) && ex.K == k0;
            if (t == 0) {
                fix_s = 0xFFFFFFFFu;
                kw0_s = (uint32_t)win[0];
            }
            // the piece [0, S) of this tile: published by the lane owning its last slot
            if ((uint32_t)x0 <= S - 1 && S - 1 < (uint32_t)x0 + chunk) {
                const uint32_t kS = (uint32_t)win[S - 1];
                FoldAgg part;
                part.F = k0;
                part.K = kS;
                part.Q = qS;
                part.fl = kFsPiece | (k0 == kS ? kFsFull : 0u);
                const FoldAgg g = fa_combine(ex, part);
                fc_put(lb[tile].agg, g, epoch);
                agg_s = g;
            }
            // The lane's head run, when it began before the lane's walk (more than lim
            // entries: the walk's sums miss its front): its slots take the re-associated
            // window-local prefix — the partial in front of x0 (ex) + the partial from x0.  Only the head run can be such a run; the owner lane fixes its own
            // slots (a fixed trip count), so the representative loop below reads sums[]
            // alone.  (Round 6 first had every slot test its owner's head run there: six
            // LDS reads a slot, and a read of the owner's ex without a barrier.)
            // (the partial from x0 recomputed here, in the walk's order: the head run is
            // contiguous from x0, so a2 is the walk's acc2 on its slots)
            const bool lngL = ys > 0 && x0 < (int)Wn && (uint32_t)win[ys - 1] == k0;
            float a2 = 0.0f;
            for (uint32_t i = 0; i < chunk; ++i) {
                const int y = x0 + (int)i;
                const uint64_t r = win[min(y, (int)Wn - 1)];
                a2 = i == 0 ? rec_val(r) : __fadd_rn(a2, rec_val(r));
                const bool fix = lngL && y < (int)Wn && (uint32_t)r == k0;
                if (fix) sums[y] = exf ? __fadd_rn(ex.Q, a2) : a2;
            }
        }
        __syncthreads();  // every lane's sums[] final before any lane reads another's
        // representatives with idx < d -> (c = p - idx, sum); the rest never move.  A run
        // that began before its owner lane's walk (more than lim entries) takes the
        // re-associated window-local prefix (fixed by the owner lane above); the carry from
        // before the window is added after the levels (below), to the
        // one record it concerns: the window's head run's, wherever the levels took it.
        uint64_t v[PER];
        {
            const uint32_t kw0 = (uint32_t)win[0];
            const uint32_t gm = (1u << G) - 1;
#pragma unroll
            for (uint32_t i = 0; i < PER; ++i) {
                const uint32_t f = t + i * NT, x = f + Hr;
                const long long p = a + f;
                const uint64_t r = win[x];
                const uint32_t idx = (uint32_t)r;
                const bool end = p == (long long)L - 1 || (uint32_t)win[x + 1] != idx;
                const float hv = sums[x];
                const bool rep = p < (long long)L && idx < d && end;
                const uint32_t c = (uint32_t)p - idx;
                v[i] = rep ? (((uint64_t)__float_as_uint(hv) << 32) | c) : CP_DUMMY;
                if (rep && idx == kw0) fix_s = f - (c & gm);  // its slot after the G levels
            }
        }
        __syncthreads();
        uint64_t *sm = win;
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) sm[t + i * NT] = v[i];
        // the look-back's first-round words, loaded now: they arrive while the levels run
        uint64_t lw[6] = {0, 0, 0, 0, 0, 0};
        {
            const long long p1 = (long long)tile - 1 - (long long)t;
            if (FLTEE_FC_LB && FLTEE_FC_LBPRE && p1 >= 0) {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    lw[i] = __hip_atomic_load(&lb[p1].inc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    lw[3 + i] = __hip_atomic_load(&lb[p1].agg[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __syncthreads();
        // the first G levels, exactly compact_pass's (contiguous: W = 1, j0 = 0); all nine at
        // compile time when the array has that many (FLTEE_CP_CT, cp_levels_ct)
        bool lv_done = false;
        if constexpr (FLTEE_CP_CT) {
            if (G == 9 && S + H == CAP) {
                cp_levels_ct<NT, PER, 9, 0, (int)CAP>(sm, 0u, t);
                lv_done = true;
            }
        }
        uint64_t nv[PER];
        for (uint32_t g = 0; g < (lv_done ? 0u : G);) {
            const uint32_t stepf = 1u << g;
            const bool two = FLTEE_CP_TWO && g + 1 < G;
            const uint32_t gl = two ? g + 1 : g;
            const uint32_t lmt = S + H - ((2u << gl) - 1);
            if (two) {
#pragma unroll
                for (uint32_t i = 0; i < PER; ++i) {
                    const uint32_t f = t + i * NT;
                    if (f < lmt) {
                        const uint64_t y0 = cp_pick(sm[f], sm[f + stepf], g);
                        const uint64_t y2 = cp_pick(sm[f + 2 * stepf], sm[f + 3 * stepf], g);
                        nv[i] = cp_pick(y0, y2, g + 1);
                    }
                }
            } else {
#pragma unroll
                for (uint32_t i = 0; i < PER; ++i) {
                    const uint32_t f = t + i * NT;
                    if (f < lmt) nv[i] = cp_pick(sm[f], sm[f + stepf], g);
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t i = 0; i < PER; ++i) {
                const uint32_t f = t + i * NT;
                if (f < lmt) sm[f] = nv[i];
            }
            __syncthreads();
            g += two ? 2 : 1;
        }
        // the carry from in front of the window (decoupled look-back; FLTEE_FC_LB=0: none,
        // an A/B of its cost only) into the window head run's record, if it began before
        FoldAgg wc = fa_empty();
        if (FLTEE_FC_LB) {
            wc = fc_lookback<NW>(lb, tile, epoch, t, status, lb_sh, lb_shf, lw);
            if (t == 0) fc_put(lb[tile].inc, fa_combine(wc, agg_s), epoch);
        }
        const bool wok = (wc.fl & kFsPiece) && wc.K == kw0_s;
        const uint32_t fx = fix_s;
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) {
            const uint32_t f = t + i * NT;
            if (f < S) {
                const long long p = a + f;
                uint64_t rv = sm[f];
                const float fv = __fadd_rn(wc.Q, rec_val(rv));
                rv = (wok && f == fx) ? ((rv & 0xFFFFFFFFull) | ((uint64_t)__float_as_uint(fv) << 32)) : rv;
                if (FINAL == 0) {
                    if (p < (long long)L) dst[p] = rv;
                } else if (p < (long long)d) {
                    const float vv = cp_out(rv);
                    out[p] = FINAL == 2 ? __fadd_rn(out[p], vv) : __fmul_rn(vv, coef);
                }
            }
        }
        if (next >= ntiles) break;
        __syncthreads();  // this tile's LDS reads retire before the next window lands
        tile = next;
    }
}

static bool g_fold_compact = true;  // fltee_debug_set_fold_compact (A/B)
void set_fold_compact(int on) { g_fold_compact = on != 0; }

// The fold (fold_len == L) + the compaction of `advanced`: sorted array A (M records,
// [0, L) meaningful) -> out.  A and B are clobbered.  hipErrorNotSupported: not fused
// here (halo wide against the 4096-record tile, or no levels): the caller folds separately.
// lb: fc_lookback_bytes() of look-back slots, zeroed when allocated; *epoch: this
// device's launch counter (the slots of earlier launches never match a later epoch).
template <int PER, int F, int X>
static hipError_t fc_launch(uint64_t ntiles, size_t lds, hipStream_t s, const uint64_t *A, uint64_t *B,
                            size_t L, size_t M, size_t d, uint32_t G, uint32_t S, size_t Hr,
                            float coef, float *out, uint32_t lim, FcLb *lb, uint32_t epoch,
                            uint32_t *status) {
    constexpr int NT = 512;
    constexpr int BPC = FLTEE_FC_BLOCKS;
    auto kern = fold_compact_first<NT, PER, F, X, BPC>;
    // the grid never exceeds the blocks resident at once (the look-back waits for tiles of
    // lower index only: they are running), whatever the occupancy turns out to be
    static int resident = 0;
    static size_t res_lds = 0;
    if (!resident || res_lds != lds) {
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  80 * 1024);
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kern, NT, lds) !=
                hipSuccess)
            return hipErrorLaunchFailure;
        if (per_cu > BPC) per_cu = BPC;
        resident = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
        res_lds = lds;
    }
    const unsigned grid = (unsigned)(ntiles < (uint64_t)resident ? ntiles : (uint64_t)resident);
    FLTEE_LAUNCH(kern, dim3(grid), dim3(NT), lds, s, A, B, (uint32_t)L, (uint32_t)M,
                       (uint32_t)d, G, S, (uint32_t)Hr, (uint32_t)ntiles, coef, out, lim, lb, epoch,
                       status);
    return hipGetLastError();
}

template <int PER>
static hipError_t fc_dispatch(int F, bool x1, uint64_t ntiles, size_t lds, hipStream_t s,
                              const uint64_t *A, uint64_t *B, size_t L, size_t M, size_t d,
                              uint32_t G, uint32_t S, size_t Hr, float coef, float *out,
                              uint32_t lim, FcLb *lb, uint32_t epoch, uint32_t *status) {
#define FC_ARGS ntiles, lds, s, A, B, L, M, d, G, S, Hr, coef, out, lim, lb, epoch, status
    if (F == 0) return x1 ? fc_launch<PER, 0, 1>(FC_ARGS) : fc_launch<PER, 0, 2>(FC_ARGS);
    if (F == 2) return x1 ? fc_launch<PER, 2, 1>(FC_ARGS) : fc_launch<PER, 2, 2>(FC_ARGS);
    return x1 ? fc_launch<PER, 1, 1>(FC_ARGS) : fc_launch<PER, 1, 2>(FC_ARGS);
#undef FC_ARGS
}

// the fused pass's tile geometry for this shape (false: not fused)
struct FcShape {
    uint32_t per, G, S, lim;
    size_t Hr, ntiles;
};
static bool fc_shape(size_t M, size_t L, size_t d, size_t halo, FcShape &o) {
    constexpr uint32_t NT = 512;
    // the window reaches lim = halo + 1 records back: every run of <= halo + 1 entries
    // (each client's indices distinct) folds bit for bit
    o.Hr = fold_context(halo + 1);
    o.lim = halo + 1 >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(halo + 1);
    // A/B in one process (scripts/ab_fold_compact.py, profiles/r02/ab/fold_compact.jsonl):
    // C3 (Hr = 112): 0.211 vs 0.214 ms with the separate fold; C5 (Hr = 1008, windows 25 %
    // wider than the tile): 17.66 vs 17.48 ms in round 2, when it stayed separate; round 3
    // (spill-free compaction): C5 13.22 vs 13.32 ms fused (`profiles/r03/ab/ab10_*`), so the
    // fold is fused whenever the halo fits two window slots per lane (Hr < 1024).
    // (Tried in round 3 and not kept: batched branch-free level rounds, 505.6 -> 517 us per
    // pass; the block-swizzled layout between the passes, 508 -> 503 us, `ab12_*`, `ab13_*`,
    // and again in round 4 with the 16-B slot pairs: 414-418 us either way,
    // `profiles/r04/ab/ab15_compact_swizzle_v2_rejected.jsonl`; 64 KiB tiles, 3 passes of 6
    // levels, as slow as 4 of 5, `ab11_*`.)
    if (!g_fold_compact || d == 0 || L <= d || o.Hr + 1 > 2 * 512 || M >= ((size_t)1 << 29) || L > M)
        return false;
    if (o.lim > kFixedWalkMax && !(o.lim <= kFixedWalkMaxSmall && M <= ((size_t)1 << 20)))
        return false;  // the streaming fold
    const uint32_t nlev = bitlen(L - d);
    o.G = nlev < 9 ? nlev : 9;
    const uint32_t H = (1u << o.G) - 1;
    // records per lane: the fewest (4, 6 or 8) that still leave at most one tile per CU —
    // each lane's walk and levels are the critical path, the window re-read is cheap
    o.per = 8;
    for (uint32_t p : {4u, 6u}) {
        if (NT * p <= 2 * H) continue;  // the halo rows would swamp the tile
        if ((L + NT * p - H - 1) / (NT * p - H) <= 256 * FLTEE_FC_TILES_PER_CU) {
            o.per = p;
            break;
        }
    }
    const uint32_t CAP = NT * o.per;
    o.S = CAP - H;
    o.ntiles = (L + o.S - 1) / o.S;
    // the window, the walks' run sums and the run partials beside it; the resident blocks
    // per CU must fit the 160 KiB LDS (lim <= 320: 71 KiB a block)
    const size_t lds = (o.Hr + CAP + 1) * 12;  // the window (8 B a slot), its sums (4 B)
    return lds * FLTEE_FC_BLOCKS <= 160 * 1024 && lds <= 80 * 1024;
}

size_t fc_lookback_bytes(size_t M, size_t L, size_t d, size_t halo) {
    FcShape o;
    return fc_shape(M, L, d, halo, o) ? o.ntiles * sizeof(FcLb) : 0;
}

hipError_t launch_fold_compact_extract(uint64_t *A, uint64_t *B, size_t M, size_t L, size_t d,
                                       size_t halo, float coef, float *out, bool accumulate,
                                       uint32_t *status, hipStream_t s, void *lb, size_t lb_cap,
                                       uint32_t *epoch) {
    constexpr uint32_t NT = 512;
    FcShape o;
    if (!fc_shape(M, L, d, halo, o)) return hipErrorNotSupported;
    if (!lb || lb_cap < o.ntiles * sizeof(FcLb) || !epoch) return hipErrorInvalidValue;
    if (++*epoch >= (1u << 30)) return hipErrorInvalidValue;  // the caller re-zeroes the slots
    const uint32_t nlev = bitlen(L - d);
    const uint32_t CAP = NT * o.per;
    const bool last = o.G == nlev;
    const size_t lds = (o.Hr + CAP + 1) * 12;  // the window (8 B a slot), its sums (4 B)
    net_account((uint64_t)(last ? 8 : 16) * L, "fold_compact_first", s);
    const bool x1 = o.Hr + 1 <= NT;  // one window slot past CAP per lane, else two
    const int F = !last ? 0 : (accumulate ? 2 : 1);
    FcLb *l = (FcLb *)lb;
    hipError_t e;
#define FC_GO(P_) fc_dispatch<P_>(F, x1, o.ntiles, lds, s, A, B, L, M, d, o.G, o.S, o.Hr, coef, out, \
                                  o.lim, l, *epoch, status)
    if (o.per == 4) e = FC_GO(4);
    else if (o.per == 6) e = FC_GO(6);
    else e = FC_GO(8);
#undef FC_GO
    if (e != hipSuccess || last) return e;
    return compact_levels(B, A, L, d, L - d, coef, out, accumulate, s, o.G);
}

// ------------------------------------------------ one range of the array ---
// Position-sharded `advanced` (SURVEY §8e Option B): after the fold, one GPU holds a
// range of c folded records whose run representatives are some indices in [0, d),
// each at most once, in ascending order.  buf = d unselected entries (u32::MAX, +0.0)
// followed by the range: every representative then sits at a position p >= d > idx,
// so the same left-moving network brings each to position idx — fixed addresses,
// no data-dependent offset (the range's first index is never used).  out[i] gets
// val * coef where this range holds index i and +0.0 elsewhere; the ranges' outputs
// are then summed (RCCL reduce): exactly one range holds each index, so the sum is
// that value, bit for bit (x + 0.0 == x: a run sum includes the +0.0 initial entry
// and is never -0.0).
__global__ void offset_copy_kernel(const uint64_t *__restrict__ chunk, size_t c, size_t d,
                                   uint64_t *__restrict__ buf) {
    const size_t L = d + c;
    for (size_t p = (size_t)blockIdx.x * 256 + threadIdx.x; p < L; p += (size_t)gridDim.x * 256)
        buf[p] = p < d ? CP_DUMMY : chunk[p - d];
}

hipError_t launch_compact_offset(const uint64_t *chunk, size_t c, size_t d, uint64_t *buf,
                                 uint64_t *tmp, float coef, float *out, hipStream_t s) {
    if (d == 0) return hipSuccess;
    const size_t L = d + c;
    if (L >= ((size_t)1 << 29)) return hipErrorInvalidValue;
    size_t blocks = (L + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    FLTEE_LAUNCH(offset_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, chunk, c, d,
                       buf);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return compact_levels(buf, tmp, L, d, L - 1, coef, out, false, s);
}

}  // namespace fltee
