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
//   mode 2: cond2 = top bit of (l ^ stepkey(seed,i,j)) * 0x9E3779B1  (nips19.rs:66-105;
//           keyed mixer replaces the running FxHash of heap addresses)
// Every compare-exchange is branch-free (v_cndmask) and every address depends
// only on (i, j, k): the memory trace is data-independent, like the cmov
// network it replaces.  Compare-exchanges of one step are disjoint, so any
// grouping of consecutive steps that keeps their order is the same network.
//
// Grouping.  R consecutive steps j = 2^jtop .. 2^(jtop-R+1) of one stage only
// pair records whose positions differ in bits [jtop-R+1, jtop]: the 2^R records
// {b + q * 2^(jtop-R+1)} form a closed group that one lane can run through all
// R steps in registers.
//   tile_sort   : stages 2..T in LDS (T = 2^t <= 8192 records = 64 KB); each lane
//                 holds 16 records per round, i.e. 4 steps per barrier.
//   per stage i > T:
//     global    : steps j >= T in passes of up to 6 steps (64 records / lane in
//                 registers), HBM traffic 2*M*8 bytes per pass;
//     merge     : steps j < T in one LDS launch (4 steps per barrier).
// LDS layout pads one slot per 16 records so that the 64 lanes of a wave hit
// distinct banks when each walks a 16-record group.
#include <map>
#include <mutex>
#include <vector>

#include "common.h"

// A/B switches of the tile kernels' code shape (compile time; scripts/ab_build.sh):
//   FLTEE_CE_BATCH   a step's swap decisions all computed before its selects
//   FLTEE_LDS_BATCH  groups per batch of a round's LDS reads issued before their
//                    compare-exchanges and writes (0: all of the lane's groups)
#ifndef FLTEE_CE_BATCH
#define FLTEE_CE_BATCH 1
#endif
#ifndef FLTEE_LDS_BATCH
#define FLTEE_LDS_BATCH 2
#endif
//   FLTEE_KEY_AFTER_DATA  the keyed comparator's step keys computed after each round's loads
#ifndef FLTEE_KEY_AFTER_DATA
#define FLTEE_KEY_AFTER_DATA 1
#endif
//   FLTEE_KEYED_SPLIT  the keyed comparator as one per-lane product per step + a scalar
//                      (off: it moves the cost to the scalar unit, C4 8.93 vs 9.01 ms with
//                      it, `profiles/r03/ab/ab6_c4.jsonl`)
#ifndef FLTEE_KEYED_SPLIT
#define FLTEE_KEYED_SPLIT 0
#endif
//   FLTEE_KEYED_DIRFOLD  the keyed comparator with the direction folded into the hashed word
//                        (keyed_swap; off: the round-3 form, for A/B)
#ifndef FLTEE_KEYED_DIRFOLD
#define FLTEE_KEYED_DIRFOLD 1
#endif
template <int G>
constexpr int kLdsBatch = (FLTEE_LDS_BATCH == 0 || FLTEE_LDS_BATCH > G) ? G : FLTEE_LDS_BATCH;
//   FLTEE_LDS_READ1   LDS reads as single ds_read_b64 (no ds_read2_b64 pairing)
#ifndef FLTEE_LDS_READ1
#define FLTEE_LDS_READ1 0
#endif
//   FLTEE_TILE_HEADREG  a strided tile's first row round on its prefetch registers
#ifndef FLTEE_TILE_HEADREG
#define FLTEE_TILE_HEADREG 1
#endif
//   FLTEE_TAIL_CT_1024  compile-time tail rounds in the 1024-lane strided tiles too
#ifndef FLTEE_TAIL_CT_1024
#define FLTEE_TAIL_CT_1024 1
#endif
//   FLTEE_PLAN_SHUFFLE  the keyed shuffle (mode 2) on the planned schedule too
#ifndef FLTEE_PLAN_SHUFFLE
#define FLTEE_PLAN_SHUFFLE 1
#endif
//   FLTEE_TID_FRESH   the lane id re-read per LDS round (see lane_tid)
#ifndef FLTEE_TID_FRESH
#define FLTEE_TID_FRESH 1
#endif
//   FLTEE_WAVE_LOCAL  the first pass's stages inside a wave's records without block barriers
#ifndef FLTEE_WAVE_LOCAL
#define FLTEE_WAVE_LOCAL 1
#endif
//   FLTEE_WAVE_SPLIT  the first pass's stages above log2(64 E): the steps that cross waves
//   block-wide, then the stage's steps inside a wave's records wave-local (1: always;
//   2: only where the split adds no LDS round; 0: the whole stage block-wide).  A/B
//   (`profiles/r04/ab/ab6_wave_split.jsonl`): 2 takes C4's first pass 1,085 -> 1,065 us and
//   C5's 1,234 -> 1,227 us; 1 is slower than 0 (the extra rounds cost more than the barriers)
#ifndef FLTEE_WAVE_SPLIT
#define FLTEE_WAVE_SPLIT 2
#endif
//   FLTEE_TILE_PAIRS  the compile-time-shaped tile passes load and store slot pairs (16 B
//   per lane: lane t holds tile elements 2t, 2t + 1 (+ 2 NT r)) instead of single records
#ifndef FLTEE_TILE_PAIRS
#define FLTEE_TILE_PAIRS 1
#endif
//   FLTEE_MERGE_PAIRS  the same for the contiguous direct merges (bitonic_merge_direct):
//   1 all, 2 the selecting last pass of nips19's shuffle only, 0 none.  A/B
//   (`profiles/r04/ab/ab9_merge_pairs_*.jsonl`): the selecting pass 552 -> 517 us, the
//   plain merges 251 -> 279 us (C4) / 335 -> 364 us (C5) — their last round then stores
//   groups of 8 instead of 4
#ifndef FLTEE_MERGE_PAIRS
#define FLTEE_MERGE_PAIRS 2
#endif
// (Measured and removed, round 4: the first pass over 2^14 tiles as 512 lanes x 32 records —
// 5 steps per LDS round, stages 1..5 in registers — 1,640 vs 1,068 us at C4, 1,821 vs 1,220
// at C5: the compile-time rounds spill at 32 records per lane and the runtime ones run
// slower; `profiles/r04/ab/ab12_first_pass_e32_rejected_*.jsonl`.  Likewise C3's 2^12 tiles as
// 256 lanes x 16: 24.0 vs 21.0 us, `ab14_first_pass_256x16_c3_rejected.jsonl`.)
//   FLTEE_SEL_STORE_OOB  the selecting pass stores every record, the unselected ones out of
//   the tile's buffer range (dropped), instead of a branch per record (A/B: 530 vs 520 us,
//   not kept; `profiles/r04/ab/ab10_sel_store_oob_c4.jsonl`)
//   FLTEE_TAIL_CT_KEYED  compile-time tail rounds for the keyed shuffle (mode 2) too (round 4:
//   no spills since the 1024-lane tiles lost theirs; C4 8.00 -> 7.89 ms, bit-identical,
//   `profiles/r04/ab/ab18_keyed_tail_ct_c4.jsonl`)
#ifndef FLTEE_TAIL_CT_KEYED
#define FLTEE_TAIL_CT_KEYED 1
#endif
//   FLTEE_TILE_W10  compile-time rounds for the 1024-lane strided tiles with rows of 2^10 too
//   (the planned passes with a 10-step tail; round 4: C4 7.90 -> 7.84 ms, C5 unchanged,
//   `profiles/r04/ab/ab19_tile_w10_*.jsonl`)
#ifndef FLTEE_TILE_W10
#define FLTEE_TILE_W10 1
#endif
//   FLTEE_TILE_MINW14  the narrowest rows (log2 records) of a planned strided 2^14 tile: 4
//   (128-B row segments) or 3 (64-B segments: 11 row steps per pass; the plan may then use
//   rows of 2^8 too, compiled with it).  At M = 2^27 the plan drops from 23 to 22 launches,
//   but the passes on 64-B rows run far slower (round 5, bit-identical: C5 12.29 -> 13.65
//   ms, C4 7.85 -> 8.45 ms; tile passes 367 -> 447 us on average,
//   `profiles/r05/ab/ab14_tile_rows_of_8_rejected.jsonl`), so 4 stays.
//   FLTEE_TILE_SKIP_SELF  a tile pass's block on its last tile prefetches nothing (round 5,
//   bit-identical: C3 0.1295 -> 0.1285 ms, C4 / C5 unchanged, `profiles/r05/ab/ab21_*`)
#ifndef FLTEE_TILE_SKIP_SELF
#define FLTEE_TILE_SKIP_SELF 1
#endif
#ifndef FLTEE_TILE_MINW14
#define FLTEE_TILE_MINW14 4
#endif
//   FLTEE_TILE_MINW12  the same for the 512-lane 2^12 tiles (M <= 2^20: C3 13 -> 12 launches,
//   0.1365 -> 0.1387 ms, same record)
#ifndef FLTEE_TILE_MINW12
#define FLTEE_TILE_MINW12 4
#endif
#ifndef FLTEE_DIRECT_MERGE
#define FLTEE_DIRECT_MERGE 0
#endif
#ifndef FLTEE_UNSW_TILES
#define FLTEE_UNSW_TILES 1
#endif
#ifndef FLTEE_SEL_STORE_OOB
#define FLTEE_SEL_STORE_OOB 0
#endif

namespace fltee {

// cond2 of the compare-exchange at position l (see the header comment)
template <int MODE>
__device__ __forceinline__ bool cond2(uint64_t a, uint64_t b, uint32_t l, uint32_t key) {
    if (MODE == 0) return (uint32_t)a < (uint32_t)b;
    if (MODE == 1) return a < b;
    return (((l ^ key) * 0x9E3779B1u) >> 31) != 0;  // multiplicative hash, top bit
}

// insert r zero bits at bit position d of g
__device__ __forceinline__ uint32_t spread(uint32_t g, uint32_t d, uint32_t r) {
    const uint32_t lo = g & ((1u << d) - 1u);
    return ((g >> d) << (d + r)) | lo;
}

// The same value, made to depend on a loaded record (an SGPR the compiler cannot see
// through): the keyed comparator's step keys and swap decisions depend on positions only,
// so without this hipcc computes those of a whole tile up front and spills them.
__device__ __forceinline__ uint32_t after_data(uint32_t s, uint32_t v) {
    asm volatile("; after_data %1" : "+s"(s) : "v"(v));
    return s;
}

// The keyed comparator (MODE 2) split into a per-lane and a wave-uniform part.  For a
// group whose first position p0 has zero bits where dq = q << dlog has ones, l = p0 + dq
// = p0 ^ dq, so l ^ key = x ^ dq = x + dq - 2 (key & dq) with x = p0 ^ key, and
//   (l ^ key) * K = x * K + (dq - 2 (key & dq)) * K   (mod 2^32):
// the top bit cond2<2> takes is the sign of X + C(dq), X = x * K once per group and step,
// C(dq) computed by the scalar unit.  One v_add per compare instead of an add, a xor and
// a v_mul_lo_u32; the same bits.
__device__ __forceinline__ uint32_t keyed_c(uint32_t key, uint32_t dq) {
    return (dq - 2u * (key & dq)) * 0x9E3779B1u;
}

// The keyed comparator (MODE 2) with the block's direction folded into the hashed word.
// swap = asc ^ top bit of ((l ^ key) * K).  For S in {0, 2^31}: (y ^ S) * K = y * K + S
// (mod 2^32; K odd), so the top bit of ((l ^ key ^ S) * K) is that of (l ^ key) * K,
// flipped when S = 2^31.  With S = 2^31 for an ascending block (l < 2^29 never has bit 31)
// swap = sign of ((l ^ key ^ S) * K): the same bits as cond2<2>, in a xor, a v_mul_lo and
// one signed compare (instead of a shift and a compare with the direction), and the key,
// the direction and the group's first position are joined once per group and step
// (l = p0 ^ (q << dlog): p0 has zeros there).
__device__ __forceinline__ uint32_t keyed_dir(bool asc) { return asc ? 0x80000000u : 0u; }
__device__ __forceinline__ bool keyed_swap(uint32_t kb, uint32_t dq) {
    return (int32_t)((kb ^ dq) * 0x9E3779B1u) < 0;
}

// The keyed comparator read from a table (round 5, FLTEE_KEYED_TABLE).  With kb = p0 ^
// dir ^ key and dq = q << dlog (p0 has zeros at dq's bits, dq < 2^31): kb & dq = key & dq,
// so (kb ^ dq) * K = kb * K + C(dq) with C(dq) = keyed_c(key, dq) — one product per group
// and step (X) and, per compare-exchange, one v_add of a per-(step, q) constant and the
// sign test, instead of a v_xor, a half-rate v_mul_lo_u32 and the sign test: 6 VALU issue
// slots per compare-exchange instead of 9.  The constants of every step a network can run
// — T[ilog][jlog][lv][q] = keyed_c(step_key(seed, ilog, jlog), q << (jlog - lv)), the
// group's steps lv = 0..3 at distance 2^(jlog - lv) — sit in a per-device table of 256 KB
// built for the network's seed before its first pass (keyed_table_prepare, stream-
// ordered), and a step's 16 constants come in as one scalar load (s_load_dwordx16) into
// SGPRs: no VALU, no LDS.  Every address is a function of (ilog, jlog, lv) — public — and
// the bits are the same (a ring identity mod 2^32).  Groups of more than 16 records (the
// register passes of 5 and 6 steps) keep the direct form.
// Measured and REJECTED (off by default): C4 8.45 vs 7.85 ms, bit-identical
// (`profiles/r05/ab/ab5_keyed_table_c4_rejected.jsonl`).  The asm has a quarter of the
// multiplies (222 vs 846 v_mul_lo_u32 in the first pass), but every scalar load is counted
// in the same lgkm counter as the LDS reads and returns out of order, so each use of a row
// waits for ALL outstanding LDS reads (lgkmcnt(0): 116 such waits in the pass against 63
// in the index sort's) — the LDS rounds lose their overlap.
#ifndef FLTEE_KEYED_TABLE
#define FLTEE_KEYED_TABLE 0
#endif
__device__ const uint32_t *g_keyed_tab;  // this device's table (set once per device)
typedef __attribute__((address_space(4))) const uint32_t kt_u32;  // scalar (constant) loads
__device__ __forceinline__ const kt_u32 *keyed_row(uint32_t ilog, uint32_t jlog, uint32_t lv) {
    return (const kt_u32 *)g_keyed_tab + ((((ilog & 31u) << 5) | (jlog & 31u)) * 4u + lv) * 16u;
}
constexpr uint32_t kKeyedTabEntries = 32u * 32u * 4u * 16u;

__global__ void keyed_table_kernel(uint32_t *__restrict__ tab, uint32_t seed) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kKeyedTabEntries) return;
    const uint32_t q = i & 15u, lv = (i >> 4) & 3u, jlog = (i >> 6) & 31u, ilog = i >> 11;
    uint32_t c = 0;
    if (lv <= jlog) c = keyed_c(shuffle_step_key(seed, ilog, jlog), q << (jlog - lv));
    tab[i] = c;
}

struct KeyedTab {
    uint32_t *ptr = nullptr;
    uint32_t seed = 0;
    bool valid = false;
};
static KeyedTab g_kt[64];

// the table for `seed` on the current device, ahead of the network's launches on s (a
// device's networks run on one stream at a time: the library's calls are serialised)
static hipError_t keyed_table_prepare(uint32_t seed, hipStream_t s) {
    if (!FLTEE_KEYED_TABLE) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess || dev < 0 || dev >= 64) return e != hipSuccess ? e : hipErrorInvalidDevice;
    KeyedTab &t = g_kt[dev];
    if (!t.ptr) {
        e = hipMalloc(&t.ptr, kKeyedTabEntries * 4);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_keyed_tab), &t.ptr, sizeof(t.ptr));
        if (e != hipSuccess) {
            t.ptr = nullptr;
            return e;
        }
        t.valid = false;
    }
    if (t.valid && t.seed == seed) return hipSuccess;
    FLTEE_LAUNCH(keyed_table_kernel, dim3(kKeyedTabEntries / 256), dim3(256), 0, s, t.ptr, seed);
    e = hipGetLastError();
    t.seed = seed;
    t.valid = e == hipSuccess;
    return e;
}

// Run steps lv = R-1..0 (distance 2^(dlog+lv)) of stage ilog on one group of 2^R
// records held in v[], whose first record sits at global position p0.  The group
// spans 2^(dlog+R) <= 2^ilog aligned positions, so the direction bit (l & i) == 0
// is the same for every compare-exchange of the group: computed once.
template <int MODE, int R>
__device__ __forceinline__ void group_steps(uint64_t (&v)[1 << R], uint32_t p0, uint32_t dlog,
                                            uint32_t ilog, uint32_t seed) {
    if constexpr (MODE == 2 && FLTEE_KEY_AFTER_DATA) seed = after_data(seed, (uint32_t)v[0]);
    const bool asc = (p0 & (1u << ilog)) == 0;
    const uint32_t pdir = MODE == 2 ? p0 ^ keyed_dir(asc) : 0u;
#pragma unroll
    for (int lv = R - 1; lv >= 0; --lv) {
        const uint32_t key = MODE == 2 ? shuffle_step_key(seed, ilog, dlog + lv) : 0u;
        const uint32_t X = (MODE == 2 && FLTEE_KEYED_SPLIT) ? (p0 ^ key) * 0x9E3779B1u : 0u;
        const uint32_t kb = pdir ^ key;
        constexpr bool kTab = MODE == 2 && FLTEE_KEYED_TABLE && R <= 4;
        const uint32_t XT = kTab ? kb * 0x9E3779B1u : 0u;
        const kt_u32 *row = kTab ? keyed_row(ilog, dlog + (uint32_t)lv, (uint32_t)lv) : nullptr;
        auto decide = [&](int q, int qm) -> bool {
            if constexpr (kTab) return (int32_t)(XT + row[q]) < 0;
            if constexpr (MODE == 2 && FLTEE_KEYED_SPLIT)
                return asc ^ ((int32_t)(X + keyed_c(key, (uint32_t)q << dlog)) < 0);
            if constexpr (MODE == 2 && FLTEE_KEYED_DIRFOLD) return keyed_swap(kb, (uint32_t)q << dlog);
            return asc ^ cond2<MODE>(v[q], v[qm], p0 + ((uint32_t)q << dlog), key);
        };
#if FLTEE_CE_BATCH
        // every swap decision of the step first, then the selects: the compares are
        // independent, so their mask chains (v_cmp -> s_xor -> v_cndmask) overlap
        bool sw[(1 << R) / 2];
#pragma unroll
        for (int q = 0, k = 0; q < (1 << R); ++q) {
            if (q & (1 << lv)) continue;
            sw[k++] = decide(q, q | (1 << lv));
        }
#pragma unroll
        for (int q = 0, k = 0; q < (1 << R); ++q) {
            if (q & (1 << lv)) continue;
            const int qm = q | (1 << lv);
            const uint64_t a = v[q], c = v[qm];
            const bool s = sw[k++];
            v[q] = s ? c : a;
            v[qm] = s ? a : c;
        }
#else
#pragma unroll
        for (int q = 0; q < (1 << R); ++q) {
            if (q & (1 << lv)) continue;
            const int qm = q | (1 << lv);
            const uint64_t a = v[q], c = v[qm];
            const bool sw = decide(q, qm);
            v[q] = sw ? c : a;
            v[qm] = sw ? a : c;
        }
#endif
    }
}

// An 8-B LDS read the compiler does not pair into ds_read2_b64: on gfx950 that form takes
// 8 LDS cycles for two 512-B wave accesses, two ds_read_b64 take 4 (MI355X_MICROARCH.md
// LDS table).  A volatile access is never merged (FLTEE_LDS_READ1).
__device__ __forceinline__ uint64_t lds_ld(const uint64_t *p) {
#if FLTEE_LDS_READ1
    typedef __attribute__((address_space(3))) const volatile uint64_t lds_cv_u64;
    return *(lds_cv_u64 *)p;
#else
    return *p;
#endif
}

// The lane id, re-defined where it is read (FLTEE_TID_FRESH): a round's per-lane LDS
// addresses are then computed in the round (a few VALU) instead of being hoisted out of
// the tile loop as loop invariants and spilled (a spill's reload waits vmcnt(0), i.e. for
// the previous tile's stores and the prefetch in flight).
// Only the 1024-lane kernels (held to 128 VGPRs) need it: at 512 lanes the recomputation
// costs more than it saves (C3 0.1518 vs 0.1484 ms, `profiles/r03/ab/`).
template <int NT>
__device__ __forceinline__ uint32_t lane_tid() {
    uint32_t t = threadIdx.x;
    if constexpr (FLTEE_TID_FRESH && NT >= 1024) asm volatile("; lane_tid" : "+v"(t));
    return t;
}

// One wave's LDS accesses stay in program order (the LDS executes a wave's DS
// instructions in issue order), so between wave-local rounds only the compiler must be
// kept from moving a later round's LDS reads above an earlier round's writes: the
// __syncwarp idiom — wavefront-scope release/acquire fences around the wave barrier.  The
// bare wave barrier touches no memory and orders nothing at the compiler level; the
// wavefront-scope fences emit no instructions (ISA unchanged, `make asm`).
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Raw buffer access: byte offset = soffset (wave-uniform, SGPR) + voffset (per lane).
typedef unsigned int bt_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int bt_u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBufNT = 2;  // cache policy: nontemporal (streaming, each byte used once)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t bt_rsrc(uint64_t *data) {
    return __builtin_amdgcn_make_buffer_rsrc(data, (short)0, (int)0xFFFFFFFF, 0x00020000);
}
template <int CP = kBufNT>
__device__ __forceinline__ uint64_t bt_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
    const bt_u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)voff, (int)soff, CP);
    return ((uint64_t)x.y << 32) | x.x;
}
template <int CP = kBufNT>
__device__ __forceinline__ void bt_store(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                         uint64_t v) {
    const bt_u32x2 x = {(uint32_t)v, (uint32_t)(v >> 32)};
    __builtin_amdgcn_raw_buffer_store_b64(x, rs, (int)voff, (int)soff, CP);
}
// tile kernels: default cache policy (nontemporal measured slower there: 504 vs 469 us).
// Where a 2^14-tile merge pass goes at M = 2^27 (MI355X, rocprofv3): 468 us in all;
// 390 us with the LDS rounds skipped (load -> LDS -> store only), 340 us with the
// global stores skipped; a register-only pass (bitonic_global R=1) streams at 321 us.
// Tried and dropped: the steps below 2^10 in registers (lane exchanges by DPP /
// v_permlane16/32_swap, no LDS) — correct, but 577 us per merge and 9.5 ms for the
// tile sort (spills at 1024 lanes; ~12 VALU per record per cross-lane step).
constexpr int kTileCP = 0;

// Block-swizzled physical layout (round 3, common.h phys) of the 2^14-tile networks (C4,
// C5): between its first and its last pass a full sort keeps logical position p at
// physical slot
//   phys(p) = p ^ (((h ^ (h >> 10)) << 4) & 0x3FF0),  h = p >> 14,
// i.e. the 128-B blocks (16 records) inside each aligned 2^14-record block are permuted
// by a function of the block's position bits >= 14.  A strided tile's rows (W = 16..128
// consecutive records, 2^dtile apart) otherwise sit at power-of-two strides that map one
// wave's rows onto the same HBM channels (MI355X: W = 16 rows 2^14 apart stream at 3.5
// TB/s, swizzled 5.1, `profiles/r03/microbench_tiles_*.jsonl`).  Properties used:
//  * bits >= 14 are unchanged, so a contiguous 2^14 tile occupies its own block in either
//    layout (the first pass reads logical and writes physical, the last pass the other
//    way round, both in place) and whole pad blocks are the same in both;
//  * bits 0..3 are unchanged, so every 16-record row segment stays contiguous;
//  * it is GF(2)-linear: phys(a ^ b) = phys(a) ^ phys(b), so for an address made of
//    bit-disjoint fields (tile base | lane part | row part) the per-lane and the uniform
//    parts are swizzled separately and combined with one XOR.
// Only addresses change: positions (directions, keys) stay logical — the same network.
// A tile record's HBM access: lane part `vl` (bytes; SW: phys(lane part) * 8) and uniform
// record index `u` (the tile base plus the record's row part, bit-disjoint from the lane
// part).  !SW: voffset + soffset as before; SW: one XOR into the voffset.
template <bool SW>
__device__ __forceinline__ uint64_t tl_load(__amdgpu_buffer_rsrc_t rs, uint32_t vl, uint32_t u) {
    if constexpr (SW) return bt_load<kTileCP>(rs, vl ^ (phys(u) * 8u), 0u);
    return bt_load<kTileCP>(rs, vl, u * 8u);
}
template <bool SW>
__device__ __forceinline__ void tl_store(__amdgpu_buffer_rsrc_t rs, uint32_t vl, uint32_t u, uint64_t v) {
    if constexpr (SW) bt_store<kTileCP>(rs, vl ^ (phys(u) * 8u), 0u, v);
    else bt_store<kTileCP>(rs, vl, u * 8u, v);
}

// Two adjacent records (16 B, the lane part even): the tile passes' slot pairs.  Stores
// fenced with s_nop 1 (the dwordx4 store data hazard, see bitonic_merge_direct).
template <bool SW>
__device__ __forceinline__ void tl_load2(__amdgpu_buffer_rsrc_t rs, uint32_t vl, uint32_t u, uint64_t &a,
                                         uint64_t &b) {
    const uint32_t off = SW ? (vl ^ (phys(u) * 8u)) : vl;
    const bt_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, SW ? 0 : (int)(u * 8u), kTileCP);
    a = ((uint64_t)x.y << 32) | x.x;
    b = ((uint64_t)x.w << 32) | x.z;
}
template <bool SW>
__device__ __forceinline__ void tl_store2(__amdgpu_buffer_rsrc_t rs, uint32_t vl, uint32_t u, uint64_t a,
                                          uint64_t b) {
    const uint32_t off = SW ? (vl ^ (phys(u) * 8u)) : vl;
    const bt_u32x4 x = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)off, SW ? 0 : (int)(u * 8u), kTileCP);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------- LDS tile ----
__device__ __forceinline__ uint32_t lpad(uint32_t e) { return e + (e >> 4); }

// Tile maps.  A tile is T = 2^tlog records: W = 2^wlog consecutive positions times
// T/W rows at stride 2^dtile (wlog <= dtile).  Contiguous tiles: wlog = dtile = tlog.
// Tile t fixes the position bits outside the tile: bits [wlog, dtile) from t's low
// bits, bits >= dtile + (tlog - wlog) from the rest.
__device__ __forceinline__ uint32_t tile_base(uint32_t t, uint32_t tlog, uint32_t wlog,
                                              uint32_t dtile) {
    const uint32_t mid = dtile - wlog;
    return ((t >> mid) << (dtile + tlog - wlog)) | ((t & ((1u << mid) - 1u)) << wlog);
}
__device__ __forceinline__ uint32_t tile_pos(uint32_t base, uint32_t e, uint32_t wlog,
                                             uint32_t dtile) {
    return base + (e & ((1u << wlog) - 1u)) + ((e >> wlog) << dtile);
}

// Tile / group t of a launch that skips the hole_len pad-only units from hole_at on
// (pad_map): units are numbered in position order, the live ones run as 0 .. n-1.
__device__ __forceinline__ uint32_t past_hole(uint32_t t, uint32_t hole_at, uint32_t hole_len) {
    return t >= hole_at ? t + hole_len : t;
}

// One LDS round: steps at tile-local bits jtop..jtop-R+1 of stage ilog over the whole
// tile of T = E * NT records.  Lane t handles the G = E >> R groups t + h*NT (R <=
// log2 E, so every lane is busy).  A round never straddles bit wlog, so the group's
// global distance is 2^dlog_g and its first record sits at tile_pos(b).
template <int MODE, int R, int E, int NT>
__device__ __forceinline__ void lds_round(uint64_t *sm, uint32_t base, uint32_t wlog,
                                          uint32_t dtile, uint32_t ilog, uint32_t jtop,
                                          uint32_t seed) {
    constexpr int G = E >> R;
    const uint32_t dlog = jtop - R + 1;
    const uint32_t dlog_g = dlog >= wlog ? dlog - wlog + dtile : dlog;
    // every group's records are read before any is written back: the LDS reads of one
    // group cannot be issued ahead of the previous group's writes otherwise (the
    // compiler cannot prove they do not alias), which left G - 1 read latencies exposed
    constexpr int BW = kLdsBatch<G>;
#pragma unroll
    for (int h0 = 0; h0 < G; h0 += BW) {
        uint64_t v[BW][1 << R];
        uint32_t b[BW];
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            b[h] = spread(lane_tid<NT>() + (uint32_t)(h0 + h) * NT, dlog, R);
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) v[h][q] = lds_ld(&sm[lpad(b[h] + ((uint32_t)q << dlog))]);
        }
#pragma unroll
        for (int h = 0; h < BW; ++h)
            group_steps<MODE, R>(v[h], tile_pos(base, b[h], wlog, dtile), dlog_g, ilog, seed);
#pragma unroll
        for (int h = 0; h < BW; ++h) {
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) sm[lpad(b[h] + ((uint32_t)q << dlog))] = v[h][q];
        }
    }
}

// tile-local steps jtop..jbot of stage ilog, up to log2(E) per barrier.  (Tried:
// wave-local rounds without block barriers for steps inside 64*E-record chunks —
// slower on MI355X: +40 us per merge pass from the extra register pressure.)
template <int MODE, int E, int NT>
__device__ __forceinline__ void lds_steps(uint64_t *sm, uint32_t base, uint32_t wlog,
                                          uint32_t dtile, uint32_t ilog, int jtop, int jbot,
                                          uint32_t seed) {
    constexpr int rmax = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    while (jtop >= jbot) {
        const int left = jtop - jbot + 1;
        const int r = left < rmax ? left : rmax;
        if (rmax >= 5 && r == 5) lds_round<MODE, (rmax >= 5 ? 5 : 1), E, NT>(sm, base, wlog, dtile, ilog, (uint32_t)jtop, seed);
        else if (rmax >= 4 && r == 4) lds_round<MODE, (rmax >= 4 ? 4 : 1), E, NT>(sm, base, wlog, dtile, ilog, (uint32_t)jtop, seed);
        else if (rmax >= 3 && r == 3) lds_round<MODE, (rmax >= 3 ? 3 : 1), E, NT>(sm, base, wlog, dtile, ilog, (uint32_t)jtop, seed);
        else if (rmax >= 2 && r == 2) lds_round<MODE, (rmax >= 2 ? 2 : 1), E, NT>(sm, base, wlog, dtile, ilog, (uint32_t)jtop, seed);
        else lds_round<MODE, 1, E, NT>(sm, base, wlog, dtile, ilog, (uint32_t)jtop, seed);
        __syncthreads();
        jtop -= r;
    }
}

// The same rounds for contiguous tiles of a size known at compile time (the direct
// merges of 2^13 / 2^14-record tiles): spread() and the slot offsets fold to constants,
// lpad(b + q*2^DLOG) = lpad(b) + q*2^DLOG + (q*2^DLOG >> 4) (b has zeros at bits
// [DLOG, DLOG+R) and its part above them is a multiple of 16), so every slot is a
// ds_read/ds_write immediate offset off one per-group address — five VALU per slot
// fewer.  Same greedy split into rounds as lds_steps: the same network.
// WL > 0: a strided tile (2^WL consecutive positions x rows 2^dtile apart): the group's
// first position from tile_pos, its global distance 2^(DLOG - WL + dtile) for the rounds
// on the row bits (>= WL) and 2^DLOG for those on the consecutive bits (< WL: a stage's
// tail fused into the tile, plan_network).
// WB > 0: a wave-local round (every group inside the wave's own 2^WB = 64 * E records:
// the wave's 64 lanes x G groups x 2^R records are tile positions wave * 2^WB + [0, 2^WB)),
// so it needs no block barrier before or after it, only the wave's own LDS order.
template <int G>
__device__ __forceinline__ uint32_t round_group(uint32_t t, int h, int NT, int WB) {
    constexpr int gl = G >= 32 ? 5 : (G >= 16 ? 4 : (G >= 8 ? 3 : (G >= 4 ? 2 : (G >= 2 ? 1 : 0))));
    if (!WB) return t + (uint32_t)h * (uint32_t)NT;
    return (t & 63u) | ((uint32_t)h << 6) | ((t >> 6) << (6 + gl));
}

template <int MODE, int R, int E, int NT, int DLOG, int WL = 0, int WB = 0>
__device__ __forceinline__ void lds_round_ct(uint64_t *sm, uint32_t base, uint32_t ilog,
                                             uint32_t seed, uint32_t dtile = 0) {
    static_assert(WL == 0 || DLOG >= WL || DLOG + R <= WL, "a round stays on one side of bit WL");
    static_assert(WB == 0 || (WL == 0 && DLOG + R <= WB && (64 * E) == (1 << WB)), "wave-local round");
    constexpr int G = E >> R;
    const uint32_t dg = (WL && DLOG >= WL) ? (uint32_t)(DLOG - WL) + dtile : (uint32_t)DLOG;
    // all G groups read first, then computed, then written (see lds_round)
    constexpr int BW = kLdsBatch<G>;
#pragma unroll
    for (int h0 = 0; h0 < G; h0 += BW) {
    uint64_t v[BW][1 << R];
    uint32_t b[BW];
#pragma unroll
    for (int h = 0; h < BW; ++h) {
        b[h] = spread(round_group<G>(lane_tid<NT>(), h0 + h, NT, WB), (uint32_t)DLOG, (uint32_t)R);
        if constexpr (DLOG + R >= 4) {
            const uint64_t *row = sm + lpad(b[h]);
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) v[h][q] = lds_ld(&row[(q << DLOG) + ((q << DLOG) >> 4)]);
        } else {  // a group inside 16 records: the padding slot may fall between its records
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) v[h][q] = lds_ld(&sm[lpad(b[h] + ((uint32_t)q << DLOG))]);
        }
    }
#pragma unroll
    for (int h = 0; h < BW; ++h) {
        const uint32_t p0 = WL ? tile_pos(base, b[h], (uint32_t)WL, dtile) : base + b[h];
        group_steps<MODE, R>(v[h], p0, dg, ilog, seed);
    }
#pragma unroll
    for (int h = 0; h < BW; ++h) {
        if constexpr (DLOG + R >= 4) {
            uint64_t *row = sm + lpad(b[h]);
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) row[(q << DLOG) + ((q << DLOG) >> 4)] = v[h][q];
        } else {
#pragma unroll
            for (int q = 0; q < (1 << R); ++q) sm[lpad(b[h] + ((uint32_t)q << DLOG))] = v[h][q];
        }
    }
    }
}
// WB > 0: wave-local rounds (see round_group), ordered by the wave's own LDS order
// (a compiler-only barrier between them) instead of block barriers
template <int MODE, int E, int NT, int JTOP, int JBOT, int WL = 0, int WB = 0>
__device__ __forceinline__ void lds_steps_ct(uint64_t *sm, uint32_t base, uint32_t ilog,
                                             uint32_t seed, uint32_t dtile = 0) {
    if constexpr (JTOP >= JBOT) {
        constexpr int rmax = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
        constexpr int r = JTOP - JBOT + 1 < rmax ? JTOP - JBOT + 1 : rmax;
        lds_round_ct<MODE, r, E, NT, JTOP - r + 1, WL, WB>(sm, base, ilog, seed, dtile);
        if constexpr (WB) wave_lds_order();
        else __syncthreads();
        lds_steps_ct<MODE, E, NT, JTOP - r, JBOT, WL, WB>(sm, base, ilog, seed, dtile);
    }
}

// stages IL..TL-1 in full and stage TL down to step RL (bitonic_sort_direct's LDS part).
// With FLTEE_WAVE_LOCAL the stages up to log2(64 E) (every step inside the wave's own
// records) run as wave-local rounds — no block barrier, so the waves drift apart and one
// wave's LDS traffic overlaps another's compare-exchanges — and one block barrier
// precedes the first stage that crosses waves.  The caller orders the LDS writes in front
// of the first round (a block barrier, or the wave's own order when WAVE_FIRST).
template <int E>
constexpr int kWaveLog = E >= 32 ? 11 : (E >= 16 ? 10 : (E >= 8 ? 9 : (E >= 4 ? 8 : 7)));
// Steps IL-1 .. JBOT of stage IL (> log2(64 E) with FLTEE_WAVE_SPLIT): the steps of
// distance >= 64 E cross waves and run block-wide; the rest stay inside each wave's 64 E
// consecutive records and run as wave-local rounds (no block barrier: the waves drift and
// overlap one another's LDS traffic with their compare-exchanges), then one block barrier.
// The same steps in the same order: the network is unchanged.  Ends in a block barrier.
template <int MODE, int E, int NT, int IL, int JBOT>
__device__ __forceinline__ void stage_steps_ct(uint64_t *sm, uint32_t base, uint32_t seed) {
    constexpr int WB = FLTEE_WAVE_LOCAL ? kWaveLog<E> : 0;
    constexpr int rmax = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    constexpr int r_all = (IL - JBOT + rmax - 1) / rmax;
    constexpr int r_split = WB ? (IL - WB + rmax - 1) / rmax + (WB - JBOT + rmax - 1) / rmax : 0;
    constexpr bool split = WB != 0 && FLTEE_WAVE_SPLIT != 0 && IL > WB && JBOT < WB &&
                           (FLTEE_WAVE_SPLIT == 1 || r_split <= r_all);
    if constexpr (split) {
        lds_steps_ct<MODE, E, NT, IL - 1, WB>(sm, base, (uint32_t)IL, seed);
        lds_steps_ct<MODE, E, NT, WB - 1, JBOT, 0, WB>(sm, base, (uint32_t)IL, seed);
        __syncthreads();
    } else {
        lds_steps_ct<MODE, E, NT, IL - 1, JBOT>(sm, base, (uint32_t)IL, seed);
    }
}

template <int MODE, int E, int NT, int IL, int TL, int RL>
__device__ __forceinline__ void sort_stages_ct(uint64_t *sm, uint32_t base, uint32_t seed) {
    constexpr int WB = FLTEE_WAVE_LOCAL ? kWaveLog<E> : 0;
    if constexpr (IL < TL) {
        if constexpr (WB && IL <= WB) {
            lds_steps_ct<MODE, E, NT, IL - 1, 0, 0, WB>(sm, base, (uint32_t)IL, seed);
            if constexpr (IL == WB) __syncthreads();  // the next stage crosses waves
        } else {
            stage_steps_ct<MODE, E, NT, IL, 0>(sm, base, seed);
        }
        sort_stages_ct<MODE, E, NT, IL + 1, TL, RL>(sm, base, seed);
    } else {
        // stage TL runs block-wide rounds: if the stage before it was wave-local and did
        // not end in a block barrier (TL <= WB), order the waves here
        if constexpr (WB && TL <= WB) __syncthreads();
        stage_steps_ct<MODE, E, NT, TL, RL>(sm, base, seed);
    }
}

// Persistent tile kernels: a block walks tiles blockIdx.x, +gridDim.x, ...; the
// next tile's records are prefetched into registers (E per lane) while the current
// tile runs its LDS rounds, so HBM and LDS work overlap (T14-style issue-early /
// write-late staging).
//   SORT  : all stages 2..T of each contiguous tile (first launch of a sort)
//   !SORT : contiguous (wlog == tlog): the steps j < T of stage ilog (merge);
//           strided: the global steps dtile + tlog-wlog-1 .. dtile of stage ilog.
// E (records per lane) and NT (lanes) are template parameters: a runtime guard
// around each prefetch load makes hipcc branch and wait vmcnt(0) per load
// (cdna_hip_programming.md §5 trap 4c), and a blockDim read inside the rounds is a
// vector load + vmcnt(0) that drains the prefetch.
template <int MODE, bool SORT, int E, int NT, int TL = 0, int WL = 0, bool LPF = true, bool SW = false,
          bool PR = false, bool UNSW = false>
__global__ __launch_bounds__(NT) void bitonic_tiles(uint64_t *__restrict__ data, uint32_t tlog,
                                                    uint32_t ilog, uint32_t wlog, uint32_t dtile,
                                                    uint32_t seed, uint32_t ntiles, uint32_t pbase,
                                                    uint32_t seg0, uint32_t hole_at, uint32_t hole_len) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    // ntiles live tiles; the hole_len tiles from hole_at on hold pads alone (pad_map)
    // record r of this lane is tile element threadIdx.x + r*NT at position
    // base + p_off + r*rstride (W <= NT for strided tiles, W = T for contiguous ones)
    // SW (static_assert: middle passes only, read and written in the swizzled layout):
    // the lane part swizzled once, each record's uniform part (tile base + row) per access
    static_assert(!SW || !SORT, "the first pass is bitonic_sort_direct");
    // P2: lane t holds the slot pairs 2t, 2t + 1 (+ 2 NT r) — adjacent positions (the
    // compile-time shapes have W >= 2; SW keeps bits 0..3), one 16-B load and store each
    // (PR: a run-time shape whose launcher checked wlog >= 1)
    constexpr bool P2 = FLTEE_TILE_PAIRS && !SORT && (TL != 0 || PR);
    constexpr uint32_t LS = P2 ? 2u : 1u;  // records per load
    auto elem = [](int r) -> uint32_t {     // the tile element held in pf[r]
        return P2 ? 2u * threadIdx.x + (uint32_t)(r & 1) + (uint32_t)(r >> 1) * (2u * NT)
                  : threadIdx.x + (uint32_t)r * NT;
    };
    const uint32_t lpos = tile_pos(0u, LS * threadIdx.x, wlog, dtile);
    const uint32_t voff = (SW ? phys(lpos) : lpos) * 8u;          // per-lane bytes
    // UNSW (a contiguous sort's last merge): read the swizzled layout, write positions in
    // order — a contiguous 2^14 tile keeps its own block in both layouts, so in place
    static_assert(!UNSW || (SW && TL != 0 && WL == 0), "UNSW: contiguous swizzled tiles");
    constexpr bool SWO_ = SW && !UNSW;
    const uint32_t voffo = (SWO_ ? phys(lpos) : lpos) * 8u;
    const uint32_t rrow = (LS * (uint32_t)NT) << (dtile - wlog);  // records per load row, uniform
    const __amdgpu_buffer_rsrc_t rs = bt_rsrc(data);
    uint64_t pf[E];
    auto load_tile = [&](uint32_t sb) {
        if constexpr (P2) {
#pragma unroll
            for (int r = 0; r < E; r += 2) tl_load2<SW>(rs, voff, sb + (uint32_t)(r >> 1) * rrow, pf[r], pf[r + 1]);
        } else {
#pragma unroll
            for (int r = 0; r < E; ++r) pf[r] = tl_load<SW>(rs, voff, sb + (uint32_t)r * rrow);
        }
    };
    load_tile(tile_base(past_hole(tile, hole_at, hole_len), tlog, wlog, dtile));
    constexpr int R1 = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    // a strided tile with no fused tail (seg0 == 0) starts with the stage's top row steps:
    // the records of lane t (one parity class with P2) differ in the top log2(E) (P2:
    // log2(E) - 1) row bits only, so that first round runs on the prefetch registers
    // before they go to LDS (one LDS write + read of the tile less, as in
    // bitonic_merge_direct)
    constexpr int RH = P2 ? R1 - 1 : R1;  // the head round's steps
    constexpr bool kHeadReg = FLTEE_TILE_HEADREG && TL != 0 && WL != 0 && !SORT && RH >= 1 && (TL - RH) >= WL;
    for (;;) {
        const uint32_t base = tile_base(past_hole(tile, hole_at, hole_len), tlog, wlog, dtile);
        const bool head_reg = kHeadReg && seg0 == 0;
        if constexpr (kHeadReg) {
            if (head_reg) {
                if constexpr (P2) {
                    uint64_t g0[E / 2], g1[E / 2];
#pragma unroll
                    for (int k = 0; k < E / 2; ++k) g0[k] = pf[2 * k], g1[k] = pf[2 * k + 1];
                    const uint32_t p0 = tile_pos(base, 2u * threadIdx.x, (uint32_t)WL, dtile) + pbase;
                    group_steps<MODE, RH>(g0, p0, (uint32_t)(TL - RH - WL) + dtile, ilog, seed);
                    group_steps<MODE, RH>(g1, p0 + 1u, (uint32_t)(TL - RH - WL) + dtile, ilog, seed);
#pragma unroll
                    for (int k = 0; k < E / 2; ++k) pf[2 * k] = g0[k], pf[2 * k + 1] = g1[k];
                } else {
                    group_steps<MODE, R1>(pf, tile_pos(base, threadIdx.x, (uint32_t)WL, dtile) + pbase,
                                          (uint32_t)(TL - R1 - WL) + dtile, ilog, seed);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r) sm[lpad(elem(r))] = pf[r];
        __syncthreads();
        const uint32_t next = tile + gridDim.x;
        // always prefetch (the last round re-reads its own tile) so no branch wraps the loads
        // FLTEE_TILE_SKIP_SELF: a block on its last tile prefetches nothing (one uniform
        // branch around the whole prefetch; else it re-reads its own tile)
        auto prefetch = [&]() {
            if (!FLTEE_TILE_SKIP_SELF || next < ntiles)
                load_tile(tile_base(past_hole(next < ntiles ? next : tile, hole_at, hole_len), tlog, wlog, dtile));
        };
        // compile-time strided tiles: the prefetch after the fused tail's rounds (its
        // registers are then not live through the tail)
        constexpr bool kLate = LPF && TL != 0 && WL != 0 && !SORT;
        if (!kLate) prefetch();
        if (SORT) {
            for (uint32_t il = 1; il <= tlog; ++il)
                lds_steps<MODE, E, NT>(sm, base + pbase, wlog, dtile, il, (int)il - 1, 0, seed);
        } else {
            // seg0 = (stage << 8) | top: first the last steps top..0 of an earlier stage on
            // the tile's low (consecutive) bits — a stage's tail fused with the next
            // stage's head (the planned schedule, plan_network)
            if (seg0) {
                // the tail on every consecutive bit (top = WL - 1, what plan_network emits):
                // compile-time rounds like the rows below; any other top: runtime rounds
                const uint32_t st = (seg0 >> 8) & 0xFFFFu;
                bool done = false;
                // (2^12 tiles of 512 lanes; the 1024-lane 2^14 tiles are held to 128 VGPRs
                // and spill with the tail unrolled: C5 14.82 -> 15.44 ms, so they keep
                // runtime tail rounds, `profiles/r02/ab/tail_ct.jsonl`)
                if constexpr (TL != 0 && WL != 0 && (MODE != 2 || FLTEE_TAIL_CT_KEYED) &&
                              (NT <= 512 || FLTEE_TAIL_CT_1024)) {
                    if ((seg0 & 0xFFu) == (uint32_t)WL - 1u) {
                        lds_steps_ct<MODE, E, NT, WL - 1, 0, WL>(sm, base + pbase, st, seed, dtile);
                        done = true;
                    }
                }
                if (!done)
                    lds_steps<MODE, E, NT>(sm, base + pbase, wlog, dtile, st, (int)(seg0 & 0xFFu), 0, seed);
            }
            if (kLate) prefetch();
            if constexpr (TL != 0 && WL == 0) {  // contiguous merge, tlog == TL (launcher)
                lds_steps_ct<MODE, E, NT, TL - 1, 0>(sm, base + pbase, ilog, seed);
            } else if constexpr (TL != 0) {  // strided, tlog == TL and wlog == WL (launcher)
                if constexpr (kHeadReg) {
                    if (head_reg)
                        lds_steps_ct<MODE, E, NT, TL - RH - 1, WL, WL>(sm, base + pbase, ilog, seed, dtile);
                    else
                        lds_steps_ct<MODE, E, NT, TL - 1, WL, WL>(sm, base + pbase, ilog, seed, dtile);
                } else {
                    lds_steps_ct<MODE, E, NT, TL - 1, WL, WL>(sm, base + pbase, ilog, seed, dtile);
                }
            } else if (ilog) {  // ilog = 0: no steps on the row bits
                lds_steps<MODE, E, NT>(sm, base + pbase, wlog, dtile, ilog, (int)tlog - 1,
                                       wlog < tlog ? (int)wlog : 0, seed);
            }
        }
        if constexpr (P2) {
#pragma unroll
            for (int r = 0; r < E; r += 2)
                tl_store2<SWO_>(rs, voffo, base + (uint32_t)(r >> 1) * rrow, lds_ld(&sm[lpad(elem(r))]),
                              lds_ld(&sm[lpad(elem(r + 1))]));
        } else {
#pragma unroll
            for (int r = 0; r < E; ++r)
                tl_store<SWO_>(rs, voffo, base + (uint32_t)r * rrow, lds_ld(&sm[lpad(threadIdx.x + r * NT)]));
        }
        if (next >= ntiles) break;
        __syncthreads();  // this tile's LDS reads retire before the next tile lands
        tile = next;
    }
}

// Contiguous merge (the steps j < T of stage ilog) with its first and last LDS round
// in registers.  Lane t prefetches records t + r*NT (r < E = 2^R1): exactly the group
// the first round needs (steps T/2 .. NT, distance log2 NT = tlog - R1), so that round
// runs on the prefetch registers before they are written to LDS.  The last round
// (steps 2^(RL-1) .. 1, groups of 2^RL consecutive records) stores its groups straight
// to HBM instead of writing LDS back for a separate store loop.  Saves
// one LDS write + read of the tile and two barriers per tile; same network.
//
// SEL (the LAST pass of nips19's shuffle only): instead of storing the tile, keep the
// entries with idx < sel_d — the ones safe_aggregate adds (common.rs:25-35) — and write
// them compacted, in position order, to the front of the tile's own slot of `data`
// (data[tile * T, + count)), and their count to sel_cnt[tile].  The last round then
// gives lane t the E consecutive records t*E .. t*E+E-1 (groups t*G .. t*G+G-1), so
// one block-wide exclusive scan of the lanes' counts orders the tile's entries.  The
// tile was read into LDS before, so the in-place writes are safe.
// SWI / SWO: the tile is read / written in the block-swizzled layout (kSwzMask; the
// contiguous merges only: a middle merge both, the last merge of a sort SWI alone).
template <int MODE, int E, int NT, int RL, bool STRIDED, bool SEL = false, int TL = 0,
          bool SWI = false, bool SWO = false>
__global__ __launch_bounds__(NT) void bitonic_merge_direct(uint64_t *__restrict__ data,
                                                           uint32_t tlog, uint32_t ilog,
                                                           uint32_t wlog, uint32_t dtile,
                                                           uint32_t seed, uint32_t ntiles,
                                                           uint32_t pbase, uint32_t sel_d,
                                                           uint32_t *__restrict__ sel_cnt,
                                                           uint32_t hole_at, uint32_t hole_len) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    __shared__ uint32_t wtot[SEL ? NT / 64 : 1];
    constexpr int R1 = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    static_assert((1 << R1) == E, "E must be a power of two <= 32");
    static_assert(RL >= 1 && RL <= R1, "last round");
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    const uint32_t t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = bt_rsrc(data);
    // contiguous: wlog = dtile = tlog.  strided: W = 2^wlog consecutive positions x T/W
    // rows at stride 2^dtile (W <= NT), as in bitonic_tiles
    static_assert(!(STRIDED && (SWI || SWO)), "swizzled layout: contiguous merges only");
    static_assert(!(SEL && SWO), "the selection is written in position order");
    // P2 (contiguous, compile-time shape): lane t loads the slot pairs 2t, 2t + 1 (+ 2 NT r),
    // 16 B each; the head round in registers then covers the top R1 - 1 steps per parity
    // class and the last round takes one step more (RL + 1): the same LDS rounds
    constexpr bool P2 = (FLTEE_MERGE_PAIRS == 1 || (FLTEE_MERGE_PAIRS == 2 && SEL)) && TL != 0 && !STRIDED && RL < R1;
    constexpr int RH = P2 ? R1 - 1 : R1;  // head round (registers)
    constexpr int RT = P2 ? RL + 1 : RL;  // last round (registers)
    auto elem = [&](int r) -> uint32_t {  // the tile element held in pf[r]
        return P2 ? 2u * t + (uint32_t)(r & 1) + (uint32_t)(r >> 1) * (2u * NT) : t + (uint32_t)r * NT;
    };
    const uint32_t lpos = tile_pos(0u, (P2 ? 2u : 1u) * t, wlog, dtile);
    const uint32_t voff = (SWI ? phys(lpos) : lpos) * 8u;
    const uint32_t rrow = ((P2 ? 2u : 1u) * (uint32_t)NT) << (dtile - wlog);  // records per load row
    const uint32_t dlog1 = tlog - (uint32_t)R1;  // == log2 NT: the first round's tile-local distance
    const uint32_t dlog1_g = STRIDED ? dlog1 - wlog + dtile : dlog1;
    const uint32_t jbot = STRIDED ? wlog : 0u;  // the tile's lowest step
    uint64_t pf[E];
    auto load_tile = [&](uint32_t sb) {
        if constexpr (P2) {
#pragma unroll
            for (int r = 0; r < E; r += 2) tl_load2<SWI>(rs, voff, sb + (uint32_t)(r >> 1) * rrow, pf[r], pf[r + 1]);
        } else {
#pragma unroll
            for (int r = 0; r < E; ++r) pf[r] = tl_load<SWI>(rs, voff, sb + (uint32_t)r * rrow);
        }
    };
    load_tile(tile_base(past_hole(tile, hole_at, hole_len), tlog, wlog, dtile));
    for (;;) {
        const uint32_t ptile = past_hole(tile, hole_at, hole_len);
        const uint32_t base = tile_base(ptile, tlog, wlog, dtile);
        if constexpr (P2) {
            uint64_t g0[E / 2], g1[E / 2];
#pragma unroll
            for (int k = 0; k < E / 2; ++k) g0[k] = pf[2 * k], g1[k] = pf[2 * k + 1];
            group_steps<MODE, RH>(g0, base + 2u * t + pbase, dlog1_g + 1u, ilog, seed);
            group_steps<MODE, RH>(g1, base + 2u * t + 1u + pbase, dlog1_g + 1u, ilog, seed);
#pragma unroll
            for (int k = 0; k < E / 2; ++k) pf[2 * k] = g0[k], pf[2 * k + 1] = g1[k];
        } else {
            group_steps<MODE, R1>(pf, tile_pos(base, t, wlog, dtile) + pbase, dlog1_g, ilog, seed);
        }
#pragma unroll
        for (int r = 0; r < E; ++r) sm[lpad(elem(r))] = pf[r];
        __syncthreads();
        const uint32_t next = tile + gridDim.x;
        load_tile(tile_base(past_hole(next < ntiles ? next : tile, hole_at, hole_len), tlog, wlog, dtile));
        if constexpr (TL != 0 && !STRIDED)  // tlog == TL (checked by the launcher)
            lds_steps_ct<MODE, E, NT, TL - 1 - RH, RT>(sm, base + pbase, ilog, seed);
        else
            lds_steps<MODE, E, NT>(sm, base + pbase, wlog, dtile, ilog, (int)dlog1 - 1,
                                   (int)(jbot + RL), seed);
        constexpr int G = E >> RT;
        if constexpr (SEL && !STRIDED) {
            uint64_t v[E];
            const uint64_t *own = sm + lpad(t * (uint32_t)E);  // E >= 16: lpad splits
#pragma unroll
            for (int q = 0; q < E; ++q) v[q] = lds_ld(&own[q + (q >> 4)]);
            uint32_t c = 0;
#pragma unroll
            for (int h = 0; h < G; ++h) {
                uint64_t (&g)[1 << RT] = *reinterpret_cast<uint64_t (*)[1 << RT]>(&v[h << RT]);
                group_steps<MODE, RT>(g, base + pbase + t * (uint32_t)E + ((uint32_t)h << RT), 0u,
                                      ilog, seed);
            }
#pragma unroll
            for (int q = 0; q < E; ++q) c += (uint32_t)v[q] < sel_d;
            // block-wide exclusive scan of c in lane order
            const uint32_t lane = t & 63, wv = t / 64;
            uint32_t inc = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o);
                if (lane >= (uint32_t)o) inc += y;
            }
            if (lane == 63) wtot[wv] = inc;
            __syncthreads();
            uint32_t pre = 0, tot = 0;
#pragma unroll
            for (uint32_t w = 0; w < NT / 64; ++w) {
                const uint32_t x = wtot[w];
                pre += w < wv ? x : 0u;
                tot += x;
            }
#if FLTEE_SEL_STORE_OOB
            // branch-free: every record is stored, the unselected ones at the first byte
            // past the tile's own slot of a tile-sized buffer resource, where the store is
            // dropped (no data-dependent branch, no per-record exec mask kept live)
            const uint32_t tbytes = (1u << tlog) * 8u;
            const __amdgpu_buffer_rsrc_t ts =
                __builtin_amdgcn_make_buffer_rsrc((void *)(data + base), (short)0, (int)tbytes, 0x00020000);
            uint32_t o = pre + inc - c;  // tile-relative
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const bool sq = (uint32_t)v[q] < sel_d;
                bt_store<kTileCP>(ts, sq ? o * 8u : tbytes, 0u, v[q]);
                o += sq ? 1u : 0u;
            }
#else
            uint32_t o = base + pre + inc - c;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                if ((uint32_t)v[q] < sel_d) {
                    bt_store<kTileCP>(rs, o * 8u, 0u, v[q]);  // per-lane offset: voffset
                    ++o;
                }
            }
#endif
            if (t == NT - 1) sel_cnt[ptile] = tot;
            if (next >= ntiles) break;
            __syncthreads();  // wtot and the last round's LDS reads retire
            tile = next;
            continue;
        }
        // every group read from LDS first (the fenced stores below would otherwise keep the
        // next group's reads behind them), then computed, then stored
        constexpr int BW = kLdsBatch<G>;
        // SWO: a contiguous tile stays in its own 2^14 block, so its records' physical
        // offsets inside the block are (tile offset ^ swz_x(base)): one uniform XOR
        const uint32_t sxb = SWO ? swz_x(base) : 0u;
#pragma unroll
        for (int h0 = 0; h0 < G; h0 += BW) {
        uint64_t vv[BW][1 << RT];
        uint32_t bb[BW];
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            const uint32_t b = bb[h] = spread(lane_tid<NT>() + (uint32_t)(h0 + h) * NT, jbot, RT);
            if (!STRIDED) {  // b = g << RT: lpad(b + q) = lpad(b) + q + (q >> 4)
                const uint64_t *row = sm + lpad(b);
#pragma unroll
                for (int q = 0; q < (1 << RT); ++q) vv[h][q] = lds_ld(&row[q + (q >> 4)]);
            } else {
#pragma unroll
                for (int q = 0; q < (1 << RT); ++q) vv[h][q] = lds_ld(&sm[lpad(b + ((uint32_t)q << jbot))]);
            }
        }
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            const uint32_t pb = tile_pos(0u, bb[h], wlog, dtile);  // tile-relative position of v[0]
            group_steps<MODE, RT>(vv[h], base + pbase + pb, STRIDED ? dtile : 0u, ilog, seed);
        }
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            uint64_t (&v)[1 << RT] = vv[h];
            const uint32_t pb = tile_pos(0u, bb[h], wlog, dtile);
            if (STRIDED) {  // v[q] sits 2^dtile positions after v[q-1]: 8-B stores
#pragma unroll
                for (int q = 0; q < (1 << RT); ++q)
                    bt_store<kTileCP>(rs, (pb + ((uint32_t)q << dtile)) * 8u, base * 8u, v[q]);
            } else {
                // 16-B stores.  hipcc (ROCm 7.2) may let the next group's VALU overwrite a
                // dwordx4 store's data registers one instruction after the store, before the
                // store has read them (measured: nondeterministic output); the explicit
                // "s_nop 1" fenced by sched_barriers gives the two wait states the hazard needs
                // (cdna_hip_programming.md §5.7: dwordx3/x4 stores end with s_nop 1).
                // (pb is a multiple of 2^RT and sxb of 16: (pb ^ sxb) + q is the physical
                // offset of record pb + q)
                const uint32_t pbs = SWO ? (pb ^ sxb) : pb;
#pragma unroll
                for (int q = 0; q < (1 << RT); q += 2) {
                    const bt_u32x4 x = {(uint32_t)v[q], (uint32_t)(v[q] >> 32), (uint32_t)v[q + 1],
                                        (uint32_t)(v[q + 1] >> 32)};
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)((pbs + (uint32_t)q) * 8u),
                                                           (int)(base * 8u), kTileCP);
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        }
        if (next >= ntiles) break;
        __syncthreads();  // the last round's LDS reads retire before the next tile lands
        tile = next;
    }
}

// Stage IL (< log2 E) on a lane's E consecutive records at positions p0..p0+E-1: the
// records form E / 2^IL whole stage blocks, each with its own direction.
template <int MODE, int IL, int E>
__device__ __forceinline__ void lane_stage(uint64_t (&v)[E], uint32_t p0, uint32_t seed) {
    constexpr int B = 1 << IL;
    if constexpr (MODE == 2 && FLTEE_KEY_AFTER_DATA) seed = after_data(seed, (uint32_t)v[0]);
#pragma unroll
    for (int lv = IL - 1; lv >= 0; --lv) {
        const uint32_t key = MODE == 2 ? shuffle_step_key(seed, IL, (uint32_t)lv) : 0u;
        // p0 is a multiple of E: l = p0 + q = p0 ^ q (keyed_c)
        const uint32_t X = (MODE == 2 && FLTEE_KEYED_SPLIT) ? (p0 ^ key) * 0x9E3779B1u : 0u;
        bool sw[E / 2];
#pragma unroll
        for (int q = 0, k = 0; q < E; ++q) {
            if (q & (1 << lv)) continue;
            const int qm = q | (1 << lv);
            const bool asc = ((p0 + (uint32_t)(q & ~(B - 1))) & (1u << IL)) == 0;
            if constexpr (MODE == 2 && FLTEE_KEYED_SPLIT)
                sw[k++] = asc ^ ((int32_t)(X + keyed_c(key, (uint32_t)q)) < 0);
            else if constexpr (MODE == 2 && FLTEE_KEYED_DIRFOLD)
                sw[k++] = keyed_swap(p0 ^ key ^ keyed_dir(asc), (uint32_t)q);
            else
                sw[k++] = asc ^ cond2<MODE>(v[q], v[qm], p0 + (uint32_t)q, key);
        }
#pragma unroll
        for (int q = 0, k = 0; q < E; ++q) {
            if (q & (1 << lv)) continue;
            const int qm = q | (1 << lv);
            const uint64_t a = v[q], c = v[qm];
            const bool s = sw[k++];
            v[q] = s ? c : a;
            v[qm] = s ? a : c;
        }
    }
}

// Producers fused into a sort's first pass (GEN != 0): the tile loads read the client
// records from `rec` and synthesize the padded entries in registers, so the padded
// array is never written by a separate init kernel and read back (one HBM pass less).
//   GEN 1: advanced_init (advanced.rs:116-142): records ++ (i, +0.0) for i < d ++
//          (u32::MAX, +0.0) pads
//   GEN 2: nips19_build (nips19.rs:18-63, common.rs:189-197): records ++ entry e =
//          i*tf + j of the d*tf dummies ((r_i < j) ? i : u32::MAX, +0.0) ++ pads
// Same entries as advanced_init_kernel / nips19_build_kernel, position for position.
struct SortGen {
    const uint64_t *rec;  // the record at global position p is rec[p - pbase] (p < nrec)
    const uint32_t *r;    // GEN 2: Laplace counts r_i
    uint32_t nrec, d, tf;
    // pad_n > 0: blocks >= grid_live store (u32::MAX, +0.0) to positions pad_begin ..
    // pad_begin + pad_n - 1 (the tiles of pads alone, which no sort step reads before
    // a later stage's live region reaches them) instead of sorting
    uint32_t grid_live = 0, pad_begin = 0, pad_n = 0;
};
template <int GEN>
__device__ __forceinline__ uint64_t gen_entry(const SortGen &g, uint32_t p, uint64_t v) {
    if (p < g.nrec) return v;
    const uint32_t e = p - g.nrec;
    if (GEN == 1) return e < g.d ? (uint64_t)e : 0xFFFFFFFFull;
    if (g.tf == 0) return 0xFFFFFFFFull;
    const uint32_t i = e / g.tf, j = e - i * g.tf;
    if (i >= g.d) return 0xFFFFFFFFull;
    return g.r[i] < j ? (uint64_t)i : 0xFFFFFFFFull;  // o_setb / o_mov, as in the build kernel
}

// The first pass of a sort (stages 1..T of every contiguous tile) with its first and
// last work in registers: lane t loads records tE .. tE+E-1 (16-B loads), runs stages
// 1..log2 E on them without LDS, and writes them to LDS; the LDS rounds run stages
// log2 E + 1 .. tlog; the last round of stage tlog (groups of 2^RL consecutive records)
// stores straight to HBM (16-B stores fenced with s_nop 1, see bitonic_merge_direct).
// SWO: the sorted tiles are written in the block-swizzled layout (kSwzMask; the loads
// are logical), for a sort whose later passes run swizzled.
template <int MODE, int E, int NT, int RL, int GEN = 0, int TL = 0, int LPF = 1, bool SWO = false>
__global__ __launch_bounds__(NT) void bitonic_sort_direct(uint64_t *__restrict__ data,
                                                          uint32_t tlog, uint32_t seed,
                                                          uint32_t ntiles, uint32_t pbase,
                                                          SortGen g) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
    constexpr int R1 = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    static_assert((1 << R1) == E && RL >= 1 && RL <= R1, "tile shape");
    const uint32_t t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = bt_rsrc(data);
    if (g.pad_n && blockIdx.x >= g.grid_live) {  // store-only blocks (replace a fill launch)
        const uint32_t nb = gridDim.x - g.grid_live;
        const bt_u32x4 pad = {0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0u};
        for (uint32_t i = (blockIdx.x - g.grid_live) * (uint32_t)NT + t; i < g.pad_n / 2u;
             i += nb * (uint32_t)NT) {
            __builtin_amdgcn_raw_buffer_store_b128(pad, rs, (int)(i * 16u), (int)(g.pad_begin * 8u),
                                                   kTileCP);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 1" ::: "memory");  // dwordx4 store data hazard (see above)
            __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
    const uint32_t stride = g.pad_n ? g.grid_live : gridDim.x;  // the sorting blocks
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    // GEN: loads come from rec, range-checked to its nloc records from pbase (beyond:
    // zeros, replaced by gen_entry)
    uint32_t nloc = 0;
    if (GEN) {
        nloc = g.nrec > pbase ? g.nrec - pbase : 0u;
        const uint32_t m = ntiles << tlog;
        if (nloc > m) nloc = m;
    }
    const uint64_t lbytes = (uint64_t)nloc * 8u;
    const __amdgpu_buffer_rsrc_t ls =
        GEN ? __builtin_amdgcn_make_buffer_rsrc((void *)g.rec, (short)0,
                                                (int)(lbytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)lbytes),
                                                0x00020000)
            : rs;
    const uint32_t voff = t * (uint32_t)E * 8u;
    // GEN: a 16-B load that straddles the end of rec (nloc odd) returns zeros whole: its
    // first record, the last client record, is read once up front and put back in
    // finish() (a select, no branch)
    uint64_t last_rec = 0;
    if (GEN && (nloc & 1u)) last_rec = g.rec[nloc - 1u];
    // GEN 2: the Laplace counts the lane's dummies read, r[gi] and r[gi + 1] (the E
    // entries of a lane span at most two counts when tf >= E), as range-checked buffer
    // loads (index >= d: 0, an entry that is a pad anyway)
    const __amdgpu_buffer_rsrc_t lr =
        GEN == 2 ? __builtin_amdgcn_make_buffer_rsrc((void *)g.r, (short)0, (int)(g.d * 4u), 0x00020000) : rs;
    uint64_t pf[E];
    uint32_t lap[2] = {0u, 0u};
    // issue(): the next tile's loads only — nothing here waits for them (a use of the
    // loaded values would make the compiler wait right after the loads and the prefetch
    // would no longer overlap the LDS rounds); finish(): the producer, on arrival
    auto first_entry = [&](uint32_t tl, uint32_t &gi, uint32_t &gj) {
        const uint32_t p0 = pbase + (tl << tlog) + t * (uint32_t)E;
        const uint32_t e0 = p0 > g.nrec ? p0 - g.nrec : 0u;
        gi = g.tf ? e0 / g.tf : 0u;
        gj = e0 - gi * g.tf;
    };
    auto issue = [&](uint32_t tl) {
        const uint32_t sb = (tl << tlog) * 8u;
#pragma unroll
        for (int r = 0; r < E; r += 2) {
            const bt_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(ls, (int)(voff + (uint32_t)r * 8u),
                                                                      (int)sb, kTileCP);
            pf[r] = ((uint64_t)x.y << 32) | x.x;
            pf[r + 1] = ((uint64_t)x.w << 32) | x.z;
        }
        if constexpr (GEN == 2) {
            uint32_t gi, gj;
            first_entry(tl, gi, gj);
            lap[0] = __builtin_amdgcn_raw_buffer_load_b32(lr, (int)(gi * 4u), 0, 0);
            lap[1] = __builtin_amdgcn_raw_buffer_load_b32(lr, (int)(gi * 4u + 4u), 0, 0);
        }
    };
    auto finish = [&](uint32_t tl) {
        if constexpr (GEN != 0) {
            const uint32_t x0 = (tl << tlog) + t * (uint32_t)E;  // local index of pf[0]
#pragma unroll
            for (int r = 0; r < E; r += 2)
                pf[r] = (x0 + (uint32_t)r + 1u == nloc) ? last_rec : pf[r];
            if constexpr (GEN == 1) {
#pragma unroll
                for (int q = 0; q < E; ++q) pf[q] = gen_entry<GEN>(g, pbase + x0 + (uint32_t)q, pf[q]);
            } else {
                uint32_t gi, gj;
                first_entry(tl, gi, gj);
                const uint32_t gi0 = gi;
                const bool two = g.tf >= (uint32_t)E;  // uniform: the prefetched counts cover the lane
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    if (pbase + x0 + (uint32_t)q >= g.nrec) {  // entry (i, j): (r_i < j) ? i : MAX
                        const uint32_t ri = two ? (gi == gi0 ? lap[0] : lap[1]) : (gi < g.d ? g.r[gi] : 0u);
                        pf[q] = (g.tf == 0 || gi >= g.d || ri >= gj) ? 0xFFFFFFFFull : (uint64_t)gi;
                        if (++gj == g.tf) { gj = 0; ++gi; }
                    }
                }
            }
        }
    };
    issue(tile);
    for (;;) {
        finish(tile);
        const uint32_t base = tile << tlog;
        const uint32_t p0 = base + pbase + t * (uint32_t)E;
        lane_stage<MODE, 1, E>(pf, p0, seed);
        if (R1 >= 2) lane_stage<MODE, (R1 >= 2 ? 2 : 1), E>(pf, p0, seed);
        if (R1 >= 3) lane_stage<MODE, (R1 >= 3 ? 3 : 1), E>(pf, p0, seed);
        if (R1 >= 4) lane_stage<MODE, (R1 >= 4 ? 4 : 1), E>(pf, p0, seed);
        if (R1 >= 5) lane_stage<MODE, (R1 >= 5 ? 5 : 1), E>(pf, p0, seed);
#pragma unroll
        for (int r = 0; r < E; ++r) sm[lpad(t * (uint32_t)E + (uint32_t)r)] = pf[r];
        // the lane's records are positions tE .. tE + E - 1: the wave's own 64 E records,
        // which its wave-local first rounds read back (TL != 0 with FLTEE_WAVE_LOCAL)
        if constexpr (TL != 0 && FLTEE_WAVE_LOCAL && R1 + 1 <= kWaveLog<E>) wave_lds_order();
        else __syncthreads();
        const uint32_t next = tile + stride;
        if constexpr (TL != 0) {  // tlog == TL (launcher)
            // the next tile's loads go out before the LAST stage's rounds, not before the
            // first: the prefetch registers stay free through the rounds of stages
            // log2 E + 1 .. TL - 1 (1024 lanes are held to 128 VGPRs; with the prefetch
            // live across every round the 2^14-tile kernels spilled), and stage TL's
            // rounds still cover the load latency (LPF 0: before the first round)
            // LPF 2: later still, before stage TL's last LDS round.  That round is forced to
            // a full R1-step round (steps kLast .. RL, kLast = RL + R1 - 1) and the steps
            // above it are regrouped greedily; this is not always lds_steps_ct's own greedy
            // split (whenever (TL - RL) % R1 != 0), but the steps still run one after the
            // other in the same order, so the network and its output are unchanged.
            constexpr int kLast = RL + R1 - 1;
            if constexpr (LPF == 2 && kLast < TL - 1) {
                sort_stages_ct<MODE, E, NT, R1 + 1, TL - 1, 0>(sm, base + pbase, seed);
                lds_steps_ct<MODE, E, NT, TL - 1, kLast + 1>(sm, base + pbase, (uint32_t)TL, seed);
                issue(next < ntiles ? next : tile);
                lds_steps_ct<MODE, E, NT, kLast, RL>(sm, base + pbase, (uint32_t)TL, seed);
            } else if constexpr (LPF != 0) {
                sort_stages_ct<MODE, E, NT, R1 + 1, TL - 1, 0>(sm, base + pbase, seed);
                issue(next < ntiles ? next : tile);
                lds_steps_ct<MODE, E, NT, TL - 1, RL>(sm, base + pbase, (uint32_t)TL, seed);
            } else {
                issue(next < ntiles ? next : tile);
                sort_stages_ct<MODE, E, NT, R1 + 1, TL, RL>(sm, base + pbase, seed);
            }
        } else {
            issue(next < ntiles ? next : tile);
            for (uint32_t il = (uint32_t)R1 + 1; il < tlog; ++il)
                lds_steps<MODE, E, NT>(sm, base + pbase, tlog, tlog, il, (int)il - 1, 0, seed);
            lds_steps<MODE, E, NT>(sm, base + pbase, tlog, tlog, tlog, (int)tlog - 1, RL, seed);
        }
        constexpr int G = E >> RL;
        // every group read from LDS first, then computed, then stored (the fenced stores
        // would otherwise hold the next group's reads behind them)
        constexpr int BW = kLdsBatch<G>;
        const uint32_t sxb = SWO ? swz_x(base) : 0u;  // the tile's block swizzle (merge_direct)
#pragma unroll
        for (int h0 = 0; h0 < G; h0 += BW) {
        uint64_t vv[BW][1 << RL];
        const uint32_t tf = lane_tid<NT>();
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            const uint32_t b = (tf + (uint32_t)(h0 + h) * NT) << RL;
#pragma unroll
            for (int q = 0; q < (1 << RL); ++q) vv[h][q] = lds_ld(&sm[lpad(b + (uint32_t)q)]);
        }
#pragma unroll
        for (int h = 0; h < BW; ++h)
            group_steps<MODE, RL>(vv[h], base + pbase + ((tf + (uint32_t)(h0 + h) * NT) << RL), 0u, tlog, seed);
#pragma unroll
        for (int h = 0; h < BW; ++h) {
            const uint32_t b = ((tf + (uint32_t)(h0 + h) * NT) << RL) ^ sxb;  // physical offset
            uint64_t (&v)[1 << RL] = vv[h];
#pragma unroll
            for (int q = 0; q < (1 << RL); q += 2) {
                const bt_u32x4 x = {(uint32_t)v[q], (uint32_t)(v[q] >> 32), (uint32_t)v[q + 1],
                                    (uint32_t)(v[q + 1] >> 32)};
                // the fence in front too: no VALU of this group sinks below the store
                // into the window the s_nop covers (seen with the compile-time rounds)
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)((b + (uint32_t)q) * 8u),
                                                       (int)(base * 8u), kTileCP);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 1" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        }
        if (next >= ntiles) break;
        __syncthreads();  // the last round's LDS reads retire before the next tile lands
        tile = next;
    }
}

// --------------------------------------------------------- global pass -----
// Steps jtop..jtop-R+1 of stage ilog straight from HBM: lane t owns group t.
// Record q of a group sits at byte (q << dlog) * 8 + b * 8: a wave-uniform part and
// a per-lane part, issued as raw buffer loads/stores with the first in soffset (an
// SGPR) and the second in voffset (one VGPR).  With plain pointers hipcc folds the
// uniform part into 64 per-record 64-bit addresses that stay live across the
// compare-exchanges (R = 6: ~290 VGPRs, one wave per SIMD).  Byte offsets are 32-bit:
// M <= 2^29 (checked by the callers).

// SW: the array is in the block-swizzled layout (a middle pass of a swizzled sort): the
// group's first record swizzled per lane, record q's uniform part per access (one XOR).
template <int MODE, int R, bool SW = false>
__global__ __launch_bounds__(256) void bitonic_global(uint64_t *__restrict__ data, uint32_t ilog,
                                                      uint32_t jtop, uint32_t seed,
                                                      uint32_t ngroups, uint32_t pbase,
                                                      uint32_t hole_at, uint32_t hole_len) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= ngroups) return;
    const uint32_t dlog = jtop - R + 1;
    const uint32_t b = spread(past_hole(t, hole_at, hole_len), dlog, R);
    const uint32_t voff = (SW ? phys(b) : b) * 8u;
    const __amdgpu_buffer_rsrc_t rs = bt_rsrc(data);
    uint64_t v[1 << R];
#pragma unroll
    for (int q = 0; q < (1 << R); ++q) {
        if constexpr (SW) v[q] = bt_load(rs, voff ^ (phys((uint32_t)q << dlog) * 8u), 0u);
        else v[q] = bt_load(rs, voff, (uint32_t)q << (dlog + 3));
    }
    group_steps<MODE, R>(v, b + pbase, dlog, ilog, seed);
    // the store addresses recomputed (one XOR each) rather than 2^R of them kept live
    uint32_t vst = voff;
    if constexpr (SW) asm volatile("; global swz" : "+v"(vst));
#pragma unroll
    for (int q = 0; q < (1 << R); ++q) {
        if constexpr (SW) bt_store(rs, vst ^ (phys((uint32_t)q << dlog) * 8u), 0u, v[q]);
        else bt_store(rs, voff, (uint32_t)q << (dlog + 3), v[q]);
    }
}

// live_groups (0 = all): only the first live_groups groups run — the rest lie in stage
// blocks made of pad records alone, which the step leaves as they are (see stage_steps)
template <int MODE>
static hipError_t launch_global(uint64_t *data, uint32_t mlog, uint32_t ilog, uint32_t jtop,
                                int R, uint32_t seed, hipStream_t s, uint32_t pbase,
                                uint32_t live_groups = 0, bool sw = false, uint32_t hole_at = 0,
                                uint32_t hole_len = 0) {
    uint32_t ngroups = 1u << (mlog - R);
    if (live_groups && live_groups < ngroups) ngroups = live_groups;
    if (hole_len >= ngroups || hole_at >= ngroups) hole_at = hole_len = 0;
    ngroups -= hole_len;
    if (ngroups == 0) return hipSuccess;
    const unsigned blocks = (ngroups + 255) / 256;
    net_account((uint64_t)16 * ngroups << R, "bitonic_global", s);
#define BG_GO(R_)                                                                                  \
    do {                                                                                           \
        if (sw) FLTEE_LAUNCH((bitonic_global<MODE, R_, true>), dim3(blocks), dim3(256), 0, s, \
                                   data, ilog, jtop, seed, ngroups, pbase, hole_at, hole_len);     \
        else FLTEE_LAUNCH((bitonic_global<MODE, R_>), dim3(blocks), dim3(256), 0, s, data,    \
                                ilog, jtop, seed, ngroups, pbase, hole_at, hole_len);              \
    } while (0)
    switch (R) {
    case 1: BG_GO(1); break;
    case 2: BG_GO(2); break;
    case 3: BG_GO(3); break;
    case 4: BG_GO(4); break;
    case 5: BG_GO(5); break;
    default: BG_GO(6); break;
    }
#undef BG_GO
    return hipGetLastError();
}

constexpr uint32_t kMaxTileLog = 14;  // 16384 records = 128 KB (+1/16 padding) of LDS

// Network shape constants (compile time; the variants measured against them are in
// profiles/r01/ab and profiles/r02/ab — the library has no runtime switches).
// Steps per register-blocked global pass: 6 (64 records / lane; fastest at M = 2^24, 2^27).
constexpr int kRegMaxSteps = 6;
// Smaller tiles until there are at least 2^8 of them (one per CU).
#ifndef FLTEE_MIN_TILES_LOG
#define FLTEE_MIN_TILES_LOG 8
#endif
constexpr uint32_t kMinTilesLog = FLTEE_MIN_TILES_LOG;
// ... but no tile under 2^FLTEE_TILE_FLOOR records for that: below 2^20 records fewer,
// larger tiles win on launch count (round 5, `profiles/r05/ab/ab7_tile_floor_*.jsonl`,
// floors 11 / 12 / 13: 2^16 records 0.071 / 0.062 / 0.076 ms, 2^18 0.107 / 0.087 / 0.115;
// 2^14 tiles were slower at every size)
#ifndef FLTEE_TILE_FLOOR
#define FLTEE_TILE_FLOOR 12
#endif
// Narrowest strided-tile row, log2: 16 records = 128-B row segments (W = 8: 14.09 vs
// 14.03 ms at 2^27, W = 4: 14.66, W = 2: 16.37).
constexpr int kMinWLog = 4;
// The first pass's prefetch of the next tile: 0 = before the first LDS round, 1 = before
// the last stage's rounds, 2 = before that stage's last round.  Round 2 kept it late (2
// for the sorts by key, 1 for the keyed shuffle) because the kernels spilled; without
// spills (lane_tid, the producer moved out of the prefetch) the earliest is fastest: C5
// 13.69 vs 13.77 ms (2), C4 9.34 vs 9.35 ms (1) (`profiles/r03/ab/ab4_*.jsonl`).
// Overridable at build time for A/B libraries only (scripts/ab_build.sh).
#ifndef FLTEE_SORT_LATEPF_KEY
#define FLTEE_SORT_LATEPF_KEY 0
#endif
#ifndef FLTEE_SORT_LATEPF_SHUFFLE
#define FLTEE_SORT_LATEPF_SHUFFLE 0
#endif
template <int MODE>
constexpr int kSortLatePf = MODE == 2 ? FLTEE_SORT_LATEPF_SHUFFLE : FLTEE_SORT_LATEPF_KEY;

template <int MODE, bool SORT, int E, int NT, int TL, int WL, bool LPF, bool SW, bool PR = false>
static hipError_t launch_tiles_pr(unsigned grid, size_t lds, hipStream_t s, uint64_t *data,
                                  uint32_t tlog, uint32_t ilog, uint32_t wlog, uint32_t dtile,
                                  uint32_t seed, uint32_t tiles, uint32_t pbase, uint32_t seg0,
                                  uint32_t hole_at, uint32_t hole_len) {
    static bool attr = false;  // > 64 KB of dynamic LDS needs the opt-in (160 KB on gfx950)
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)bitonic_tiles<MODE, SORT, E, NT, TL, WL, LPF, SW, PR>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    net_account((uint64_t)16 * tiles << tlog, "bitonic_tiles", s);
    FLTEE_LAUNCH((bitonic_tiles<MODE, SORT, E, NT, TL, WL, LPF, SW, PR>), dim3(grid), dim3(NT), lds, s,
                       data, tlog, ilog, wlog, dtile, seed, tiles, pbase, seg0, hole_at, hole_len);
    return hipGetLastError();
}
// the run-time-shaped 2^14 tiles take the slot pairs too when their rows have >= 2 records
#ifndef FLTEE_TILE_PAIRS_RT
#define FLTEE_TILE_PAIRS_RT 1
#endif
template <int MODE, bool SORT, int E, int NT, int TL, int WL, bool LPF, bool SW>
static hipError_t launch_tiles_sw(unsigned grid, size_t lds, hipStream_t s, uint64_t *data,
                                  uint32_t tlog, uint32_t ilog, uint32_t wlog, uint32_t dtile,
                                  uint32_t seed, uint32_t tiles, uint32_t pbase, uint32_t seg0,
                                  uint32_t hole_at, uint32_t hole_len) {
    if constexpr (FLTEE_TILE_PAIRS_RT && TL == 0 && !SORT && NT == 1024 && E == 16) {
        if (wlog >= 1)
            return launch_tiles_pr<MODE, SORT, E, NT, TL, WL, LPF, SW, true>(grid, lds, s, data, tlog, ilog, wlog,
                                                                            dtile, seed, tiles, pbase, seg0,
                                                                            hole_at, hole_len);
    }
    return launch_tiles_pr<MODE, SORT, E, NT, TL, WL, LPF, SW>(grid, lds, s, data, tlog, ilog, wlog, dtile,
                                                               seed, tiles, pbase, seg0, hole_at, hole_len);
}

// sw: the pass reads and writes the block-swizzled layout (2^14 tiles of 1024 lanes only)
template <int MODE, bool SORT, int E, int NT, int TL, int WL, bool LPF>
static hipError_t launch_tiles_lpf(unsigned grid, size_t lds, hipStream_t s, uint64_t *data,
                                   uint32_t tlog, uint32_t ilog, uint32_t wlog, uint32_t dtile,
                                   uint32_t seed, uint32_t tiles, uint32_t pbase, uint32_t seg0,
                                   bool sw, uint32_t hole_at, uint32_t hole_len) {
    if constexpr (!SORT && NT == 1024 && E == 16) {
        if (sw)
            return launch_tiles_sw<MODE, SORT, E, NT, TL, WL, LPF, true>(grid, lds, s, data, tlog, ilog,
                                                                         wlog, dtile, seed, tiles, pbase, seg0,
                                                                         hole_at, hole_len);
    } else {
        if (sw) return hipErrorInvalidValue;
    }
    return launch_tiles_sw<MODE, SORT, E, NT, TL, WL, LPF, false>(grid, lds, s, data, tlog, ilog, wlog,
                                                                  dtile, seed, tiles, pbase, seg0, hole_at,
                                                                  hole_len);
}

template <int MODE, bool SORT, int E, int NT, int TL = 0, int WL = 0>
static hipError_t launch_tiles_e(unsigned grid, size_t lds, hipStream_t s, uint64_t *data,
                                 uint32_t tlog, uint32_t ilog, uint32_t wlog, uint32_t dtile,
                                 uint32_t seed, uint32_t tiles, uint32_t pbase, uint32_t seg0 = 0,
                                 bool sw = false, uint32_t hole_at = 0, uint32_t hole_len = 0) {
    // the compile-time strided tiles' prefetch goes after their fused tail, except for the
    // tiles with a tail on rows of 2^5 (their 9 row steps cover the load less well: 514 ->
    // 553 us at C5 with it late, while every other shape gains,
    // `profiles/r02/ab/tile_late_prefetch.jsonl`)
    if constexpr (TL != 0 && WL == 5 && !SORT) {
        if (seg0 != 0)
            return launch_tiles_lpf<MODE, SORT, E, NT, TL, WL, false>(grid, lds, s, data, tlog, ilog, wlog,
                                                                      dtile, seed, tiles, pbase, seg0, sw,
                                                                      hole_at, hole_len);
    }
    return launch_tiles_lpf<MODE, SORT, E, NT, TL, WL, true>(grid, lds, s, data, tlog, ilog, wlog, dtile,
                                                             seed, tiles, pbase, seg0, sw, hole_at, hole_len);
}

// The block-swizzled layout (kSwzMask) of a pass's input and output
struct Swz {
    bool in = false, out = false;
};

struct TileCfg {
    uint32_t tlog, E, NT;
    unsigned tiles, grid;  // tiles: the live tiles a launch runs (the hole excluded)
    size_t lds;
    unsigned hole_at = 0, hole_len = 0;  // pad-only tiles skipped inside the range (pad_map)
};
// the selection sink of the last pass (see bitonic_merge_direct SEL)
struct SelSink {
    uint32_t d = 0;
    uint32_t *cnt = nullptr;  // null: no sink
};

template <int MODE, int E, int NT, bool STRIDED>
static hipError_t launch_direct(const TileCfg &c, hipStream_t s, uint64_t *data, uint32_t ilog,
                                uint32_t wlog, uint32_t dtile, uint32_t seed, uint32_t pbase,
                                const SelSink &sink = SelSink{}, Swz sw = Swz{}) {
    constexpr int R1 = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    const int rest = (int)c.tlog - (int)(STRIDED ? wlog : 0u) - R1;  // steps after the register round
    const int rl = rest <= 0 ? 0 : (rest - 1) % R1 + 1;  // lds_steps' greedy split leaves this last
    if (rl == 0) return hipErrorInvalidValue;
    // the select pass writes ~nothing
    net_account((uint64_t)(sink.cnt ? 8 : 16) * c.tiles << c.tlog,
                sink.cnt ? "bitonic_merge_direct(select)" : "bitonic_merge_direct", s);
#define BD_GO2(RL_, SEL_, TL_, SWI_, SWO_)                                                         \
    do {                                                                                           \
        static bool attr = false;                                                                  \
        if (!attr) {                                                                               \
            (void)hipFuncSetAttribute(                                                             \
                (const void *)bitonic_merge_direct<MODE, E, NT, RL_, STRIDED, SEL_, TL_, SWI_, SWO_>, \
                hipFuncAttributeMaxDynamicSharedMemorySize,                                        \
                160 * 1024 - (SEL_ ? 256 : 0)); /* static wtot[] counts against the 160 KB */      \
            attr = true;                                                                           \
        }                                                                                          \
        FLTEE_LAUNCH((bitonic_merge_direct<MODE, E, NT, RL_, STRIDED, SEL_, TL_, SWI_, SWO_>), \
                           dim3(c.grid), dim3(NT), c.lds, s, data, c.tlog, ilog, wlog, dtile, seed, \
                           c.tiles, pbase, sink.d, sink.cnt, c.hole_at, c.hole_len);               \
    } while (0)
#define BD_GO1(RL_, SEL_, TL_) BD_GO2(RL_, SEL_, TL_, false, false)
#define BD_GO(RL_, TL_)                                                                            \
    do {                                                                                           \
        if (!STRIDED && sink.cnt) BD_GO1(RL_, true, TL_);                                          \
        else BD_GO1(RL_, false, TL_);                                                              \
    } while (0)
    // contiguous tiles of the usual sizes: the LDS rounds unrolled at compile time
    if constexpr (!STRIDED) {
        if constexpr (E == 16 && NT == 1024) {
            if (c.tlog == 14 && rl == 2) {
                if (sw.in && sw.out && !sink.cnt) BD_GO2(2, false, 14, true, true);  // a middle merge
                else if (sw.in && !sw.out && sink.cnt) BD_GO2(2, true, 14, true, false);  // the last
                else if (sw.in && !sw.out) BD_GO2(2, false, 14, true, false);
                else if (sw.out) return hipErrorInvalidValue;
                else BD_GO(2, 14);
                return hipGetLastError();
            }
        }
        if constexpr (E == 16 && NT == 512) {
            if (c.tlog == 13 && rl == 1) { BD_GO(1, 13); return hipGetLastError(); }
        }
    }
    if (sw.in || sw.out) return hipErrorInvalidValue;  // swizzled: 2^14 contiguous tiles only
    switch (rl) {
    case 1: BD_GO(1, 0); break;
    case 2: if constexpr (R1 >= 2) BD_GO(2, 0); break;
    case 3: if constexpr (R1 >= 3) BD_GO(3, 0); break;
    case 4: if constexpr (R1 >= 4) BD_GO(4, 0); break;
    default: if constexpr (R1 >= 5) BD_GO(5, 0); break;
    }
#undef BD_GO
#undef BD_GO1
#undef BD_GO2
    return hipGetLastError();
}

template <int MODE, int E, int NT, int GEN = 0>
static hipError_t launch_sort_direct(const TileCfg &c, hipStream_t s, uint64_t *data,
                                     uint32_t seed, uint32_t pbase, const SortGen &g = SortGen{},
                                     bool swo = false) {
    constexpr int R1 = E >= 32 ? 5 : (E >= 16 ? 4 : (E >= 8 ? 3 : (E >= 4 ? 2 : 1)));
    const int rl = ((int)c.tlog - 1) % R1 + 1;  // lds_steps' greedy split of stage tlog
    SortGen gg = g;
    unsigned grid = c.grid;
    // the live tiles' read + write (GEN: the read is the client records; the initial
    // entries, dummies and pads are made in registers) ...
    uint64_t bytes = (uint64_t)16 * c.tiles << c.tlog;
    if (GEN) {
        const uint64_t live = (uint64_t)c.tiles << c.tlog;
        const uint64_t rd = g.nrec > pbase ? (uint64_t)g.nrec - pbase : 0u;
        bytes = 8 * live + 8 * (rd < live ? rd : live);
    }
    if (gg.pad_n) {  // + store-only blocks for the pad tiles, about 8 stores per lane
        gg.grid_live = c.grid;
        uint32_t nb = (gg.pad_n / 2u + NT * 8u - 1u) / (NT * 8u);
        grid += nb < 1024u ? nb : 1024u;
        bytes += (uint64_t)8 * gg.pad_n;  // ... + the pad tiles' stores
    }
    net_account(bytes, "bitonic_sort_direct", s);
#define BS_GO_SW(RL_, TL_, LPF_, SWO_)                                                             \
    do {                                                                                           \
        static bool attr = false;                                                                  \
        if (!attr) {                                                                               \
            (void)hipFuncSetAttribute((const void *)bitonic_sort_direct<MODE, E, NT, RL_, GEN, TL_, LPF_, SWO_>, \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);     \
            attr = true;                                                                           \
        }                                                                                          \
        FLTEE_LAUNCH((bitonic_sort_direct<MODE, E, NT, RL_, GEN, TL_, LPF_, SWO_>), dim3(grid), \
                           dim3(NT), c.lds, s, data, c.tlog, seed, c.tiles, pbase, gg);            \
    } while (0)
#define BS_GO_PF(RL_, TL_, LPF_) BS_GO_SW(RL_, TL_, LPF_, false)
#define BS_GO(RL_, TL_) BS_GO_PF(RL_, TL_, ((TL_) != 0 ? kSortLatePf<MODE> : 1))
    // the usual tile sizes: every stage's LDS rounds unrolled at compile time
    if constexpr (E == 16 && NT == 1024) {
        if (c.tlog == 14 && rl == 2) {
            if (swo) BS_GO_SW(2, 14, kSortLatePf<MODE>, true);
            else BS_GO(2, 14);
            return hipGetLastError();
        }
    }
    if (swo) return hipErrorInvalidValue;  // swizzled: 2^14 tiles of 1024 lanes only
    if constexpr (E == 16 && NT == 512) {
        if (c.tlog == 13 && rl == 1) { BS_GO(1, 13); return hipGetLastError(); }
    }
    if constexpr (E == 8 && NT == 512) {
        if (c.tlog == 12 && rl == 3) { BS_GO(3, 12); return hipGetLastError(); }
    }
    switch (rl) {
    case 1: BS_GO(1, 0); break;
    case 2: if constexpr (R1 >= 2) BS_GO(2, 0); break;
    case 3: if constexpr (R1 >= 3) BS_GO(3, 0); break;
    case 4: if constexpr (R1 >= 4) BS_GO(4, 0); break;
    default: if constexpr (R1 >= 5) BS_GO(5, 0); break;
    }
#undef BS_GO
#undef BS_GO_PF
#undef BS_GO_SW
    return hipGetLastError();
}

// sw: the block-swizzled layout of the pass's input / output (2^14 tiles of 1024 lanes:
// the first pass writes it, the middle passes read and write it, the last reads it)
template <int MODE, bool SORT>
static hipError_t launch_tiles(const TileCfg &c, hipStream_t s, uint64_t *data, uint32_t ilog,
                               uint32_t wlog, uint32_t dtile, uint32_t seed, uint32_t pbase,
                               const SelSink &sink = SelSink{}, uint32_t seg0 = 0, Swz sw = Swz{}) {
    if (c.tiles == 0) return hipSuccess;  // every tile in pad-only stage blocks
    const bool plain = seg0 == 0 && ilog != 0;  // one segment over every row bit
    if (SORT && wlog == c.tlog && c.tlog > 6) {
        if (sw.in) return hipErrorInvalidValue;
        if (c.NT == 1024) return launch_sort_direct<MODE, 16, 1024>(c, s, data, seed, pbase, SortGen{}, sw.out);
        if (sw.out) return hipErrorInvalidValue;
        if (c.NT == 512 && c.E == 16) return launch_sort_direct<MODE, 16, 512>(c, s, data, seed, pbase);
        if (c.NT == 512 && c.E == 8) return launch_sort_direct<MODE, 8, 512>(c, s, data, seed, pbase);
    }
    // contiguous merges of 2^13 / 2^14 tiles: first and last round in registers
    // (A/B at 2^27: 13.89 vs 14.63 ms mode 0, 14.55 vs 15.65 ms mode 2; 2^24: -6 %)
    // FLTEE_DIRECT_MERGE 0 (round 4): a merge that neither selects nor changes layout runs as
    // a plain contiguous tile pass with 16-B slot pairs instead of the direct merge (8-B
    // loads for its register head round): C4 8.02 -> 8.00 ms, C5 12.28 -> 12.26 ms
    // (`profiles/r04/ab/ab16_tile_merges_*.jsonl`); the selecting last pass and the last
    // merge of a swizzled sort (reads swizzled, writes in order) stay direct
    const bool direct = FLTEE_DIRECT_MERGE || sink.cnt || (sw.in != sw.out && !FLTEE_UNSW_TILES);
    if constexpr (!SORT) {
        // the last merge of a swizzled sort as a slot-pair tile pass that reads swizzled and
        // writes in order (FLTEE_UNSW_TILES)
        if (!direct && sw.in && !sw.out && plain && wlog == c.tlog && c.NT == 1024 && c.E == 16 &&
            c.tlog == 14) {
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute(
                    (const void *)bitonic_tiles<MODE, false, 16, 1024, 14, 0, true, true, false, true>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr = true;
            }
            net_account((uint64_t)16 * c.tiles << c.tlog, "bitonic_tiles", s);
            FLTEE_LAUNCH((bitonic_tiles<MODE, false, 16, 1024, 14, 0, true, true, false, true>), dim3(c.grid),
                               dim3(1024), c.lds, s, data, c.tlog, ilog, wlog, dtile, seed, c.tiles, pbase, 0u,
                               c.hole_at, c.hole_len);
            return hipGetLastError();
        }
    }
    if (!SORT && plain && wlog == c.tlog && c.tlog > 6 && direct) {
        if (c.NT == 1024) return launch_direct<MODE, 16, 1024, false>(c, s, data, ilog, wlog, dtile, seed, pbase, sink, sw);
        if (c.NT == 512 && c.E == 16 && !sw.in && !sw.out)
            return launch_direct<MODE, 16, 512, false>(c, s, data, ilog, wlog, dtile, seed, pbase, sink);
    }  // (E <= 8 tiles, M <= 2^20: measured no faster, 175 vs 169 us at 2^20)
    if (sink.cnt) return hipErrorNotSupported;  // only the direct contiguous merge selects
    // the other tile passes are in place: a swizzled one reads and writes that layout
    if (sw.in != sw.out || (sw.in && (SORT || c.NT != 1024 || c.E != 16))) return hipErrorInvalidValue;
    // (strided tiles with the first / last round in registers were slower: 14.64 vs
    // 14.03 ms at 2^27, the last round's 8-B stores land 2^dtile apart)
    // strided passes of the usual tile sizes, rows of 2^4 .. 2^7 (and, for 2^12 tiles, the
    // planned tiles' 2^8 .. 2^9, whose tails fill the consecutive bits): compile-time rounds
    const uint32_t wmin = c.NT == 1024 ? (uint32_t)FLTEE_TILE_MINW14 : (uint32_t)FLTEE_TILE_MINW12;
    if (!SORT && ilog != 0 && wlog < c.tlog && wlog >= wmin && (1u << wlog) <= c.NT &&
        ((c.NT == 1024 && c.E == 16 && c.tlog == 14) || (c.NT == 512 && c.E == 8 && c.tlog == 12)) &&
        (wlog <= 7 || (seg0 && MODE != 2 && c.NT <= 512) || (FLTEE_TILE_W10 && c.NT == 1024 && wlog == 10) ||
         (FLTEE_TILE_MINW14 < 4 && c.NT == 1024 && wlog == 8))) {
#define BT_ST_CASE(E_, NT_, TL_, W_)                                                               \
    case W_: return launch_tiles_e<MODE, SORT, E_, NT_, TL_, W_>(c.grid, c.lds, s, data, c.tlog, ilog, wlog, dtile, seed, c.tiles, pbase, seg0, sw.in, c.hole_at, c.hole_len);
        if (c.NT == 1024) {
            switch (wlog) {
                BT_ST_CASE(16, 1024, 14, 4) BT_ST_CASE(16, 1024, 14, 5) BT_ST_CASE(16, 1024, 14, 6)
                BT_ST_CASE(16, 1024, 14, 7)
#if FLTEE_TILE_MINW14 < 4
                BT_ST_CASE(16, 1024, 14, 3) BT_ST_CASE(16, 1024, 14, 8)
#endif
#if FLTEE_TILE_W10
                BT_ST_CASE(16, 1024, 14, 10)  // rows of 2^10 (the planned tails on 10 low bits)
#endif
            default: break;
            }
        } else {
            switch (wlog) {
                BT_ST_CASE(8, 512, 12, 4) BT_ST_CASE(8, 512, 12, 5) BT_ST_CASE(8, 512, 12, 6)
                BT_ST_CASE(8, 512, 12, 7)
#if FLTEE_TILE_MINW12 < 4
                BT_ST_CASE(8, 512, 12, 3)
#endif
            default: break;
            }
            if constexpr (MODE != 2) {  // planned tiles only (the keyed shuffle runs per stage)
                switch (wlog) {
                    BT_ST_CASE(8, 512, 12, 8) BT_ST_CASE(8, 512, 12, 9)
                default: break;
                }
            }
        }
#undef BT_ST_CASE
    }
#define BT_GO(E_, NT_) \
    return launch_tiles_e<MODE, SORT, E_, NT_>(c.grid, c.lds, s, data, c.tlog, ilog, wlog, dtile, seed, c.tiles, pbase, seg0, sw.in, c.hole_at, c.hole_len)
    if (!FLTEE_DIRECT_MERGE && !SORT && plain && wlog == c.tlog && c.NT == 1024 && c.E == 16 && c.tlog == 14)
        return launch_tiles_e<MODE, SORT, 16, 1024, 14>(c.grid, c.lds, s, data, c.tlog, ilog, wlog, dtile, seed,
                                                        c.tiles, pbase, 0u, sw.in, c.hole_at, c.hole_len);
    if (c.NT == 1024) BT_GO(16, 1024);
    if (c.NT == 256) BT_GO(2, 256);
    if (c.NT == 128) BT_GO(2, 128);
    if (c.NT == 64) BT_GO(2, 64);
    if (!SORT && plain && wlog == c.tlog && c.E == 8 && c.tlog == 12)  // contiguous 2^12 merge
        return launch_tiles_e<MODE, SORT, 8, 512, 12>(c.grid, c.lds, s, data, c.tlog, ilog, wlog,
                                                      dtile, seed, c.tiles, pbase, 0u, false, c.hole_at,
                                                      c.hole_len);
    switch (c.E) {
    case 2: BT_GO(2, 512);
    case 4: BT_GO(4, 512);
    case 8: BT_GO(8, 512);
    default: BT_GO(16, 512);
    }
#undef BT_GO
}

// Tile configuration for an m = 2^mlog record array whose sort runs stages 1..slog.
// 2^14-record tiles (1024 lanes x 16) when there are enough of them to fill the CUs;
// else up to 2^13 with 512 lanes; small sorts use E = 2 and T/2 lanes; tlog <= 6
// means every stage is one register pass (no tiles).
static TileCfg make_cfg(uint32_t mlog, uint32_t slog) {
    TileCfg c{};
    const uint32_t tmax = kMaxTileLog;
    uint32_t tlog = mlog < tmax ? mlog : tmax;
    if (tlog > slog) tlog = slog;
    const uint32_t mt = kMinTilesLog;
    if (tlog == 14 && mlog - tlog < mt) tlog = 13;
    while (tlog > FLTEE_TILE_FLOOR && tlog <= 13 && (mlog - tlog) < mt) --tlog;  // >= 2^mt tiles
    c.tlog = tlog;
    if (tlog <= 6) return c;
    const uint32_t T = 1u << tlog;
    if (tlog == 14) {  // (512 lanes x 32 records, 5 steps per round: 15.07 vs 14.05 ms at 2^27)
        c.E = 16;
        c.NT = 1024;
    } else if (T >= 1024) {
        c.E = T / 512 > 16 ? 16 : T / 512;  // 512 lanes
        c.NT = 512;
    } else {
        c.E = 2;
        c.NT = T / 2;  // 64, 128 or 256 lanes
    }
    c.tiles = 1u << (mlog - tlog);
    c.lds = (size_t)(T + T / 16 + 1) * 8;
    // persistent: one (2^14) or two resident tiles per CU, each prefetching its next tile
    const unsigned resident = tlog == 14 ? 256 : 512;
    c.grid = c.tiles < resident ? c.tiles : resident;
    return c;
}

// Pad-only stage blocks.  Positions >= `valid` hold identical pad records (u32::MAX,
// +0.0) — or ~0 composite keys — and a stage-ilog step only pairs positions inside one
// aligned 2^ilog block, so every such block lying at or past roundup(valid, 2^ilog)
// holds pads alone before and after the whole stage: swapping equal records changes
// nothing.  Tiles and groups are numbered in position order (strided tiles by their
// 2^(dtile+R) superblock first), so the live ones are a prefix: T-record tiles <
// skip_from / T, 2^R-record groups < skip_from / 2^R.  The bound depends only on the
// public sizes (n, k, d, T): the network stays oblivious, and bit-identical.
static uint32_t skip_from(uint32_t valid, uint32_t ilog, uint32_t mlog) {
    if (valid == 0 || ilog >= mlog) return 0;
    const uint64_t b = ((uint64_t)valid + ((uint64_t)1 << ilog) - 1) >> ilog << ilog;
    return b >= ((uint64_t)1 << mlog) ? 0u : (uint32_t)b;
}
static TileCfg live_tiles(const TileCfg &c, uint32_t skip) {
    if (!skip) return c;
    TileCfg l = c;
    const uint32_t live = skip >> c.tlog;
    if (live < l.tiles) l.tiles = live;
    if (l.grid > l.tiles) l.grid = l.tiles;
    return l;
}
// fltee_debug_set_pad_skip (A/B): 0 off, 1 pad-only stage blocks, 2 (default) also the pad-only
// units inside a stage's mixed block on the planned schedule (pad_map)
static int g_pad_skip = 2;
void set_pad_skip(int on) { g_pad_skip = on < 0 ? 0 : (on > 2 ? 2 : on); }
bool pad_skip_enabled() { return g_pad_skip != 0; }

// Pads inside a stage's mixed block.  Sorting by key (MODE 0 / 1), the pads are the largest
// keys, so a compare-exchange of a pad with a record always leaves the pad on the side its
// direction sends the larger key to, and one of two pads with another pad: the set of
// positions holding pads after every step depends on `valid` alone (public), not on the
// data.  At stage ilog one aligned 2^ilog block holds `valid` (the mixed block: below it no
// pads, above it pads alone).  Its two halves come sorted in opposite directions, so the
// block is bitonic and each step's half-cleaner sends min(p, half) of its p pads to the
// half its direction fills with the larger keys (the 0-1 principle): one half is then
// clean (pads alone, or none) and the other holds the rest.  Pads alone fill
//   ascending block:  [end, M)                  (a suffix, growing down from the top)
//   descending block: [hlo, hhi) and [end, M)   (growing up from the block's start)
// at the start of step 2^jstep (steps ilog-1 .. jstep+1 done).  A unit of a launch (tile or
// register group) whose positions all lie there holds pads alone and its compare-exchanges
// pair pads with pads: skipping it leaves the array as it is.  (A record whose key equals
// the pads' — idx u32::MAX — shares their key: the positions holding that key still follow
// the same map (monotone in the set: a superset of it), only records of that key may end
// in another order among themselves; none of them has idx < d, so no output changes.)
// The keyed shuffle (MODE 2) moves pads by a secret permutation: stage blocks only.
struct PadMap {
    uint64_t end, hlo, hhi;
};
static PadMap pad_map(uint64_t valid, uint32_t mlog, uint32_t ilog, uint32_t jstep, uint32_t pbase,
                      bool fine) {
    const uint64_t M = (uint64_t)1 << mlog;
    PadMap r{M, 0, 0};
    if (valid == 0 || valid >= M || ilog > mlog) return r;
    const uint64_t B = (uint64_t)1 << ilog;
    const uint64_t a = valid & ~(B - 1), bend = a + B;  // the block holding position `valid`
    if (a == valid) { r.end = valid; return r; }        // aligned: whole pad blocks from valid on
    r.end = bend;
    if (!fine) return r;
    const bool asc = ((((uint64_t)pbase + a) >> ilog) & 1u) == 0;
    uint64_t lo = a, size = B, p = bend - valid, padlo = bend, padhi = a;
    for (int k = (int)ilog - 1; k > (int)jstep && p != 0 && p != size; --k) {
        const uint64_t half = (uint64_t)1 << k;
        if (p >= half) {  // the half taking the larger keys is pads alone
            if (asc) padlo = lo + half;
            else { padhi = lo + half; lo += half; }
            p -= half;
        } else if (asc) {
            lo += half;  // the lower half has none left: the upper one holds all p
        }
        size = half;
    }
    if (p == size) {  // the rest of the block is pads too
        if (asc) padlo = lo;
        else padhi = lo + size;
    }
    if (asc) r.end = padlo;
    else { r.hlo = a; r.hhi = padhi; }
    return r;
}

// The live units of a launch whose units (2^uplog per aligned superblock of 2^sblog
// positions, numbered in position order) start at step 2^jstep of stage ilog: every unit
// before `live` runs except the hole_len units from hole_at on.
struct PadUnits {
    uint32_t live, hole_at, hole_len;
};
template <int MODE>
static PadUnits pad_units(uint32_t valid, uint32_t mlog, uint32_t pbase, uint32_t ilog, uint32_t jstep,
                          uint32_t sblog, uint32_t uplog) {
    const uint64_t nunits = ((uint64_t)1 << (mlog - sblog)) << uplog;
    PadUnits u{(uint32_t)nunits, 0u, 0u};
    if (!g_pad_skip || valid == 0) return u;
    const PadMap pm = pad_map(valid, mlog, ilog, jstep, pbase, MODE != 2 && g_pad_skip >= 2);
    const uint64_t sb = (uint64_t)1 << sblog;
    auto up = [&](uint64_t x) { return ((x + sb - 1) >> sblog) << uplog; };
    auto dn = [&](uint64_t x) { return (x >> sblog) << uplog; };
    const uint64_t live = up(pm.end);
    u.live = (uint32_t)(live < nunits ? live : nunits);
    if (pm.hhi > pm.hlo) {
        const uint64_t h0 = up(pm.hlo), h1 = dn(pm.hhi);
        if (h1 > h0 && h1 <= u.live) { u.hole_at = (uint32_t)h0; u.hole_len = (uint32_t)(h1 - h0); }
    }
    return u;
}

// Steps jtop..0 of stage ilog (ilog > c.tlog) over the m = 2^mlog records at global
// positions pbase..pbase+m-1: the steps with j >= T in register passes (up to 6 steps)
// or strided LDS passes (more than 6), then one merge tile pass for the steps j < T.
// valid: positions >= valid hold identical pads (0: unknown, nothing skipped).
template <int MODE>
static hipError_t stage_steps(uint64_t *data, uint32_t mlog, const TileCfg &c0, uint32_t ilog,
                              int jtop, uint32_t seed, uint32_t pbase, hipStream_t s,
                              const SelSink &sink = SelSink{}, uint32_t valid = 0) {
    // a register pass of R steps runs M / 2^R lanes: keep >= 2^16 of them (256 lanes per
    // CU) down to R = 4 — at M = 2^20 (C3) R = 6 left 64 blocks of 256 for the whole chip (10.1 us for
    // that pass; the cap, as R = 4 there: 0.1894 vs 0.1916 ms per aggregate)
    const int rcap = (int)mlog - 16 < 4 ? 4 : (int)mlog - 16;
    const int kMaxGlobalR = kRegMaxSteps < rcap ? kRegMaxSteps : rcap;
    const uint32_t skip = g_pad_skip ? skip_from(valid, ilog, mlog) : 0u;
    const TileCfg c = live_tiles(c0, skip);
    const uint32_t tlog = c.tlog, T = 1u << tlog;
    const int rs = (int)tlog - kMinWLog;  // global steps per strided LDS pass (W >= 2^kMinWLog)
    const int nglobal = jtop - (int)tlog + 1;  // steps with j >= T
    hipError_t e;
    if (nglobal > 0) {
        const int per = rs > kMaxGlobalR ? rs : kMaxGlobalR;
        const int passes = (nglobal + per - 1) / per;
        for (int p = 0; p < passes; ++p) {
            const int left = jtop - (int)tlog + 1;
            const int R = (left + (passes - p) - 1) / (passes - p);  // balanced split
            if (R > kMaxGlobalR && (T >> R) <= c.NT) {  // strided LDS tile: W = T / 2^R consecutive x 2^R rows
                const uint32_t dtile = (uint32_t)(jtop - R + 1);
                e = launch_tiles<MODE, false>(c, s, data, ilog, tlog - (uint32_t)R, dtile, seed, pbase);
            } else {
                e = launch_global<MODE>(data, mlog, ilog, (uint32_t)jtop, R, seed, s, pbase,
                                        skip >> R);
            }
            if (e != hipSuccess) return e;
            jtop -= R;
        }
    }
    return launch_tiles<MODE, false>(c, s, data, ilog, tlog, tlog, seed, pbase, sink);
}


// ------------------------------------------------------------ planned schedule --
// The steps of stages T+1 .. M (after the first pass) split into launches by a shortest
// path over the step sequence, instead of "per stage: register / strided passes for the
// steps j >= T, then one merge for j < T".  A launch is
//   * a register pass: up to rmax consecutive steps of one stage (bitonic_global);
//   * an LDS tile pass over 2^tlog records whose positions vary in bits [0, wlog) (W >= 16
//     consecutive records: coalesced) and in tlog - wlog row bits from dtile up.  It runs
//     at most two segments, in network order: a stage's LAST steps on bits aTop..0 (low
//     bits) and then the next stage's FIRST steps on every row bit (a tail fused with the
//     next head), or one of them alone.
// Each launch costs about the same whatever the steps (HBM or launch bound), so fewer
// launches win: at M = 2^27 / 2^14 tiles 23 instead of 35, at 2^20 / 2^12 tiles 13
// instead of 17.  The steps and their order are the reference network's: bit-identical.
// The last launch is always the contiguous merge of stage M's last tlog steps (the direct
// merge, and the only pass that can carry the selection sink).
struct NetPass {
    bool reg = false;
    uint32_t ilog = 0, jtop = 0, R = 0;  // register pass
    uint32_t ilogA = 0, aTop = 0;        // tile: segment A (0: none), steps aTop..0
    uint32_t ilogB = 0;                  // tile: segment B (0: none), steps on every row bit
    uint32_t wlog = 0, dtile = 0;        // tile shape
    uint32_t stage = 0;                  // the last stage the launch touches (pad skip)
};

static std::vector<NetPass> plan_network(uint32_t mlog, uint32_t tlog, uint32_t NT, int rmax) {
    const bool t14 = tlog == 14 && NT == 1024, t12 = tlog == 12 && NT == 512;
    const uint32_t minw = t14 ? (uint32_t)FLTEE_TILE_MINW14
                              : t12 ? (uint32_t)FLTEE_TILE_MINW12 : (uint32_t)kMinWLog;
    uint32_t ntl = 0;
    while ((1u << (ntl + 1)) <= NT) ++ntl;  // log2 NT: W <= NT for strided tiles
    // narrower rows than 2^4: only the row widths launch_tiles has compile-time rounds for
    auto w_ok = [&](uint32_t w) {
        if (minw >= 4) return true;
        return t14 ? ((w >= 3 && w <= 8) || (FLTEE_TILE_W10 && w == 10)) : (w >= 3 && w <= 9);
    };
    // relative launch costs (MI355X rocprof, `profiles/r02/`): register passes R <= 4 one
    // unit (2^27: 268-280 us, 2^20: 4.5-5.2 us), R = 5 / 6 at 2^27 1.19 / 1.43; strided and
    // two-segment tiles 1.5 (2^27: 404 us) / 1.45 (2^20: 7.3 us); the direct contiguous merge
    // 1.35 (2^27: 360 us) / 1.55 (2^20: 7.8 us)
    const bool large = mlog >= 23;
    auto creg = [&](int R) { return R <= 4 ? 1.0 : (large ? (R == 5 ? 1.19 : 1.43) : 1.0); };
    const double ctile = large ? 1.50 : 1.45, cmerge = large ? 1.35 : 1.55;
    // steps: stage s (tlog < s <= mlog) has bits s-1 .. 0
    std::vector<uint32_t> st, bt, first;  // stage, bit of step k; first step of stage s
    first.assign(mlog + 2, 0);
    for (uint32_t s = tlog + 1; s <= mlog; ++s) {
        first[s] = (uint32_t)st.size();
        for (int b = (int)s - 1; b >= 0; --b) st.push_back(s), bt.push_back((uint32_t)b);
    }
    const size_t N = st.size();
    first[mlog + 1] = (uint32_t)N;
    std::vector<double> best(N + 1, 1e30);
    std::vector<NetPass> choice(N + 1);
    std::vector<size_t> nxt(N + 1, N);
    best[N] = 0.0;
    for (size_t i = N; i-- > 0;) {
        const uint32_t s = st[i], b = bt[i];
        const size_t stage_end = first[s + 1];  // index after stage s's bit 0
        auto consider = [&](size_t j, double c, const NetPass &p) {
            if (j > N || best[j] >= 1e29) return;
            if (c + best[j] < best[i] - 1e-9) {
                best[i] = c + best[j];
                choice[i] = p;
                nxt[i] = j;
            }
        };
        const bool last_stage = s == mlog;
        // the last stage's steps below tlog belong to the final contiguous merge only
        if (last_stage && b < tlog) {
            if (b == tlog - 1) {
                NetPass p;
                p.ilogA = s; p.aTop = b; p.wlog = p.dtile = tlog; p.stage = s;
                consider(N, cmerge, p);
            }
            continue;
        }
        // register pass: R steps b .. b-R+1 of stage s
        for (int R = 1; R <= rmax && R <= (int)b + 1; ++R) {
            if (last_stage && (int)b - R + 1 < (int)tlog) break;
            NetPass p;
            p.reg = true; p.ilog = s; p.jtop = b; p.R = (uint32_t)R; p.stage = s;
            consider(i + (size_t)R, creg(R), p);
        }
        // tail of stage s alone (contiguous tile): steps b .. 0
        if (!last_stage && b <= tlog - 1) {
            NetPass p;
            p.ilogA = s; p.aTop = b; p.wlog = p.dtile = tlog; p.stage = s;
            consider(stage_end, b == tlog - 1 ? cmerge : ctile, p);
        }
        // middle of stage s (strided tile, low bits idle): steps b .. lo on the row bits
        for (uint32_t rows = 1; rows <= b && rows < tlog; ++rows) {
            const uint32_t lo = b - rows + 1, w = tlog - rows;
            if (w < minw || w > ntl || lo < w || !w_ok(w)) continue;
            if (last_stage && lo < tlog) continue;
            NetPass p;
            p.ilogB = s; p.wlog = w; p.dtile = lo; p.stage = s;
            consider(i + rows, ctile, p);
        }
        // tail of stage s (bits b..0, low bits) + head of stage s+1 (bits s .. lo, row bits)
        if (s < mlog) {
            for (uint32_t rows = 1; rows < tlog; ++rows) {
                const uint32_t w = tlog - rows;
                if (w < b + 1 || w < minw || w > ntl || !w_ok(w)) continue;
                if (rows > s) break;
                const uint32_t lo = s - rows + 1;
                if (lo < w) continue;
                if (s + 1 == mlog && lo < tlog) continue;
                NetPass p;
                p.ilogA = s; p.aTop = b; p.ilogB = s + 1; p.wlog = w; p.dtile = lo; p.stage = s + 1;
                consider(first[s + 1] + rows, ctile, p);
            }
        }
    }
    std::vector<NetPass> plan;
    for (size_t i = 0; i < N;) {
        if (best[i] >= 1e29) return {};  // no schedule (cannot happen for tlog >= 4): old path
        plan.push_back(choice[i]);
        i = nxt[i];
    }
    return plan;
}

static const std::vector<NetPass> &cached_plan(uint32_t mlog, uint32_t tlog, uint32_t NT, int rmax) {
    static std::mutex mu;
    static std::map<uint64_t, std::vector<NetPass>> plans;
    const uint64_t key = ((uint64_t)mlog << 40) | ((uint64_t)tlog << 32) | ((uint64_t)NT << 8) | (uint64_t)rmax;
    std::lock_guard<std::mutex> lk(mu);
    auto it = plans.find(key);
    if (it == plans.end()) it = plans.emplace(key, plan_network(mlog, tlog, NT, rmax)).first;
    return it->second;
}

// test hook (fltee_debug_pad_units): pad_units of a sort by key (mode 0/1) or the keyed
// shuffle (mode 2) at the current pad-skip level: {live, hole_at, hole_len}
void debug_pad_units(uint32_t mode, uint32_t valid, uint32_t mlog, uint32_t pbase, uint32_t ilog,
                     uint32_t jstep, uint32_t sblog, uint32_t uplog, uint32_t out[3]) {
    const PadUnits u = mode == 2 ? pad_units<2>(valid, mlog, pbase, ilog, jstep, sblog, uplog)
                                 : pad_units<0>(valid, mlog, pbase, ilog, jstep, sblog, uplog);
    out[0] = u.live;
    out[1] = u.hole_at;
    out[2] = u.hole_len;
}

// test hook: the plan as rows of 8 words {reg, ilog, jtop, R, ilogA, aTop, ilogB, wlog|dtile<<8}
size_t debug_plan(uint32_t mlog, uint32_t tlog, uint32_t NT, int rmax, uint32_t *out, size_t cap) {
    const std::vector<NetPass> &plan = cached_plan(mlog, tlog, NT, rmax);
    for (size_t k = 0; k < plan.size() && k < cap; ++k) {
        const NetPass &p = plan[k];
        const uint32_t row[8] = {p.reg ? 1u : 0u, p.ilog, p.jtop, p.R, p.ilogA, p.aTop, p.ilogB,
                                 p.wlog | (p.dtile << 8)};
        for (int q = 0; q < 8; ++q) out[k * 8 + q] = row[q];
    }
    return plan.size();
}

// the planned schedule of a full sort (empty: none, the per-stage one runs)
template <int MODE>
static const std::vector<NetPass> *plan_for(uint32_t mlog, const TileCfg &c0) {
    // (the keyed shuffle planned too since round 3: FLTEE_PLAN_SHUFFLE, `profiles/r03/ab`)
    if ((MODE == 2 && !FLTEE_PLAN_SHUFFLE) || c0.tlog <= 6 || mlog <= c0.tlog) return nullptr;
    const int rcap = (int)mlog - 16 < 4 ? 4 : (int)mlog - 16;
    const int rmax = kRegMaxSteps < rcap ? kRegMaxSteps : rcap;
    const std::vector<NetPass> &plan = cached_plan(mlog, c0.tlog, c0.NT, rmax);
    return plan.empty() ? nullptr : &plan;
}

// Whether a full sort runs in the block-swizzled layout (kSwzMask): planned, 2^14 tiles of
// 1024 lanes, its last launch the contiguous merge (plan_network always ends with it).
static bool g_swizzle = true;  // fltee_debug_set_swizzle (A/B)
void set_swizzle(int on) { g_swizzle = on != 0; }
static bool swizzled(const std::vector<NetPass> *plan, const TileCfg &c0) {
    if (!g_swizzle || !plan || c0.tlog != 14 || c0.NT != 1024 || c0.E != 16) return false;
    const NetPass &l = plan->back();
    return !l.reg && l.ilogA && !l.ilogB && l.aTop == c0.tlog - 1;
}

// stages tlog+1 .. mlog of a full sort by the planned launches (false: no plan, use
// stage_steps).  sw: the first pass wrote the block-swizzled layout; the middle launches
// read and write it and the last one (the contiguous merge) writes positions in order.
template <int MODE>
static bool run_plan(uint64_t *data, uint32_t mlog, const TileCfg &c0, uint32_t seed, uint32_t pbase,
                     hipStream_t s, const SelSink &sink, uint32_t valid, hipError_t &e,
                     bool sw = false) {
    const std::vector<NetPass> *pl = plan_for<MODE>(mlog, c0);
    if (!pl) return false;
    const std::vector<NetPass> &plan = *pl;
    e = hipSuccess;
    for (size_t k = 0; k < plan.size() && e == hipSuccess; ++k) {
        const NetPass &p = plan[k];
        const bool last = k + 1 == plan.size();
        const Swz io{sw, sw && !last};
        if (p.reg) {  // groups of 2^R: 2^(jtop+1-R) per superblock of 2^(jtop+1)
            if (io.in != io.out) { e = hipErrorInvalidValue; break; }
            const PadUnits u = pad_units<MODE>(valid, mlog, pbase, p.ilog, p.jtop, p.jtop + 1, p.jtop + 1 - p.R);
            if (u.live == u.hole_len) continue;  // pads alone
            e = launch_global<MODE>(data, mlog, p.ilog, p.jtop, (int)p.R, seed, s, pbase, u.live, sw,
                                    u.hole_at, u.hole_len);
            continue;
        }
        // tiles: contiguous ones one per 2^tlog; strided ones 2^(dtile-wlog) per superblock of
        // 2^(dtile+rows); the launch starts with segment A's top step (else segment B's)
        const uint32_t rows = c0.tlog - p.wlog;
        const bool contig = p.wlog == c0.tlog;
        const PadUnits u = pad_units<MODE>(valid, mlog, pbase, p.ilogA ? p.ilogA : p.ilogB,
                                           p.ilogA ? p.aTop : p.dtile + rows - 1,
                                           contig ? c0.tlog : p.dtile + rows, contig ? 0u : p.dtile - p.wlog);
        TileCfg c = c0;
        c.tiles = u.live - u.hole_len;
        c.hole_at = u.hole_at;
        c.hole_len = u.hole_len;
        if (c.grid > c.tiles) c.grid = c.tiles;
        if (p.ilogA && !p.ilogB && p.aTop == c0.tlog - 1)  // a whole contiguous merge
            e = launch_tiles<MODE, false>(c, s, data, p.ilogA, c0.tlog, c0.tlog, seed, pbase,
                                          last ? sink : SelSink{}, 0u, io);
        else
            e = launch_tiles<MODE, false>(c, s, data, p.ilogB, p.wlog, p.dtile, seed, pbase, SelSink{},
                                          p.ilogA ? ((p.ilogA << 8) | p.aTop) : 0u, io);
    }
    return true;
}

// Stages 1..slog of the network over m records at global positions pbase.. (pbase a
// multiple of m; slog = log2 m: the full sort of this range, ascending where bit slog
// of pbase is 0 and descending where it is 1 — the reference network's direction).
// With slog < log2 m every aligned segment of 2^slog records comes out sorted,
// ascending where bit slog of its first position is 0 and descending where it is 1.
template <int MODE>
static hipError_t sort_impl(uint64_t *data, size_t m, uint32_t seed, hipStream_t s,
                            uint32_t slog, uint32_t pbase, uint32_t valid = 0) {
    const uint32_t mlog = log2_pow2(m);
    const TileCfg c = make_cfg(mlog, slog);
    if (!g_pad_skip) valid = 0;
    hipError_t e;
    if constexpr (MODE == 2) {
        e = keyed_table_prepare(seed, s);
        if (e != hipSuccess) return e;
    }
    if (c.tlog <= 6) {  // tiles of <= 64 records: every stage is one register pass
        for (uint32_t ilog = 1; ilog <= slog; ++ilog) {
            e = launch_global<MODE>(data, mlog, ilog, ilog - 1, (int)ilog, seed, s, pbase,
                                    skip_from(valid, ilog, mlog) >> ilog);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // a full sort on the planned schedule runs in the block-swizzled layout where it can
    const bool sw = slog == mlog && swizzled(plan_for<MODE>(mlog, c), c);
    e = launch_tiles<MODE, true>(live_tiles(c, skip_from(valid, c.tlog, mlog)), s, data, 0u, c.tlog,
                                 c.tlog, seed, pbase, SelSink{}, 0u, Swz{false, sw});
    if (e != hipSuccess) return e;
    if (slog == mlog && run_plan<MODE>(data, mlog, c, seed, pbase, s, SelSink{}, valid, e, sw)) return e;
    for (uint32_t ilog = c.tlog + 1; ilog <= slog; ++ilog) {
        e = stage_steps<MODE>(data, mlog, c, ilog, (int)ilog - 1, seed, pbase, s, SelSink{}, valid);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// The steps j = m/2 .. 1 of stage ilog > log2 m on the m records at global positions
// pbase..: what a stage leaves to each range once its steps j >= m (the exchanges
// between ranges, bitonic_exchange) are done.
template <int MODE>
static hipError_t merge_impl(uint64_t *data, size_t m, uint32_t seed, hipStream_t s,
                             uint32_t ilog, uint32_t pbase) {
    const uint32_t mlog = log2_pow2(m);
    if (mlog == 0) return hipSuccess;
    if constexpr (MODE == 2) {
        const hipError_t e = keyed_table_prepare(seed, s);
        if (e != hipSuccess) return e;
    }
    const TileCfg c = make_cfg(mlog, mlog);
    if (c.tlog <= 6)
        return launch_global<MODE>(data, mlog, ilog, mlog - 1, (int)mlog, seed, s, pbase);
    return stage_steps<MODE>(data, mlog, c, ilog, (int)mlog - 1, seed, pbase, s);
}

// Step j = 2^jlog >= m of stage ilog between two ranges of m records, `mine` at
// positions pos_mine.. and the partner's copy `theirs` at pos_mine ^ j..: position x
// of one pairs with position x of the other (l = the lower one, m = l + j), and
// `mine` takes the partner's record iff that pair swaps.  Same comparator as
// group_steps, so the ranges together run the reference network's step exactly.
template <int MODE>
__global__ __launch_bounds__(256) void bitonic_exchange_kernel(uint4 *__restrict__ mine,
                                                               const uint4 *__restrict__ theirs,
                                                               size_t m2, uint32_t pos_lo,
                                                               uint32_t lower, uint32_t ilog,
                                                               uint32_t key) {
    for (size_t x = (size_t)blockIdx.x * 256 + threadIdx.x; x < m2; x += (size_t)gridDim.x * 256) {
        const uint4 a4 = mine[x], b4 = theirs[x];
        const uint64_t a[2] = {((uint64_t)a4.y << 32) | a4.x, ((uint64_t)a4.w << 32) | a4.z};
        const uint64_t b[2] = {((uint64_t)b4.y << 32) | b4.x, ((uint64_t)b4.w << 32) | b4.z};
        uint64_t r[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t lo = lower ? a[h] : b[h], hi = lower ? b[h] : a[h];
            const uint32_t l = pos_lo + (uint32_t)(2 * x + h);
            const bool asc = (l & (1u << ilog)) == 0;
            const bool sw = asc ^ cond2<MODE>(lo, hi, l, key);
            r[h] = sw ? b[h] : a[h];
        }
        mine[x] = make_uint4((uint32_t)r[0], (uint32_t)(r[0] >> 32), (uint32_t)r[1],
                             (uint32_t)(r[1] >> 32));
    }
}

hipError_t bitonic_sort(uint64_t *data, size_t m, uint32_t mode, uint32_t seed, hipStream_t s,
                        size_t valid) {
    if (m < 2) return hipSuccess;
    if (m > ((size_t)1 << 29)) return hipErrorInvalidValue;  // 32-bit byte offsets (4 GiB)
    const uint32_t mlog = log2_pow2(m);
    const uint32_t v = valid >= m ? 0u : (uint32_t)valid;
    switch (mode) {
    case 0: return sort_impl<0>(data, m, seed, s, mlog, 0u, v);
    case 1: return sort_impl<1>(data, m, seed, s, mlog, 0u, v);
    default: return sort_impl<2>(data, m, seed, s, mlog, 0u, v);
    }
}

hipError_t bitonic_sort_segments(uint64_t *data, size_t m, size_t seg, uint32_t mode,
                                 hipStream_t s) {
    if (m < 2 || seg < 2) return hipSuccess;
    if (m > ((size_t)1 << 29)) return hipErrorInvalidValue;
    const uint32_t slog = log2_pow2(seg);
    switch (mode) {
    case 0: return sort_impl<0>(data, m, 0, s, slog, 0u);
    case 1: return sort_impl<1>(data, m, 0, s, slog, 0u);
    default: return sort_impl<2>(data, m, 0, s, slog, 0u);
    }
}

// ------------------------------------------- sorts with a fused producer ---
// The sort of the padded array that `g` describes (GEN 1: advanced's, 2: nips19's),
// written into data[0, m): the producer runs inside the first pass's loads.
// hipErrorNotSupported when that pass is not the direct tile sort (small m, fused
// init off): the caller then builds the array and sorts it.
static bool g_fused_init = true;  // fltee_debug_set_fused_init (A/B)
void set_fused_init(int on) { g_fused_init = on != 0; }

// whether the last pass of an m-record sort is the direct contiguous merge (the only
// pass that can carry the selection sink)
static bool last_pass_is_direct_merge(size_t m) {
    const uint32_t mlog = log2_pow2(m);
    const TileCfg c = make_cfg(mlog, mlog);
    return c.tlog > 6 && mlog > c.tlog && (c.NT == 1024 || (c.NT == 512 && c.E == 16));
}

template <int MODE, int GEN>
static hipError_t sort_gen_impl(uint64_t *data, size_t m, uint32_t seed, const SortGen &g,
                                hipStream_t s, const SelSink &sink = SelSink{}) {
    if (!g_fused_init || m < 2 || m > ((size_t)1 << 29)) return hipErrorNotSupported;
    const uint32_t mlog = log2_pow2(m);
    const TileCfg c0 = make_cfg(mlog, mlog);
    if (c0.tlog <= 6) return hipErrorNotSupported;
    if (sink.cnt && !last_pass_is_direct_merge(m)) return hipErrorNotSupported;
    if constexpr (MODE == 2) {
        const hipError_t e = keyed_table_prepare(seed, s);
        if (e != hipSuccess) return e;
    }
    // the padded array's records (advanced: records ++ initial entries; nips19: records ++
    // dummies); past them only (u32::MAX, +0.0) pads
    const uint64_t nvalid = (uint64_t)g.nrec + (GEN == 1 ? (uint64_t)g.d : (uint64_t)g.d * g.tf);
    const uint32_t valid = (g_pad_skip && nvalid < m) ? (uint32_t)nvalid : 0u;
    // the first pass skips the tiles of pads alone and a store-only pass writes them
    const TileCfg c = live_tiles(c0, skip_from(valid, c0.tlog, mlog));
    const size_t done = (size_t)c.tiles << c.tlog;
    SortGen gp = g;  // the pad tiles are stored by extra blocks of the same launch
    gp.pad_begin = (uint32_t)done;
    gp.pad_n = (uint32_t)(m - done);
    hipError_t e;
    const bool sw = swizzled(plan_for<MODE>(mlog, c0), c0);  // (pad blocks: whole 2^14 blocks)
    if (c.NT == 1024) e = launch_sort_direct<MODE, 16, 1024, GEN>(c, s, data, seed, 0u, gp, sw);
    else if (c.NT == 512 && c.E == 16) e = launch_sort_direct<MODE, 16, 512, GEN>(c, s, data, seed, 0u, gp);
    else if (c.NT == 512 && c.E == 8) e = launch_sort_direct<MODE, 8, 512, GEN>(c, s, data, seed, 0u, gp);
    else return hipErrorNotSupported;
    if (e != hipSuccess) return e;
    if (run_plan<MODE>(data, mlog, c0, seed, 0u, s, sink, valid, e, sw)) return e;
    for (uint32_t ilog = c0.tlog + 1; ilog <= mlog; ++ilog) {
        e = stage_steps<MODE>(data, mlog, c0, ilog, (int)ilog - 1, seed, 0u, s,
                              ilog == mlog ? sink : SelSink{}, valid);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t bitonic_sort_advanced(uint64_t *data, size_t m, const void *rec, size_t nrec, size_t d,
                                 hipStream_t s) {
    if (nrec + d > m) return hipErrorInvalidValue;
    const SortGen g{(const uint64_t *)rec, nullptr, (uint32_t)nrec, (uint32_t)d, 0u};
    return sort_gen_impl<0, 1>(data, m, 0u, g, s);
}

hipError_t bitonic_sort_nips19(uint64_t *data, size_t m, uint32_t seed, const void *rec, size_t nrec,
                               const uint32_t *r, size_t d, size_t tf, hipStream_t s) {
    if (nrec + d * tf > m) return hipErrorInvalidValue;
    const SortGen g{(const uint64_t *)rec, r, (uint32_t)nrec, (uint32_t)d, (uint32_t)tf};
    return sort_gen_impl<2, 2>(data, m, seed, g, s);
}

size_t bitonic_select_tiles(size_t m) {
    if (m < 2 || m > ((size_t)1 << 29) || !last_pass_is_direct_merge(m)) return 0;
    const TileCfg c = make_cfg(log2_pow2(m), log2_pow2(m));
    return c.tiles;
}

hipError_t bitonic_sort_nips19_select(uint64_t *data, size_t m, uint32_t seed, const void *rec,
                                      size_t nrec, const uint32_t *r, size_t d, size_t tf,
                                      uint32_t *tile_cnt, hipStream_t s) {
    if (nrec + d * tf > m || d > 0xFFFFFFFFull || !tile_cnt) return hipErrorInvalidValue;
    const SortGen g{(const uint64_t *)rec, r, (uint32_t)nrec, (uint32_t)d, (uint32_t)tf};
    SelSink sink;
    sink.d = (uint32_t)d;
    sink.cnt = tile_cnt;
    return sort_gen_impl<2, 2>(data, m, seed, g, s, sink);
}

// ---------------------------------------------- position-range pieces -----
// One range of an M-record network split into M/m ranges of m records (one per GPU,
// SURVEY §8e Option B): the caller runs sort_range on every range, then for each
// stage ilog > log2 m the exchange steps j >= m (bitonic_exchange with the partner
// range pbase ^ j) and merge_range.  Together: the reference network, step for step.
hipError_t bitonic_sort_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                              uint32_t pbase, hipStream_t s, uint32_t valid) {
    if (m < 2) return hipSuccess;
    if (m > ((size_t)1 << 29)) return hipErrorInvalidValue;
    const uint32_t mlog = log2_pow2(m);
    if (valid >= m) valid = 0;
    switch (mode) {
    case 0: return sort_impl<0>(data, m, seed, s, mlog, pbase, valid);
    case 1: return sort_impl<1>(data, m, seed, s, mlog, pbase, valid);
    default: return sort_impl<2>(data, m, seed, s, mlog, pbase, valid);
    }
}

hipError_t bitonic_merge_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                               uint32_t ilog, uint32_t pbase, hipStream_t s) {
    if (m < 2) return hipSuccess;
    if (m > ((size_t)1 << 29)) return hipErrorInvalidValue;
    switch (mode) {
    case 0: return merge_impl<0>(data, m, seed, s, ilog, pbase);
    case 1: return merge_impl<1>(data, m, seed, s, ilog, pbase);
    default: return merge_impl<2>(data, m, seed, s, ilog, pbase);
    }
}

// Steps 2^jtop .. 2^jbot (jtop < ilog, all < log2 m) of stage ilog on the m records at
// positions pbase.. as register passes of up to 6 steps (the few high steps a
// transposed range runs, fltee/parallel.py).
hipError_t bitonic_steps_range(uint64_t *data, size_t m, uint32_t mode, uint32_t seed,
                               uint32_t ilog, uint32_t jtop, uint32_t jbot, uint32_t pbase,
                               hipStream_t s) {
    if (m > ((size_t)1 << 29)) return hipErrorInvalidValue;
    const uint32_t mlog = log2_pow2(m);
    if (jtop >= mlog || jbot > jtop || jtop >= ilog) return hipErrorInvalidValue;
    if (mode == 2) {
        const hipError_t e = keyed_table_prepare(seed, s);
        if (e != hipSuccess) return e;
    }
    const int kMaxGlobalR = kRegMaxSteps;
    int top = (int)jtop;
    while (top >= (int)jbot) {
        const int left = top - (int)jbot + 1;
        const int R = left < kMaxGlobalR ? left : kMaxGlobalR;
        hipError_t e;
        if (mode == 0) e = launch_global<0>(data, mlog, ilog, (uint32_t)top, R, seed, s, pbase);
        else if (mode == 1) e = launch_global<1>(data, mlog, ilog, (uint32_t)top, R, seed, s, pbase);
        else e = launch_global<2>(data, mlog, ilog, (uint32_t)top, R, seed, s, pbase);
        if (e != hipSuccess) return e;
        top -= R;
    }
    return hipSuccess;
}

hipError_t bitonic_exchange(uint64_t *mine, const uint64_t *theirs, size_t m, uint32_t pos_mine,
                            uint32_t pos_theirs, uint32_t mode, uint32_t seed, uint32_t ilog,
                            uint32_t jlog, hipStream_t s) {
    if (m == 0) return hipSuccess;
    if (m & 1) return hipErrorInvalidValue;  // 16-B pairs of records
    const size_t m2 = m / 2;
    size_t blocks = (m2 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    const uint32_t lower = pos_mine < pos_theirs;
    const uint32_t pos_lo = lower ? pos_mine : pos_theirs;
    const uint32_t key = mode == 2 ? shuffle_step_key(seed, ilog, jlog) : 0u;
    net_account((uint64_t)24 * m, "bitonic_exchange_kernel", s);
#define BX_GO(MD)                                                                                  \
    FLTEE_LAUNCH((bitonic_exchange_kernel<MD>), dim3((unsigned)blocks), dim3(256), 0, s,     \
                       (uint4 *)mine, (const uint4 *)theirs, m2, pos_lo, lower, ilog, key)
    if (mode == 0) BX_GO(0); else if (mode == 1) BX_GO(1); else BX_GO(2);
#undef BX_GO
    return hipGetLastError();
}

}  // namespace fltee
