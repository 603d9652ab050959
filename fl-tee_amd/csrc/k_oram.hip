// k_oram.hip — path_oram as a tree Path ORAM on the GPU (oram.rs:64-118; the mobilecoin
// PathORAM the enclave instantiates: bucket size Z = 4, stash 20, next_pow2(d) blocks).
//
// The enclave's access sequence (oram.rs), which this runs one access for one access:
//   prepare()            d writes of 0.0, blocks 0..d-1 (:79-82)
//   per uploaded record  oram.read(idx), then oram.write(idx, value + val) (:100-105)
//   readout              d reads, blocks 0..d-1 -> global_params (:111-113), then x 1f32/n
// = A = 2 n k + 2 d accesses (FLTEE_OPT_ORAM_LAZY instead: one read-modify-write per
// record, blocks created on first use, and the readout through `advanced`'s oblivious
// network: n k accesses).  Each is one Path ORAM access (Stefanov et al.): the block's
// current leaf, a fresh random leaf for it; read the path root..leaf into the pool (path
// buckets + stash); take the block out (or +0.0: a block never written), put it back
// with its new value and leaf; evict greedily — every block to the deepest bucket of
// the path it may live in, four per bucket — keep what does not fit in the stash;
// write the whole path back.
//
// The position map.  The whole access sequence is known when the call starts (its
// blocks are the public positions plus the uploaded indices, its fresh leaves come from
// Philox4x32-10 under the call's seed), so the leaf each access finds its block under —
// the fresh leaf of the previous access to the same block, or the block's initial random
// leaf — is computed up front by two oblivious sorts: the keys (block << 32 | access) in
// the order of the reference bitonic network (mode 1), each access linked to its
// predecessor in the sorted order (a fixed-address pass), and the (access << 32 | leaf)
// pairs sorted back into access order.  Every address in that is a function of the array
// size (no position map read or written at a secret address: the recursive U32PositionMap
// of the crate hides the same thing by another ORAM).  The accesses then read their leaf
// at their own (public) index, so N is bounded by the path fitting the wave (<= 2^22
// blocks, d up to 4M), not by an LDS map.
//
// GPU form of the accesses: ONE persistent wave (they are sequential: each path read
// needs the previous access's path write; lane j holds pool entries j and 64 + j).  Its
// LDS holds the stash and a ring of the next accesses' descriptors; the tree of
// 4 (2N - 1) 16-B slots (idx, leaf, f32 value) lives in HBM.  Obliviousness, as the
// enclave's (ZeroTrace-style) ORAM has it:
//  * the HBM trace of an access is one whole path, root to a uniformly random leaf,
//    written; read, the part of it below the buckets it shares with the previous
//    accesses' paths (a function of the public random leaves);
//  * inside the pool every step is branch-free over all Z (L + 1) + 20 entries: the
//    block is found and taken out by compares and selects, eviction ranks come from
//    wave ballots, and the new path and stash are GATHERED slot by slot through the
//    register crossbar (ds_bpermute: no LDS bank), never scattered; LDS addresses are
//    fixed per lane (stash) or the public access index (ring);
//  * the readout's reads write out[i] at the public position i.
// The output is the in-order f32 sum of each index's values from +0.0, x 1f32/n — bit for
// bit the oracle's fo_path_oram (and non_oblivious / baseline).
#include "common.h"

namespace fltee {

#define FLTEE_STREAM_ORAM 0x4F52414Du
constexpr uint32_t kOramZ = 4, kOramStash = 20;
constexpr uint32_t kOramEmpty = 0xFFFFFFFFu;
constexpr uint32_t kOramMaxLog = 22;  // the path (Z (Lh + 1) + stash <= 128 entries) in one wave;
                                      // slot offsets < 2^31 (buffer resource)
// access kinds (the descriptor ring's top bits)
constexpr uint32_t kOpPrep = 0, kOpRead = 1, kOpWrite = 2, kOpFinal = 3, kOpRmw = 4;
constexpr uint32_t kOpShift = 28, kBlockMask = (1u << kOpShift) - 1u;

__device__ __forceinline__ uint32_t oram_leaf(uint32_t k0, uint32_t k1, uint32_t ctr, uint32_t mask) {
    uint32_t c[4] = {ctr, FLTEE_STREAM_ORAM, 0u, 0u};
    philox4x32_10(c, k0, k1);
    return c[0] & mask;
}


// slot s of the path to leaf x: level s / Z, bucket (2^l - 1) + (x >> (Lh - l))
__device__ __forceinline__ uint32_t oram_slot(uint32_t s, uint32_t x, uint32_t Lh) {
    const uint32_t l = s / kOramZ;
    return (((1u << l) - 1u) + (x >> (Lh - l))) * kOramZ + (s % kOramZ);
}

// the z-th set bit (z = 0, 1, ...) of a 128-bit mask (m0 | m1 << 64), one per call:
// the lowest remaining bit is returned (index, or 0xFF) and cleared.  Uniform (SALU).
__device__ __forceinline__ uint32_t take_lowest(uint64_t &m0, uint64_t &m1) {
    // branch-free (ffsll is defined at 0; m & (m - 1) keeps 0 at 0)
    const bool h0 = m0 != 0, h1 = m1 != 0;
    const uint32_t f0 = (uint32_t)__builtin_ffsll((long long)m0) - 1u;
    const uint32_t f1 = (uint32_t)__builtin_ffsll((long long)m1) - 1u;
    const uint32_t i = h0 ? f0 : (h1 ? 64u + f1 : 0xFFu);
    const uint64_t keep1 = h0 ? ~0ull : m1 - 1;
    m0 &= m0 - 1;
    m1 &= keep1;
    return i;
}

// the path slot words of leaf x for lane j (slot j, and slot 64 + j when P > 64)
struct OramLane {
    uint32_t a0, l0, w0, a1, l1, w1;
};
typedef unsigned int oram_u32x4 __attribute__((ext_vector_type(4)));
// The tree as a buffer resource of its slots: a slot offset at or past the end reads zeros
// and stores nothing, so every lane issues the same loads and stores each access (a
// skipped slot at the out-of-range offset: no memory access) — the compiler's vmcnt waits
// then count them exactly instead of waiting for everything.
constexpr uint32_t kOramOob = 0x7FFFFFF0u;
__device__ __forceinline__ void oram_load_path(__amdgpu_buffer_rsrc_t rs, uint32_t x, uint32_t Lh,
                                               uint32_t lane, bool p0, bool p1, OramLane &r) {
    const oram_u32x4 b0 = __builtin_amdgcn_raw_buffer_load_b128(
        rs, (int)(p0 ? oram_slot(lane, x, Lh) * 16u : kOramOob), 0, 1);
    const oram_u32x4 b1 = __builtin_amdgcn_raw_buffer_load_b128(
        rs, (int)(p1 ? oram_slot(64 + lane, x, Lh) * 16u : kOramOob), 0, 1);
    r.a0 = b0.x, r.l0 = b0.y, r.w0 = b0.z;
    r.a1 = b1.x, r.l1 = b1.y, r.w1 = b1.z;
}
__device__ __forceinline__ void oram_store_slot(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t a,
                                                uint32_t l, uint32_t w) {
    const oram_u32x4 v = {a, l, w, 0u};
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1" ::: "memory");  // dwordx4 store data hazard (k_bitonic.hip)
    __builtin_amdgcn_sched_barrier(0);
}

// The descriptor of access q (public q; the block of a record access is the record's idx):
// REF (oram.rs's sequence): q < d prepare block q; then per record r two accesses (read,
// write of idx_r); then the readout of block q - d - 2 nrec.  LAZY: record q, one RMW.
__device__ __forceinline__ uint2 oram_desc(const uint2 *__restrict__ rec, uint32_t q, uint32_t nrec,
                                           uint32_t d, bool ref, uint32_t mask) {
    if (!ref) {
        const uint2 r = rec[q];
        return make_uint2((r.x & mask) | (kOpRmw << kOpShift), r.y);
    }
    if (q < d) return make_uint2(q | (kOpPrep << kOpShift), 0u);
    const uint32_t u = q - d;
    if (u < 2u * nrec) {
        const uint2 r = rec[u >> 1];
        return make_uint2((r.x & mask) | (((u & 1u) ? kOpWrite : kOpRead) << kOpShift), r.y);
    }
    return make_uint2((u - 2u * nrec) | (kOpFinal << kOpShift), 0u);
}

// Leaf precompute (see the header): keys[q] = block(q) << 32 | q for q < A, ~0 past it.
__global__ void oram_keys_kernel(const uint2 *__restrict__ rec, uint32_t nrec, uint32_t d, uint32_t A,
                                 uint32_t MA, uint32_t mask, int ref, uint64_t *__restrict__ keys) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < MA; q += gridDim.x * 256) {
        uint64_t k = ~0ull;
        if (q < A) {
            const uint32_t a = oram_desc(rec, q, nrec, d, ref != 0, mask).x & kBlockMask;
            k = ((uint64_t)a << 32) | q;
        }
        keys[q] = k;
    }
}

// sorted (block, access) pairs -> (access << 32 | the leaf its block is found under): the
// fresh leaf of the previous access to the block (the pair before it), else the block's
// initial leaf.  Reads positions p - 1 and p: fixed addresses.
__global__ void oram_link_kernel(const uint64_t *__restrict__ sorted, uint32_t A, uint32_t MA,
                                 uint32_t k0, uint32_t k1, uint32_t mask, uint64_t *__restrict__ out) {
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < MA; p += gridDim.x * 256) {
        uint64_t v = ~0ull;
        if (p < A) {
            const uint64_t k = sorted[p], kp = p ? sorted[p - 1] : ~0ull;
            const uint32_t blk = (uint32_t)(k >> 32);
            const bool seen = p > 0 && (uint32_t)(kp >> 32) == blk;
            const uint32_t x = oram_leaf(k0, k1, seen ? (uint32_t)kp : A + blk, mask);
            v = ((uint64_t)(uint32_t)k << 32) | x;
        }
        out[p] = v;
    }
}

// rec: the uploaded records (idx < N checked by the caller's range pass; masked here);
// xs[q]: the leaf access q finds its block under (low word; oram_link + the sort back);
// tree: 4 (2N - 1) slots (all empty on entry) followed by the 20 stash slots (written at
// the end for the lazy readout).  One wave: lane j holds pool entries j and 64 + j (the
// path slots first, then the stash), as (idx, leaf, value) words — plain registers, never
// an indexed array (which would go to scratch).
// Per access, after its own path is in registers: the path of the access TWO ahead has
// its loads issued (its leaf is xs[q + 2]), to land during this access and the next; the
// buckets a path shares with the previous one (the top levels: l <= Lh - bitlen(x ^ x'))
// are taken from that access's output, those it shares with the one before only from
// that one's output (kept in registers), and only the rest are loaded.  Each output lives
// in the same lanes (slot l*Z + z of any path).  A lane only ever stores and reloads its
// own slots, so program order orders them.
// The eviction: every block's rank by (deepest legal level, pool index) from one ballot
// pair per level (mbcnt), the rank each slot receives from the per-level counts (uniform),
// the pool entry holding that rank by matching its 7 bits against one ballot per bit;
// every lane then fetches its new content from that pool entry with ds_bpermute (a
// register crossbar: no LDS bank, so the same time for any pattern).  All lane-parallel
// selects over fixed ballots: no per-slot scalar search (round 4: 1,810 SALU per access
// before, `profiles/r04/oram_sq.txt`).
// zlim (debug, default 4): blocks a bucket may take on eviction (0 forces the stash).
template <bool REF, bool ACC>
__global__ __launch_bounds__(64) void oram_tree_kernel(const uint2 *__restrict__ rec,
                                                       uint32_t nrec, uint32_t d, uint32_t A,
                                                       const uint64_t *__restrict__ xs,
                                                       uint32_t Lh, uint4 *__restrict__ tree,
                                                       uint32_t k0, uint32_t k1, uint32_t zlim,
                                                       float coef, float *__restrict__ out,
                                                       uint32_t *status) {
    __shared__ __attribute__((aligned(16))) uint4 st[kOramStash];  // the stash
    __shared__ uint2 rb[128];     // descriptors of the accesses in flight: a ring of 128
    __shared__ uint32_t lb[128];  // their fresh leaves
    __shared__ uint32_t xb[128];  // and the leaves their blocks are found under
    const uint32_t N = 1u << Lh, mask = N - 1u;
    const uint32_t P = kOramZ * (Lh + 1), POOL = P + kOramStash;
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc((void *)tree, (short)0, (int)(kOramZ * (2u * N - 1u) * 16u), 0x00020000);
    if (lane < kOramStash) st[lane] = make_uint4(kOramEmpty, 0u, 0u, 0u);
    // accesses q0 .. q0 + 63 into their half of the ring (read by broadcast afterwards):
    // the loads are waited for once per 64 accesses, off the access path
    auto batch = [&](uint32_t q0) {
        const uint32_t q = q0 + lane;
        const bool ok = q < A;
        rb[q & 127u] = ok ? oram_desc(rec, q, nrec, d, REF, mask) : make_uint2(0u, 0u);
        lb[q & 127u] = oram_leaf(k0, k1, q, mask);
        xb[q & 127u] = ok ? (uint32_t)xs[q] : 0u;
    };
    batch(0);
    batch(64);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const bool v0 = lane < POOL, v1 = 64 + lane < POOL;
    const bool p0 = lane < P, p1 = 64 + lane < P;  // path slot (else stash entry)
    const uint32_t s0i = lane - P, s1i = 64 + lane - P;  // stash index of a stash entry
    const uint32_t lev0 = lane / kOramZ, lev1 = (64 + lane) / kOramZ;  // their levels
    // the deepest level the paths to leaves u and v share
    auto top = [&](uint32_t u, uint32_t v) { return Lh - (32u - (uint32_t)__clz((int)(u ^ v))); };
    uint32_t over = 0;
    float last = 0.0f;  // REF: the value the read before a write returned (oram.rs:101-103)
    const OramLane none = {kOramEmpty, 0u, 0u, kOramEmpty, 0u, 0u};
    // cur: access q's path; nxt1: the loads of access q+1's path (its buckets not shared
    // with the paths of q or q-1); keep: access q-1's output
    OramLane cur = none, nxt1 = none, keep = none;
    uint32_t x = 0, x1 = 0, xp = 0;  // the leaves of accesses q, q+1, q-1
    if (A) {
        x = xb[0];
        oram_load_path(trs, x, Lh, lane, p0, p1, cur);
        xp = x;  // no access -1: its buckets are never taken (top(xp, x1) = top(x, x1))
        x1 = x;
    }
    if (A > 1) {
        x1 = xb[1];
        const uint32_t t01 = top(x, x1);
        oram_load_path(trs, x1, Lh, lane, p0 && lev0 > t01, p1 && lev1 > t01, nxt1);
    }
    // every load landed before the loop: the loop's own waits then cover only what it
    // issued (the compiler otherwise keeps the first paths "pending" at every iteration)
    __builtin_amdgcn_s_waitcnt(0);
    // one access; nin: the loads of access q+1's path (issued one access earlier), nout:
    // where this access issues access q+2's.  The loop runs two accesses per trip with the
    // two load sets in swapped roles, so no register copy of a load in flight (which would
    // wait for it) is ever made.
    auto access = [&](uint32_t q, OramLane &nin, OramLane &nout) {
        const uint2 r = rb[q & 127u];
        const uint32_t a = r.x & kBlockMask, op = r.x >> kOpShift;
        const float w = __uint_as_float(r.y);
        const uint32_t nleaf = lb[q & 127u];
        if ((q & 63u) == 0 && q) {  // accesses q + 64 .. q + 127 into the half q - 64 .. q - 1 left
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            batch(q + 64);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        // two accesses ahead: access q+2's path loads — only the buckets it shares with
        // neither path q nor path q+1 (which come from those accesses' outputs; which
        // levels is a function of the public leaves).  A load then has a whole access more
        // to land, and never waits behind the stores of the buckets just written.
        const bool more2 = q + 2 < A;
        const uint32_t x2 = more2 ? xb[(q + 2) & 127u] : x1;
        const uint32_t sk2 = max(top(x1, x2), top(x, x2));
        oram_load_path(trs, x2, Lh, lane, more2 && p0 && lev0 > sk2, more2 && p1 && lev1 > sk2, nout);
        // the pool: this path (registers) and the stash (LDS)
        uint32_t a0 = cur.a0, l0 = cur.l0, w0 = cur.w0, a1 = cur.a1, l1 = cur.l1, w1 = cur.w1;
        if (!p0) {
            const uint4 e = v0 ? st[s0i] : make_uint4(kOramEmpty, 0u, 0u, 0u);
            a0 = e.x, l0 = e.y, w0 = e.z;
        }
        if (!p1) {
            const uint4 e = v1 ? st[s1i] : make_uint4(kOramEmpty, 0u, 0u, 0u);
            a1 = e.x, l1 = e.y, w1 = e.z;
        }
        // the block (at most one entry holds it), or +0.0 (never written)
        const bool m0 = a0 == a, m1 = a1 == a;
        // the holder's value by one readlane at the ballot's lowest set bit (uniform), not a
        // 6-step shuffle reduction (each step a crossbar round trip)
        const uint64_t bm0 = __ballot(m0), bm1 = __ballot(m1);
        const bool found = (bm0 | bm1) != 0;
        const uint32_t hl0 = (uint32_t)__builtin_ffsll((long long)bm0) - 1u;
        const uint32_t hl1 = (uint32_t)__builtin_ffsll((long long)bm1) - 1u;
        const uint32_t vb0 = (uint32_t)__builtin_amdgcn_readlane((int)w0, (int)(hl0 & 63u));
        const uint32_t vb1 = (uint32_t)__builtin_amdgcn_readlane((int)w1, (int)(hl1 & 63u));
        const float fv = found ? __uint_as_float(bm0 ? vb0 : vb1) : 0.0f;
        // the value the block keeps (the access kind is public: a function of q)
        float nv = fv;                                  // read / readout
        if (op == kOpPrep) nv = 0.0f;                   // prepare(): write 0.0
        if (op == kOpRead) last = fv;                   // oram.read(idx)
        if (op == kOpWrite) nv = __fadd_rn(last, w);    // oram.write(idx, read + val)
        if (op == kOpRmw) nv = __fadd_rn(fv, w);        // LAZY: one access per record
        if (REF && op == kOpFinal && lane == 0)         // global_params[i] = oram.read(i)
            out[a] = ACC ? __fadd_rn(out[a], fv) : __fmul_rn(fv, coef);
        a0 = m0 ? kOramEmpty : a0;
        a1 = m1 ? kOramEmpty : a1;
        // write: the block with its new leaf into the first free entry
        uint64_t f0 = __ballot(v0 && a0 == kOramEmpty), f1 = __ballot(v1 && a1 == kOramEmpty);
        const uint32_t fi = take_lowest(f0, f1);
        over |= fi == 0xFFu;
        const bool i0 = fi == lane, i1 = fi == 64u + lane;
        a0 = i0 ? a : a0, l0 = i0 ? nleaf : l0, w0 = i0 ? __float_as_uint(nv) : w0;
        a1 = i1 ? a : a1, l1 = i1 ? nleaf : l1, w1 = i1 ? __float_as_uint(nv) : w1;
        // eviction: the deepest level each block may take on this path (lm), zlim (4) per
        // bucket, deepest first.  The blocks ranked by (lm descending, pool index): level
        // l then takes the next min(4, #(lm >= l) - placed) ranks, the stash the rest —
        // the greedy's count at every level, whichever blocks it picks, so the same
        // stash size as any deepest-first eviction.
        const bool o0 = v0 && a0 != kOramEmpty, o1 = v1 && a1 != kOramEmpty;
        const uint32_t lm0 = Lh - (32u - (uint32_t)__clz((int)(l0 ^ x)));
        const uint32_t lm1 = Lh - (32u - (uint32_t)__clz((int)(l1 ^ x)));
        uint32_t rank0 = 0, rank1 = 0;  // this lane's blocks' ranks
        uint32_t rw0, rw1;              // the rank this lane's slots receive
        bool fill0, fill1;
        uint32_t tfirst = 0, tcount = 0;  // lane l: level l's first rank and count
        uint32_t before = 0, placed = 0;  // blocks with lm > l; ranks handed out so far
        for (int l = (int)Lh; l >= 0; --l) {
            const bool e0 = o0 && lm0 == (uint32_t)l, e1 = o1 && lm1 == (uint32_t)l;
            const uint64_t mv0 = __ballot(e0), mv1 = __ballot(e1);
            const uint32_t c0 = (uint32_t)__popcll(mv0);
            const uint32_t below0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(mv0 >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mv0, 0u));
            const uint32_t below1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(mv1 >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mv1, 0u));
            rank0 = e0 ? before + below0 : rank0;
            rank1 = e1 ? before + c0 + below1 : rank1;
            before += c0 + (uint32_t)__popcll(mv1);
            const uint32_t pl = min(zlim, before - placed);
            // level l's first rank and count, kept in lane l
            tfirst = lane == (uint32_t)l ? placed : tfirst;
            tcount = lane == (uint32_t)l ? pl : tcount;
            placed += pl;
        }
        // slot l*Z + z (lane-static l, z) takes rank first(l) + z when z < count(l): the
        // level's pair fetched from lane l (a lane-static crossbar read)
        {
            const uint32_t f0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lev0 & 63u) * 4u), (int)tfirst);
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lev0 & 63u) * 4u), (int)tcount);
            const uint32_t f1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lev1 & 63u) * 4u), (int)tfirst);
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lev1 & 63u) * 4u), (int)tcount);
            rw0 = f0 + (lane & 3u);
            rw1 = f1 + (lane & 3u);
            fill0 = p0 && (lane & 3u) < n0;
            fill1 = p1 && (lane & 3u) < n1;
        }
        // the rest to the stash, by rank
        const uint32_t nst = before - placed;
        over |= nst > kOramStash;
        rw0 = (!p0 && v0) ? placed + s0i : rw0;
        rw1 = (!p1 && v1) ? placed + s1i : rw1;
        fill0 = (!p0 && v0) ? s0i < nst : fill0;
        fill1 = (!p1 && v1) ? s1i < nst : fill1;
        // src0 / src1: the pool entry holding the wanted rank (0xFF = empty slot), by
        // matching the rank's bits against one ballot per bit (uniform masks, selects)
        uint64_t m00 = __ballot(o0), m01 = __ballot(o1);
        uint64_t m10 = m00, m11 = m01;
#pragma unroll
        for (uint32_t b = 0; b < 7; ++b) {
            const uint64_t B0 = __ballot(o0 && ((rank0 >> b) & 1u)), B1 = __ballot(o1 && ((rank1 >> b) & 1u));
            const bool q0 = (rw0 >> b) & 1u, q1 = (rw1 >> b) & 1u;
            m00 &= q0 ? B0 : ~B0;
            m01 &= q0 ? B1 : ~B1;
            m10 &= q1 ? B0 : ~B0;
            m11 &= q1 ? B1 : ~B1;
        }
        const uint32_t src0 = !fill0 ? 0xFFu
                                     : (m00 ? (uint32_t)__builtin_ffsll((long long)m00) - 1u
                                            : 63u + (uint32_t)__builtin_ffsll((long long)m01));
        const uint32_t src1 = !fill1 ? 0xFFu
                                     : (m10 ? (uint32_t)__builtin_ffsll((long long)m10) - 1u
                                            : 63u + (uint32_t)__builtin_ffsll((long long)m11));
        // gather through the register crossbar: from set 0 or set 1 of lane src & 63
        const int ad0 = (int)((src0 & 63u) * 4u), ad1 = (int)((src1 & 63u) * 4u);
        const bool h0 = src0 != 0xFFu, h1 = src1 != 0xFFu, hi0 = src0 >= 64u, hi1 = src1 >= 64u;
        const uint32_t ga0x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)a0),
                       ga0y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)a1);
        const uint32_t gl0x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)l0),
                       gl0y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)l1);
        const uint32_t gw0x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)w0),
                       gw0y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad0, (int)w1);
        const uint32_t ga1x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)a0),
                       ga1y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)a1);
        const uint32_t gl1x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)l0),
                       gl1y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)l1);
        const uint32_t gw1x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)w0),
                       gw1y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad1, (int)w1);
        const uint32_t ga0 = !h0 ? kOramEmpty : (hi0 ? ga0y : ga0x), gl0 = hi0 ? gl0y : gl0x,
                       gw0 = hi0 ? gw0y : gw0x;
        const uint32_t ga1 = !h1 ? kOramEmpty : (hi1 ? ga1y : ga1x), gl1 = hi1 ? gl1y : gl1x,
                       gw1 = hi1 ? gw1y : gw1x;
        // access q+1's path: the buckets it shares with path q from this output, those it
        // shares with path q-1 only from that access's output, the rest from the loads
        // (merged before this access's stores are issued: the wait for the loads then does
        // not also wait for these stores — CDNA counts both in vmcnt, in order)
        const uint32_t t01 = top(x, x1), tp1 = top(xp, x1);
        const bool sh0 = lev0 <= t01, sh1 = lev1 <= t01, kp0 = lev0 <= tp1, kp1 = lev1 <= tp1;
        OramLane nc;
        nc.a0 = sh0 ? ga0 : (kp0 ? keep.a0 : nin.a0);
        nc.l0 = sh0 ? gl0 : (kp0 ? keep.l0 : nin.l0);
        nc.w0 = sh0 ? gw0 : (kp0 ? keep.w0 : nin.w0);
        nc.a1 = sh1 ? ga1 : (kp1 ? keep.a1 : nin.a1);
        nc.l1 = sh1 ? gl1 : (kp1 ? keep.l1 : nin.l1);
        nc.w1 = sh1 ? gw1 : (kp1 ? keep.w1 : nin.w1);
        // pin the merge here (the compiler would sink it past the stores, and its wait for
        // the loads would then wait for them too)
        asm volatile("" : "+v"(nc.a0), "+v"(nc.l0), "+v"(nc.w0), "+v"(nc.a1), "+v"(nc.l1), "+v"(nc.w1)
                     :
                     : "memory");
        // write the path back (the whole path, fixed addresses) and the stash
        oram_store_slot(trs, p0 ? oram_slot(lane, x, Lh) * 16u : kOramOob, ga0, gl0, gw0);
        oram_store_slot(trs, p1 ? oram_slot(64 + lane, x, Lh) * 16u : kOramOob, ga1, gl1, gw1);
        if (!p0 && v0) st[s0i] = make_uint4(ga0, gl0, gw0, 0u);
        if (!p1 && v1) st[s1i] = make_uint4(ga1, gl1, gw1, 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        keep = {ga0, gl0, gw0, ga1, gl1, gw1};
        cur = nc;
        xp = x;
        x = x1;
        x1 = x2;
    };
    OramLane nxt2 = none;
    for (uint32_t q = 0; q < A; q += 2) {
        access(q, nxt1, nxt2);
        if (q + 1 < A) access(q + 1, nxt2, nxt1);
    }
    // the stash, after the tree, for the lazy readout
    if (lane < kOramStash) tree[(size_t)kOramZ * (2u * N - 1u) + lane] = st[lane];
    if (__ballot(over != 0) && lane == 0) atomicOr(status, FLTEE_DEV_ERR_ORAM_STASH);
}

__global__ void oram_fill_kernel(uint4 *__restrict__ tree, size_t ns) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < ns; i += (size_t)gridDim.x * 256)
        tree[i] = make_uint4(kOramEmpty, 0u, 0u, 0u);
}

// tree + stash slots -> 8-B records (idx, value); an empty slot j gets idx N + j (unique,
// never < d): every index appears at most once
__global__ void oram_records_kernel(const uint4 *__restrict__ tree, size_t ns, uint32_t N,
                                    uint2 *__restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < ns; i += (size_t)gridDim.x * 256) {
        const uint4 s = tree[i];
        out[i] = make_uint2(s.x == kOramEmpty ? N + (uint32_t)i : s.x, s.z);
    }
}

static uint32_t g_oram_zlim = kOramZ;  // fltee_debug_set_oram_bucket (tests: force the stash)
void set_oram_bucket(int z) { g_oram_zlim = z < 0 ? 0u : (z > (int)kOramZ ? kOramZ : (uint32_t)z); }

size_t oram_slots(size_t d) {
    const size_t N = next_pow2_sz(d ? d : 1);
    return kOramZ * (2 * N - 1) + kOramStash;
}

bool oram_supported(size_t d) { return next_pow2_sz(d ? d : 1) <= ((size_t)1 << kOramMaxLog); }

size_t oram_accesses(size_t nrec, size_t d, bool lazy) { return lazy ? nrec : 2 * nrec + 2 * d; }

// the tree runs this shape: its block count, and the leaf precompute's (and the lazy
// readout's) sorts within the networks' 2^29-entry bound (k_bitonic.hip)
bool oram_fits(size_t nrec, size_t d, bool lazy) {
    constexpr size_t kMaxNet = (size_t)1 << 29;
    if (!oram_supported(d) || oram_accesses(nrec, d, lazy) >= 0x7F000000ull) return false;
    if (next_pow2_sz(oram_accesses(nrec, d, lazy)) > kMaxNet) return false;
    return !lazy || next_pow2_sz(oram_slots(d) + d) <= kMaxNet;
}

hipError_t launch_oram_tree(const void *rec, size_t nrec, size_t d, bool lazy, void *tree,
                            uint64_t seed, uint64_t *keys, uint64_t *keys2, uint64_t *records,
                            float coef, bool accumulate, float *out, uint32_t *status,
                            hipStream_t s) {
    const size_t A = oram_accesses(nrec, d, lazy);
    if (!oram_supported(d) || A >= 0x7FFFFFFFull - ((size_t)1 << kOramMaxLog)) return hipErrorInvalidValue;
    const size_t N = next_pow2_sz(d ? d : 1);
    const uint32_t Lh = log2_pow2(N), mask = (uint32_t)N - 1u;
    const size_t ns = oram_slots(d);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    size_t blocks = (ns + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    FLTEE_LAUNCH(oram_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint4 *)tree, ns);
    if (A == 0) {
        if (lazy)
            FLTEE_LAUNCH(oram_records_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                               (const uint4 *)tree, ns, (uint32_t)N, (uint2 *)records);
        return hipGetLastError();
    }
    // the leaves: keys sorted by (block, access), linked, sorted back by access
    const size_t MA = next_pow2_sz(A);
    size_t kb = (MA + 255) / 256;
    if (kb > 65536) kb = 65536;
    FLTEE_LAUNCH(oram_keys_kernel, dim3((unsigned)kb), dim3(256), 0, s, (const uint2 *)rec,
                       (uint32_t)nrec, (uint32_t)d, (uint32_t)A, (uint32_t)MA, mask, lazy ? 0 : 1, keys);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = bitonic_sort(keys, MA, 1, 0, s, A);
    if (e != hipSuccess) return e;
    FLTEE_LAUNCH(oram_link_kernel, dim3((unsigned)kb), dim3(256), 0, s, keys, (uint32_t)A,
                       (uint32_t)MA, k0, k1, mask, keys2);
    e = hipGetLastError();
    if (e == hipSuccess) e = bitonic_sort(keys2, MA, 1, 0, s, A);
    if (e != hipSuccess) return e;
#define OT_GO(REF_, ACC_)                                                                          \
    FLTEE_LAUNCH((oram_tree_kernel<REF_, ACC_>), dim3(1), dim3(64), 0, s, (const uint2 *)rec, \
                       (uint32_t)nrec, (uint32_t)d, (uint32_t)A, (const uint64_t *)keys2, Lh,       \
                       (uint4 *)tree, k0, k1, g_oram_zlim, coef, out, status)
    if (lazy) OT_GO(false, false);
    else if (accumulate) OT_GO(true, true);
    else OT_GO(true, false);
#undef OT_GO
    if (lazy)
        FLTEE_LAUNCH(oram_records_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                           (const uint4 *)tree, ns, (uint32_t)N, (uint2 *)records);
    return hipGetLastError();
}

}  // namespace fltee
