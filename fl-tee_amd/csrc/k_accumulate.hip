// k_accumulate.hip — element-wise accumulate across clients (gfx950).
//
// Reference semantics (non_oblivious.rs:6-15, baseline.rs:7-60, oram.rs:86-118):
// out[idx] += val for every record in upload order (client order, then each
// client's own order), starting from +0.0 (the SGX bridge zero-fills [out],
// Enclave_t.c:626), then out *= 1f32/n (common.rs:14-19).  All kernels here
// keep that exact per-index order, so results are bit-identical.
//
// dense_accumulate : records are dense (client c, slot j has idx j — the
//   serialize_dense layout, utils.py:171-190).  One thread owns 2*V adjacent
//   outputs, walks the n clients in order with 16-B non-temporal loads, U
//   clients in flight.  HBM-read bound: n*d*8 + d*4 bytes per launch.  The
//   access pattern does not depend on the data (every record is read once at
//   a fixed address), so it is oblivious; idx != position is reported, not
//   followed (FLTEE_DEV_ERR_DENSE_ORDER).
// sweep_ordered : sparse records, oblivious and exact for ANY upload.  GPU form of
//   baseline.rs's o_update (and oram.rs's output): lane j owns out[j] and walks every
//   record in upload order, adding the record's value where its idx is j and +0.0
//   elsewhere (a select, no branch; +0.0 is the identity of a sum that started at +0.0).
//   The same per-index order as the enclave whatever the data — a client may repeat an
//   index — so no status word, no rerun: the cost is n*k*d compare-selects, fixed by the
//   public sizes.
#include <atomic>

#include "common.h"

namespace fltee {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// streaming (non-temporal) loads: every byte is read exactly once
static __device__ __forceinline__ uint4 ld_nt(const uint4 *p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
static __device__ __forceinline__ uint2 ld_nt(const uint2 *p) {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t *>(p));
    return make_uint2(v.x, v.y);
}
static __device__ __forceinline__ float4 ld_nt(const float4 *p) {
    const f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------------- dense ----
// rec viewed as uint4 = two records {idx0, val0, idx1, val1}; row stride d2 = d/2.
// A block covers V*NTH consecutive uint4 columns; lane t owns columns
// base + t + v*NTH (v < V), so every load instruction of a wave is 1 KB contiguous.
template <typename T4>
static __device__ __forceinline__ uint4 ld4(const uint4 *p, bool nt) {
    return nt ? ld_nt(p) : *p;
}

// Small d (MLP-MNIST: d/2 = 25,445 output pairs = 398 waves, under one wave per SIMD):
// one lane per output pair with a whole batch of U clients' 16-B loads in flight at once —
// the wave may take the whole register file (one wave per SIMD: up to 512 VGPRs + AGPRs),
// so one HBM latency covers the batch instead of one per 16 clients.  Full batches, then
// one clamped batch for the rest (clients past n re-read the last row; their adds are
// selected away, branch-free: a branch per client kept 100 conditions live in spilled
// SGPRs; REM = false when U divides n).  The same adds in the same order as
// dense_accumulate_v: bit-identical.  A/B (MI355X, 50,890 params, cold inputs,
// `profiles/r03/ab/ab17_dense_small_d.jsonl`): n = 100 9.2-9.5 us against 10.4-10.6 us for
// the LDS-staged kernel below; n = 64 8.8 vs 9.1; n <= 32 and n > 100 no faster (those keep
// the LDS kernel).
template <int U, bool CLIP, bool ACC, bool NTL = true>
__device__ __forceinline__ void dw_batch(const uint4 *__restrict__ p, size_t d2, uint32_t n, uint32_t c,
                                         bool clamp, uint32_t jx, const float *__restrict__ ccoef,
                                         float &a0, float &a1, uint32_t &bad) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t cc = (clamp && c + (uint32_t)u >= n) ? n - 1 : c + (uint32_t)u;
        x[u] = NTL ? ld_nt(p + (size_t)cc * d2) : p[(size_t)cc * d2];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool take = !clamp || c + (uint32_t)u < n;
        float a = __uint_as_float(x[u].y), b = __uint_as_float(x[u].w);
        if (CLIP) {
            const float cf = ccoef[take ? c + u : n - 1];
            a = __fmul_rn(a, cf);
            b = __fmul_rn(b, cf);
        }
        const float s0 = __fadd_rn(a0, a), s1 = __fadd_rn(a1, b);
        a0 = take ? s0 : a0;
        a1 = take ? s1 : a1;
        bad |= take ? (x[u].x ^ jx) | (x[u].z ^ (jx + 1)) : 0u;
    }
}

// per (< 64: the balanced-grid A/B, variants 50-52): output pairs per wave, so that the
// waves spread evenly over the CUs (MLP-MNIST: 398 full waves leave 142 CUs with two and
// 114 with one)
template <int U, bool REM, bool CLIP, bool ACC, bool NTL = true>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void dense_accumulate_w(
    const uint4 *__restrict__ rec, size_t d2, uint32_t n, float coef, float *__restrict__ out,
    const float *__restrict__ ccoef, uint32_t *status, uint32_t per = 64) {
    const size_t j = (size_t)blockIdx.x * per + threadIdx.x;
    if (threadIdx.x >= per || j >= d2) return;
    const uint4 *p = rec + j;
    const uint32_t jx = (uint32_t)(2 * j);
    float a0 = 0.0f, a1 = 0.0f;
    uint32_t bad = 0, c = 0;
    for (; c + U <= n; c += U) dw_batch<U, CLIP, ACC, NTL>(p, d2, n, c, false, jx, ccoef, a0, a1, bad);
    if (REM && c < n) dw_batch<U, CLIP, ACC, NTL>(p, d2, n, c, true, jx, ccoef, a0, a1, bad);
    float2 *o = reinterpret_cast<float2 *>(out) + j;
    float2 r;
    if (ACC) {
        const float2 prev = *o;
        r = make_float2(__fadd_rn(prev.x, a0), __fadd_rn(prev.y, a1));
    } else {
        r = make_float2(__fmul_rn(a0, coef), __fmul_rn(a1, coef));
    }
    *o = r;
    if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

// One lane per output index (8-B loads): twice the waves of dense_accumulate_w (796 at
// MLP-MNIST), 2 VGPRs per client in flight, so two waves fit a SIMD.  Same adds, same
// order: bit-identical.  A/B variant 47.
template <int U, bool ACC>
__global__ __launch_bounds__(64) void dense_accumulate_w1(const uint2 *__restrict__ rec, size_t d,
                                                          uint32_t n, float coef,
                                                          float *__restrict__ out, uint32_t *status) {
    const size_t j = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (j >= d) return;
    const uint2 *p = rec + j;
    const uint32_t jx = (uint32_t)j;
    float a = 0.0f;
    uint32_t bad = 0;
    for (uint32_t c = 0; c < n; c += U) {
        uint2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t cc = c + (uint32_t)u < n ? c + (uint32_t)u : n - 1;
            x[u] = ld_nt(p + (size_t)cc * d);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool take = c + (uint32_t)u < n;
            const float s = __fadd_rn(a, __uint_as_float(x[u].y));
            a = take ? s : a;
            bad |= take ? (x[u].x ^ jx) : 0u;
        }
    }
    out[j] = ACC ? __fadd_rn(out[j], a) : __fmul_rn(a, coef);
    if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

// The same output pairs with the clients split over W waves of one block (wave w: clients
// [w*UC, (w+1)*UC)): every wave issues its UC rows' loads at once, so W times the waves
// (and SIMDs) pull the batch; the in-order sum then passes from wave to wave through LDS —
// wave w adds its clients to wave w-1's partial sums, after a block barrier — the same adds
// in the same order as dense_accumulate_w: bit-identical.  n <= W * UC (clients past n are
// clamped and selected away as in dw_batch).
template <int W, int UC, bool ACC>
__global__ __launch_bounds__(64 * W) void dense_accumulate_wk(const uint4 *__restrict__ rec,
                                                            size_t d2, uint32_t n, float coef,
                                                            float *__restrict__ out,
                                                            uint32_t *status) {
    __shared__ float2 part[W][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t j = (size_t)blockIdx.x * 64 + lane;
    const bool live = j < d2;
    const uint4 *p = rec + (live ? j : 0);
    const uint32_t jx = (uint32_t)(2 * j), c0 = w * (uint32_t)UC;
    uint4 x[UC];
#pragma unroll
    for (int u = 0; u < UC; ++u) {
        const uint32_t cc = c0 + (uint32_t)u < n ? c0 + (uint32_t)u : n - 1;
        x[u] = ld_nt(p + (size_t)cc * d2);
    }
    float a0 = 0.0f, a1 = 0.0f;
    uint32_t bad = 0;
    for (uint32_t s = 0; s < (uint32_t)W; ++s) {
        if (s) __syncthreads();
        if (s == w) {
            if (s) {
                const float2 pr = part[s - 1][lane];
                a0 = pr.x;
                a1 = pr.y;
            }
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const bool take = c0 + (uint32_t)u < n;
                const float s0 = __fadd_rn(a0, __uint_as_float(x[u].y));
                const float s1 = __fadd_rn(a1, __uint_as_float(x[u].w));
                a0 = take ? s0 : a0;
                a1 = take ? s1 : a1;
                bad |= take ? (x[u].x ^ jx) | (x[u].z ^ (jx + 1)) : 0u;
            }
            part[s][lane] = make_float2(a0, a1);
        }
    }
    if (w == W - 1 && live) {
        float2 *o = reinterpret_cast<float2 *>(out) + j;
        float2 r;
        if (ACC) {
            const float2 prev = *o;
            r = make_float2(__fadd_rn(prev.x, a0), __fadd_rn(prev.y, a1));
        } else {
            r = make_float2(__fmul_rn(a0, coef), __fmul_rn(a1, coef));
        }
        *o = r;
    }
    if (live && bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

template <int V, int U, bool CLIP, bool ACC, bool NT, int NTH = 256>
__global__ __launch_bounds__(NTH) void dense_accumulate_v(const uint4 *__restrict__ rec, size_t d2,
                                                          uint32_t n, float coef,
                                                          float *__restrict__ out,
                                                          const float *__restrict__ ccoef,
                                                          uint32_t *status) {
    const size_t base = (size_t)blockIdx.x * (NTH * V) + threadIdx.x;
    float acc[2 * V];
    bool live[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        acc[2 * v] = acc[2 * v + 1] = 0.0f;
        live[v] = base + (size_t)v * NTH < d2;
    }
    if (!live[0]) return;
    uint32_t bad = 0;
    const uint4 *p = rec + base;
    uint32_t c = 0;
    const bool full = live[V - 1];
    if (full) {
        for (; c + U <= n; c += U) {
            uint4 x[U][V];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int v = 0; v < V; ++v) x[u][v] = ld4<uint4>(p + (size_t)(c + u) * d2 + v * NTH, NT);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float cc = CLIP ? ccoef[c + u] : 1.0f;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float a = __uint_as_float(x[u][v].y), b = __uint_as_float(x[u][v].w);
                    if (CLIP) { a = __fmul_rn(a, cc); b = __fmul_rn(b, cc); }
                    acc[2 * v] = __fadd_rn(acc[2 * v], a);
                    acc[2 * v + 1] = __fadd_rn(acc[2 * v + 1], b);
                    const uint32_t j = (uint32_t)(2 * (base + (size_t)v * NTH));
                    bad |= (x[u][v].x ^ j) | (x[u][v].z ^ (j + 1));
                }
            }
        }
    }
    for (; c < n; ++c) {
        const float cc = CLIP ? ccoef[c] : 1.0f;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            if (!live[v]) continue;
            const uint4 x = ld4<uint4>(p + (size_t)c * d2 + v * NTH, NT);
            float a = __uint_as_float(x.y), b = __uint_as_float(x.w);
            if (CLIP) { a = __fmul_rn(a, cc); b = __fmul_rn(b, cc); }
            acc[2 * v] = __fadd_rn(acc[2 * v], a);
            acc[2 * v + 1] = __fadd_rn(acc[2 * v + 1], b);
            const uint32_t j = (uint32_t)(2 * (base + (size_t)v * NTH));
            bad |= (x.x ^ j) | (x.z ^ (j + 1));
        }
    }
    float2 *o = reinterpret_cast<float2 *>(out) + base;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        if (!live[v]) continue;
        float2 r;
        if (ACC) {
            const float2 prev = o[v * NTH];
            r = make_float2(__fadd_rn(prev.x, acc[2 * v]), __fadd_rn(prev.y, acc[2 * v + 1]));
        } else {
            r = make_float2(__fmul_rn(acc[2 * v], coef), __fmul_rn(acc[2 * v + 1], coef));
        }
        o[v * NTH] = r;
    }
    if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

// odd d or misaligned base: one record (8 B) per lane per client.
template <bool CLIP, bool ACC>
__global__ __launch_bounds__(256) void dense_accumulate_s(const uint2 *__restrict__ rec, size_t d,
                                                          uint32_t n, float coef,
                                                          float *__restrict__ out,
                                                          const float *__restrict__ ccoef,
                                                          uint32_t *status) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= d) return;
    float acc = 0.0f;
    uint32_t bad = 0;
    for (uint32_t c = 0; c < n; ++c) {
        uint2 x = ld_nt(rec + (size_t)c * d + j);
        float a = __uint_as_float(x.y);
        if (CLIP) a = __fmul_rn(a, ccoef[c]);
        acc = __fadd_rn(acc, a);
        bad |= x.x ^ (uint32_t)j;
    }
    out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
    if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

// one record (8 B) per lane and client, U clients in flight (A/B variant)
template <int U, bool CLIP, bool ACC>
__global__ __launch_bounds__(256) void dense_accumulate_r(const uint2 *__restrict__ rec, size_t d,
                                                          uint32_t n, float coef,
                                                          float *__restrict__ out,
                                                          const float *__restrict__ ccoef,
                                                          uint32_t *status) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= d) return;
    const uint2 *p = rec + j;
    float acc = 0.0f;
    uint32_t bad = 0, c = 0;
    for (; c + U <= n; c += U) {
        uint2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld_nt(p + (size_t)(c + u) * d);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float a = __uint_as_float(x[u].y);
            if (CLIP) a = __fmul_rn(a, ccoef[c + u]);
            acc = __fadd_rn(acc, a);
            bad |= x[u].x ^ (uint32_t)j;
        }
    }
    for (; c < n; ++c) {
        const uint2 x = ld_nt(p + (size_t)c * d);
        float a = __uint_as_float(x.y);
        if (CLIP) a = __fmul_rn(a, ccoef[c]);
        acc = __fadd_rn(acc, a);
        bad |= x.x ^ (uint32_t)j;
    }
    out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
    if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
}

// Small d (MLP-MNIST, d = 50,890): one lane per output pair leaves most CUs idle and
// each lane's U-client batches run back to back (latency-bound, 19 us for 100 clients).
// Here a block of 256 lanes owns DS_OB outputs and stages DS_CC clients of them at a
// time through LDS: every lane issues its share of the chunk's loads at once (next chunk
// in flight while the current one is summed), then lanes < DS_OB sum their output over
// the chunk's clients in client order from LDS.  Same adds in the same order as
// dense_accumulate_v: bit-identical.
constexpr int DS_NT = 256;

template <bool VEC, bool CLIP, bool ACC, int DS_OB = 128, int DS_CC = 32>
__global__ __launch_bounds__(DS_NT) void dense_accumulate_lds(const uint2 *__restrict__ rec, size_t d,
                                                              uint32_t n, float coef,
                                                              float *__restrict__ out,
                                                              const float *__restrict__ ccoef,
                                                              uint32_t *status) {
    constexpr int DS_LD = DS_OB * DS_CC / 2 / DS_NT;  // 16-B loads per lane per chunk
    static_assert(DS_LD >= 1 && DS_LD * 2 * DS_NT == DS_OB * DS_CC && DS_OB <= DS_NT, "shape");
    __shared__ uint4 buf[2][DS_CC][DS_OB / 2];  // record pairs (conflict-free 16-B writes)
    const uint32_t t = threadIdx.x;
    const size_t j0 = (size_t)blockIdx.x * DS_OB;
    const uint32_t nch = (n + DS_CC - 1) / DS_CC;
    // lane t, load i: client cl = q / (DS_OB/2), pair pr = q % (DS_OB/2), q = t + i*DS_NT
    uint4 r[DS_LD];
    auto load = [&](uint32_t ch) {
#pragma unroll
        for (int i = 0; i < DS_LD; ++i) {
            const uint32_t q = t + (uint32_t)i * DS_NT;
            const uint32_t cl = q / (DS_OB / 2), pr = q % (DS_OB / 2);
            const uint32_t c = ch * DS_CC + cl;
            const size_t j = j0 + 2 * pr;
            uint4 x = make_uint4(0u, 0u, 0u, 0u);
            if (c < n) {
                const uint2 *p = rec + (size_t)c * d + j;
                if (VEC) {
                    if (j < d) x = ld_nt(reinterpret_cast<const uint4 *>(p));  // d even: j+1 < d too
                } else {
                    if (j < d) { const uint2 a = ld_nt(p); x.x = a.x; x.y = a.y; }
                    if (j + 1 < d) { const uint2 b = ld_nt(p + 1); x.z = b.x; x.w = b.y; }
                }
            }
            r[i] = x;
        }
    };
    auto stash = [&](int b) {
#pragma unroll
        for (int i = 0; i < DS_LD; ++i) {
            const uint32_t q = t + (uint32_t)i * DS_NT;
            const uint32_t cl = q / (DS_OB / 2), pr = q % (DS_OB / 2);
            buf[b][cl][pr] = r[i];
        }
    };
    float acc = 0.0f;
    uint32_t bad = 0;
    const size_t j = j0 + t;
    load(0);
    stash(0);
    __syncthreads();
    for (uint32_t ch = 0; ch < nch; ++ch) {
        if (ch + 1 < nch) load(ch + 1);
        if (t < DS_OB && j < d) {
            const uint32_t cend = n - ch * DS_CC < DS_CC ? n - ch * DS_CC : DS_CC;
            for (uint32_t cl = 0; cl < cend; ++cl) {
                const uint2 x = reinterpret_cast<const uint2 *>(buf[ch & 1][cl])[t];
                float a = __uint_as_float(x.y);
                if (CLIP) a = __fmul_rn(a, ccoef[ch * DS_CC + cl]);
                acc = __fadd_rn(acc, a);
                bad |= x.x ^ (uint32_t)j;
            }
        }
        if (ch + 1 < nch) stash((ch + 1) & 1);
        __syncthreads();
    }
    if (t < DS_OB && j < d) {
        out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
        if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
    }
}

// Small d, LDS-DMA ring: a 256-lane block owns 64 outputs; chunks of 16 clients (8 KB)
// land in a 4-slot LDS ring straight from HBM (global_load_lds, 16 B per lane: one wave
// instruction fills two clients' 512-B rows), so 4 chunks are in flight per block and a
// CU holds 4-5 blocks — about 128 KB of loads in flight per CU, where the register-staged
// kernel above has one 32 KB chunk per block.  Wave 0 sums each chunk's clients in client
// order (lane = output), exactly the adds of dense_accumulate_v: bit-identical.  Waits
// are counted per wave (each wave's own LDS-DMA, vmcnt) and the block syncs with raw
// s_barrier: __syncthreads() would drain every load in flight (vmcnt(0)).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Four separately named ring slots with the slot of every access known at compile time
// (the chunk loop unrolled by 4): hipcc's wait insertion then sees that a slot's reads
// cannot alias the LDS-DMA still in flight into the other three, and waits only for the
// counted vmcnt above instead of draining every load (vmcnt(0)) before the first read.
constexpr int DG_OB = 64, DG_CC = 16;
__shared__ __attribute__((aligned(16))) uint2 dg_ring0[DG_CC][DG_OB];
__shared__ __attribute__((aligned(16))) uint2 dg_ring1[DG_CC][DG_OB];
__shared__ __attribute__((aligned(16))) uint2 dg_ring2[DG_CC][DG_OB];
__shared__ __attribute__((aligned(16))) uint2 dg_ring3[DG_CC][DG_OB];
template <int S>
__device__ __forceinline__ uint2 (&dg_slot())[DG_CC][DG_OB] {
    if constexpr (S == 0) return dg_ring0;
    else if constexpr (S == 1) return dg_ring1;
    else if constexpr (S == 2) return dg_ring2;
    else return dg_ring3;
}

template <int S>
__device__ __forceinline__ void dg_issue(const uint2 *__restrict__ rec, size_t d, uint32_t n,
                                         uint32_t ch, uint32_t w, uint32_t l, size_t jl) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t row = 2 * (w + 4 * (uint32_t)i);
        uint32_t c = ch * DG_CC + row + (l >> 5);
        if (c >= n) c = n - 1;  // clamped, never summed
        __builtin_amdgcn_global_load_lds((const void *)(rec + (size_t)c * d + jl),
                                         (void __attribute__((address_space(3))) *)&dg_slot<S>()[row][0],
                                         16, 0, 0);
    }
}

// one chunk: wait for this wave's loads of it, sum it (wave 0), free the slot, refill it
template <int S, bool CLIP>
__device__ __forceinline__ void dg_step(const uint2 *__restrict__ rec, size_t d, uint32_t n,
                                        uint32_t nch, uint32_t ch, uint32_t w, uint32_t l,
                                        size_t jl, size_t j, const float *__restrict__ ccoef,
                                        float &acc, uint32_t &bad) {
    const uint32_t ahead = nch - ch - 1 < 3u ? nch - ch - 1 : 3u;  // later chunks in flight
    if (ahead >= 3) wait_vmcnt<6>();
    else if (ahead == 2) wait_vmcnt<4>();
    else if (ahead == 1) wait_vmcnt<2>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (w == 0 && j < d) {
        const uint32_t cend = n - ch * DG_CC < (uint32_t)DG_CC ? n - ch * DG_CC : (uint32_t)DG_CC;
        for (uint32_t cl = 0; cl < cend; ++cl) {
            const uint2 x = dg_slot<S>()[cl][l];
            float a = __uint_as_float(x.y);
            if (CLIP) a = __fmul_rn(a, ccoef[ch * DG_CC + cl]);
            acc = __fadd_rn(acc, a);
            bad |= x.x ^ (uint32_t)j;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): wave 0's reads of the slot retired
    __builtin_amdgcn_s_barrier();
    if (ch + 4 < nch) dg_issue<S>(rec, d, n, ch + 4, w, l, jl);
}

template <bool CLIP, bool ACC>
__global__ __launch_bounds__(256) void dense_accumulate_glds(const uint2 *__restrict__ rec, size_t d,
                                                             uint32_t n, float coef,
                                                             float *__restrict__ out,
                                                             const float *__restrict__ ccoef,
                                                             uint32_t *status) {
    const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
    const size_t j0 = (size_t)blockIdx.x * DG_OB;
    const uint32_t nch = (n + DG_CC - 1) / DG_CC;
    // lane l of wave w, instruction i: client 2*(w + 4i) + (l >> 5) of the chunk, record
    // pair l & 31 (one wave instruction = two clients' 512-B rows, lane-linear in LDS)
    size_t jl = j0 + 2 * (l & 31);
    if (jl + 2 > d) jl = d - 2;  // d even (launcher); past d: clamped, never stored
    dg_issue<0>(rec, d, n, 0, w, l, jl);
    if (nch > 1) dg_issue<1>(rec, d, n, 1, w, l, jl);
    if (nch > 2) dg_issue<2>(rec, d, n, 2, w, l, jl);
    if (nch > 3) dg_issue<3>(rec, d, n, 3, w, l, jl);
    float acc = 0.0f;
    uint32_t bad = 0;
    const size_t j = j0 + l;
    for (uint32_t ch = 0; ch < nch; ch += 4) {
        dg_step<0, CLIP>(rec, d, n, nch, ch, w, l, jl, j, ccoef, acc, bad);
        if (ch + 1 < nch) dg_step<1, CLIP>(rec, d, n, nch, ch + 1, w, l, jl, j, ccoef, acc, bad);
        if (ch + 2 < nch) dg_step<2, CLIP>(rec, d, n, nch, ch + 2, w, l, jl, j, ccoef, acc, bad);
        if (ch + 3 < nch) dg_step<3, CLIP>(rec, d, n, nch, ch + 3, w, l, jl, j, ccoef, acc, bad);
    }
    if (w == 0 && j < d) {
        out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
        if (bad) atomicOr(status, FLTEE_DEV_ERR_DENSE_ORDER);
    }
}

// Tuning hook (fltee_debug_set_dense_variant): 0 is the shipped configuration.
static int g_dense_variant = 0;

template <int V, int U, bool CLIP, bool ACC, bool NT, int NTH = 256>
static void launch_v(const void *rec, size_t n, size_t d2, float coef, float *out,
                     const float *ccoef, uint32_t *status, hipStream_t s) {
    const unsigned blocks = (unsigned)((d2 + NTH * V - 1) / (NTH * V));
    FLTEE_LAUNCH((dense_accumulate_v<V, U, CLIP, ACC, NT, NTH>), dim3(blocks), dim3(NTH), 0, s,
                       (const uint4 *)rec, d2, (uint32_t)n, coef, out, ccoef, status);
}
template <int U, bool CLIP, bool ACC>
static void launch_r(const void *rec, size_t n, size_t d, float coef, float *out,
                     const float *ccoef, uint32_t *status, hipStream_t s) {
    FLTEE_LAUNCH((dense_accumulate_r<U, CLIP, ACC>), dim3((unsigned)((d + 255) / 256)), dim3(256),
                       0, s, (const uint2 *)rec, d, (uint32_t)n, coef, out, ccoef, status);
}

template <bool CLIP, bool ACC, int OB, int CC>
static void launch_lds(bool vec, const void *rec, size_t n, size_t d, float coef, float *out,
                       const float *ccoef, uint32_t *status, hipStream_t s) {
    const unsigned blocks = (unsigned)((d + OB - 1) / OB);
    if (vec)
        FLTEE_LAUNCH((dense_accumulate_lds<true, CLIP, ACC, OB, CC>), dim3(blocks), dim3(DS_NT), 0, s,
                           (const uint2 *)rec, d, (uint32_t)n, coef, out, ccoef, status);
    else
        FLTEE_LAUNCH((dense_accumulate_lds<false, CLIP, ACC, OB, CC>), dim3(blocks), dim3(DS_NT), 0,
                           s, (const uint2 *)rec, d, (uint32_t)n, coef, out, ccoef, status);
}

template <int U, bool REM, bool ACC>
static void dw_launch(unsigned blocks, const void *rec, size_t n, size_t d, float coef, float *out,
                      uint32_t *status, hipStream_t s, uint32_t per = 64) {
    FLTEE_LAUNCH((dense_accumulate_w<U, REM, false, ACC>), dim3(blocks), dim3(64), 0, s,
                       (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, nullptr, status, per);
}

static int cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

template <bool CLIP, bool ACC>
static hipError_t dense_dispatch(const void *rec, size_t n, size_t d, float coef, float *out,
                                 const float *ccoef, uint32_t *status, hipStream_t s) {
    const bool aligned = ((uintptr_t)rec % 16 == 0) && ((uintptr_t)out % 8 == 0) && (d % 2 == 0);
    if (d < ((size_t)1 << 18) && n > 1 && (g_dense_variant == 0 || g_dense_variant >= 20)) {
        // small d: LDS-staged chunks (variants 20-23: other block shapes, A/B)
        const bool vec = ((uintptr_t)rec % 16 == 0) && (d % 2 == 0);
        switch (g_dense_variant) {
        case 20: launch_lds<CLIP, ACC, 64, 32>(vec, rec, n, d, coef, out, ccoef, status, s); break;
        case 21: launch_lds<CLIP, ACC, 128, 16>(vec, rec, n, d, coef, out, ccoef, status, s); break;
        case 22: launch_lds<CLIP, ACC, 256, 16>(vec, rec, n, d, coef, out, ccoef, status, s); break;
        case 23: launch_lds<CLIP, ACC, 64, 16>(vec, rec, n, d, coef, out, ccoef, status, s); break;
        // 40-43: dense_accumulate_w, batches of 100 / 32 / 64 / 50 clients
        case 40: case 41: case 42: case 43:
            if (vec) {
                const unsigned blocks = (unsigned)((d / 2 + 63) / 64);
#define DW_GO(U_) FLTEE_LAUNCH((dense_accumulate_w<U_, true, CLIP, ACC>), dim3(blocks), dim3(64), 0, s, \
                                     (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, ccoef, status)
                if (g_dense_variant == 40) DW_GO(100);
                else if (g_dense_variant == 41) DW_GO(32);
                else if (g_dense_variant == 42) DW_GO(64);
                else DW_GO(50);
#undef DW_GO
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        // 44-46: dense_accumulate_wk, the clients of a pair over 2 / 4 / 3 waves (n <= 100)
        case 44: case 45: case 46:
            if (vec && !CLIP && n <= 100) {
                const unsigned blocks = (unsigned)((d / 2 + 63) / 64);
                if (g_dense_variant == 44)
                    FLTEE_LAUNCH((dense_accumulate_wk<2, 50, ACC>), dim3(blocks), dim3(128), 0, s,
                                       (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, status);
                else if (g_dense_variant == 45)
                    FLTEE_LAUNCH((dense_accumulate_wk<4, 25, ACC>), dim3(blocks), dim3(256), 0, s,
                                       (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, status);
                else
                    FLTEE_LAUNCH((dense_accumulate_wk<3, 34, ACC>), dim3(blocks), dim3(192), 0, s,
                                       (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, status);
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        // 49: dense_accumulate_w with plain (not nontemporal) loads
        case 49:
            if (vec && !CLIP && n <= 100) {
                const unsigned blocks = (unsigned)((d / 2 + 63) / 64);
                FLTEE_LAUNCH((dense_accumulate_w<100, true, false, ACC, false>), dim3(blocks), dim3(64), 0, s,
                                   (const uint4 *)rec, d / 2, (uint32_t)n, coef, out, nullptr, status);
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        // 47 / 48: dense_accumulate_w1, one lane per index, 100 / 50 clients in flight
        case 47: case 48:
            if (!CLIP && ((uintptr_t)rec % 8 == 0)) {
                const unsigned blocks = (unsigned)((d + 63) / 64);
                if (g_dense_variant == 47)
                    FLTEE_LAUNCH((dense_accumulate_w1<100, ACC>), dim3(blocks), dim3(64), 0, s,
                                       (const uint2 *)rec, d, (uint32_t)n, coef, out, status);
                else
                    FLTEE_LAUNCH((dense_accumulate_w1<50, ACC>), dim3(blocks), dim3(64), 0, s,
                                       (const uint2 *)rec, d, (uint32_t)n, coef, out, status);
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        case 24:
            if (vec && d >= 2) {
                FLTEE_LAUNCH((dense_accumulate_glds<CLIP, ACC>), dim3((unsigned)((d + 63) / 64)),
                                   dim3(256), 0, s, (const uint2 *)rec, d, (uint32_t)n, coef, out,
                                   ccoef, status);
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        // 50-52: dense_accumulate_w on a grid of 2 / 3 / 4 waves per CU (balanced)
        case 50: case 51: case 52:
            if (vec && !CLIP && n > 32 && n <= 100) {
                const size_t waves = (size_t)cu_count() * (size_t)(g_dense_variant - 48);
                const uint32_t per = (uint32_t)((d / 2 + waves - 1) / waves);
                if (per <= 64 && per > 0) {
                    const unsigned blocks = (unsigned)((d / 2 + per - 1) / per);
                    if (n == 100) dw_launch<100, false, ACC>(blocks, rec, n, d, coef, out, status, s, per);
                    else if (n > 64) dw_launch<100, true, ACC>(blocks, rec, n, d, coef, out, status, s, per);
                    else if (n == 64) dw_launch<64, false, ACC>(blocks, rec, n, d, coef, out, status, s, per);
                    else dw_launch<64, true, ACC>(blocks, rec, n, d, coef, out, status, s, per);
                    break;
                }
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        default:
            if (vec && !CLIP && n > 32 && n <= 100) {  // dense_accumulate_w, one batch in flight
                const unsigned blocks = (unsigned)((d / 2 + 63) / 64);
                if (n == 100) dw_launch<100, false, ACC>(blocks, rec, n, d, coef, out, status, s);
                else if (n > 64) dw_launch<100, true, ACC>(blocks, rec, n, d, coef, out, status, s);
                else if (n == 64) dw_launch<64, false, ACC>(blocks, rec, n, d, coef, out, status, s);
                else dw_launch<64, true, ACC>(blocks, rec, n, d, coef, out, status, s);
                break;
            }
            launch_lds<CLIP, ACC, 128, 32>(vec, rec, n, d, coef, out, ccoef, status, s);
            break;
        }
        return hipGetLastError();
    }
    if (aligned) {
        const size_t d2 = d / 2;
        switch (g_dense_variant) {
        case 1: launch_v<1, 8, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 2: launch_v<1, 32, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 3: launch_v<2, 8, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 4: launch_v<2, 16, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 5: launch_v<1, 16, CLIP, ACC, false>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 6: launch_v<4, 4, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 7: launch_v<4, 8, CLIP, ACC, true>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 9: launch_v<1, 16, CLIP, ACC, true, 128>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 10: launch_r<16, CLIP, ACC>(rec, n, d, coef, out, ccoef, status, s); break;
        case 11: launch_r<32, CLIP, ACC>(rec, n, d, coef, out, ccoef, status, s); break;
        case 12: launch_v<1, 16, CLIP, ACC, true, 64>(rec, n, d2, coef, out, ccoef, status, s); break;
        case 13: launch_v<1, 16, CLIP, ACC, true, 256>(rec, n, d2, coef, out, ccoef, status, s); break;
        // shipped: 512-lane blocks, 16 clients in flight, 16-B nontemporal loads
        // (A/B, 100 x 1M: 122.3 us vs 124.2 us for 256-lane blocks; profiles/r01/dense_variants_ab2.jsonl)
        default: launch_v<1, 16, CLIP, ACC, true, 512>(rec, n, d2, coef, out, ccoef, status, s); break;
        }
    } else {
        const unsigned blocks = (unsigned)((d + 255) / 256);
        FLTEE_LAUNCH((dense_accumulate_s<CLIP, ACC>), dim3(blocks), dim3(256), 0, s,
                           (const uint2 *)rec, d, (uint32_t)n, coef, out, ccoef, status);
    }
    return hipGetLastError();
}

void set_dense_variant(int v) { g_dense_variant = v; }

hipError_t launch_dense_accumulate(const void *rec, size_t n, size_t d, float coef, float *out,
                                   const float *client_coef, bool accumulate, uint32_t *status,
                                   hipStream_t s) {
    if (d == 0) return hipSuccess;
    if (client_coef)
        return accumulate ? dense_dispatch<true, true>(rec, n, d, coef, out, client_coef, status, s)
                          : dense_dispatch<true, false>(rec, n, d, coef, out, client_coef, status, s);
    return accumulate ? dense_dispatch<false, true>(rec, n, d, coef, out, nullptr, status, s)
                      : dense_dispatch<false, false>(rec, n, d, coef, out, nullptr, status, s);
}

// ---------------------------------------------------------------- sparse ---
// sweep_ordered: one lane per output, every record in upload order.  The records stream
// through LDS in chunks of SO_CH (each lane loads 16 of them one chunk ahead, 8-B
// non-temporal loads), and every lane reads each chunk back as 16-B broadcasts (two
// records per ds_read, the same address for the whole wave: no bank conflict).  Per
// record and output: one compare, one select, one add — 3 VALU.  The parallelism is the
// d outputs: 64-lane blocks while d / 64 waves do not fill the chip (MLP-MNIST: 796 waves
// for 1,024 SIMDs), 256-lane blocks sharing each chunk when there are waves to spare.
// Positions past nrec read as (u32::MAX, +0.0), which no output j < d matches.
constexpr int SO_CH = 1024;  // records per LDS chunk (8 KB)
// (Round 5, rejected: EXEC-masked adds — v_cmpx + v_add + EXEC restore, two VALU per
// record — 2.06 vs 1.22 ms at MLP-MNIST n = 30: each EXEC write stalls the next VALU.)

template <int NT, bool ACC>
__global__ __launch_bounds__(NT) void sweep_ordered(const uint2 *__restrict__ rec, uint32_t nrec,
                                                    uint32_t d, float coef, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint2 tile[SO_CH];
    constexpr int PER = SO_CH / NT;  // records each lane stages per chunk
    const uint32_t t = threadIdx.x;
    const uint32_t j = blockIdx.x * NT + t;
    uint2 pf[PER];
    auto load = [&](uint32_t c0) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t q = c0 + (uint32_t)i * NT + t;
            pf[i] = q < nrec ? ld_nt(rec + q) : make_uint2(0xFFFFFFFFu, 0u);
        }
    };
    load(0);
    float acc = 0.0f;
    const uint4 *t4 = reinterpret_cast<const uint4 *>(tile);
    for (uint32_t c0 = 0; c0 < nrec; c0 += SO_CH) {
        __syncthreads();  // every lane is done reading the previous chunk
#pragma unroll
        for (int i = 0; i < PER; ++i) tile[i * NT + t] = pf[i];
        __syncthreads();
        if (c0 + SO_CH < nrec) load(c0 + SO_CH);
        // 16 records per step, the next step's reads issued before this step's adds; the
        // whole 16-B reads are pinned in registers (as one 128-bit tuple each: no copies):
        // otherwise hipcc turns the select into a load of the value under an EXEC mask of
        // the matching lanes — a read whose lanes depend on the data, one LDS round trip
        // per record
        u32x4_t ra[8], rb[8];
        auto rd = [&](u32x4_t (&r)[8], int q) {
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const u32x4_t *>(t4 + q + i);
        };
        // 4 records at a time by hand: four compares into four SGPR-pair masks, the four
        // selects, the four adds in upload order, so every mask is read four VALU after it
        // is written (hipcc puts every compare in VCC, then needs two wait states before the
        // select that reads it, and turns selects of loaded values into loads under an EXEC
        // mask of the matching lanes).  (Round 5: a software-pipelined form — compare i + 2,
        // select i, add i - 1 — measured 2 % slower: `profiles/r05/ab/ab6_*`.)
        auto add4 = [&](const u32x4_t &a0, const u32x4_t &a1) {
            uint64_t m0, m1, m2, m3;
            uint32_t t0, t1, t2, t3;
            asm volatile(
                "v_cmp_eq_u32_e64 %[m0], %[i0], %[j]\n\t"
                "v_cmp_eq_u32_e64 %[m1], %[i1], %[j]\n\t"
                "v_cmp_eq_u32_e64 %[m2], %[i2], %[j]\n\t"
                "v_cmp_eq_u32_e64 %[m3], %[i3], %[j]\n\t"
                "v_cndmask_b32_e64 %[t0], 0, %[v0], %[m0]\n\t"
                "v_cndmask_b32_e64 %[t1], 0, %[v1], %[m1]\n\t"
                "v_cndmask_b32_e64 %[t2], 0, %[v2], %[m2]\n\t"
                "v_cndmask_b32_e64 %[t3], 0, %[v3], %[m3]\n\t"
                "v_add_f32_e32 %[acc], %[acc], %[t0]\n\t"
                "v_add_f32_e32 %[acc], %[acc], %[t1]\n\t"
                "v_add_f32_e32 %[acc], %[acc], %[t2]\n\t"
                "v_add_f32_e32 %[acc], %[acc], %[t3]"
                : [acc] "+v"(acc), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
                  [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                : [i0] "v"(a0.x), [v0] "v"(a0.y), [i1] "v"(a0.z), [v1] "v"(a0.w), [i2] "v"(a1.x),
                  [v2] "v"(a1.y), [i3] "v"(a1.z), [v3] "v"(a1.w), [j] "v"(j));
        };
        auto add = [&](const u32x4_t (&r)[8]) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) add4(r[i], r[i + 1]);
        };
        rd(ra, 0);
        for (int q = 0; q < SO_CH / 2; q += 16) {
            rd(rb, q + 8);
            add(ra);
            if (q + 16 < SO_CH / 2) rd(ra, q + 16);
            add(rb);
        }
    }
    if (j < d) out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
}

// rows [n][d] f32 summed in row order: out[j] = sum_c mat[c][j] (* coef)
template <int U, bool ACC>
__global__ __launch_bounds__(256) void rows_accumulate(const float4 *__restrict__ mat, size_t d4,
                                                       uint32_t n, float coef,
                                                       float4 *__restrict__ out) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= d4) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t c = 0;
    for (; c + U <= n; c += U) {
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld_nt(mat + (size_t)(c + u) * d4 + t);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc.x = __fadd_rn(acc.x, x[u].x); acc.y = __fadd_rn(acc.y, x[u].y);
            acc.z = __fadd_rn(acc.z, x[u].z); acc.w = __fadd_rn(acc.w, x[u].w);
        }
    }
    for (; c < n; ++c) {
        float4 x = ld_nt(mat + (size_t)c * d4 + t);
        acc.x = __fadd_rn(acc.x, x.x); acc.y = __fadd_rn(acc.y, x.y);
        acc.z = __fadd_rn(acc.z, x.z); acc.w = __fadd_rn(acc.w, x.w);
    }
    if (ACC) {
        float4 p = out[t];
        out[t] = make_float4(__fadd_rn(p.x, acc.x), __fadd_rn(p.y, acc.y), __fadd_rn(p.z, acc.z),
                             __fadd_rn(p.w, acc.w));
    } else {
        out[t] = make_float4(__fmul_rn(acc.x, coef), __fmul_rn(acc.y, coef),
                             __fmul_rn(acc.z, coef), __fmul_rn(acc.w, coef));
    }
}

template <bool ACC>
__global__ __launch_bounds__(256) void rows_accumulate_s(const float *__restrict__ mat, size_t d,
                                                         uint32_t n, float coef,
                                                         float *__restrict__ out) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= d) return;
    float acc = 0.0f;
    for (uint32_t c = 0; c < n; ++c) acc = __fadd_rn(acc, mat[(size_t)c * d + j]);
    out[j] = ACC ? __fadd_rn(out[j], acc) : __fmul_rn(acc, coef);
}

hipError_t launch_rows_accumulate(const float *mat, size_t n, size_t d, float coef, float *out,
                                  bool accumulate, hipStream_t s) {
    if (d == 0) return hipSuccess;
    if (d % 4 == 0 && (uintptr_t)out % 16 == 0) {
        const size_t d4 = d / 4;
        const unsigned blocks = (unsigned)((d4 + 255) / 256);
        if (accumulate)
            FLTEE_LAUNCH((rows_accumulate<8, true>), dim3(blocks), dim3(256), 0, s,
                               (const float4 *)mat, d4, (uint32_t)n, coef, (float4 *)out);
        else
            FLTEE_LAUNCH((rows_accumulate<8, false>), dim3(blocks), dim3(256), 0, s,
                               (const float4 *)mat, d4, (uint32_t)n, coef, (float4 *)out);
    } else {
        const unsigned blocks = (unsigned)((d + 255) / 256);
        if (accumulate)
            FLTEE_LAUNCH(rows_accumulate_s<true>, dim3(blocks), dim3(256), 0, s, mat, d,
                               (uint32_t)n, coef, out);
        else
            FLTEE_LAUNCH(rows_accumulate_s<false>, dim3(blocks), dim3(256), 0, s, mat, d,
                               (uint32_t)n, coef, out);
    }
    return hipGetLastError();
}

hipError_t launch_sweep_accumulate(const void *rec, size_t nrec, size_t d, float coef, float *out,
                                   bool accumulate, hipStream_t s) {
    if (d == 0) return hipSuccess;
    if (nrec >= 0xFFFFFFFFull || d >= 0xFFFFFFFFull) return hipErrorInvalidValue;
    // 256-lane blocks: a block's four waves go to the CU's four SIMDs, one each (64-lane
    // blocks left SIMDs holding two of them while others idled: 1.8 vs 0.8 ms at MLP-MNIST
    // n = 30); 64-lane blocks only for a d too small to give every CU a block
    const bool wide = d >= (size_t)256 * 64;
    const unsigned blocks = (unsigned)((d + (wide ? 255 : 63)) / (wide ? 256 : 64));
#define SO_GO(NT_, ACC_)                                                                         \
    FLTEE_LAUNCH((sweep_ordered<NT_, ACC_>), dim3(blocks), dim3(NT_), 0, s,                \
                       (const uint2 *)rec, (uint32_t)nrec, (uint32_t)d, coef, out)
    if (wide) {
        if (accumulate) SO_GO(256, true);
        else SO_GO(256, false);
    } else {
        if (accumulate) SO_GO(64, true);
        else SO_GO(64, false);
    }
#undef SO_GO
    return hipGetLastError();
}

// ------------------------------------------------- sparse non_oblivious ----
// non_oblivious.rs:6-15 is a plain scatter-add with no obliviousness to keep, so
// its GPU form is a scatter too.  Client c's records land at mat[c][idx] (mat
// pre-filled with the empty sentinel), then the rows are summed in client order
// with the sentinel read as +0.0 — adding +0.0 to a running sum that started at
// +0.0 is the identity (such a sum is never -0.0), so every output is the
// reference's in-order sum, bit for bit.  That needs a client's indices to be
// distinct (top-k, utils.py:327-354): a repeated index, or a value whose bits are
// the sentinel, sets *dup and the row pass switches (uniformly, same launch) to
// the in-order sequential sweep over every record.  Traffic: n*k*8 + n*d*4*2 + d*4.
constexpr uint32_t kEmptySlot = 0xFFFFFFFFu;
constexpr int SW_CHUNK = 2048;  // records staged per LDS pass of the repeated-index path

__global__ __launch_bounds__(256) void scatter_rows_kernel(const uint2 *__restrict__ rec, size_t n,
                                                           size_t k, size_t d,
                                                           uint32_t *__restrict__ mat,
                                                           uint32_t *dup, uint32_t epoch,
                                                           uint32_t *status) {
    uint32_t bad = 0, rep = 0;
    for (size_t c = blockIdx.y; c < n; c += gridDim.y) {
        for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < k; e += (size_t)gridDim.x * 256) {
            const uint2 r = rec[c * k + e];
            if (r.x >= d) { bad = 1; continue; }
            const uint32_t old = atomicCAS(mat + c * d + r.x, kEmptySlot, r.y);
            rep |= (old != kEmptySlot) | (r.y == kEmptySlot);
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, FLTEE_DEV_ERR_INDEX_RANGE);
    if (__any(rep) && (threadIdx.x & 63) == 0) atomicMax(dup, epoch);  // this call's mark
}

// One lane per output j: the n rows' slots j are read U at a time (wave-coalesced
// 256-B loads) and added in client order.  Every slot a record filled is set back to the
// sentinel (on the repeated-index path: the whole column), so the rows are empty again
// for the next call and no fill launch is needed (launch_scatter_sum).
template <bool ACC, int U>
__global__ __launch_bounds__(256) void scatter_rows_sum(uint32_t *__restrict__ mat, size_t d,
                                                        uint32_t n, const uint2 *__restrict__ rec,
                                                        size_t nrec, const uint32_t *dup,
                                                        uint32_t epoch, float coef,
                                                        float *__restrict__ out) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    float acc = 0.0f;
    bool hit = false;
    if (*dup != epoch) {
        if (j >= d) return;
        uint32_t *col = mat + j;
        uint32_t c = 0;
        for (; c + U <= n; c += U) {
            uint32_t x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(col + (size_t)(c + u) * d);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool h = x[u] != kEmptySlot;
                acc = __fadd_rn(acc, h ? __uint_as_float(x[u]) : 0.0f);
                hit |= h;
                if (h) col[(size_t)(c + u) * d] = kEmptySlot;
            }
        }
        if (c < n) {  // the last n % U rows as one predicated batch (all loads in flight)
            uint32_t x[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                x[u] = c + u < n ? __builtin_nontemporal_load(col + (size_t)(c + u) * d) : kEmptySlot;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (c + u < n) {
                    const bool h = x[u] != kEmptySlot;
                    acc = __fadd_rn(acc, h ? __uint_as_float(x[u]) : 0.0f);
                    hit |= h;
                    if (h) col[(size_t)(c + u) * d] = kEmptySlot;
                }
            }
        }
    } else {  // a client repeated an index: every record, in upload order
        __shared__ uint2 tile[SW_CHUNK];
        for (size_t c0 = 0; c0 < nrec; c0 += SW_CHUNK) {
            const uint32_t m = (uint32_t)((nrec - c0) < SW_CHUNK ? (nrec - c0) : SW_CHUNK);
            __syncthreads();
            for (uint32_t e = threadIdx.x; e < m; e += 256) tile[e] = rec[c0 + e];
            __syncthreads();
            for (uint32_t q = 0; q < m; ++q) {
                const uint2 r = tile[q];
                const bool h = r.x == j;
                acc = __fadd_rn(acc, h ? __uint_as_float(r.y) : 0.0f);
                hit |= h;
            }
        }
        if (j >= d) return;
        for (uint32_t c = 0; c < n; ++c) mat[(size_t)c * d + j] = kEmptySlot;
    }
    if (ACC) {
        if (hit) out[j] = __fadd_rn(out[j], acc);
    } else {
        out[j] = __fmul_rn(acc, coef);
    }
}

hipError_t launch_scatter_sum(const void *rec, size_t n, size_t k, size_t d, uint32_t *mat,
                              size_t *mat_clean, uint32_t *dup, float coef, float *out, bool accumulate,
                              uint32_t *status, hipStream_t s) {
    if (d == 0) return hipSuccess;
    // *dup holds the epoch of the last call that saw a repeated index: a fresh epoch per
    // call replaces a memset of the flag (one launch less)
    static std::atomic<uint32_t> epochs{0};
    uint32_t epoch = ++epochs;
    if (epoch == 0) epoch = ++epochs;
    // the rows [0, n*d) must hold the sentinel: filled once per buffer, then kept so by
    // scatter_rows_sum, which empties every slot it consumed
    if (*mat_clean < n * d * 4) {
        hipError_t e = fl_memset_async(mat, 0xFF, n * d * 4, s);
        if (e != hipSuccess) return e;
        *mat_clean = n * d * 4;
    }
    if (k) {
        const size_t bx = (k + 255) / 256 < 1024 ? (k + 255) / 256 : 1024;
        const size_t by = n < 65535 ? n : 65535;
        FLTEE_LAUNCH(scatter_rows_kernel, dim3((unsigned)bx, (unsigned)by), dim3(256), 0, s,
                           (const uint2 *)rec, n, k, d, mat, dup, epoch, status);
    }
    const unsigned blocks = (unsigned)((d + 255) / 256);
    const size_t nrec = n * k;
    if (accumulate)
        FLTEE_LAUNCH((scatter_rows_sum<true, 32>), dim3(blocks), dim3(256), 0, s, mat, d,
                           (uint32_t)n, (const uint2 *)rec, nrec, dup, epoch, coef, out);
    else
        FLTEE_LAUNCH((scatter_rows_sum<false, 32>), dim3(blocks), dim3(256), 0, s, mat, d,
                           (uint32_t)n, (const uint2 *)rec, nrec, dup, epoch, coef, out);
    return hipGetLastError();
}

// ------------------------------------------------------------- helpers -----
__global__ void scale_kernel(float *out, size_t d, float coef) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j < d) out[j] = __fmul_rn(out[j], coef);
}

// Measurement only (bench.py: the achievable floor beside the metric's literal config): a
// plain streaming read of `bytes` with 16-B non-temporal loads, 8 in flight per lane, the
// words xor-folded so the loads stay (a store to sink only on one fold value).
__global__ __launch_bounds__(256) void read_floor_kernel(const uint4 *__restrict__ src, size_t n16,
                                                         uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        uint4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = ld_nt(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    for (; i < n16; i += stride) {
        const uint4 x = ld_nt(src + i);
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = threadIdx.x;  // keeps the loads; (almost) never taken
}

hipError_t launch_read_floor(const void *src, size_t bytes, uint32_t *sink, unsigned blocks,
                             hipStream_t s) {
    FLTEE_LAUNCH(read_floor_kernel, dim3(blocks), dim3(256), 0, s, (const uint4 *)src, bytes / 16,
                       sink);
    return hipGetLastError();
}

hipError_t launch_scale(float *out, size_t d, float coef, hipStream_t s) {
    if (d == 0) return hipSuccess;
    FLTEE_LAUNCH(scale_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, out, d,
                       coef);
    return hipGetLastError();
}

// status |= INDEX_RANGE if any record idx >= limit
__global__ void check_range_kernel(const uint2 *rec, size_t nrec, uint32_t limit,
                                   uint32_t *status) {
    uint32_t bad = 0;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < nrec; e += (size_t)gridDim.x * 256)
        bad |= rec[e].x >= limit;
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, FLTEE_DEV_ERR_INDEX_RANGE);
}

hipError_t launch_check_range(const void *rec, size_t nrec, uint32_t limit, uint32_t *status,
                              hipStream_t s) {
    if (nrec == 0) return hipSuccess;
    size_t blocks = (nrec + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    FLTEE_LAUNCH(check_range_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint2 *)rec, nrec, limit, status);
    return hipGetLastError();
}

}  // namespace fltee
