// engine.hip — device-side orchestration of the aggregation algorithms.
//
// fltee_aggregate_device() is the aggregation of ecall_secure_aggregation
// (lib.rs:355-408) on records already decrypted into HBM: the dispatcher on
// aggregation_alg (lib.rs:359-397), optional DP noise (lib.rs:399-408), with
// the enclave's 1f32/n averaging (common.rs:14-19).  Scratch HBM is held per
// device, grow-only, so steady-state calls do no hipMalloc (graph-capturable
// once reserved).
#include <sys/random.h>
#include <time.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "engine.h"

namespace fltee {

hipError_t launch_rows_accumulate(const float *mat, size_t n, size_t d, float coef, float *out,
                                  bool accumulate, hipStream_t s);
hipError_t launch_scatter_sum(const void *rec, size_t n, size_t k, size_t d, uint32_t *mat,
                              size_t *mat_clean,
                              uint32_t *dup, float coef, float *out, bool accumulate,
                              uint32_t *status, hipStream_t s);

// Sparse non_oblivious: scatter into per-client rows (k_accumulate.hip) when the
// [n][d] row matrix costs less HBM traffic than the stable sort it replaces
// (rows: ~8*n*d bytes; sort: >= 16*M bytes per pass), or when the rows are small enough
// (<= 2^24 cells, 128 MB of traffic: ~25 us) that the counting sort's nine launches and
// its count readback cost more than they move (round 5: MLP-MNIST n = 3, k = 508 took
// ~100 us through the sort, `profiles/r05/small_ecall/`).
static bool use_scatter_rows(size_t n, size_t k, size_t d) {
    const size_t cells = n * d;
    return cells <= ((size_t)1 << 30) &&
           (cells <= ((size_t)1 << 24) || cells <= 64 * next_pow2_sz(n * k));
}

// Sparse baseline / path_oram (the sweep otherwise): uploads of dense size (k = d, e.g.
// fl_main.py --alpha 1.0, whose top-k orders each client's records by |val|, utils.py:
// 346-352), where the sweep's n*k*d compare-selects (n*d^2) would dominate, go through the
// ordered fold in the composite-key network's order (idx, upload position): the
// enclave's o_update result for any upload, bit for bit (baseline.rs:28-60 adds each
// index's records in upload order).  A public-size decision.
static bool flat_ordered(size_t n, size_t k, size_t d) { return k == d && n * k > 0; }

static DeviceCtx g_ctx[kMaxDevices];
static std::mutex g_ctx_mu;
static std::atomic<uint64_t> g_debug_seed{0};
static std::atomic<uint64_t> g_seed_calls{0};

static std::atomic<uint64_t> g_net_launches{0}, g_net_bytes{0};
struct NetLaunch {
    const char *kernel;  // nullptr: the final event
    uint64_t bytes;
    hipEvent_t ev;
};
static std::mutex g_net_mu;
static std::vector<NetLaunch> g_net_log;
static std::atomic<bool> g_net_timing{false};
constexpr size_t kNetLogCap = 16384;

// the launch trace (common.h): one text line per launch / copy / memset / sync / RCCL op
static std::atomic<bool> g_trace{false};
static std::mutex g_trace_mu;
static std::string g_trace_text;
static size_t g_trace_lines = 0;
constexpr size_t kTraceCap = (size_t)64 << 20;

bool trace_on() { return g_trace.load(std::memory_order_relaxed); }

void trace_event(const char *what, const char *site, uint64_t a, uint64_t b, uint64_t c) {
    char line[512];
    const int len = std::snprintf(line, sizeof line, "%s|%s|%llu|%llu|%llu\n", what, site,
                                  (unsigned long long)a, (unsigned long long)b, (unsigned long long)c);
    std::lock_guard<std::mutex> lk(g_trace_mu);
    if (len > 0 && g_trace_text.size() + (size_t)len < kTraceCap) {
        g_trace_text.append(line, (size_t)len < sizeof line ? (size_t)len : sizeof line - 1);
        ++g_trace_lines;
    }
}

void net_account(uint64_t bytes, const char *kernel, hipStream_t s) {
    if (trace_on()) trace_event("bytes", kernel, bytes, 0, 0);
    g_net_launches.fetch_add(1, std::memory_order_relaxed);
    g_net_bytes.fetch_add(bytes, std::memory_order_relaxed);
    if (!g_net_timing.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> lk(g_net_mu);
    if (g_net_log.size() >= kNetLogCap) return;
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return;
    if (hipEventRecord(e, s) != hipSuccess) { (void)hipEventDestroy(e); return; }
    g_net_log.push_back({kernel, bytes, e});
}

static void net_log_clear() {
    for (auto &r : g_net_log) (void)hipEventDestroy(r.ev);
    g_net_log.clear();
}

uint64_t next_seed() {
    const uint64_t s = g_debug_seed.load();
    if (s) return s + 0x9E3779B97F4A7C15ull * (++g_seed_calls);
    uint64_t r = 0;
    if (getrandom(&r, sizeof r, 0) != (ssize_t)sizeof r) r = (uint64_t)time(nullptr) * 0x2545F4914F6CDD1Dull;
    return r ? r : 1;
}

void set_debug_seed(uint64_t seed) {
    g_debug_seed.store(seed);
    g_seed_calls.store(0);
}

DeviceCtx *device_ctx(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    DeviceCtx &c = g_ctx[dev];
    if (!c.ready) {
        if (hipSetDevice(dev) != hipSuccess) return nullptr;
        if (hipMalloc(&c.status, 256) != hipSuccess) return nullptr;
        if (fl_memset(c.status, 0, 256) != hipSuccess) return nullptr;
        c.device = dev;
        c.ready = true;
    }
    return &c;
}

DeviceCtx *current_ctx() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    return device_ctx(dev);
}

bool Buffer::reserve(size_t bytes) {
    if (bytes <= cap) return true;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    const size_t want = bytes + bytes / 8 + 256;
    if (hipMalloc(&ptr, want) != hipSuccess) { ptr = nullptr; return false; }
    cap = want;
    return true;
}

bool HostBuffer::reserve(size_t bytes) {
    if (bytes <= cap) return true;
    if (ptr) (void)hipHostFree(ptr);
    ptr = dptr = nullptr;
    cap = 0;
    const size_t want = bytes + bytes / 8 + 4096;
    if (hipHostMalloc(&ptr, want, hipHostMallocDefault) != hipSuccess) { ptr = nullptr; return false; }
    if (hipHostGetDevicePointer(&dptr, ptr, 0) != hipSuccess) dptr = ptr;  // one address space
    cap = want;
    return true;
}

void Buffer::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
}

float nips19_threshold(size_t d, size_t k, size_t n) {
    const float epsilon = 100.0f, delta = 1.0f / (float)n;
    const float l1 = 2.0f * (float)k;
    return l1 / epsilon * logf((float)d / delta);
}

static size_t f32_to_usize_sat(float x) {
    if (!(x > 0.0f)) return 0;
    if (x >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)x;
}

// scratch plan per algorithm
struct Plan {
    size_t a_bytes = 0, b_bytes = 0, mat_bytes = 0, r_bytes = 0, coef_bytes = 0, rec_bytes = 0;
    size_t keys_bytes = 0, radix_bytes = 0;  // ordered fold: sorted records, sort scratch
    size_t side_bytes = 0;                   // advanced's streaming fold: side records
    size_t lb_bytes = 0;                     // advanced's fused fold: look-back slots
    size_t oram_bytes = 0;                   // path_oram tree: slots (16 B) + their records (8 B)
};

// the side records of advanced's streaming fold over its array (M) or its compaction
// prefix (run_advanced's mf), whichever has more lanes
static size_t advanced_side_bytes(size_t n, size_t k, size_t d, size_t halo) {
    const size_t L = n * k + d, M = next_pow2_sz(L);
    size_t mf = (L + 1 + 15) / 16 * 16;
    if (mf > M) mf = M;
    const size_t a = fold_side_bytes(M, M, halo, 0, 0), b = mf >= 2 ? fold_side_bytes(mf, L, halo, 0, 0) : 0;
    return a > b ? a : b;
}

static Plan plan_for(uint32_t alg, size_t n, size_t k, size_t d, const fltee_device_opts &o) {
    Plan p;
    const bool dense = (o.flags & FLTEE_OPT_DENSE) != 0;
    const bool clip = (o.flags & FLTEE_OPT_CLIP) != 0;
    // (aggregate() refuses a tree shape that does not fit before it plans: tree_shape)
    const bool tree = alg == FLTEE_ALG_PATH_ORAM && (o.flags & FLTEE_OPT_ORAM_TREE);
    if (clip) {
        p.coef_bytes = n * 4;
        if (!dense || tree) p.rec_bytes = n * k * 8;  // the tree reads records: clipped copies
    }
    switch (alg) {
    case FLTEE_ALG_PATH_ORAM:
        if (tree) {
            const bool lazy = (o.flags & FLTEE_OPT_ORAM_LAZY) != 0;
            const size_t ns = oram_slots(d);
            p.oram_bytes = ns * (lazy ? 24 : 16);
            // the leaf precompute's two key arrays; lazy: the readout network too
            size_t m = next_pow2_sz(oram_accesses(n * k, d, lazy));
            if (lazy && next_pow2_sz(ns + d) > m) m = next_pow2_sz(ns + d);
            p.a_bytes = p.b_bytes = m * 8;
        } else if (!dense && flat_ordered(n, k, d)) {
            p.keys_bytes = n * k * 8, p.radix_bytes = next_pow2_sz(n * k) * 8;
        }
        break;
    case FLTEE_ALG_BASELINE:
        if (!dense && flat_ordered(n, k, d))  // the composite-key network + its gather
            p.keys_bytes = n * k * 8, p.radix_bytes = next_pow2_sz(n * k) * 8;
        break;
    case FLTEE_ALG_NON_OBLIVIOUS:
        if (!dense) {
            if (use_scatter_rows(n, k, d)) p.mat_bytes = n * d * 4;
            else p.keys_bytes = n * k * 8, p.radix_bytes = radix_scratch_bytes(n * k, d);
        }
        break;
    case FLTEE_ALG_ADVANCED:
        p.a_bytes = p.b_bytes = next_pow2_sz(n * k + d) * 8;
        p.side_bytes = advanced_side_bytes(n, k, d, o.fold_halo ? o.fold_halo : n);
        p.lb_bytes = fc_lookback_bytes(next_pow2_sz(n * k + d), n * k + d, d, o.fold_halo ? o.fold_halo : n);
        break;
    case FLTEE_ALG_OPTIMIZED: {
        size_t b = o.batch ? (o.batch < n ? o.batch : n) : n;
        p.a_bytes = p.b_bytes = next_pow2_sz(b * k + d) * 8;
        p.side_bytes = advanced_side_bytes(b, k, d, o.fold_halo ? o.fold_halo : b);
        p.lb_bytes = fc_lookback_bytes(next_pow2_sz(b * k + d), b * k + d, d, o.fold_halo ? o.fold_halo : b);
        break;
    }
    case FLTEE_ALG_NIPS19: {
        const size_t kq = (o.flags & FLTEE_OPT_K_REQ) ? o.k_req : k;  // nips19.rs:38
        const float T = nips19_threshold(d, kq, n);
        p.a_bytes = next_pow2_sz(n * k + d * f32_to_usize_sat(T)) * 8;
        p.r_bytes = d * 4;
        break;
    }
    default: break;
    }
    return p;
}

// the fused fold's look-back slots: grown zeroed (a stale slot must never carry a live
// epoch), the epochs starting over
static bool reserve_lb(DeviceCtx *c, size_t bytes) {
    if (bytes <= c->ws_lb.cap) return true;
    if (!c->ws_lb.reserve(bytes) || fl_memset(c->ws_lb.ptr, 0, c->ws_lb.cap) != hipSuccess) return false;
    c->fc_epoch = 0;
    return true;
}

static bool reserve_plan(DeviceCtx *c, const Plan &p) {
    return c->ws_a.reserve(p.a_bytes) && c->ws_b.reserve(p.b_bytes) &&
           c->ws_mat.reserve(p.mat_bytes) && c->ws_r.reserve(p.r_bytes) &&
           c->ws_coef.reserve(p.coef_bytes) && c->ws_rec.reserve(p.rec_bytes) &&
           c->ws_keys.reserve(p.keys_bytes) && c->ws_radix.reserve(p.radix_bytes) &&
           c->ws_oram.reserve(p.oram_bytes) && c->ws_side.reserve(p.side_bytes) &&
           reserve_lb(c, p.lb_bytes);
}

// The ordered fold of n records (common.rs:25-35, non_oblivious.rs:11-13): the records in
// stable order by idx, then out[i] = the in-order sum of index i's.  The order comes from
// the hand-written counting sort (k_radix.hip: the sequence of indices in list order is
// what the enclave's own g[idx] += val loop touches) — or, fltee_debug_set_radix_order(0),
// from the composite-key bitonic sort, the records gathered by its keys (the same order,
// bit for bit: test_gpu_parity.py).
static bool g_radix_order = true;
void set_radix_order(int on) { g_radix_order = on != 0; }
static bool g_exact_runs = false;  // the ECALLs' advanced / alg 6: reject runs > n + 1 unless set
void set_exact_runs(int on) { g_exact_runs = on != 0; }
bool exact_runs_default() { return g_exact_runs; }
static bool g_oram_tree = false;  // the ECALLs' path_oram: the sweep unless set
void set_oram_tree(int on) { g_oram_tree = on != 0; }
bool oram_tree_default() { return g_oram_tree; }

static hipError_t ordered_fold_records(DeviceCtx *c, const void *rec, size_t n, size_t d,
                                       float coef, float *out, bool acc, uint32_t *status,
                                       hipStream_t s, bool network_order = false) {
    if (n == 0) return acc ? hipSuccess : fl_memset_async(out, 0, d * 4, s);
    if (!c->ws_keys.reserve(n * 8)) return hipErrorOutOfMemory;
    uint64_t *sorted = (uint64_t *)c->ws_keys.ptr;
    hipError_t e;
    if (g_radix_order && !network_order) {
        if (!c->ws_radix.reserve(radix_scratch_bytes(n, d))) return hipErrorOutOfMemory;
        e = launch_sort_records_by_idx(rec, n, d, c->ws_radix.ptr, c->ws_radix.cap, sorted, status,
                                       acc ? nullptr : out, d, s);
    } else {
        const size_t mc = next_pow2_sz(n);
        if (!c->ws_radix.reserve(mc * 8)) return hipErrorOutOfMemory;
        uint64_t *keys = (uint64_t *)c->ws_radix.ptr;
        e = launch_composite_init(rec, n, d, mc, keys, status, s);
        if (e == hipSuccess) e = bitonic_sort(keys, mc, 1, 0, s, n);  // ~0 keys past n
        if (e == hipSuccess) e = launch_gather_by_keys(keys, n, rec, sorted, s);
        if (e == hipSuccess && !acc) e = fl_memset_async(out, 0, d * 4, s);
    }
    if (e == hipSuccess) e = launch_fold_sorted(sorted, n, d, coef, out, acc, s);
    return e;
}

// the selected list sel[0, lc) (entries with idx < d in position order) -> out: stable
// order by idx (list position within an index), then the ordered fold
hipError_t ordered_from_list(DeviceCtx *c, const uint64_t *sel, size_t lc, size_t d, float coef,
                             float *out, bool acc, uint32_t *status, hipStream_t s) {
    if (lc == 0) return acc ? hipSuccess : fl_memset_async(out, 0, d * 4, s);
    return ordered_fold_records(c, sel, lc, d, coef, out, acc, status, s);
}

hipError_t read_device_word(DeviceCtx *c, const uint32_t *dev_word, size_t *out, hipStream_t s) {
    if (!c->host_word && hipHostMalloc((void **)&c->host_word, 64, hipHostMallocDefault) != hipSuccess) {
        c->host_word = nullptr;
        return hipErrorOutOfMemory;
    }
    hipError_t e = fl_memcpy_async(c->host_word, dev_word, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = fl_stream_sync(s);
    if (e == hipSuccess) *out = *c->host_word;
    return e;
}

hipError_t safe_aggregate_ordered(DeviceCtx *c, const uint64_t *src, size_t m, size_t d,
                                  float coef, float *out, bool acc, uint32_t *status,
                                  hipStream_t s) {
    if (d == 0) return hipSuccess;
    if (m == 0) return acc ? hipSuccess : fl_memset_async(out, 0, d * 4, s);
    const size_t nb = select_tiles(m);
    if (!c->ws_cnt.reserve((2 * nb + 2) * 4)) return hipErrorOutOfMemory;
    uint32_t *cnt = (uint32_t *)c->ws_cnt.ptr, *base = cnt + nb + 1;
    hipError_t e = launch_select_count(src, m, d, cnt, base, s);
    size_t lc = 0;  // entries with idx < d (the DP-noised histogram total)
    if (e == hipSuccess) e = read_device_word(c, base + nb, &lc, s);
    if (e != hipSuccess) return e;
    if (!c->ws_sel.reserve(lc * 8 + 8)) return hipErrorOutOfMemory;
    uint64_t *sel = (uint64_t *)c->ws_sel.ptr;
    if (lc) e = launch_select_write(src, m, d, base, sel, s);
    if (e != hipSuccess) return e;
    return ordered_from_list(c, sel, lc, d, coef, out, acc, status, s);
}

// nips19's shuffle + safe_aggregate with the selection fused into the shuffle's last
// pass (bitonic_sort_nips19_select): the 2^27-entry array is never written out or read
// back.  hipErrorNotSupported: shape not fusable (the caller shuffles, then selects).
static hipError_t nips19_shuffle_aggregate(DeviceCtx *c, uint64_t *A, size_t M, uint32_t key,
                                           const void *rec, size_t nrec, const uint32_t *r,
                                           size_t d, size_t tf, float coef, float *out, bool acc,
                                           uint32_t *status, hipStream_t s) {
    const size_t ntl = bitonic_select_tiles(M);
    if (ntl == 0 || d == 0) return hipErrorNotSupported;
    if (!c->ws_cnt.reserve((2 * ntl + 2) * 4)) return hipErrorOutOfMemory;
    uint32_t *cnt = (uint32_t *)c->ws_cnt.ptr, *base = cnt + ntl + 1;
    // tiles of pads alone are skipped by the last pass and keep a zero count
    hipError_t e = fl_memset_async(cnt, 0, ntl * 4, s);
    if (e == hipSuccess) e = bitonic_sort_nips19_select(A, M, key, rec, nrec, r, d, tf, cnt, s);
    if (e != hipSuccess) return e;
    e = launch_select_scan(cnt, ntl, base, s);
    size_t lc = 0;
    if (e == hipSuccess) e = read_device_word(c, base + ntl, &lc, s);
    if (e != hipSuccess) return e;
    if (!c->ws_sel.reserve(lc * 8 + 8)) return hipErrorOutOfMemory;
    uint64_t *sel = (uint64_t *)c->ws_sel.ptr;
    if (lc) e = launch_select_gather(A, log2_pow2(M / ntl), ntl, cnt, base, sel, s);
    if (e != hipSuccess) return e;
    return ordered_from_list(c, sel, lc, d, coef, out, acc, status, s);
}

// `advanced` over n clients' records into out (coef or accumulate).
#ifndef FLTEE_FOLD_CEMIT
#define FLTEE_FOLD_CEMIT 1
#endif
static bool g_advanced_compaction = true;  // fltee_debug_set_advanced_compaction
static bool g_nips19_fused_select = true;  // fltee_debug_set_nips19_fused_select (A/B)

static hipError_t run_advanced(DeviceCtx *c, const void *rec, size_t n, size_t k, size_t d,
                               size_t k_req, size_t halo, float coef, float *out, bool acc,
                               uint32_t *status, hipStream_t s) {
    const size_t L = n * k + d, M = next_pow2_sz(L);
    const size_t fold_len = n * k_req + d;
    uint64_t *A = (uint64_t *)c->ws_a.ptr, *B = (uint64_t *)c->ws_b.ptr;
    hipError_t e = bitonic_sort_advanced(A, M, rec, n * k, d, s);  // init fused into the sort
    if (e == hipErrorNotSupported) {
        e = launch_advanced_init(rec, n * k, d, M, A, s);
        if (e == hipSuccess) e = bitonic_sort(A, M, 0, 0, s, L);
    }
    if (e != hipSuccess) return e;
    // Second sort (advanced.rs:106-111): with fold_len == L its [0, d) prefix is the
    // order-preserving compaction of the idx < d representatives (k_compact.hip), and
    // the fold runs inside the compaction's first pass; the k_req != k quirk leaves
    // unfolded records competing for that prefix and keeps the full network.
    if (fold_len == L && g_advanced_compaction) {
        const size_t lbb = fc_lookback_bytes(M, L, d, halo ? halo : n);
        if (lbb && (lbb > c->ws_lb.cap || c->fc_epoch >= (1u << 30) - 1)) {
            // new slots hold whatever was there: zero them (the epochs start over)
            if (!c->ws_lb.reserve(lbb) || fl_memset_async(c->ws_lb.ptr, 0, c->ws_lb.cap, s) != hipSuccess)
                return hipErrorOutOfMemory;
            c->fc_epoch = 0;
        }
        e = launch_fold_compact_extract(A, B, M, L, d, halo ? halo : n, coef, out, acc, status, s,
                                        c->ws_lb.ptr, c->ws_lb.cap, &c->fc_epoch);
        if (e != hipErrorNotSupported) return e;
    }
    if (fold_len == L && g_advanced_compaction) {
        // the compaction reads [0, L) only: fold up to the first pad (position L is
        // read as the run-end test of L - 1), not the pads after it
        size_t mf = (L + 1 + 15) / 16 * 16;
        if (mf > M) mf = M;
        // the fold emits the compaction's first-pass form (no conversion there, 16-B pairs;
        // FLTEE_FOLD_CEMIT=0: the enclave's folded array, converted by that pass; and a
        // one-entry array — d = 1 and no records — which has nothing to fold: copied)
        if (!c->ws_side.reserve(fold_side_bytes(mf, fold_len, halo ? halo : n, 0, 0)))
            return hipErrorOutOfMemory;
        if (FLTEE_FOLD_CEMIT && mf >= 2) {
            e = launch_fold(A, B, mf, fold_len, halo ? halo : n, c->ws_side.ptr, c->ws_side.cap, s,
                            d, compact_dummy());
            if (e != hipSuccess) return e;
            return launch_compact_extract_converted(B, A, L, d, coef, out, acc, s);
        }
        e = launch_fold(A, B, mf, fold_len, halo ? halo : n, c->ws_side.ptr, c->ws_side.cap, s);
        if (e != hipSuccess) return e;
        return launch_compact_extract(B, A, L, d, coef, out, acc, s);
    }
    if (!c->ws_side.reserve(fold_side_bytes(M, fold_len, halo ? halo : n, 0, 0)))
        return hipErrorOutOfMemory;
    e = launch_fold(A, B, M, fold_len, halo ? halo : n, c->ws_side.ptr, c->ws_side.cap, s);
    if (e != hipSuccess) return e;
    e = bitonic_sort(B, M, 0, 0, s, L);  // the fold copies the pads past fold_len
    if (e == hipSuccess) e = launch_extract(B, d, coef, out, acc, s);
    return e;
}

// `advanced` of n clients' records into out[d] un-averaged (coef 1, overwrite): one
// batch sum of alg 6 (advanced.rs:10-21), on the current device's scratch
hipError_t advanced_batch(const void *rec, size_t n, size_t k, size_t d, size_t halo, float *out,
                          uint32_t *status, hipStream_t s) {
    DeviceCtx *c = current_ctx();
    if (!c) return hipErrorInvalidDevice;
    fltee_device_opts o;
    std::memset(&o, 0, sizeof o);
    if (!reserve_plan(c, plan_for(FLTEE_ALG_ADVANCED, n, k, d, o))) return hipErrorOutOfMemory;
    return run_advanced(c, rec, n, k, d, k, halo, 1.0f, out, false, status, s);
}

fltee_status_t aggregate(uint32_t alg, const void *rec, size_t n, size_t k, size_t d, float *out,
                         const fltee_device_opts &o, hipStream_t s, uint32_t *status) {
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_UNEXPECTED;
    if (n == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    if (n * k + d >= ((size_t)1 << 31)) return FLTEE_ERROR_INVALID_PARAMETER;  // 32-bit positions
    // the networks address records with 32-bit byte offsets: arrays of <= 2^29 records
    // (k_bitonic.hip, k_compact.hip); refuse larger ones before reserving scratch
    constexpr size_t kMaxNet = (size_t)1 << 29;
    if ((alg == FLTEE_ALG_ADVANCED && next_pow2_sz(n * k + d) > kMaxNet) ||
        (alg == FLTEE_ALG_OPTIMIZED &&
         next_pow2_sz((o.batch && o.batch < n ? o.batch : n) * k + d) > kMaxNet) ||
        (alg == FLTEE_ALG_NON_OBLIVIOUS && !(o.flags & FLTEE_OPT_DENSE) &&
         !use_scatter_rows(n, k, d) && next_pow2_sz(n * k) > kMaxNet))
        return FLTEE_ERROR_INVALID_PARAMETER;
    // the tree Path ORAM: a shape outside oram_fits is refused before any scratch is sized
    // for it (the ECALL gates the tree on the same predicate and takes the sweep instead)
    const bool tree = alg == FLTEE_ALG_PATH_ORAM && (o.flags & FLTEE_OPT_ORAM_TREE);
    if (tree && !oram_fits(n * k, d, (o.flags & FLTEE_OPT_ORAM_LAZY) != 0))
        return FLTEE_ERROR_INVALID_PARAMETER;
    if ((alg == FLTEE_ALG_BASELINE || (alg == FLTEE_ALG_PATH_ORAM && !tree)) &&
        !(o.flags & FLTEE_OPT_DENSE) && flat_ordered(n, k, d) && next_pow2_sz(n * k) > kMaxNet)
        return FLTEE_ERROR_INVALID_PARAMETER;
    if (alg == FLTEE_ALG_NIPS19) {
        const size_t kq = (o.flags & FLTEE_OPT_K_REQ) ? o.k_req : k;
        const size_t tf = f32_to_usize_sat(nips19_threshold(d, kq, n));
        if (tf > ((size_t)1 << 31) / (d ? d : 1) || next_pow2_sz(n * k + d * tf) > kMaxNet)
            return FLTEE_ERROR_INVALID_PARAMETER;
    }
    const bool dense = (o.flags & FLTEE_OPT_DENSE) != 0;
    if (dense && k != d) return FLTEE_ERROR_INVALID_PARAMETER;
    const bool acc = (o.flags & FLTEE_OPT_ACCUMULATE) != 0;
    const size_t n_avg = o.n_avg ? o.n_avg : n;
    const float coef = (o.flags & FLTEE_OPT_NO_AVERAGE) ? 1.0f : 1.0f / (float)n_avg;
    const Plan p = plan_for(alg, n, k, d, o);
    if (!reserve_plan(c, p)) return FLTEE_ERROR_OUT_OF_MEMORY;

    // per-client L2 clip (update.py:187-204), off by default
    const float *ccoef = nullptr;
    if (o.flags & FLTEE_OPT_CLIP) {
        float *cf = (float *)c->ws_coef.ptr;
        if (launch_client_clip_coef(rec, n, k, o.clipping, cf, s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
        ccoef = cf;
        if (!dense || tree) {  // plan_for reserved ws_rec on the same predicate
            if (fl_memcpy_async(c->ws_rec.ptr, rec, n * k * 8, hipMemcpyDeviceToDevice, s) != hipSuccess ||
                launch_apply_clip(c->ws_rec.ptr, n, k, cf, s) != hipSuccess)
                return FLTEE_ERROR_UNEXPECTED;
            rec = c->ws_rec.ptr;
        }
    }

    hipError_t e = hipSuccess;
    switch (alg) {
    case FLTEE_ALG_PATH_ORAM:
        if (tree) {  // the tree Path ORAM (k_oram.hip); oram_fits checked above
            const bool lazy = (o.flags & FLTEE_OPT_ORAM_LAZY) != 0;
            const size_t ns = oram_slots(d);
            uint8_t *tree = (uint8_t *)c->ws_oram.ptr;
            uint64_t *recs = lazy ? (uint64_t *)(tree + ns * 16) : nullptr;
            const uint64_t seed = o.seed ? o.seed : next_seed();
            e = launch_check_range(rec, n * k, (uint32_t)next_pow2_sz(d), status, s);  // oram.rs panics
            if (e == hipSuccess)
                e = launch_oram_tree(rec, n * k, d, lazy, tree, seed, (uint64_t *)c->ws_a.ptr,
                                     (uint64_t *)c->ws_b.ptr, recs, coef, acc, out, status, s);
            // lazy readout: every slot's (idx, value) through advanced's oblivious network
            // (one "client" of ns records: each index at most once, runs of <= 2 entries)
            if (e == hipSuccess && lazy) e = run_advanced(c, recs, 1, ns, d, ns, 1, coef, out, acc, status, s);
            break;
        }
        [[fallthrough]];
    case FLTEE_ALG_BASELINE:
    case FLTEE_ALG_NON_OBLIVIOUS:
        if (dense) {
            e = launch_dense_accumulate(rec, n, d, coef, out, ccoef, acc, status, s);
        } else if (alg == FLTEE_ALG_NON_OBLIVIOUS && use_scatter_rows(n, k, d)) {
            if (c->mat_clean_ptr != c->ws_mat.ptr || c->mat_clean_cap != c->ws_mat.cap) {
                c->mat_clean = 0;  // a new allocation: contents unknown
                c->mat_clean_ptr = c->ws_mat.ptr;
                c->mat_clean_cap = c->ws_mat.cap;
            }
            e = launch_scatter_sum(rec, n, k, d, (uint32_t *)c->ws_mat.ptr, &c->mat_clean,
                                   c->status + 16, coef, out, acc, status, s);
            if (e != hipSuccess) c->mat_clean = 0;  // the emptying pass may not have run
        } else if (alg == FLTEE_ALG_NON_OBLIVIOUS) {
            e = ordered_fold_records(c, rec, n * k, d, coef, out, acc, status, s);
        } else {
            // baseline / path_oram on sparse uploads: the ordered sweep (exact for any
            // upload, a client may repeat an index; fixed cost n*k*d compare-selects) —
            // or, for dense-sized uploads (flat_ordered), the composite-key network's
            // ordered fold (exact for any upload too).  Records with idx >= d are ignored
            // (o_update's compare never matches): the network's range flag goes to a
            // scratch word.
            if (alg == FLTEE_ALG_PATH_ORAM)  // oram.rs: blocks beyond next_pow2(d) do not exist
                e = launch_check_range(rec, n * k, (uint32_t)next_pow2_sz(d), status, s);
            if (e == hipSuccess && flat_ordered(n, k, d))
                e = ordered_fold_records(c, rec, n * k, d, coef, out, acc, c->status + 32, s, true);
            else if (e == hipSuccess)
                e = launch_sweep_accumulate(rec, n * k, d, coef, out, acc, s);
        }
        break;
    case FLTEE_ALG_ADVANCED: {
        const size_t k_req = (o.flags & FLTEE_OPT_K_REQ) ? o.k_req : k;
        const size_t fold_len = n * k_req + d;
        if (fold_len > n * k + d) return FLTEE_ERROR_INVALID_PARAMETER;  // advanced.rs:72 panic
        e = run_advanced(c, rec, n, k, d, k_req, o.fold_halo, coef, out, acc, status, s);
        break;
    }
    case FLTEE_ALG_OPTIMIZED: {
        const size_t batch = o.batch ? o.batch : n;
        if (!acc) e = fl_memset_async(out, 0, d * 4, s);
        for (size_t c0 = 0; e == hipSuccess && c0 < n; c0 += batch) {
            const size_t nb = (c0 + batch < n) ? batch : n - c0;
            e = run_advanced(c, (const uint8_t *)rec + c0 * k * 8, nb, k, d, k, o.fold_halo, 1.0f,
                             out, true, status, s);
        }
        if (e == hipSuccess && coef != 1.0f) e = launch_scale(out, d, coef, s);
        break;
    }
    case FLTEE_ALG_NIPS19: {
        // nips19.rs:38 takes T and the Laplace scale from the REQUEST's
        // num_of_sparse_parameters (0 for fl_main.py's dense uploads), not the payload
        const size_t kq = (o.flags & FLTEE_OPT_K_REQ) ? o.k_req : k;
        const float T = nips19_threshold(d, kq, n);
        const size_t tf = f32_to_usize_sat(T);
        const size_t L = n * k + d * tf, M = next_pow2_sz(L);
        if (L >= ((size_t)1 << 31) || M > kMaxNet) return FLTEE_ERROR_INVALID_PARAMETER;
        const uint64_t seed = o.seed ? o.seed : next_seed();
        uint32_t *r = (uint32_t *)c->ws_r.ptr;
        uint64_t *A = (uint64_t *)c->ws_a.ptr;
        e = launch_laplace_r(d, kq, T, seed, r, s);
        const uint32_t key = (uint32_t)(seed ^ (seed >> 32));
        bool done = false;
        if (e == hipSuccess && g_nips19_fused_select) {  // build + shuffle + select fused
            e = nips19_shuffle_aggregate(c, A, M, key, rec, n * k, r, d, tf, coef, out, acc,
                                         status, s);
            done = e != hipErrorNotSupported;
            if (!done) e = hipSuccess;
        }
        if (e == hipSuccess && !done) {  // build fused into the shuffle's first pass where it can be
            e = bitonic_sort_nips19(A, M, key, rec, n * k, r, d, tf, s);
            if (e == hipErrorNotSupported) {
                e = launch_nips19_build(rec, n * k, r, d, tf, M, A, s);
                if (e == hipSuccess) e = bitonic_sort(A, M, 2, key, s, L);
            }
            if (e == hipSuccess) e = safe_aggregate_ordered(c, A, M, d, coef, out, acc, status, s);
        }
        break;
    }
    default:
        return FLTEE_ERROR_INVALID_PARAMETER;  // lib.rs:396 panics on unknown algs
    }
    if (e == hipSuccess && (o.flags & FLTEE_OPT_DP)) {
        const uint64_t seed = o.seed ? o.seed : next_seed();
        e = launch_dp_noise(out, d, o.sigma, o.clipping, n_avg, seed, s);
    }
    if (e != hipSuccess)
        std::fprintf(stderr, "[fltee] aggregate(alg %u, n %zu, k %zu, d %zu): %s\n", alg, n, k, d,
                     hipGetErrorString(e));
    return e == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}

size_t workspace_bytes(uint32_t alg, size_t n, size_t k, size_t d, const fltee_device_opts &o) {
    const Plan p = plan_for(alg, n, k, d, o);
    return p.a_bytes + p.b_bytes + p.mat_bytes + p.r_bytes + p.coef_bytes + p.rec_bytes +
           p.keys_bytes + p.radix_bytes + p.oram_bytes + p.side_bytes + p.lb_bytes;
}

bool reserve(uint32_t alg, size_t n, size_t k, size_t d, const fltee_device_opts &o) {
    DeviceCtx *c = current_ctx();
    return c && reserve_plan(c, plan_for(alg, n, k, d, o));
}

}  // namespace fltee

// ============================================================ C ABI =========
using namespace fltee;

static fltee_device_opts default_opts() {
    fltee_device_opts o;
    std::memset(&o, 0, sizeof o);
    return o;
}

extern "C" fltee_status_t fltee_aggregate_device(uint32_t alg, const void *d_records, size_t n,
                                                 size_t k, size_t d, float *d_out,
                                                 const fltee_device_opts *opts, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    const fltee_device_opts o = opts ? *opts : default_opts();
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_UNEXPECTED;
    uint32_t *status = o.d_status ? o.d_status : c->status;
    hipStream_t s = (hipStream_t)stream;
    if (!o.d_status && fl_memset_async(c->status, 0, 4, s) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    return aggregate(alg, d_records, n, k, d, d_out, o, s, status);
}

extern "C" size_t fltee_workspace_bytes(uint32_t alg, size_t n, size_t k, size_t d,
                                        const fltee_device_opts *opts) {
    const fltee_device_opts o = opts ? *opts : default_opts();
    return workspace_bytes(alg, n, k, d, o);
}

extern "C" fltee_status_t fltee_reserve(uint32_t alg, size_t n, size_t k, size_t d,
                                        const fltee_device_opts *opts) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    const fltee_device_opts o = opts ? *opts : default_opts();
    return reserve(alg, n, k, d, o) ? FLTEE_SUCCESS : FLTEE_ERROR_OUT_OF_MEMORY;
}

extern "C" fltee_status_t fltee_device_status(void *stream, uint32_t *status) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c || !status) return FLTEE_ERROR_UNEXPECTED;
    hipStream_t s = (hipStream_t)stream;
    if (fl_stream_sync(s) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    if (fl_memcpy(status, c->status, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    if (fl_memset(c->status, 0, 4) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    return FLTEE_SUCCESS;
}

extern "C" fltee_status_t fltee_bitonic_device(void *d_records, size_t m, uint32_t mode,
                                               uint32_t seed, void *stream) {
    if (m & (m - 1)) return FLTEE_ERROR_INVALID_PARAMETER;
    if (m >= ((size_t)1 << 31)) return FLTEE_ERROR_INVALID_PARAMETER;
    return bitonic_sort((uint64_t *)d_records, m, mode, seed, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_fold_device(const void *d_src, void *d_dst, size_t m,
                                            size_t fold_len, size_t halo, uint32_t *d_status,
                                            void *stream) {
    if (fold_len == 0 || fold_len > m || !d_status) return FLTEE_ERROR_INVALID_PARAMETER;
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c || !c->ws_side.reserve(fold_side_bytes(m, fold_len, halo, 0, 0)))
        return FLTEE_ERROR_OUT_OF_MEMORY;
    return launch_fold((const uint64_t *)d_src, (uint64_t *)d_dst, m, fold_len, halo,
                       c->ws_side.ptr, c->ws_side.cap, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_INVALID_PARAMETER;
}

extern "C" fltee_status_t fltee_laplace_r_device(size_t d, size_t k, size_t n, uint64_t seed,
                                                 uint32_t *d_r, float *T_out, void *stream) {
    if (n == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    const float T = nips19_threshold(d, k, n);
    if (T_out) *T_out = T;
    return launch_laplace_r(d, k, T, seed, d_r, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

// ---- position-range pieces of `advanced` (SURVEY §8e Option B) ----------
static bool range_ok(size_t m, size_t pos_base) {
    return m >= 2 && !(m & (m - 1)) && pos_base % m == 0 && pos_base + m <= ((size_t)1 << 31);
}

extern "C" fltee_status_t fltee_advanced_init_range_device(const void *d_records, size_t nrec,
                                                           size_t d, size_t pos_base, size_t m,
                                                           void *d_dst, void *stream) {
    return launch_advanced_init_range(d_records, nrec, d, pos_base, m, (uint64_t *)d_dst,
                                      (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_bitonic_range_sort_device(void *d_records, size_t m,
                                                          size_t pos_base, uint32_t mode,
                                                          uint32_t seed, void *stream) {
    if (!range_ok(m, pos_base)) return FLTEE_ERROR_INVALID_PARAMETER;
    return bitonic_sort_range((uint64_t *)d_records, m, mode, seed, (uint32_t)pos_base,
                              (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_bitonic_range_sort_padded_device(void *d_records, size_t m,
                                                                 size_t pos_base, size_t valid,
                                                                 uint32_t mode, uint32_t seed,
                                                                 void *stream) {
    if (!range_ok(m, pos_base)) return FLTEE_ERROR_INVALID_PARAMETER;
    if (valid == 0) return FLTEE_SUCCESS;  // pads alone: sorted as they are
    return bitonic_sort_range((uint64_t *)d_records, m, mode, seed, (uint32_t)pos_base,
                              (hipStream_t)stream, valid >= m ? 0u : (uint32_t)valid) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_bitonic_range_merge_device(void *d_records, size_t m,
                                                           size_t pos_base, uint32_t mode,
                                                           uint32_t seed, uint32_t stage_log,
                                                           void *stream) {
    if (!range_ok(m, pos_base) || ((size_t)1 << stage_log) <= m || stage_log > 31)
        return FLTEE_ERROR_INVALID_PARAMETER;
    return bitonic_merge_range((uint64_t *)d_records, m, mode, seed, stage_log,
                               (uint32_t)pos_base, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_bitonic_range_exchange_device(void *d_mine, const void *d_theirs,
                                                              size_t m, size_t pos_mine,
                                                              size_t pos_theirs, uint32_t mode,
                                                              uint32_t seed, uint32_t stage_log,
                                                              void *stream) {
    if (!range_ok(m, pos_mine) || !range_ok(m, pos_theirs) || stage_log > 31)
        return FLTEE_ERROR_INVALID_PARAMETER;
    const size_t j = pos_mine > pos_theirs ? pos_mine - pos_theirs : pos_theirs - pos_mine;
    if ((j & (j - 1)) || j < m || j >= ((size_t)1 << stage_log) || (pos_mine ^ pos_theirs) != j)
        return FLTEE_ERROR_INVALID_PARAMETER;
    return bitonic_exchange((uint64_t *)d_mine, (const uint64_t *)d_theirs, m, (uint32_t)pos_mine,
                            (uint32_t)pos_theirs, mode, seed, stage_log, log2_pow2(j),
                            (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_bitonic_range_steps_device(void *d_records, size_t m,
                                                           size_t pos_base, uint32_t mode,
                                                           uint32_t seed, uint32_t stage_log,
                                                           uint32_t step_top, uint32_t step_bot,
                                                           void *stream) {
    if (!range_ok(m, pos_base) || stage_log > 31 || step_bot > step_top ||
        step_top >= stage_log || ((size_t)1 << step_top) >= m)
        return FLTEE_ERROR_INVALID_PARAMETER;
    return bitonic_steps_range((uint64_t *)d_records, m, mode, seed, stage_log, step_top,
                               step_bot, (uint32_t)pos_base, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" size_t fltee_fold_context(size_t halo) { return fold_context(halo); }

extern "C" size_t fltee_fold_side_bytes(size_t span, size_t halo) {
    return fold_side_bytes(span, (size_t)1 << 62, halo, 1, 1);
}

extern "C" fltee_status_t fltee_fold_range_device(const void *d_src, void *d_dst, size_t m,
                                                  size_t origin, size_t end, int64_t pos_base,
                                                  size_t fold_len, size_t halo, void *d_side,
                                                  void *stream) {
    // range mode: [0, origin) holds >= fold_context(halo) + 1 records of context
    if (!d_side || origin < fold_context(halo) + 1 || end > m || origin >= end || (origin & 1) ||
        (end & 1) || (m & 1))
        return FLTEE_ERROR_INVALID_PARAMETER;
    if (end < m ? false : (int64_t)end + pos_base < (int64_t)fold_len)
        return FLTEE_ERROR_INVALID_PARAMETER;  // needs the next range's first record
    return launch_fold_range((const uint64_t *)d_src, (uint64_t *)d_dst, m, origin, end,
                             (long long)pos_base, fold_len, halo, (FoldSide *)d_side,
                             (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_fold_range_total_device(const void *d_side, size_t span,
                                                        size_t halo, void *d_total, void *stream) {
    if (!d_side || !d_total) return FLTEE_ERROR_INVALID_PARAMETER;
    const size_t lanes = fold_lanes(span, (size_t)1 << 62, halo, 1, 1);
    return launch_fold_range_total((const FoldSide *)d_side, lanes, (FoldAgg *)d_total,
                                   (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_fold_range_patch_device(void *d_dst, size_t origin, size_t end,
                                                        int64_t pos_base, size_t fold_len,
                                                        size_t halo, const void *d_side,
                                                        const void *d_prev_totals, size_t n_prev,
                                                        void *stream) {
    if (!d_dst || !d_side || origin >= end || (n_prev && !d_prev_totals))
        return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_fold_range_patch((uint64_t *)d_dst, end - origin, origin, (long long)pos_base,
                                   fold_len, halo, (const FoldSide *)d_side,
                                   (const FoldAgg *)d_prev_totals, n_prev, (hipStream_t)stream) ==
                   hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_compact_range_device(const void *d_chunk, size_t c, size_t d,
                                                     void *d_buf, void *d_tmp, float coef,
                                                     float *d_out, void *stream) {
    if (d + c >= ((size_t)1 << 29)) return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_compact_offset((const uint64_t *)d_chunk, c, d, (uint64_t *)d_buf,
                                 (uint64_t *)d_tmp, coef, d_out, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_nips19_build_range_device(const void *d_records, size_t nrec,
                                                          const uint32_t *d_r, size_t d,
                                                          size_t tf, size_t pos_base, size_t m,
                                                          void *d_dst, void *stream) {
    if (nrec + d * tf >= ((size_t)1 << 31)) return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_nips19_build_range(d_records, nrec, d_r, d, tf, pos_base, m, (uint64_t *)d_dst,
                                     (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_safe_aggregate_device(const void *d_src, size_t m, size_t d,
                                                      float *d_out, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_UNEXPECTED;
    if (m >= ((size_t)1 << 31)) return FLTEE_ERROR_INVALID_PARAMETER;
    return safe_aggregate_ordered(c, (const uint64_t *)d_src, m, d, 1.0f, d_out, false, c->status,
                                  (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

// safe_aggregate split for position ranges (nips19 over several GPUs): each range's
// entries with idx < d in position order, then the ordered fold of their concatenation
// in range order on the root — the one-GPU result bit for bit.
extern "C" fltee_status_t fltee_select_device(const void *d_src, size_t m, size_t d, void *d_list,
                                              size_t cap, size_t *count, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c || !count || m >= ((size_t)1 << 31)) return FLTEE_ERROR_INVALID_PARAMETER;
    hipStream_t s = (hipStream_t)stream;
    *count = 0;
    if (m == 0 || d == 0) return FLTEE_SUCCESS;
    const size_t nb = select_tiles(m);
    if (!c->ws_cnt.reserve((2 * nb + 2) * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
    uint32_t *cnt = (uint32_t *)c->ws_cnt.ptr, *base = cnt + nb + 1;
    size_t lc = 0;
    if (launch_select_count((const uint64_t *)d_src, m, d, cnt, base, s) != hipSuccess ||
        read_device_word(c, base + nb, &lc, s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    *count = lc;
    if (lc > cap || (lc && !d_list)) return FLTEE_ERROR_INVALID_PARAMETER;  // caller grows the list
    if (lc && launch_select_write((const uint64_t *)d_src, m, d, base, (uint64_t *)d_list, s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    return FLTEE_SUCCESS;
}

extern "C" fltee_status_t fltee_ordered_list_device(const void *d_list, size_t lc, size_t d,
                                                    float coef, float *d_out, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c || lc >= ((size_t)1 << 29)) return FLTEE_ERROR_INVALID_PARAMETER;
    if (d == 0) return FLTEE_SUCCESS;
    return ordered_from_list(c, (const uint64_t *)d_list, lc, d, coef, d_out, false, c->status,
                             (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" void fltee_debug_set_seed(uint64_t seed) { set_debug_seed(seed); }

// test hook: the launch trace (common.h).  on = 1 clears it and starts recording, 0 stops.
extern "C" void fltee_debug_trace(int on) {
    std::lock_guard<std::mutex> lk(fltee::g_trace_mu);
    if (on) {
        fltee::g_trace_text.clear();
        fltee::g_trace_lines = 0;
    }
    fltee::g_trace.store(on != 0);
}

// the trace so far as text (one line per event: what|site|a|b|c); returns its length
// (copies at most cap - 1 bytes and a NUL into buf when buf is given)
extern "C" size_t fltee_debug_trace_text(char *buf, size_t cap) {
    std::lock_guard<std::mutex> lk(fltee::g_trace_mu);
    const std::string &t = fltee::g_trace_text;
    if (buf && cap) {
        const size_t n = t.size() < cap - 1 ? t.size() : cap - 1;
        std::memcpy(buf, t.data(), n);
        buf[n] = 0;
    }
    return t.size();
}

// the planned network schedule (k_bitonic.hip plan_network), 8 words per launch
extern "C" size_t fltee_debug_network_plan(uint32_t mlog, uint32_t tlog, uint32_t nt, int rmax,
                                           uint32_t *out, size_t cap) {
    return fltee::debug_plan(mlog, tlog, nt, rmax, out, cap);
}

// the pad-only units a network launch skips (k_bitonic.hip pad_units): {live, hole_at, hole_len}
extern "C" void fltee_debug_pad_units(uint32_t mode, uint32_t valid, uint32_t mlog, uint32_t pbase,
                                      uint32_t ilog, uint32_t jstep, uint32_t sblog, uint32_t uplog,
                                      uint32_t *out) {
    fltee::debug_pad_units(mode, valid, mlog, pbase, ilog, jstep, sblog, uplog, out);
}

// measurement hook: streaming passes launched and the bytes they sweep since the last reset
extern "C" void fltee_debug_net_stats(uint64_t *launches, uint64_t *bytes, int reset) {
    if (launches) *launches = fltee::g_net_launches.load();
    if (bytes) *bytes = fltee::g_net_bytes.load();
    if (reset) {
        fltee::g_net_launches.store(0);
        fltee::g_net_bytes.store(0);
    }
}

// measurement hook: per-launch log of the accounted launches.  on = 1 clears the log and
// starts recording (an event on the launch's stream before each accounted launch); on = 0
// records the final event on `stream` (after the last launch of the timed call) and stops.
extern "C" void fltee_debug_net_timing(int on, void *stream) {
    std::lock_guard<std::mutex> lk(fltee::g_net_mu);
    if (on) {
        fltee::net_log_clear();
        fltee::g_net_timing.store(true);
        return;
    }
    fltee::g_net_timing.store(false);
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) == hipSuccess) {
        if (hipEventRecord(e, (hipStream_t)stream) == hipSuccess)
            fltee::g_net_log.push_back({nullptr, 0, e});
        else
            (void)hipEventDestroy(e);
    }
}

// entry i of the log (the caller has synchronised the stream): kernel name, launch-side
// bytes and the time to the next entry's event (ms).  Returns the number of launches
// logged (the final event not counted); i past it fills nothing.
extern "C" size_t fltee_debug_net_log(size_t i, char *name, size_t name_cap, uint64_t *bytes,
                                      float *ms) {
    std::lock_guard<std::mutex> lk(fltee::g_net_mu);
    const auto &L = fltee::g_net_log;
    const size_t nl = L.empty() ? 0 : (L.back().kernel ? L.size() : L.size() - 1);
    if (i < nl) {
        if (name && name_cap) {
            std::snprintf(name, name_cap, "%s", L[i].kernel ? L[i].kernel : "");
        }
        if (bytes) *bytes = L[i].bytes;
        if (ms) {
            *ms = -1.0f;
            if (i + 1 < L.size()) (void)hipEventElapsedTime(ms, L[i].ev, L[i + 1].ev);
        }
    }
    return nl;
}

extern "C" fltee_status_t fltee_sum_rows_device(const float *d_rows, size_t nrows, size_t d,
                                                float coef, float *d_out, void *stream) {
    if (nrows == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_rows_accumulate(d_rows, nrows, d, coef, d_out, false, (hipStream_t)stream) ==
                   hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_dp_noise_device(float *d_out, size_t d, float sigma,
                                                float clipping, size_t n, uint64_t seed,
                                                void *stream) {
    if (n == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_dp_noise(d_out, d, sigma, clipping, n, seed ? seed : next_seed(),
                           (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

namespace fltee {
void set_dense_variant(int v); void set_compact_variant(int v); void set_fold_compact(int on);
hipError_t launch_read_floor(const void *src, size_t bytes, uint32_t *sink, unsigned blocks, hipStream_t s);
}
// measurement hook (bench.py): a plain streaming read of `bytes` (16-B multiple) of d_src;
// d_sink: `blocks` words
extern "C" int fltee_debug_read_floor(const void *d_src, size_t bytes, void *d_sink, unsigned blocks,
                                      void *stream) {
    return fltee::launch_read_floor(d_src, bytes, (uint32_t *)d_sink, blocks, (hipStream_t)stream) ==
                   hipSuccess ? 0 : 1;
}
// tuning hook (not part of the public header)
extern "C" void fltee_debug_set_dense_variant(int v) { fltee::set_dense_variant(v); }
// A/B hook: 0 runs advanced's second bitonic sort instead of the compaction network
extern "C" void fltee_debug_set_advanced_compaction(int on) { fltee::g_advanced_compaction = on != 0; }
extern "C" void fltee_debug_set_compact_variant(int v) { fltee::set_compact_variant(v); }
// A/B hook: 0 runs advanced's fold as its own pass before the compaction
extern "C" void fltee_debug_set_fold_compact(int on) { fltee::set_fold_compact(on); }
// A/B hook: 0 runs the networks over the pad-only stage blocks too
extern "C" void fltee_debug_set_pad_skip(int on) { fltee::set_pad_skip(on); }
extern "C" void fltee_debug_set_radix_order(int on) { fltee::set_radix_order(on); }
extern "C" void fltee_set_path_oram_tree(int on) {
    std::lock_guard<std::recursive_mutex> lk(fltee::api_mutex());
    fltee::set_oram_tree(on);
}
extern "C" void fltee_set_advanced_exact_runs(int on) {
    std::lock_guard<std::recursive_mutex> lk(fltee::api_mutex());
    fltee::set_exact_runs(on);
}
// test hook: blocks a bucket of the tree ORAM takes on eviction (4; 0 forces the stash)
extern "C" void fltee_debug_set_oram_bucket(int z) {
    std::lock_guard<std::recursive_mutex> lk(fltee::api_mutex());
    fltee::set_oram_bucket(z);
}
extern "C" void fltee_debug_set_aes_variant(int v) {
    std::lock_guard<std::recursive_mutex> lk(fltee::api_mutex());
    fltee::set_aes_variant(v);
}
extern "C" void fltee_debug_set_swizzle(int on) { fltee::set_swizzle(on); }
extern "C" void fltee_debug_set_fused_init(int on) { fltee::set_fused_init(on); }
// A/B hook: 0 writes nips19's shuffled array out and selects in separate passes
extern "C" void fltee_debug_set_nips19_fused_select(int on) { fltee::g_nips19_fused_select = on != 0; }
// test hook: the fused-producer sort alone (gen 1: advanced, 2: nips19 with key seed),
// into d_data[0, m); INVALID_PARAMETER when m is too small to fuse
extern "C" fltee_status_t fltee_debug_sort_fused(uint32_t gen, void *d_data, size_t m,
                                                 const void *d_rec, size_t nrec, const uint32_t *d_r,
                                                 size_t d, size_t tf, uint32_t seed, void *stream) {
    if (!d_data || (nrec && !d_rec) || (gen == 2 && d && tf && !d_r)) return FLTEE_ERROR_INVALID_PARAMETER;
    hipError_t e;
    if (gen == 1) e = fltee::bitonic_sort_advanced((uint64_t *)d_data, m, d_rec, nrec, d, (hipStream_t)stream);
    else if (gen == 2)
        e = fltee::bitonic_sort_nips19((uint64_t *)d_data, m, seed, d_rec, nrec, d_r, d, tf, (hipStream_t)stream);
    else return FLTEE_ERROR_INVALID_PARAMETER;
    if (e == hipErrorNotSupported || e == hipErrorInvalidValue) return FLTEE_ERROR_INVALID_PARAMETER;
    return e == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}
