// ecalls.hip — the four ECALLs of Enclave.edl on an MI355X (host side).
//
// State machine restated from secure_aggregation/enclave/src/lib.rs:
//   FL_CONFIG_MAP (lib.rs:83-91, fl_config.rs)      -> g_cfg
//   SESSION_KEYS (lib.rs:93-101, session_key_store) -> g_keys (id set; the key is
//                                                      a pure function of the id)
//   single TCS (Enclave.config.xml:6)               -> api_mutex()
// The data path runs on the eid's GPU: "Loading" = H2D of the ciphertext,
// "Decryption" = AES-128-CTR kernel, "Aggregation" = engine.hip + DP noise.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <vector>

#include "common.h"
#include "engine.h"
#include "group.h"

namespace fltee {

std::recursive_mutex &api_mutex() {
    static std::recursive_mutex mu;
    return mu;
}

struct FLConfig {  // fl_config.rs:29-44
    std::vector<uint32_t> client_ids;
    size_t d = 0, k = 0;
    float sigma = 0, clipping = 0, alpha = 0, ratio = 0;
    uint32_t alg = 0, round = 0;
    uint8_t verbose = 0, dp = 0;
    std::set<uint32_t> sampled;  // current_sampled_clients (HashSet)
};

static std::map<uint32_t, FLConfig> g_cfg;
static std::set<uint32_t> g_keys;
static bool g_have_keys = false;
static std::vector<int> g_eid_dev;  // eid - 1 -> hip device (a group's root device)
static std::map<fltee_eid_t, Group *> g_groups;  // eids from fltee_device_init_multi

static Group *group_of(fltee_eid_t eid) {
    auto it = g_groups.find(eid);
    return it == g_groups.end() ? nullptr : it->second;
}

void aes128_expand_key(const uint8_t key[16], uint32_t rk[44]);

static inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static size_t f32_to_usize_sat(float x) {
    if (!(x > 0.0f)) return 0;
    if (x >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)x;
}

// sgx_rand::sample reservoir (common.rs:101-105) driven by Philox4x32-10.
static void sample_client_ids(const std::vector<uint32_t> &ids, size_t amount, uint64_t seed,
                              std::vector<uint32_t> &out) {
    const size_t take = std::min(amount, ids.size());
    out.assign(ids.begin(), ids.begin() + take);
    if (take != amount) return;
    uint64_t counter = 0;
    auto draw = [&]() {
        uint32_t c[4] = {(uint32_t)counter, (uint32_t)(counter >> 32), 0u, FLTEE_STREAM_SAMPLE};
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        ++counter;
        return ((uint64_t)c[1] << 32) | c[0];
    };
    for (size_t i = 0; i + amount < ids.size(); ++i) {
        const uint64_t range = (uint64_t)(i + 1 + amount);
        const uint64_t zone = UINT64_MAX - UINT64_MAX % range;
        uint64_t v;
        do { v = draw(); } while (v >= zone);
        const uint64_t kk = v % range;
        if (kk < amount) out[kk] = ids[amount + i];
    }
}

static DeviceCtx *eid_ctx(fltee_eid_t eid) {
    if (eid == 0 || eid > g_eid_dev.size() || g_eid_dev[eid - 1] < 0) return nullptr;
    const int dev = g_eid_dev[eid - 1];
    if (hipSetDevice(dev) != hipSuccess) return nullptr;
    DeviceCtx *c = device_ctx(dev);
    if (c && !c->stream) {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
        for (int i = 0; i < DeviceCtx::kCopyEvents; ++i)
            if (hipEventCreateWithFlags(&c->copy_ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
    }
    return c;
}

static uint32_t check_uploaded(const FLConfig &cfg, const uint32_t *ids, size_t n) {
    if (n != cfg.sampled.size()) {  // lib.rs:269-272
        std::printf("[VERIFICATION ERROR] Uploaded client id is not matched for secure sampled one.\n");
        return FLTEE_ERROR_INVALID_PARAMETER;
    }
    for (size_t i = 0; i < n; ++i)
        if (!cfg.sampled.count(ids[i])) {
            std::printf("[VERIFICATION ERROR] Uploaded client id is not matched for secure sampled one.\n");
            return FLTEE_ERROR_INVALID_PARAMETER;
        }
    return FLTEE_SUCCESS;
}

// AES-128 round keys of the n clients' session keys (session_key_store.rs:21-22)
static void client_round_keys(const uint32_t *ids, size_t n, std::vector<uint32_t> &rk) {
    rk.resize(n * 44);
    aes128_session_round_keys(ids, n, rk.data());
}

// H2D + GPU AES-CTR decrypt of n slices of bpc bytes -> c->records (n * (bpc/8) records)
// Loading + decryption (lib.rs:285-343), pipelined: the ciphertext crosses PCIe in
// client chunks of ~64 MB on the copy stream, and each chunk's AES-CTR kernel runs on
// the ECALL stream as soon as its copy lands, under the next chunk's copy.  Timers
// (execution_time_results[0..1]): t_load = until the last chunk has landed; t_dec =
// the decryption left after it (the part not hidden under the copies).
constexpr size_t kLoadChunkBytes = (size_t)64 << 20;

static uint32_t load_and_decrypt(DeviceCtx *c, const uint32_t *ids, size_t n, const uint8_t *enc,
                                 size_t bpc, float *t_load, float *t_dec) {
    const size_t rpc = bpc / 8;
    const double t0 = now_s();
    if (!c->cipher.reserve(n * bpc) || !c->records.reserve(n * rpc * 8) ||
        !c->round_keys.reserve(n * 44 * 4))
        return FLTEE_ERROR_OUT_OF_MEMORY;
    std::vector<uint32_t> rk;
    client_round_keys(ids, n, rk);
    if (fl_memcpy_async(c->round_keys.ptr, rk.data(), rk.size() * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    size_t per = bpc ? kLoadChunkBytes / bpc : n;
    if (per == 0) per = 1;
    if ((n + per - 1) / per > (size_t)DeviceCtx::kCopyEvents) per = (n + DeviceCtx::kCopyEvents - 1) / DeviceCtx::kCopyEvents;
    const uint8_t *cipher = (const uint8_t *)c->cipher.ptr;
    int ev = 0;
    for (size_t c0 = 0; c0 < n && bpc; c0 += per, ++ev) {
        const size_t nc = c0 + per < n ? per : n - c0;
        if (fl_memcpy_async((uint8_t *)c->cipher.ptr + c0 * bpc, enc + c0 * bpc, nc * bpc,
                           hipMemcpyHostToDevice, c->copy_stream) != hipSuccess ||
            hipEventRecord(c->copy_ev[ev], c->copy_stream) != hipSuccess ||
            hipStreamWaitEvent(c->stream, c->copy_ev[ev], 0) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
        if (launch_aes_ctr(cipher + c0 * bpc, nc, bpc, rpc, (const uint32_t *)c->round_keys.ptr + c0 * 44,
                           (uint8_t *)c->records.ptr + c0 * rpc * 8, c->stream) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (fl_stream_sync(c->copy_stream) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    const double t1 = now_s();
    if (t_load) *t_load = (float)(t1 - t0);
    // rk lives on this stack frame: the decrypt (and the key upload) must finish here
    if (fl_stream_sync(c->stream) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    if (t_dec) *t_dec = (float)(now_s() - t1);
    return FLTEE_SUCCESS;
}

static uint32_t read_status(DeviceCtx *c, uint32_t *st) {
    if (fl_memcpy_async(st, c->status, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        fl_stream_sync(c->stream) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    return FLTEE_SUCCESS;
}

// The options aggregate_records gives aggregate() for an ECALL's alg (shared with the
// staged path below).
static fltee_device_opts ecall_opts(uint32_t alg, size_t n, size_t rpc, size_t d, size_t k_req,
                                    size_t batch, uint64_t seed) {
    fltee_device_opts o;
    std::memset(&o, 0, sizeof o);
    o.k_req = k_req;
    o.flags |= FLTEE_OPT_K_REQ;
    o.batch = batch;
    const bool flat = alg == FLTEE_ALG_BASELINE || alg == FLTEE_ALG_PATH_ORAM ||
                      alg == FLTEE_ALG_NON_OBLIVIOUS;
    if (flat && rpc == d) o.flags |= FLTEE_OPT_DENSE;
    if (alg == FLTEE_ALG_PATH_ORAM && oram_tree_default() && oram_fits(n * rpc, d, false))
        o.flags |= FLTEE_OPT_ORAM_TREE;  // (a shape past the tree's bounds takes the sweep)
    if (alg == FLTEE_ALG_NIPS19) o.seed = seed ? seed : next_seed();
    // advanced's fold (advanced.rs:66-101) runs once with halo = n: bit for bit for every
    // run of up to n + 1 entries — every upload whose clients each send distinct indices
    // (n records + the initial entry) — and a run of more (some client repeated an index)
    // is finished by the fold's long-run carry in the same fixed-cost sequence (round 6,
    // k_fold.hip / k_compact.hip), its sum re-associated at the walk boundaries.  With the
    // exact-runs policy the halo is the public worst case (every record one index): one
    // sequential walk, bit for bit for any run.  Either way the cost is fixed by the
    // public sizes; no data-dependent relaunch.
    o.fold_halo = exact_runs_default() ? n * rpc + d : n;
    return o;
}

// What an ECALL returns for the device status word of one aggregate (aggregate_records'
// rules); *retry: a dense-sized upload out of position, to rerun sparse.
static uint32_t status_to_retval(uint32_t dev_st, uint32_t alg, bool *retry) {
    *retry = false;
    if (dev_st == 0) return FLTEE_SUCCESS;
    if (dev_st & FLTEE_DEV_ERR_INDEX_RANGE) return FLTEE_ERROR_INVALID_PARAMETER;
    if (dev_st & FLTEE_DEV_ERR_ORAM_STASH) return FLTEE_ERROR_UNEXPECTED;
    if (dev_st & FLTEE_DEV_ERR_DENSE_ORDER) {
        // a dense-sized upload (k = d) with a record out of position — not serialize_dense's
        // layout, e.g. fl_main.py --alpha 1.0, whose top-k orders the records by |val|.
        // Every flat alg reruns it sparse, with the reference's result for any upload:
        // non_oblivious by its scatter / ordered fold, baseline and path_oram by the
        // ordered fold in the composite-key network's order (engine.hip flat_ordered,
        // baseline.rs:28-60's upload order).  The rerun follows the upload's layout (one
        // bit: in position or not, the same for every round of a given client code), not
        // its values.
        (void)alg;
        *retry = true;
        return FLTEE_SUCCESS;
    }
    return FLTEE_ERROR_UNEXPECTED;
}

// Aggregate c->records (n clients x rpc records) with alg into the device out buffer,
// reading the status word back (one sync) and rerunning only where status_to_retval says.
static uint32_t aggregate_records(DeviceCtx *c, uint32_t alg, size_t n, size_t rpc, size_t d,
                                  size_t k_req, size_t batch, float *d_out, uint64_t seed = 0) {
    fltee_device_opts o = ecall_opts(alg, n, rpc, d, k_req, batch, seed);
    if (alg == FLTEE_ALG_OPTIMIZED) o.flags &= ~FLTEE_OPT_K_REQ;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (fl_memset_async(c->status, 0, 4, c->stream) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        uint32_t st = aggregate(alg, c->records.ptr, n, rpc, d, d_out, o, c->stream, c->status);
        if (st != FLTEE_SUCCESS) return st;
        uint32_t dev_st = 0;
        if (read_status(c, &dev_st)) return FLTEE_ERROR_UNEXPECTED;
        bool retry = false;
        st = status_to_retval(dev_st, alg, &retry);
        if (!retry) return st;
        o.flags &= ~FLTEE_OPT_DENSE;  // the sparse path: exact for any upload
    }
    return FLTEE_ERROR_INVALID_PARAMETER;
}

// Small calls (payload <= kStagedBytes) on one GPU with ONE host synchronisation. The
// round keys are computed straight into pinned memory and read from there by the AES-CTR
// kernel (which also zeroes the status word); the ciphertext is read the same way up to
// kZeroCopyBytes (one host memcpy into the pinned buffer; the kernel issues its loads
// before its rounds), and above that crosses in one DMA straight from the caller's
// buffer (the runtime's pageable path pipelines its own staging: 1.2 MB in 47 us against
// 67 us through a memcpy into our pinned buffer + a DMA, `profiles/r05/small_ecall/
// h2d_probe_r05l.jsonl`).  The aggregation follows on the stream, and the f32[d] output
// leaves with the device status word (it sits right after the output in HBM) through a
// copy kernel storing into pinned memory — then one stream sync.  The runtime's copy
// commands started ~10 us after the command before them in the kernel traces of small
// calls (`profiles/r05/small_ecall/`), so the small path avoids them.  The large-payload
// path (pageable 64 MB chunks with the decryption pipelined under the copies) pays a
// stream sync per phase.  Timers (execution_time_results, lib.rs:280-353): [0] = the
// host staging + the H2D (when there is one), [1] = the AES kernel (hipEvents), [2] =
// the rest of the call (alg 6: [1] = decrypt + aggregate, [2] = 0, lib.rs:425-592).
// alg: an ECALL alg, or FLTEE_ALG_OPTIMIZED with batch.
constexpr size_t kStagedBytes = (size_t)16 << 20;
constexpr size_t kZeroCopyBytes = (size_t)256 << 10;

__global__ __launch_bounds__(256) void copy_out_kernel(const uint4 *__restrict__ src,
                                                       uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        dst[i] = src[i];
}

static hipError_t launch_copy_out(const void *src, void *dst, size_t bytes, hipStream_t s) {
    const size_t n16 = (bytes + 15) / 16;  // both ends 16-B aligned, padded
    size_t blocks = (n16 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    FLTEE_LAUNCH(copy_out_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4 *)src,
                       (uint4 *)dst, n16);
    return hipGetLastError();
}

static uint32_t staged_ecall(DeviceCtx *c, uint32_t alg, const uint32_t *ids, size_t n,
                             const uint8_t *enc, size_t bpc, size_t d, size_t k_req, size_t batch,
                             uint64_t seed, const FLConfig &cfg, float *host_out, float *times) {
    const double t0 = now_s();
    const size_t rpc = bpc / 8;
    const size_t rkb = (n * 44 * 4 + 15) / 16 * 16, cb = n * bpc;
    const size_t d4 = (d * 4 + 15) / 16 * 16;
    const bool zero_copy = 16 + rkb + cb <= kZeroCopyBytes;
    // device [out: d4][status: 16][ciphertext: cb, DMA only]; pinned in [16][round keys:
    // rkb][ciphertext: cb, zero-copy only], pinned out [out: d4][status: 16]
    if (!c->stage.reserve(d4 + 16 + (zero_copy ? 0 : cb) + 16) ||
        !c->records.reserve(n * rpc * 8 + 16) ||
        !c->pin_in.reserve(16 + rkb + (zero_copy ? cb : 0) + 16) || !c->pin_out.reserve(d4 + 16))
        return FLTEE_ERROR_OUT_OF_MEMORY;
    for (int i = 0; i < 3; ++i)
        if (!c->call_ev[i] && hipEventCreate(&c->call_ev[i]) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    uint8_t *pin = (uint8_t *)c->pin_in.ptr;
    aes128_session_round_keys(ids, n, (uint32_t *)(pin + 16));  // session_key_store.rs:21-22
    if (cb && zero_copy) std::memcpy(pin + 16 + rkb, enc, cb);
    const double t1 = now_s();  // host staging done; the DMA (if any) is timed by events
    hipStream_t s = c->stream;
    uint8_t *stage = (uint8_t *)c->stage.ptr;
    float *d_out = (float *)stage;
    uint32_t *d_st = (uint32_t *)(stage + d4);
    const uint32_t *d_rk = (const uint32_t *)((const uint8_t *)c->pin_in.dptr + 16);
    const uint8_t *d_cipher = zero_copy ? (const uint8_t *)d_rk + rkb : stage + d4 + 16;
    // (no H2D to time on the zero-copy path: no marker in front of the first kernel)
    if ((!zero_copy && hipEventRecord(c->call_ev[0], s) != hipSuccess) ||
        (!zero_copy && fl_memcpy_async(stage + d4 + 16, enc, cb, hipMemcpyHostToDevice, s) != hipSuccess) ||
        (!cb && fl_memset_async(d_st, 0, 4, s) != hipSuccess))
        return FLTEE_ERROR_UNEXPECTED;
    fltee_device_opts o = ecall_opts(alg == FLTEE_ALG_OPTIMIZED ? FLTEE_ALG_ADVANCED : alg, n, rpc, d,
                                     k_req, batch, seed);
    if (alg == FLTEE_ALG_OPTIMIZED) o.flags &= ~FLTEE_OPT_K_REQ;
    // the call's device work: AES (timed by events) -> aggregation (-> DP) -> copy-out
    auto enqueue = [&](bool retry_pass) -> uint32_t {
        if (retry_pass && fl_memset_async(d_st, 0, 4, s) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        if (!retry_pass &&
            (hipEventRecord(c->call_ev[1], s) != hipSuccess ||
             (cb && launch_aes_ctr(d_cipher, n, bpc, rpc, d_rk, (uint8_t *)c->records.ptr, s, d_st) !=
                        hipSuccess) ||
             hipEventRecord(c->call_ev[2], s) != hipSuccess))
            return FLTEE_ERROR_UNEXPECTED;
        const uint32_t a = aggregate(alg, c->records.ptr, n, rpc, d, d_out, o, s, d_st);
        if (a != FLTEE_SUCCESS) return a;
        if (cfg.dp && launch_dp_noise(d_out, d, cfg.sigma, cfg.clipping, n, next_seed(), s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
        return launch_copy_out(d_out, c->pin_out.dptr, d4 + 16, s) == hipSuccess
                   ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
    };
    // (Round 5, measured and not kept: this device work captured once per call shape as a
    // graph and replayed with one launch — MLP-MNIST n = 3 `advanced` 99-119 vs 101-110 us
    // per call: the replay still dispatches kernel by kernel, `profiles/r05/small_ecall/
    // graph_replay_r05g2.jsonl`.)
    uint32_t st = FLTEE_SUCCESS;
    for (int attempt = 0; attempt < 2; ++attempt) {
        st = enqueue(attempt > 0);
        if (st != FLTEE_SUCCESS) return st;
        if (fl_stream_sync(s) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        bool retry = false;
        st = status_to_retval(*(const volatile uint32_t *)((const uint8_t *)c->pin_out.ptr + d4), alg,
                              &retry);
        if (!retry) break;
        o.flags &= ~FLTEE_OPT_DENSE;  // the sparse path: exact for any upload
    }
    if (st) return st;
    std::memcpy(host_out, c->pin_out.ptr, d * 4);
    float h2d = 0, aes = 0;
    if (!zero_copy) (void)hipEventElapsedTime(&h2d, c->call_ev[0], c->call_ev[1]);
    (void)hipEventElapsedTime(&aes, c->call_ev[1], c->call_ev[2]);
    const float wall = (float)(now_s() - t0);
    times[0] = (float)(t1 - t0) + h2d * 1e-3f;
    times[1] = aes * 1e-3f;
    times[2] = wall - times[0] - times[1];
    if (alg == FLTEE_ALG_OPTIMIZED) {
        times[1] += times[2];
        times[2] = 0;
    }
    return FLTEE_SUCCESS;
}

}  // namespace fltee

using namespace fltee;

// fltee_version(): build/version.cpp, generated by the Makefile (source hash + tune flags)

extern "C" fltee_status_t fltee_device_init(int hip_device, fltee_eid_t *eid) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (!eid) return FLTEE_ERROR_INVALID_PARAMETER;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || hip_device < 0 || hip_device >= count)
        return FLTEE_ERROR_UNEXPECTED;
    if (hipSetDevice(hip_device) != hipSuccess || !device_ctx(hip_device)) return FLTEE_ERROR_UNEXPECTED;
    g_eid_dev.push_back(hip_device);
    *eid = (fltee_eid_t)g_eid_dev.size();
    return FLTEE_SUCCESS;
}

extern "C" fltee_status_t fltee_device_init_multi(const int *hip_devices, int n, fltee_eid_t *eid) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (!eid || !hip_devices) return FLTEE_ERROR_INVALID_PARAMETER;
    uint32_t st = 0;
    Group *G = group_create(hip_devices, n, &st);
    if (!G) return st;
    if (hipSetDevice(hip_devices[0]) != hipSuccess || !device_ctx(hip_devices[0])) {
        group_destroy(G);
        return FLTEE_ERROR_UNEXPECTED;
    }
    g_eid_dev.push_back(hip_devices[0]);
    *eid = (fltee_eid_t)g_eid_dev.size();
    g_groups[*eid] = G;
    return FLTEE_SUCCESS;
}

extern "C" int fltee_device_count(fltee_eid_t eid) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (eid == 0 || eid > g_eid_dev.size() || g_eid_dev[eid - 1] < 0) return 0;
    Group *G = group_of(eid);
    return G ? group_size(G) : 1;
}

extern "C" fltee_status_t fltee_device_fini(fltee_eid_t eid) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (eid == 0 || eid > g_eid_dev.size() || g_eid_dev[eid - 1] < 0) return FLTEE_ERROR_INVALID_ENCLAVE_ID;
    const int dev = g_eid_dev[eid - 1];
    g_eid_dev[eid - 1] = -1;
    if (Group *G = group_of(eid)) {
        group_destroy(G);
        g_groups.erase(eid);
    }
    if (hipSetDevice(dev) == hipSuccess) (void)fl_device_sync();
    return FLTEE_SUCCESS;
}

// lib.rs:113-180
extern "C" fltee_status_t ecall_fl_init(fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id,
                                        const uint32_t *client_ids, size_t client_size,
                                        size_t num_of_parameters, size_t num_of_sparse_parameters,
                                        float sigma, float clipping, float alpha,
                                        float sampling_ratio, uint32_t aggregation_alg,
                                        uint8_t verbose, uint8_t dp) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (eid == 0 || eid > g_eid_dev.size() || g_eid_dev[eid - 1] < 0) return FLTEE_ERROR_INVALID_ENCLAVE_ID;
    if (!retval) return FLTEE_ERROR_INVALID_PARAMETER;
    FLConfig cfg;
    cfg.client_ids.assign(client_ids, client_ids + client_size);
    cfg.d = num_of_parameters;
    cfg.k = num_of_sparse_parameters;
    cfg.sigma = sigma;
    cfg.clipping = clipping;
    cfg.alpha = alpha;
    cfg.ratio = sampling_ratio;
    cfg.alg = aggregation_alg;
    cfg.verbose = verbose;
    cfg.dp = dp;
    cfg.round = 0;
    if (!g_have_keys && verbose) std::printf("[FLTEE] remote attestation mock\n");
    for (size_t i = 0; i < client_size; ++i) g_keys.insert(client_ids[i]);  // lib.rs:163-174
    g_have_keys = true;
    g_cfg[fl_id] = std::move(cfg);
    if (verbose) std::printf("[FLTEE] make fl config id %u\n", fl_id);
    *retval = FLTEE_SUCCESS;
    return FLTEE_SUCCESS;
}

// lib.rs:182-219
extern "C" fltee_status_t ecall_start_round(fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id,
                                            uint32_t round, size_t sample_size,
                                            uint32_t *sampled_client_ids) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (eid == 0 || eid > g_eid_dev.size() || g_eid_dev[eid - 1] < 0) return FLTEE_ERROR_INVALID_ENCLAVE_ID;
    if (!retval) return FLTEE_ERROR_INVALID_PARAMETER;
    auto it = g_cfg.find(fl_id);
    if (it == g_cfg.end()) { *retval = FLTEE_ERROR_UNEXPECTED; return FLTEE_SUCCESS; }
    FLConfig &cfg = it->second;
    if (cfg.round != round) { *retval = FLTEE_ERROR_INVALID_PARAMETER; return FLTEE_SUCCESS; }
    std::memset(sampled_client_ids, 0, sample_size * 4);  // [out] zero-fill
    const size_t calc = f32_to_usize_sat((float)cfg.client_ids.size() * cfg.ratio);
    if (calc != sample_size) { *retval = FLTEE_ERROR_INVALID_PARAMETER; return FLTEE_SUCCESS; }
    std::vector<uint32_t> sampled;
    sample_client_ids(cfg.client_ids, calc, next_seed(), sampled);
    std::copy(sampled.begin(), sampled.end(), sampled_client_ids);
    cfg.sampled = std::set<uint32_t>(sampled.begin(), sampled.end());
    if (cfg.verbose)
        std::printf("[FLTEE] sampling for round %u is done and store %zu/%zu client ids.\n", round,
                    sample_size, cfg.client_ids.size());
    *retval = FLTEE_SUCCESS;
    return FLTEE_SUCCESS;
}

// lib.rs:221-423
extern "C" fltee_status_t ecall_secure_aggregation(
    fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id, uint32_t round,
    const uint32_t *client_ids, size_t client_size, const uint8_t *encrypted_parameters_data,
    size_t encrypted_parameters_size, size_t num_of_parameters, size_t num_of_sparse_parameters,
    uint32_t aggregation_alg, float *updated_parameters_data, float *execution_time_results) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (!retval) return FLTEE_ERROR_INVALID_PARAMETER;
    DeviceCtx *c = eid_ctx(eid);
    if (!c) return FLTEE_ERROR_INVALID_ENCLAVE_ID;
    const size_t d = num_of_parameters;
    // Enclave_t.c:626 zero-fills [out]: every successful path writes all of it, so the
    // zeros are written where a call fails (200 KB at MLP-MNIST: ~10 us saved per call)
    std::memset(execution_time_results, 0, 3 * sizeof(float));
    auto fail = [&](uint32_t st) {
        std::memset(updated_parameters_data, 0, d * sizeof(float));
        *retval = st;
        return FLTEE_SUCCESS;
    };
    auto it = g_cfg.find(fl_id);
    if (it == g_cfg.end()) return fail(FLTEE_ERROR_UNEXPECTED);
    FLConfig &cfg = it->second;
    if (cfg.round != round || cfg.alg != aggregation_alg) return fail(FLTEE_ERROR_INVALID_PARAMETER);
    const size_t n = client_size;
    if (n == 0) return fail(FLTEE_ERROR_INVALID_PARAMETER);  // lib.rs:305 would divide by zero
    if (uint32_t st = check_uploaded(cfg, client_ids, n)) return fail(st);
    for (size_t i = 0; i < n; ++i)
        if (!g_keys.count(client_ids[i])) return fail(FLTEE_ERROR_UNEXPECTED);  // lib.rs:319-322
    switch (aggregation_alg) {  // lib.rs:359-397 (6 and 7 are not dispatched here: panic)
    case FLTEE_ALG_ADVANCED: case FLTEE_ALG_NIPS19: case FLTEE_ALG_BASELINE:
    case FLTEE_ALG_NON_OBLIVIOUS: case FLTEE_ALG_PATH_ORAM: break;
    default: return fail(FLTEE_ERROR_INVALID_PARAMETER);
    }
    // lib.rs:305-306: bytes per client floored, records per client floored; slice i
    // starts at i*bpc even when that is not a record boundary (ragged payloads)
    const size_t bpc = encrypted_parameters_size / n;
    const size_t rpc = bpc / 8;
    if (aggregation_alg == FLTEE_ALG_ADVANCED && n * num_of_sparse_parameters > n * rpc)
        return fail(FLTEE_ERROR_INVALID_PARAMETER);  // advanced.rs:72 out-of-bounds panic

    if (!c->outbuf.reserve(d * 4 + 16)) return fail(FLTEE_ERROR_OUT_OF_MEMORY);
    float *d_out = (float *)c->outbuf.ptr;
    const size_t k_req = num_of_sparse_parameters;
    const float coef = 1.0f / (float)n;
    Group *G = group_of(eid);
    uint32_t st = FLTEE_GROUP_FALLBACK;
    double t2 = 0;
    const bool flat = aggregation_alg == FLTEE_ALG_BASELINE || aggregation_alg == FLTEE_ALG_PATH_ORAM ||
                      aggregation_alg == FLTEE_ALG_NON_OBLIVIOUS;
    const bool tree = aggregation_alg == FLTEE_ALG_PATH_ORAM && oram_tree_default() &&
                      oram_fits(n * rpc, d, false);
    if (G && flat && !tree && rpc == d && bpc == d * 8) {
        // dense uploads over a multi-GPU eid: every GPU loads and decrypts its own
        // parameter range (group.hip); "Loading" = the parallel H2D, "Decryption" = the
        // decrypt + aggregate + gather
        std::vector<uint32_t> rk;
        client_round_keys(client_ids, n, rk);
        st = group_dense_ecall(G, rk.data(), n, encrypted_parameters_data, d, coef, d_out,
                               &execution_time_results[0], &execution_time_results[1],
                               false);  // out of position: the root's sparse rerun, every alg
        t2 = now_s();
        if (st != FLTEE_SUCCESS && st != FLTEE_GROUP_FALLBACK) return fail(st);
    }
    // (the exact-runs policy folds on one GPU: one sequential walk of the sorted array)
    const bool sharded = G && ((aggregation_alg == FLTEE_ALG_ADVANCED && k_req == rpc &&
                                !exact_runs_default()) ||
                               aggregation_alg == FLTEE_ALG_NIPS19);
    // nips19 draws its seed (Laplace counts, shuffle key) once per call, whichever path
    // runs it, so a multi-GPU eid consumes the seed sequence exactly as one GPU does
    const uint64_t seed = aggregation_alg == FLTEE_ALG_NIPS19 ? next_seed() : 0;
    bool group_tried = false;  // a shape the group declined is not offered to it again
    if (st == FLTEE_GROUP_FALLBACK && sharded && group_splits_host_copy(G)) {
        // every GPU copies and decrypts the clients of its own position range
        std::vector<uint32_t> rk;
        client_round_keys(client_ids, n, rk);
        GroupInput in;
        in.enc = encrypted_parameters_data;
        in.rk = rk.data();
        in.bpc = bpc;
        in.t_load = &execution_time_results[0];
        in.t_dec = &execution_time_results[1];
        const double ta = now_s();
        if (aggregation_alg == FLTEE_ALG_ADVANCED)
            st = group_advanced(G, in, n, rpc, d, coef, d_out);
        else
            st = group_nips19(G, c, in, n, rpc, k_req, d, seed, coef, d_out);
        group_tried = true;
        if (st != FLTEE_SUCCESS && st != FLTEE_GROUP_FALLBACK) return fail(st);
        // "Aggregation" = the call minus its load and decrypt phases
        t2 = ta + execution_time_results[0] + execution_time_results[1];
    }
    if (st == FLTEE_GROUP_FALLBACK && !G && n * bpc <= kStagedBytes) {
        // one GPU, a small payload: one DMA each way, one host synchronisation
        st = staged_ecall(c, aggregation_alg, client_ids, n, encrypted_parameters_data, bpc, d, k_req,
                          0, seed, cfg, updated_parameters_data, execution_time_results);
        if (st) {
            std::memset(updated_parameters_data, 0, d * sizeof(float));
            std::memset(execution_time_results, 0, 3 * sizeof(float));
            return fail(st);
        }
        if (cfg.verbose)
            std::printf("[FLTEE CLOCK] Loading %.6f Decryption %.6f Aggregation %.6f seconds\n",
                        execution_time_results[0], execution_time_results[1], execution_time_results[2]);
        cfg.round += 1;  // lib.rs:421
        *retval = FLTEE_SUCCESS;
        return FLTEE_SUCCESS;
    }
    if (st == FLTEE_GROUP_FALLBACK) {  // (a shape the per-GPU path declines comes here too)
        st = load_and_decrypt(c, client_ids, n, encrypted_parameters_data, bpc,
                              &execution_time_results[0], &execution_time_results[1]);
        if (st) return fail(st);
        t2 = now_s();
        st = FLTEE_GROUP_FALLBACK;
        GroupInput in;
        in.root_rec = (const uint64_t *)c->records.ptr;
        if (sharded && !group_tried) {
            if (aggregation_alg == FLTEE_ALG_ADVANCED)
                st = group_advanced(G, in, n, rpc, d, coef, d_out);
            else
                st = group_nips19(G, c, in, n, rpc, k_req, d, seed, coef, d_out);
        }
        if (st == FLTEE_GROUP_FALLBACK)  // one device (or a shape the group does not shard)
            st = aggregate_records(c, aggregation_alg, n, rpc, d, k_req, 0, d_out, seed);
    }
    if (!st && cfg.dp) {  // lib.rs:399-408
        if (launch_dp_noise(d_out, d, cfg.sigma, cfg.clipping, n, next_seed(), c->stream) != hipSuccess)
            st = FLTEE_ERROR_UNEXPECTED;
    }
    if (!st && fl_memcpy_async(updated_parameters_data, d_out, d * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        st = FLTEE_ERROR_UNEXPECTED;
    if (fl_stream_sync(c->stream) != hipSuccess) st = FLTEE_ERROR_UNEXPECTED;
    if (st) {
        std::memset(updated_parameters_data, 0, d * sizeof(float));
        return fail(st);
    }
    execution_time_results[2] = (float)(now_s() - t2);
    if (cfg.verbose)
        std::printf("[FLTEE CLOCK] Loading %.6f Decryption %.6f Aggregation %.6f seconds\n",
                    execution_time_results[0], execution_time_results[1], execution_time_results[2]);
    cfg.round += 1;  // lib.rs:421
    *retval = FLTEE_SUCCESS;
    return FLTEE_SUCCESS;
}

// lib.rs:425-592
extern "C" fltee_status_t ecall_client_size_optimized_secure_aggregation(
    fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id, uint32_t round,
    size_t optimal_num_of_clients, const uint32_t *client_ids, size_t client_size,
    const uint8_t *encrypted_parameters_data_ptr, size_t num_of_parameters,
    size_t num_of_sparse_parameters, uint32_t aggregation_alg, float *updated_parameters_data,
    float *execution_time_results) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    if (!retval) return FLTEE_ERROR_INVALID_PARAMETER;
    DeviceCtx *c = eid_ctx(eid);
    if (!c) return FLTEE_ERROR_INVALID_ENCLAVE_ID;
    const size_t d = num_of_parameters, k = num_of_sparse_parameters, n = client_size;
    std::memset(execution_time_results, 0, 3 * sizeof(float));
    auto fail = [&](uint32_t st) {  // [out] zero-filled where the call fails (see above)
        std::memset(updated_parameters_data, 0, d * sizeof(float));
        *retval = st;
        return FLTEE_SUCCESS;
    };
    auto it = g_cfg.find(fl_id);
    if (it == g_cfg.end()) return fail(FLTEE_ERROR_UNEXPECTED);
    FLConfig &cfg = it->second;
    if (cfg.round != round || cfg.alg != aggregation_alg) return fail(FLTEE_ERROR_INVALID_PARAMETER);
    if (n == 0 || optimal_num_of_clients == 0) return fail(FLTEE_ERROR_INVALID_PARAMETER);
    if (uint32_t st = check_uploaded(cfg, client_ids, n)) return fail(st);
    for (size_t i = 0; i < n; ++i)
        if (!g_keys.count(client_ids[i])) return fail(FLTEE_ERROR_UNEXPECTED);

    float t_load = 0, t_dec = 0;
    const double t1 = now_s();
    const size_t halo6 = exact_runs_default() ? n * k + d : n;  // as aggregate_records
    float *d_out = nullptr;
    if (!c->outbuf.reserve(d * 4 + 16)) return fail(FLTEE_ERROR_OUT_OF_MEMORY);
    d_out = (float *)c->outbuf.ptr;
    uint32_t st;
    Group *G = group_of(eid);
    if (G && group_splits_host_copy(G)) {
        // the batches split over the eid's GPUs, each loading its own clients (group.hip)
        std::vector<uint32_t> rk;
        client_round_keys(client_ids, n, rk);
        GroupInput in;
        in.enc = encrypted_parameters_data_ptr;
        in.rk = rk.data();
        in.bpc = k * 8;
        in.t_load = &t_load;
        in.t_dec = &t_dec;
        st = group_optimized(G, in, n, k, d, optimal_num_of_clients, 1.0f / (float)n, d_out, halo6);
        execution_time_results[0] = t_load;
    } else if (!G && n * k * 8 <= kStagedBytes) {
        // one GPU, a small payload: one DMA each way, one host synchronisation
        st = staged_ecall(c, FLTEE_ALG_OPTIMIZED, client_ids, n, encrypted_parameters_data_ptr, k * 8, d,
                          k, optimal_num_of_clients, 0, cfg, updated_parameters_data, execution_time_results);
        if (st) {
            std::memset(updated_parameters_data, 0, d * sizeof(float));
            std::memset(execution_time_results, 0, 3 * sizeof(float));
            return fail(st);
        }
        cfg.round += 1;
        *retval = FLTEE_SUCCESS;
        return FLTEE_SUCCESS;
    } else {
        st = load_and_decrypt(c, client_ids, n, encrypted_parameters_data_ptr, k * 8, &t_load, &t_dec);
        if (st) return fail(st);
        execution_time_results[0] = t_load;
        if (G) {
            GroupInput in;
            in.root_rec = (const uint64_t *)c->records.ptr;
            st = group_optimized(G, in, n, k, d, optimal_num_of_clients, 1.0f / (float)n, d_out, halo6);
        } else {
            st = aggregate_records(c, FLTEE_ALG_OPTIMIZED, n, k, d, k, optimal_num_of_clients, d_out);
        }
    }
    if (!st && cfg.dp) {  // lib.rs:586-588
        if (launch_dp_noise(d_out, d, cfg.sigma, cfg.clipping, n, next_seed(), c->stream) != hipSuccess)
            st = FLTEE_ERROR_UNEXPECTED;
    }
    if (!st && fl_memcpy_async(updated_parameters_data, d_out, d * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        st = FLTEE_ERROR_UNEXPECTED;
    if (fl_stream_sync(c->stream) != hipSuccess) st = FLTEE_ERROR_UNEXPECTED;
    if (st) {
        std::memset(updated_parameters_data, 0, d * sizeof(float));
        return fail(st);
    }
    execution_time_results[1] = (float)(now_s() - t1) - t_load;  // decrypt + aggregate
    cfg.round += 1;
    *retval = FLTEE_SUCCESS;
    return FLTEE_SUCCESS;
}

// AES-128-CTR over n client slices with the session keys of lib.rs:312-343 (key
// bytes[4..8] = id BE; the client's 2-byte layout, utils.py:276-278, is the same for
// every id it can encode).  CTR is its own inverse: decrypt == encrypt.
static fltee_status_t aes_ctr_device(const uint32_t *client_ids, size_t n, const void *d_in,
                                     size_t bytes_per_client, void *d_out, hipStream_t s) {
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_INVALID_PARAMETER;
    if (!c->round_keys.reserve(n * 44 * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
    std::vector<uint32_t> rk(n * 44);
    aes128_session_round_keys(client_ids, n, rk.data());
    if (fl_memcpy_async(c->round_keys.ptr, rk.data(), rk.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    if (launch_aes_ctr((const uint8_t *)d_in, n, bytes_per_client, bytes_per_client / 8,
                       (const uint32_t *)c->round_keys.ptr, (uint8_t *)d_out, s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    // rk lives on this stack frame: wait for the (tiny) copy + kernel
    return fl_stream_sync(s) == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_decrypt_device(const uint32_t *client_ids, size_t n,
                                               const void *d_cipher, size_t bytes_per_client,
                                               void *d_records, void *stream) {
    return aes_ctr_device(client_ids, n, d_cipher, bytes_per_client, d_records, (hipStream_t)stream);
}

// ------------------------------------------- client-side producers (§8f.4) ----
extern "C" fltee_status_t fltee_encrypt_device(const uint32_t *client_ids, size_t n,
                                               const void *d_plain, size_t bytes_per_client,
                                               void *d_cipher, void *stream) {
    for (size_t i = 0; i < n; ++i)  // encrypt_parameters: int(id).to_bytes(2, 'big')
        if (client_ids[i] > 0xFFFFu) return FLTEE_ERROR_INVALID_PARAMETER;
    return aes_ctr_device(client_ids, n, d_plain, bytes_per_client, d_cipher, (hipStream_t)stream);
}

namespace fltee {
hipError_t launch_client_topk(const float *values, size_t n, size_t d, size_t k, uint64_t *keys,
                              uint64_t *rec, hipStream_t s);
size_t client_topk_workspace(size_t n, size_t d);
hipError_t launch_client_dense(const float *values, size_t n, size_t d, uint64_t *rec,
                               hipStream_t s);
}  // namespace fltee

extern "C" fltee_status_t fltee_client_topk_device(const float *d_values, size_t n, size_t d,
                                                   size_t k, void *d_records, void *stream) {
    if (n == 0 || d == 0 || k > d || d > 0xFFFFFFFFull) return FLTEE_ERROR_INVALID_PARAMETER;
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_INVALID_PARAMETER;
    if (k == 0) return FLTEE_SUCCESS;
    if (!c->ws_client.reserve(client_topk_workspace(n, d))) return FLTEE_ERROR_OUT_OF_MEMORY;
    return launch_client_topk(d_values, n, d, k, (uint64_t *)c->ws_client.ptr,
                              (uint64_t *)d_records, (hipStream_t)stream) == hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_client_serialize_dense_device(const float *d_values, size_t n,
                                                              size_t d, void *d_records,
                                                              void *stream) {
    if (n == 0 || d == 0 || d > 0xFFFFFFFFull) return FLTEE_ERROR_INVALID_PARAMETER;
    return launch_client_dense(d_values, n, d, (uint64_t *)d_records, (hipStream_t)stream) ==
                   hipSuccess
               ? FLTEE_SUCCESS
               : FLTEE_ERROR_UNEXPECTED;
}

extern "C" fltee_status_t fltee_client_clip_device(void *d_records, size_t n, size_t k,
                                                   float clipping, void *stream) {
    if (n == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    std::lock_guard<std::recursive_mutex> lk(api_mutex());
    DeviceCtx *c = current_ctx();
    if (!c) return FLTEE_ERROR_INVALID_PARAMETER;
    if (!c->ws_client_coef.reserve(n * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
    hipStream_t s = (hipStream_t)stream;
    float *cf = (float *)c->ws_client_coef.ptr;
    if (launch_client_clip_coef(d_records, n, k, clipping, cf, s) != hipSuccess ||
        launch_apply_clip(d_records, n, k, cf, s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    return FLTEE_SUCCESS;
}

// CPU self-test hook: the clients' round keys by the AES-NI schedule (when the CPU has
// it) or by the portable bitsliced one (portable != 0); returns 1 when AES-NI was used.
namespace fltee {
void aes128_session_round_keys_portable(const uint32_t *ids, size_t n, uint32_t *rk);
bool host_has_aesni();
}
extern "C" int fltee_debug_session_round_keys(const uint32_t *ids, size_t n, uint32_t *rk, int portable) {
    if (portable || !fltee::host_has_aesni()) {
        fltee::aes128_session_round_keys_portable(ids, n, rk);
        return 0;
    }
    fltee::aes128_session_round_keys(ids, n, rk);
    return 1;
}

// CPU self-test hook: one AES-128 block with the library's tables (no GPU).
namespace fltee { void aes128_encrypt_block_host(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]); }
extern "C" void fltee_debug_aes_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    fltee::aes128_encrypt_block_host(key, in, out);
}
