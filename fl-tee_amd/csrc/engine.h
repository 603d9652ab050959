// engine.h — per-device state and the internal aggregation entry points.
#pragma once
#include <mutex>

#include "common.h"

namespace fltee {

constexpr int kMaxDevices = 64;

struct Buffer {
    void *ptr = nullptr;
    size_t cap = 0;
    bool reserve(size_t bytes);  // grow-only hipMalloc
    void release();              // hipFree (the owning device must be current)
};

// grow-only pinned host memory (the ECALL's staging: one DMA each way per call)
struct HostBuffer {
    void *ptr = nullptr;   // host address
    void *dptr = nullptr;  // the same pinned bytes as kernels address them (zero-copy)
    size_t cap = 0;
    bool reserve(size_t bytes);
};

struct DeviceCtx {
    bool ready = false;
    int device = -1;
    uint32_t *status = nullptr;  // library-owned device status word
    Buffer ws_a, ws_b, ws_mat, ws_r, ws_coef, ws_rec;  // aggregation scratch
    // bytes of ws_mat (from its start) known to hold the scatter path's empty sentinel:
    // the scatter sum restores every slot it used, so the fill runs once per buffer
    size_t mat_clean = 0, mat_clean_cap = 0;
    void *mat_clean_ptr = nullptr;
    Buffer cipher, records, round_keys, outbuf;         // ECALL staging
    Buffer stage;                                        // small ECALLs: out, status, keys, ciphertext
    HostBuffer pin_in, pin_out;                          // small ECALLs: pinned staging both ways
    hipEvent_t call_ev[3] = {};                          // small ECALLs: the phase timers
    Buffer ws_client, ws_client_coef;                   // client-side producers
    Buffer ws_cnt, ws_sel;                               // nips19's selected list
    Buffer ws_keys, ws_radix;  // ordered folds: records sorted by idx, the counting sort's scratch
    Buffer ws_oram;            // path_oram tree mode: the tree + stash slots, then their records
    Buffer ws_side;            // advanced's streaming fold: its side records (k_fold.hip)
    Buffer ws_lb;              // the fused fold's look-back slots (k_compact.hip), zeroed
    uint32_t fc_epoch = 0;     // their launch counter
    uint32_t *host_word = nullptr;                       // pinned readback word
    hipStream_t stream = nullptr;                        // ECALL stream
    hipStream_t copy_stream = nullptr;                   // ECALL H2D (pipelined load)
    static constexpr int kCopyEvents = 64;
    hipEvent_t copy_ev[kCopyEvents] = {};
};

// One process-wide lock: the enclave had a single TCS (Enclave.config.xml:6).
std::recursive_mutex &api_mutex();

DeviceCtx *device_ctx(int dev);
DeviceCtx *current_ctx();
uint64_t next_seed();
void set_debug_seed(uint64_t seed);
float nips19_threshold(size_t d, size_t k, size_t n);

// path_oram as the tree Path ORAM for the ECALLs (fltee_set_path_oram_tree); the device
// API selects it per call with FLTEE_OPT_ORAM_TREE
void set_oram_tree(int on);
bool oram_tree_default();
// advanced / alg 6 in the ECALLs: the one-lane sequential fold at the public worst-case
// cost (fltee_set_advanced_exact_runs: the enclave's sums bit for bit for any run length),
// else the halo fold (bit for bit up to n + 1 entries a run, re-associated beyond)
void set_exact_runs(int on);
bool exact_runs_default();

fltee_status_t aggregate(uint32_t alg, const void *rec, size_t n, size_t k, size_t d, float *out,
                         const fltee_device_opts &o, hipStream_t s, uint32_t *status);
// common.rs:25-35 on m entries of src (the shuffled array), bit-exact: out[i] = coef *
// (+0 + v1 + v2 ...) over the entries with idx == i in position order (accumulate:
// out[i] += the un-scaled sum).  Synchronises `s` once to read the selected count.
hipError_t safe_aggregate_ordered(DeviceCtx *c, const uint64_t *src, size_t m, size_t d,
                                  float coef, float *out, bool accumulate, uint32_t *status,
                                  hipStream_t s);
// the selected list sel[0, lc) (nips19 entries with idx < d, in shuffled order) -> out
hipError_t ordered_from_list(DeviceCtx *c, const uint64_t *sel, size_t lc, size_t d, float coef,
                             float *out, bool acc, uint32_t *status, hipStream_t s);
// one alg-6 batch: `advanced` of n clients into out[d], un-averaged (current device)
hipError_t advanced_batch(const void *rec, size_t n, size_t k, size_t d, size_t halo, float *out,
                          uint32_t *status, hipStream_t s);
hipError_t read_device_word(DeviceCtx *c, const uint32_t *dev_word, size_t *out, hipStream_t s);
size_t workspace_bytes(uint32_t alg, size_t n, size_t k, size_t d, const fltee_device_opts &o);
bool reserve(uint32_t alg, size_t n, size_t k, size_t d, const fltee_device_opts &o);

}  // namespace fltee
