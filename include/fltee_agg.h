/*
 * fltee_agg.h — C ABI of libfltee_agg.so, the MI355X-native replacement for
 * FL-TEE's SGX aggregation enclave (secure_aggregation/enclave).
 *
 * Drop-in boundary.  The four ECALLs below keep the exact symbol names and
 * argument lists that the Rust host binds in
 *     secure_aggregation/app/src/ecalls.rs:6-64
 * (EDL contract: secure_aggregation/enclave/Enclave.edl:23-84), including the
 * leading (eid, *retval) pair that sgx_edger8r's untrusted bridge adds.  A host
 * that linked the edger8r bridge (app/Enclave_u.c) links this library instead;
 * see INTEGRATION.md for the ecalls.rs / build.rs diff.
 *
 * Conventions:
 *   - return value  = "bridge" status: always FLTEE_SUCCESS for an in-process
 *                     call (the SGX bridge could fail; this one cannot), except
 *                     FLTEE_ERROR_INVALID_ENCLAVE_ID for an unknown eid.
 *   - *retval       = the enclave's status: 0 success, 0x1 unexpected
 *                     (unknown fl_id / missing session key / device failure),
 *                     0x2 invalid parameter (round / alg / id-set / size
 *                     mismatch, and every case where the reference enclave
 *                     would panic: unknown alg (lib.rs:396), out-of-range
 *                     index in non_oblivious (non_oblivious.rs:12), fold
 *                     longer than the payload (advanced.rs:70-72)).
 *   - ownership     : the caller owns every buffer; nothing is retained.
 *   - [out] buffers : zero-filled by the callee before anything else (the SGX
 *                     bridge did this, Enclave_t.c:626); execution_time_results
 *                     is always fully written.
 *   - threading     : calls may arrive from any thread (tokio workers,
 *                     server.rs:241-245); the library serialises them with one
 *                     process-wide mutex (the enclave had one TCS,
 *                     Enclave.config.xml:6) and binds the eid's device per call.
 *                     The device-resident entry points below share per-device
 *                     scratch: calls for one device must not overlap in time on
 *                     different streams (the mutex orders the host calls; the
 *                     kernels of two streams could still interleave).
 */
#ifndef FLTEE_AGG_H
#define FLTEE_AGG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* sgx_status_t subset (sgx_error.h values) */
typedef uint32_t fltee_status_t;
#define FLTEE_SUCCESS 0x0000u
#define FLTEE_ERROR_UNEXPECTED 0x0001u
#define FLTEE_ERROR_INVALID_PARAMETER 0x0002u
#define FLTEE_ERROR_OUT_OF_MEMORY 0x0003u
#define FLTEE_ERROR_INVALID_ENCLAVE_ID 0x2002u

/* sgx_enclave_id_t */
typedef uint64_t fltee_eid_t;

/* aggregation_alg codes, src/option.py:131-145 */
#define FLTEE_ALG_ADVANCED 1u
#define FLTEE_ALG_NIPS19 2u
#define FLTEE_ALG_BASELINE 3u
#define FLTEE_ALG_NON_OBLIVIOUS 4u
#define FLTEE_ALG_PATH_ORAM 5u
#define FLTEE_ALG_OPTIMIZED 6u

/* ------------------------------------------------------------------------ */
/* Device lifetime — replaces init_enclave() / SgxEnclave::destroy()         */
/* (app/src/ecalls.rs:66-83, server.rs:224-235,257).                          */
/* ------------------------------------------------------------------------ */
fltee_status_t fltee_device_init(int hip_device, fltee_eid_t *eid);
fltee_status_t fltee_device_fini(fltee_eid_t eid);

/* One enclave id over n GPUs of this node (n a power of two): the four ECALLs of that
 * eid shard the aggregation internally and return the same bits as one
 * GPU.  Dense uploads (baseline / non_oblivious / path_oram with k = d): parameter-range
 * shards, each GPU copies and decrypts only its columns of the host ciphertext over its
 * own PCIe link, RCCL gathers the averaged slices on the root (hip_devices[0]).
 * advanced: position-range sharded bitonic network (RCCL all-to-alls), halo fold,
 * compaction and one RCCL reduce.  nips19: the same network (pairwise exchanges), the
 * ranges' selected entries gathered in order to the root.  alg 6: the batches split
 * over the GPUs, the batch sums summed in order on the root.  Sparse flat algorithms
 * run on the root.  Devices all distinct: RCCL over xGMI; the same device repeated n
 * times: n virtual ranks on that GPU (exchanges are device copies; for tests). */
fltee_status_t fltee_device_init_multi(const int *hip_devices, int n, fltee_eid_t *eid);
/* GPUs (ranks) behind an eid: 1 for fltee_device_init, n for _multi, 0 if unknown. */
int fltee_device_count(fltee_eid_t eid);

/* ------------------------------------------------------------------------ */
/* The four ECALLs (ecalls.rs:6-64 / Enclave.edl:26-73)                      */
/* ------------------------------------------------------------------------ */

/* lib.rs:113-180 — (re)create the config of fl_id, mock session keys. */
fltee_status_t ecall_fl_init(fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id,
                             const uint32_t *client_ids, size_t client_size,
                             size_t num_of_parameters, size_t num_of_sparse_parameters,
                             float sigma, float clipping, float alpha, float sampling_ratio,
                             uint32_t aggregation_alg, uint8_t verbose, uint8_t dp);

/* lib.rs:182-219 — sample (|ids| * ratio) clients for `round`.  The EDL types
 * sample_size as uint32_t (Enclave.edl:72) but Rust passes usize
 * (ecalls.rs:29): size_t is accepted. */
fltee_status_t ecall_start_round(fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id,
                                 uint32_t round, size_t sample_size,
                                 uint32_t *sampled_client_ids);

/* lib.rs:221-423 — load (H2D), decrypt (AES-128-CTR on the GPU), aggregate
 * with `aggregation_alg`, optional DP noise; writes the averaged f32[d] and
 * execution_time_results[3] = {load, decrypt, aggregate} seconds. */
fltee_status_t ecall_secure_aggregation(fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id,
                                        uint32_t round, const uint32_t *client_ids,
                                        size_t client_size,
                                        const uint8_t *encrypted_parameters_data,
                                        size_t encrypted_parameters_size,
                                        size_t num_of_parameters,
                                        size_t num_of_sparse_parameters,
                                        uint32_t aggregation_alg,
                                        float *updated_parameters_data,
                                        float *execution_time_results);

/* lib.rs:425-592 — alg 6: `advanced` over batches of optimal_num_of_clients
 * clients; the payload pointer is [user_check]: client_size * k * 8 bytes are
 * read. execution_time_results = {load, decrypt+aggregate, 0}. */
fltee_status_t ecall_client_size_optimized_secure_aggregation(
    fltee_eid_t eid, fltee_status_t *retval, uint32_t fl_id, uint32_t round,
    size_t optimal_num_of_clients, const uint32_t *client_ids, size_t client_size,
    const uint8_t *encrypted_parameters_data_ptr, size_t num_of_parameters,
    size_t num_of_sparse_parameters, uint32_t aggregation_alg, float *updated_parameters_data,
    float *execution_time_results);

/* ------------------------------------------------------------------------ */
/* Device-resident entry points: the aggregation below the ECALL, on records */
/* already decrypted into HBM.  Used by the bench (device-resident metric),  */
/* the multi-GPU driver and the parity tests.  All pointers are device       */
/* pointers; `stream` is a hipStream_t (NULL = legacy default stream).       */
/* Calls are asynchronous: errors found on the device are OR-ed into the     */
/* 32-bit status word (opts.d_status, or the library's own word read back by */
/* fltee_device_status()).                                                    */
/* ------------------------------------------------------------------------ */

/* device status bits */
#define FLTEE_DEV_ERR_DENSE_ORDER 0x1u   /* dense input with idx != position */
#define FLTEE_DEV_ERR_INDEX_RANGE 0x2u   /* idx >= d where the reference panics */
#define FLTEE_DEV_ERR_FOLD_OVERFLOW 0x4u /* retired in round 6 (advanced's fold finishes runs
                                           of any length); never set */
#define FLTEE_DEV_ERR_ORAM_STASH 0x8u    /* path_oram tree mode: the stash (20) overflowed */
#define FLTEE_DEV_ERR_LAUNCH 0x80000000u

/* option flags */
#define FLTEE_OPT_DENSE 0x1u      /* records are dense: client c, slot j has idx j */
#define FLTEE_OPT_DP 0x2u         /* add N(0, clipping*sigma)/n noise (common.rs:56-72) */
#define FLTEE_OPT_CLIP 0x4u       /* server-side per-client L2 clip (update.py:187-204) */
#define FLTEE_OPT_ACCUMULATE 0x8u /* out += sum (no averaging): alg-6 batches, shards */
#define FLTEE_OPT_NO_AVERAGE 0x10u /* skip the 1/n scaling (partial sums for RCCL) */
#define FLTEE_OPT_K_REQ 0x20u      /* advanced: fold over n*k_req+d even if k_req != k
                                      (advanced.rs:70 uses the REQUEST's k; 0 when
                                      fl_main.py sends dense uploads without --alpha) */
#define FLTEE_OPT_ORAM_TREE 0x40u  /* path_oram as a tree Path ORAM (oram.rs:64-118: Z = 4,
                                      stash 20, next_pow2(d) <= 2^22 blocks) running oram.rs's
                                      access sequence (d prepare writes, read + write per
                                      record, d readout reads) instead of the
                                      output-equivalent oblivious sweep */
#define FLTEE_OPT_ORAM_LAZY 0x80u  /* with ORAM_TREE: one read-modify-write access per record,
                                      blocks created on first use, readout by an oblivious
                                      sort of the tree's slots (n*k accesses instead of
                                      2*n*k + 2*d) */

typedef struct fltee_device_opts {
    uint32_t flags;     /* FLTEE_OPT_* */
    float sigma;        /* DP noise multiplier */
    float clipping;     /* DP / clip norm bound C */
    uint64_t seed;      /* RNG seed for nips19 / DP; 0 = draw from getrandom() */
    size_t k_req;       /* advanced: request num_of_sparse_parameters (with FLTEE_OPT_K_REQ) */
    size_t batch;       /* alg 6: optimal_num_of_clients */
    size_t n_avg;       /* divisor for averaging (0 = n) */
    size_t fold_halo;   /* advanced fold halo H (0 = n): runs of <= H + 1 entries (each client's
                           indices distinct) bit for bit, longer ones re-associated at the
                           fold's walk boundaries */
    uint32_t *d_status; /* optional device status word (never cleared by the library) */
} fltee_device_opts;

/* Aggregate n clients x k records (8 B each: u32 LE idx, f32 LE val),
 * client-major, into d_out[d] (overwritten, or accumulated with
 * FLTEE_OPT_ACCUMULATE).  Returns FLTEE_ERROR_INVALID_PARAMETER for
 * host-detectable argument errors. */
fltee_status_t fltee_aggregate_device(uint32_t alg, const void *d_records, size_t n, size_t k,
                                      size_t d, float *d_out, const fltee_device_opts *opts,
                                      void *stream);

/* Bytes of scratch HBM the library will hold for this shape (grow-only). */
size_t fltee_workspace_bytes(uint32_t alg, size_t n, size_t k, size_t d,
                             const fltee_device_opts *opts);
/* Pre-size the scratch so the first timed call does no hipMalloc. */
fltee_status_t fltee_reserve(uint32_t alg, size_t n, size_t k, size_t d,
                             const fltee_device_opts *opts);

/* AES-128-CTR decrypt of n client slices (bytes_per_client each, zero counter
 * block per client, key = session key of client_ids[i]) into compact records
 * (n * (bytes_per_client/8) * 8 bytes).  lib.rs:312-343. */
fltee_status_t fltee_decrypt_device(const uint32_t *client_ids, size_t n, const void *d_cipher,
                                    size_t bytes_per_client, void *d_records, void *stream);

/* ---- client-side producers (fl_main.py:221-238) -------
 * For a GPU-resident client simulator: n clients' flattened updates d_values
 * [n][d] (f32) -> the encrypted payload of the Aggregate request, in HBM. */
/* utils.py:327-354 zero_except_top_k_weights + utils.py:193-209 serialize_sparse:
 * per client the k records (idx, val) of largest |val|, in the reference's order
 * (|val| descending, equal magnitudes by ascending idx; Python's stable sort). */
fltee_status_t fltee_client_topk_device(const float *d_values, size_t n, size_t d, size_t k,
                                        void *d_records, void *stream);
/* utils.py:171-190 serialize_dense: records (i, v[i]), i < d, per client. */
fltee_status_t fltee_client_serialize_dense_device(const float *d_values, size_t n, size_t d,
                                                   void *d_records, void *stream);
/* update.py:187-204 l2clipping on serialized records (n clients x k records, in
 * place): val *= min(1, clipping / ||client's values||_2). */
fltee_status_t fltee_client_clip_device(void *d_records, size_t n, size_t k, float clipping,
                                        void *stream);
/* utils.py:268-290 encrypt_parameters for n clients (ids < 65536: the client's
 * 2-byte key layout), bytes_per_client each; the inverse of fltee_decrypt_device. */
fltee_status_t fltee_encrypt_device(const uint32_t *client_ids, size_t n, const void *d_plain,
                                    size_t bytes_per_client, void *d_cipher, void *stream);

/* out[j] = coef * sum_r rows[r*d + j], rows added in order (exact fp32): the
 * root-side combine of per-GPU partial sums, in the batch order of alg 6
 * (lib.rs:564-573: global[i] += batch_sum[i], then average). */
fltee_status_t fltee_sum_rows_device(const float *d_rows, size_t nrows, size_t d, float coef,
                                     float *d_out, void *stream);

/* common.rs:56-72 on a device vector: out[i] += (N(0, clipping*sigma) / n) as f32. */
fltee_status_t fltee_dp_noise_device(float *d_out, size_t d, float sigma, float clipping,
                                     size_t n, uint64_t seed, void *stream);

/* Synchronise `stream` and return (and clear) the library's status word. */
fltee_status_t fltee_device_status(void *stream, uint32_t *status);

/* ---- intermediate stages, exposed for the permutation-parity tests ------ */
/* In-place oblivious bitonic network on M = 2^m 8-byte records.
 * mode 0: sort by u32 idx with the reference comparator (advanced.rs:147-176)
 * mode 1: sort by the whole u64 (stable-by-construction composite keys)
 * mode 2: keyed shuffle network (nips19.rs:66-105 structure, seed)          */
fltee_status_t fltee_bitonic_device(void *d_records, size_t m, uint32_t mode, uint32_t seed,
                                    void *stream);
/* advanced.rs:66-101 fold over [0, fold_len) of src (length m) into dst. */
fltee_status_t fltee_fold_device(const void *d_src, void *d_dst, size_t m, size_t fold_len,
                                 size_t halo, uint32_t *d_status, void *stream);
/* common.rs:77-98,151-161 — nips19 Laplace counts r[d] and threshold T. */
fltee_status_t fltee_laplace_r_device(size_t d, size_t k, size_t n, uint64_t seed, uint32_t *d_r,
                                      float *T_out, void *stream);

/* ---- position-range pieces of `advanced` (multi-GPU, SURVEY §8e Option B) --
 * The padded array of advanced.rs:116-142 (M = 2^m entries) is split into W
 * contiguous ranges of m = M/W records, one per GPU; range r holds global
 * positions [r*m, (r+1)*m).  Run on every range, in this order, these pieces are
 * the reference's network and fold step for step (fl-tee_amd/fltee/parallel.py
 * drives them over RCCL):
 *   init_range -> range_sort -> for each stage 2^s > m: (range_exchange with the
 *   partner range for every step 2^j >= m) then range_merge -> fold_range ->
 *   compact_range -> sum of the W outputs (RCCL reduce) on the root.          */
/* entries pos_base .. pos_base+m-1 of records ++ (i, 0.0) for i < d ++ (u32::MAX,
 * 0.0) pads (advanced.rs:116-142); d_records holds the records at positions
 * pos_base.. (read where position < nrec). */
fltee_status_t fltee_advanced_init_range_device(const void *d_records, size_t nrec, size_t d,
                                                size_t pos_base, size_t m, void *d_dst,
                                                void *stream);
/* stages 2 .. m of the bitonic network (advanced.rs:147-176) on one range; the
 * direction of every compare-exchange comes from its GLOBAL position. */
fltee_status_t fltee_bitonic_range_sort_device(void *d_records, size_t m, size_t pos_base,
                                               uint32_t mode, uint32_t seed, void *stream);
/* the same, knowing that entries valid .. m-1 of the range are identical (u32::MAX,
 * +0.0) pads (valid >= m: none): stage blocks made of pads alone are skipped, which
 * leaves them as they are — the same permutation.  valid = 0: nothing to do. */
fltee_status_t fltee_bitonic_range_sort_padded_device(void *d_records, size_t m, size_t pos_base,
                                                      size_t valid, uint32_t mode, uint32_t seed,
                                                      void *stream);
/* the steps j = m/2 .. 1 of stage 2^stage_log (> m) on one range. */
fltee_status_t fltee_bitonic_range_merge_device(void *d_records, size_t m, size_t pos_base,
                                                uint32_t mode, uint32_t seed, uint32_t stage_log,
                                                void *stream);
/* the step j = |pos_mine - pos_theirs| (>= m, a power of two) of stage 2^stage_log
 * between this range and a copy of its partner's: d_mine takes the partner's
 * record wherever that compare-exchange swaps. */
fltee_status_t fltee_bitonic_range_exchange_device(void *d_mine, const void *d_theirs, size_t m,
                                                   size_t pos_mine, size_t pos_theirs,
                                                   uint32_t mode, uint32_t seed,
                                                   uint32_t stage_log, void *stream);
/* the steps j = 2^step_top .. 2^step_bot (< m, step_top < stage_log) of stage
 * 2^stage_log on one range (register passes).  Mode 0 only needs directions, so a
 * range whose position bits were permuted by an all-to-all can run its cross-range
 * steps locally through this call (fltee/parallel.py, transposed exchange). */
fltee_status_t fltee_bitonic_range_steps_device(void *d_records, size_t m, size_t pos_base,
                                                uint32_t mode, uint32_t seed, uint32_t stage_log,
                                                uint32_t step_top, uint32_t step_bot,
                                                void *stream);
/* records of context the fold needs in front of a range: halo rounded up to 16 (the
 * range fold reads one more record in front, see below). */
size_t fltee_fold_context(size_t halo);
/* advanced.rs:66-101 on [origin, end) of d_src (length m, global position =
 * pos_base + local): [0, origin) holds >= fltee_fold_context(halo) + 1 records of the
 * previous range, d_src[end] the next range's first record (unless end + pos_base
 * >= fold_len).  Writes d_dst[origin, end) and the fold's side records into d_side
 * (fltee_fold_side_bytes(end - origin, halo) bytes).  Runs of any length (a client
 * repeating an index): a run begun before a walk boundary is finished by the patch
 * below — bit for bit for every run of <= halo + 1 entries, re-associated at the
 * walk boundaries beyond. */
size_t fltee_fold_side_bytes(size_t span, size_t halo);
fltee_status_t fltee_fold_range_device(const void *d_src, void *d_dst, size_t m, size_t origin,
                                       size_t end, int64_t pos_base, size_t fold_len, size_t halo,
                                       void *d_side, void *stream);
/* the range's segmented total (16 bytes into d_total) from its side records: the
 * carry the ranges after it need */
fltee_status_t fltee_fold_range_total_device(const void *d_side, size_t span, size_t halo,
                                             void *d_total, void *stream);
/* the long-run patch of one range's fold output d_dst (the same origin, end, pos_base,
 * fold_len and halo as fltee_fold_range_device): d_prev_totals = the totals of the
 * n_prev ranges before this one, in range order.  Writes every walk's first position
 * (fixed addresses). */
fltee_status_t fltee_fold_range_patch_device(void *d_dst, size_t origin, size_t end,
                                             int64_t pos_base, size_t fold_len, size_t halo,
                                             const void *d_side, const void *d_prev_totals,
                                             size_t n_prev, void *stream);
/* one folded range (c records) -> d_out[d]: val * coef at each run representative's
 * index i < d held by this range, +0.0 elsewhere (oblivious compaction; scratch
 * d_buf, d_tmp of d + c records each).  The sum of every range's d_out is the
 * aggregate, bit for bit. */
fltee_status_t fltee_compact_range_device(const void *d_chunk, size_t c, size_t d, void *d_buf,
                                          void *d_tmp, float coef, float *d_out, void *stream);

/* nips19 by position range (the shuffle is the same kind of network): entries
 * pos_base .. pos_base+m-1 of records ++ d*tf Laplace dummies (common.rs:189-197;
 * d_r from fltee_laplace_r_device, tf = (usize)T) ++ (u32::MAX, 0.0) pads; and
 * safe_aggregate (common.rs:25-35) of m entries into d_out[d] (zeroed first,
 * un-averaged: the ranges' partial sums are added by the caller's reduce). */
fltee_status_t fltee_nips19_build_range_device(const void *d_records, size_t nrec,
                                               const uint32_t *d_r, size_t d, size_t tf,
                                               size_t pos_base, size_t m, void *d_dst,
                                               void *stream);
fltee_status_t fltee_safe_aggregate_device(const void *d_src, size_t m, size_t d, float *d_out,
                                           void *stream);
/* safe_aggregate split over ranges, bit-exact: the entries of one range with idx < d in
 * position order into d_list (at most cap; *count = how many there are, also when they
 * do not fit: INVALID_PARAMETER), synchronising `stream`; then, on the root, the ordered
 * fold of the ranges' lists concatenated in range order (the shuffled order):
 * d_out[i] = coef * (+0 + v1 + v2 ...) over the entries with idx i. */
fltee_status_t fltee_select_device(const void *d_src, size_t m, size_t d, void *d_list,
                                   size_t cap, size_t *count, void *stream);
fltee_status_t fltee_ordered_list_device(const void *d_list, size_t lc, size_t d, float coef,
                                         float *d_out, void *stream);

/* Test hooks: deterministic RNG seed for sampling / nips19 / DP (0 = off). */
/* The ECALLs' path_oram (aggregation_alg 5): on = the tree Path ORAM of oram.rs:64-118
 * (Z = 4, stash 20, next_pow2(d) blocks, oram.rs's access sequence; k_oram.hip) where
 * next_pow2(d) <= 2^22, the sweep beyond; off (default) = the output-equivalent oblivious
 * sweep.  Both give the in-order sum bit for bit.  The device API selects it per call
 * with FLTEE_OPT_ORAM_TREE. */
void fltee_set_path_oram_tree(int on);
/* The ECALLs' advanced and alg 6 when some index has a run of more than n + 1 entries
 * (a client repeated an index inside its upload; fl_main.py's top-k never does):
 * off (default) = the fixed-cost fold with its long-run carry: such a run's sum is the
 * enclave's re-associated at the fold's walk boundaries (runs of <= n + 1 entries bit for
 * bit); on = the enclave's exact fold for ANY run length (advanced.rs:66-101), at the
 * public worst-case cost: one sequential walk of the whole sorted array whatever the data. */
void fltee_set_advanced_exact_runs(int on);
void fltee_debug_set_seed(uint64_t seed);
/* Library build/version string. */
const char *fltee_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FLTEE_AGG_H */
