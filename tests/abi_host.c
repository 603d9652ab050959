/*
 * abi_host.c — a compiled (non-Python) host over include/fltee_agg.h.
 *
 * What it proves: the library links and runs the way the Rust host would bind it.
 *   1. The four ECALL prototypes are re-declared below exactly as the Rust FFI block
 *      spells them (secure_aggregation/app/src/ecalls.rs:6-64), with Rust's types
 *      mapped to C: sgx_enclave_id_t = u64, *mut sgx_status_t = uint32_t * (the SGX
 *      enum is repr(u32)), usize = size_t, f32 = float, u8 = uint8_t.  A C compiler
 *      rejects a redeclaration whose type differs from the header's, and the
 *      function-pointer assignments in check_abi() are compiled with -Werror: any
 *      drift between fltee_agg.h and ecalls.rs fails the build.
 *   2. main() runs the call sequence of the tonic server (server.rs:44-215):
 *        Start:     init_enclave -> ecall_fl_init -> ecall_start_round(0)
 *        Aggregate: optimal_num_of_clients check, alg 6 -> the client-size-optimized
 *                   ECALL else ecall_secure_aggregation, host wall time, then
 *                   ecall_start_round(round + 1, |ids|)
 *      and panics (exit 101, like a Rust panic) wherever server.rs panics.
 *
 * Input file (little-endian): u32 magic 'FLTH', u32 n, u32 alg, u32 fl_id, u64 d,
 * u64 k, u64 optimal_num_of_clients, f32 sampling_ratio, u32 dp, u64 bytes_per_client,
 * then n u32 client ids, then n ciphertext slices of bytes_per_client bytes, one per
 * id in that order (each client's AES-128-CTR payload, utils.py:268-304).  The host
 * concatenates the slices in the order the enclave sampled, as fl_main.py:221-249
 * does with secure_sampled_client_ids.
 * Output file: u32 retvals[4], u32 sampled[n_sampled], f32 updated[d], f32 times[4]
 * (load, decrypt, aggregate, host total: server.rs:184-186), u32 next_round, u32
 * next_ids[n_sampled].
 *
 * Exit codes: 0 ok, 2 usage/IO, 3 device init failed (no GPU), 101 panic.
 * Built by __graft_entry__.build() (gcc, C11); run by tests/test_abi_host.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fltee_agg.h"

/* ---- ecalls.rs:6-64, transcribed type for type ---------------------------- */
typedef uint64_t sgx_enclave_id_t;
typedef uint32_t sgx_status_t;

extern sgx_status_t ecall_fl_init(sgx_enclave_id_t eid, sgx_status_t *retval, uint32_t fl_id,
                                  const uint32_t *client_ids, size_t client_size,
                                  size_t num_of_parameters, size_t num_of_sparse_parameters,
                                  float sigma, float clipping, float alpha, float sampling_ratio,
                                  uint32_t aggregation_alg, uint8_t verbose, uint8_t dp);
extern sgx_status_t ecall_start_round(sgx_enclave_id_t eid, sgx_status_t *retval, uint32_t fl_id,
                                      uint32_t round, size_t sample_size,
                                      uint32_t *sampled_client_ids);
extern sgx_status_t ecall_secure_aggregation(sgx_enclave_id_t eid, sgx_status_t *retval,
                                             uint32_t fl_id, uint32_t round,
                                             const uint32_t *client_ids, size_t client_size,
                                             const uint8_t *encrypted_parameters_data,
                                             size_t encrypted_parameters_size,
                                             size_t num_of_parameters,
                                             size_t num_of_sparse_parameters,
                                             uint32_t aggregation_alg,
                                             float *updated_parameters_data,
                                             float *execution_time_results);
extern sgx_status_t ecall_client_size_optimized_secure_aggregation(
    sgx_enclave_id_t eid, sgx_status_t *retval, uint32_t fl_id, uint32_t round,
    size_t optimal_num_of_clients, const uint32_t *client_ids, size_t client_size,
    const uint8_t *encrypted_parameters_data_ptr, size_t num_of_parameters,
    size_t num_of_sparse_parameters, uint32_t aggregation_alg, float *updated_parameters_data,
    float *execution_time_results);

typedef sgx_status_t (*fl_init_fn)(sgx_enclave_id_t, sgx_status_t *, uint32_t, const uint32_t *,
                                   size_t, size_t, size_t, float, float, float, float, uint32_t,
                                   uint8_t, uint8_t);
typedef sgx_status_t (*start_round_fn)(sgx_enclave_id_t, sgx_status_t *, uint32_t, uint32_t,
                                       size_t, uint32_t *);
typedef sgx_status_t (*secure_aggregation_fn)(sgx_enclave_id_t, sgx_status_t *, uint32_t,
                                              uint32_t, const uint32_t *, size_t, const uint8_t *,
                                              size_t, size_t, size_t, uint32_t, float *, float *);
typedef sgx_status_t (*optimized_fn)(sgx_enclave_id_t, sgx_status_t *, uint32_t, uint32_t, size_t,
                                     const uint32_t *, size_t, const uint8_t *, size_t, size_t,
                                     uint32_t, float *, float *);

static void check_abi(void) {
    fl_init_fn a = ecall_fl_init;
    start_round_fn b = ecall_start_round;
    secure_aggregation_fn c = ecall_secure_aggregation;
    optimized_fn e = ecall_client_size_optimized_secure_aggregation;
    _Static_assert(sizeof(sgx_enclave_id_t) == sizeof(fltee_eid_t), "eid width");
    _Static_assert(sizeof(sgx_status_t) == sizeof(fltee_status_t), "status width");
    _Static_assert(sizeof(size_t) == 8, "usize is 64-bit on x86_64");
    (void)a; (void)b; (void)c; (void)e;
}

#define PANIC(msg)                                    \
    do {                                              \
        fprintf(stderr, "[Server] panic: %s\n", msg); \
        exit(101);                                    \
    } while (0)

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int read_exact(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

int main(int argc, char **argv) {
    check_abi();
    if (argc != 3) {
        fprintf(stderr, "usage: %s <in> <out>\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t magic, n, alg, fl_id, dp;
    uint64_t d, k, optimal, bpc;
    float ratio;
    if (read_exact(f, &magic, 4) || magic != 0x48544C46u || read_exact(f, &n, 4) ||
        read_exact(f, &alg, 4) || read_exact(f, &fl_id, 4) || read_exact(f, &d, 8) ||
        read_exact(f, &k, 8) || read_exact(f, &optimal, 8) || read_exact(f, &ratio, 4) ||
        read_exact(f, &dp, 4) || read_exact(f, &bpc, 8))
        return 2;
    uint32_t *ids = malloc((size_t)n * 4 + 4);
    uint8_t *slices = malloc((size_t)n * bpc + 1);
    if (!ids || !slices || read_exact(f, ids, (size_t)n * 4) || read_exact(f, slices, (size_t)n * bpc))
        return 2;
    fclose(f);

    /* init_enclave (ecalls.rs:66-83) -> device init */
    fltee_eid_t eid = 0;
    if (fltee_device_init(0, &eid) != FLTEE_SUCCESS) {
        fprintf(stderr, "[Server] Init Enclave Failed (no HIP device)\n");
        return 3;
    }
    uint32_t rvs[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

    /* ---- Start (server.rs:44-108) ---- */
    sgx_status_t retval = 0;
    sgx_status_t result = ecall_fl_init(eid, &retval, fl_id, ids, n, (size_t)d, (size_t)k, 1.12f,
                                        1.0f, 0.1f, ratio, alg, 0, (uint8_t)dp);
    rvs[0] = retval;
    if (result != 0 || retval != 0) PANIC("Error at ecall_fl_init");
    const size_t sample_size = (size_t)(ratio * (float)n); /* server.rs:84 */
    uint32_t *sampled = calloc(sample_size + 1, 4);
    result = ecall_start_round(eid, &retval, fl_id, 0, sample_size, sampled);
    rvs[1] = retval;
    if (result != 0 || retval != 0) PANIC("Error at ecall_start_round");

    /* ---- the client side: payloads concatenated in the sampled order ---- */
    uint8_t *enc = malloc(sample_size * bpc + 1);
    for (size_t i = 0; i < sample_size; ++i) {
        size_t j = 0;
        while (j < n && ids[j] != sampled[i]) ++j;
        if (j == n) PANIC("sampled id not in the client list");
        memcpy(enc + i * bpc, slices + j * bpc, bpc);
    }

    /* ---- Aggregate (server.rs:111-215) ---- */
    const uint32_t round = 0;
    if (optimal > sample_size && alg == 6) /* server.rs:126-128 (alg 6 only: SURVEY §8b) */
        PANIC("optimal_num_of_clients is more than client size");
    float *updated = calloc((size_t)d + 1, sizeof(float));
    float times[4] = {0, 0, 0, 0};
    const double t0 = now_s();
    if (alg == 6) {
        result = ecall_client_size_optimized_secure_aggregation(
            eid, &retval, fl_id, round, (size_t)optimal, sampled, sample_size, enc, (size_t)d,
            (size_t)k, alg, updated, times);
        rvs[2] = retval;
        if (result != 0 || retval != 0) PANIC("Error at ecall_client_size_optimized_secure_aggregation");
    } else {
        result = ecall_secure_aggregation(eid, &retval, fl_id, round, sampled, sample_size, enc,
                                          sample_size * bpc, (size_t)d, (size_t)k, alg, updated,
                                          times);
        rvs[2] = retval;
        if (result != 0 || retval != 0) PANIC("Error at ecall_secure_aggregation");
    }
    times[3] = (float)(now_s() - t0);
    const uint32_t next_round = round + 1;
    uint32_t *next_ids = calloc(sample_size + 1, 4);
    result = ecall_start_round(eid, &retval, fl_id, next_round, sample_size, next_ids);
    rvs[3] = retval;
    if (result != 0 || retval != 0) PANIC("[Server] Error at ecall_start_round");
    fltee_device_fini(eid);

    FILE *o = fopen(argv[2], "wb");
    if (!o) return 2;
    fwrite(rvs, 4, 4, o);
    fwrite(sampled, 4, sample_size, o);
    fwrite(updated, 4, (size_t)d, o);
    fwrite(times, 4, 4, o);
    fwrite(&next_round, 4, 1, o);
    fwrite(next_ids, 4, sample_size, o);
    fclose(o);
    printf("[Server] complete the round (alg %u, %zu clients, d %llu, %.6f s)\n", alg, sample_size,
           (unsigned long long)d, times[3]);
    free(ids); free(slices); free(sampled); free(enc); free(updated); free(next_ids);
    return 0;
}
