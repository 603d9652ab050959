/*
 * fltee_oracle.c — CPU restatement of FL-TEE's SGX enclave aggregation path
 * (secure_aggregation/enclave/src/ Rust files).  TEST INFRASTRUCTURE ONLY: see the
 * header for what may load it and for its parity status.
 *
 * Restated line-for-line, keeping the reference's loop structure and its x86
 * cmov primitives (oblivious_primitives.rs) so that the CPU timing taken from
 * here (bench.py cpu_baseline, kind "port") is faithful to the 1-TCS enclave.
 * Built single-threaded with -O2 like secure_aggregation/Makefile:54.
 */
#define _GNU_SOURCE
#include "fltee_oracle.h"

#include <math.h>
#include <openssl/evp.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* oblivious_primitives.rs — branch-free x86 primitives                      */
/* ------------------------------------------------------------------------ */

/* oblivious_primitives.rs:2-15  (cmp; sete) */
static inline int o_equal(uint64_t x, uint64_t y) {
    uint8_t r;
    __asm__ volatile("cmp %2, %1\n\tsete %0" : "=q"(r) : "r"(x), "r"(y) : "cc");
    return r;
}

/* oblivious_primitives.rs:19-32  (cmp; setb) — returns x < y (unsigned) */
static inline int o_setb(uint64_t x, uint64_t y) {
    uint8_t r;
    __asm__ volatile("cmp %2, %1\n\tsetb %0" : "=q"(r) : "r"(x), "r"(y) : "cc");
    return r;
}

/* oblivious_primitives.rs:39-56 — 8-byte cmov swap of a whole Weight */
static inline void o_swap(int64_t flag, uint64_t *x, uint64_t *y) {
    uint64_t a = *x, b = *y, t = a;
    __asm__ volatile("test %3, %3\n\tcmovnz %1, %0\n\tcmovnz %2, %1"
                     : "+&r"(a), "+&r"(b)
                     : "r"(t), "r"(flag)
                     : "cc");
    *x = a;
    *y = b;
}

/* oblivious_primitives.rs:61-76 — returns flag ? val : src */
static inline uint64_t o_mov(int64_t flag, uint64_t src, uint64_t val) {
    __asm__ volatile("test %2, %2\n\tcmovnz %1, %0" : "+&r"(src) : "r"(val), "r"(flag) : "cc");
    return src;
}

static inline uint64_t w2u(fo_weight w) { uint64_t u; memcpy(&u, &w, 8); return u; }
static inline fo_weight u2w(uint64_t u) { fo_weight w; memcpy(&w, &u, 8); return w; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* Rust `f32 as u32 / as usize` saturating casts */
static inline uint32_t f32_to_u32_sat(float x) {
    if (!(x > 0.0f)) return 0;            /* NaN and negatives -> 0 */
    if (x >= 4294967296.0f) return UINT32_MAX;
    return (uint32_t)x;
}
static inline size_t f32_to_usize_sat(float x) {
    if (!(x > 0.0f)) return 0;
    if (x >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)x;
}

/* Test-only parallelism for the comparator networks (each step's compare-exchanges
 * are independent, so the result is the same for any thread count).  Default 1: the
 * CPU baseline (bench.py) stays single-threaded like the 1-TCS enclave. */
static int g_threads = 1;
void fo_set_threads(int t) { g_threads = t > 0 ? t : 1; }

size_t fo_next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

/* ------------------------------------------------------------------------ */
/* shared counter-based generators (product uses the same definitions)        */
/* ------------------------------------------------------------------------ */

void fo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* lowbias32 integer mixer (a bijection on u32) */
uint32_t fo_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

uint32_t fo_shuffle_step_key(uint32_t seed, uint32_t stage_log2, uint32_t step_log2) {
    return fo_mix32(fo_mix32(seed) + ((stage_log2 << 8) | step_log2) * 0x9E3779B9u);
}

#define STREAM_DP 0x44504E5Au      /* "DPNZ" */
#define STREAM_LAPLACE 0x4C41504Cu /* "LAPL" */
#define STREAM_SAMPLE 0x534D504Cu  /* "SMPL" */

static inline double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------ */
/* crypto: lib.rs:312-343, session_key_store.rs:17-32                         */
/* ------------------------------------------------------------------------ */

void fo_session_key(uint32_t client_id, uint8_t key[16]) {
    memset(key, 0, 16);
    key[4] = (uint8_t)(client_id >> 24); /* client_id.to_be_bytes() into [4..8] */
    key[5] = (uint8_t)(client_id >> 16);
    key[6] = (uint8_t)(client_id >> 8);
    key[7] = (uint8_t)client_id;
}

/* sgx_tcrypto::rsgx_aes_ctr_decrypt with a zero 16-byte counter block and
 * ctr_inc_bits = 128: standard AES-128-CTR, big-endian 128-bit counter. */
int fo_aes128_ctr(const uint8_t key[16], const uint8_t *src, size_t len, uint8_t *dst) {
    uint8_t iv[16] = {0};
    int outl = 0, ok = 0;
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    if (!ctx) return -1;
    if (EVP_EncryptInit_ex(ctx, EVP_aes_128_ctr(), NULL, key, iv) == 1) {
        size_t done = 0;
        ok = 1;
        while (done < len) {
            int chunk = (len - done) > (1u << 30) ? (1 << 30) : (int)(len - done);
            if (EVP_EncryptUpdate(ctx, dst + done, &outl, src + done, chunk) != 1) { ok = 0; break; }
            done += (size_t)chunk;
        }
    }
    EVP_CIPHER_CTX_free(ctx);
    return ok ? 0 : -1;
}

int fo_decrypt_and_parse(const uint32_t *client_ids, size_t n, const uint8_t *enc,
                         size_t enc_len, fo_weight *out, size_t *n_out) {
    size_t bpc = enc_len / n;                 /* lib.rs:305 */
    size_t given_k = bpc / 8;                 /* lib.rs:306 */
    uint8_t *tmp = (uint8_t *)malloc(bpc ? bpc : 1);
    for (size_t i = 0; i < n; ++i) {
        uint8_t key[16];
        fo_session_key(client_ids[i], key);
        if (fo_aes128_ctr(key, enc + i * bpc, bpc, tmp) != 0) { free(tmp); return -1; }
        /* parameters.rs:53-67: [u32 LE idx][f32 LE val] records */
        memcpy(out + i * given_k, tmp, given_k * 8);
    }
    free(tmp);
    *n_out = n * given_k;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* common.rs                                                                  */
/* ------------------------------------------------------------------------ */

/* common.rs:14-19 — multiply by the f32 reciprocal (NOT a division) */
void fo_average_params(float *g, size_t d, size_t n) {
    float coef = 1.0f / (float)n;
    for (size_t i = 0; i < d; ++i) g[i] *= coef;
}

/* common.rs:25-35 */
void fo_safe_aggregate(float *g, size_t d, const fo_weight *s, size_t ns, size_t n) {
    uint32_t k = (uint32_t)d;
    for (size_t i = 0; i < ns; ++i)
        if (s[i].idx < k) g[s[i].idx] += s[i].val;
    fo_average_params(g, d, n);
}

/* ------------------------------------------------------------------------ */
/* non_oblivious.rs:6-15                                                      */
/* ------------------------------------------------------------------------ */
uint32_t fo_non_oblivious(float *g, size_t d, const fo_weight *w, size_t nw, size_t n) {
    for (size_t i = 0; i < nw; ++i) {
        if ((size_t)w[i].idx >= d) return FO_ERROR_ENCLAVE_CRASHED; /* Rust bounds panic */
        g[w[i].idx] += w[i].val;
    }
    fo_average_params(g, d, n);
    return FO_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* baseline.rs:7-60 — per pair, one cmov RMW in every 64-byte line           */
/* ------------------------------------------------------------------------ */
#define CACHE_LINE_NUM_OF_WEIGHT 16
static inline void o_update(float *dst_base, int64_t num, int64_t addr_off, float val) {
    float *addr = dst_base + addr_off;
    int64_t ith = addr_off % CACHE_LINE_NUM_OF_WEIGHT;
    int64_t last = 0;
    for (int64_t i = 0; i < num / CACHE_LINE_NUM_OF_WEIGHT; ++i) {
        float *cl = dst_base + CACHE_LINE_NUM_OF_WEIGHT * i + ith;
        int64_t flag = (cl == addr);
        float cur = *cl, upd = cur + val;
        *cl = u2f((uint32_t)o_mov(flag, f2u(cur), f2u(upd)));
        last += 1;
    }
    float *cl = dst_base + CACHE_LINE_NUM_OF_WEIGHT * last;
    for (int64_t j = 0; j < num % CACHE_LINE_NUM_OF_WEIGHT; ++j) {
        float *rv = cl + j;
        int64_t flag = (rv == addr);
        float cur = *rv, upd = cur + val;
        *rv = u2f((uint32_t)o_mov(flag, f2u(cur), f2u(upd)));
    }
}

void fo_baseline(float *g, size_t d, const fo_weight *w, size_t nw, size_t n) {
    for (size_t i = 0; i < nw; ++i) o_update(g, (int64_t)d, (int64_t)w[i].idx, w[i].val);
    fo_average_params(g, d, n);
}

/* ------------------------------------------------------------------------ */
/* oram.rs:86-118 — output semantics of the PathORAM aggregation: each pair  */
/* is read-modify-written in upload order, then d reads.  The ORAM holds     */
/* next_pow2(d) blocks; writes to [d, next_pow2(d)) are accepted but never   */
/* read back, anything beyond is an out-of-range ORAM access (panic).        */
/* ------------------------------------------------------------------------ */
uint32_t fo_path_oram(float *g, size_t d, const fo_weight *w, size_t nw, size_t n) {
    size_t cap = fo_next_pow2(d);
    for (size_t i = 0; i < nw; ++i) {
        if ((size_t)w[i].idx >= cap) return FO_ERROR_ENCLAVE_CRASHED;
        if ((size_t)w[i].idx < d) g[w[i].idx] += w[i].val;
    }
    fo_average_params(g, d, n);
    return FO_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* advanced.rs                                                                */
/* ------------------------------------------------------------------------ */

/* advanced.rs:147-176 — swap iff ((l & i) == 0) ^ (key[l] < key[m]) */
void fo_bitonic_sort_by_idx(fo_weight *s, size_t size) {
    size_t half = size >> 1;
    for (size_t i = 2; i <= size; i <<= 1) {
        for (size_t j = i >> 1; j > 0; j >>= 1) {
            size_t ml = j - 1, mh = ~ml;
#pragma omp parallel for if (g_threads > 1 && half >= 65536) num_threads(g_threads) schedule(static)
            for (size_t k = 0; k < half; ++k) {
                size_t l = ((k & mh) << 1) | (k & ml);
                size_t m = l + j;
                int cond1 = (l & i) == 0;
                int cond2 = s[l].idx < s[m].idx;
                o_swap((int64_t)(cond1 ^ cond2), (uint64_t *)&s[l], (uint64_t *)&s[m]);
            }
        }
    }
}

/* advanced.rs:66-101 — oblivious fold over the first fold_len entries */
void fo_fold(fo_weight *s, size_t fold_len) {
    uint32_t pre_idx = s[0].idx;
    float pre_val = s[0].val;
    uint32_t dummy_idx = UINT32_MAX;
    for (size_t i = 1; i < fold_len; ++i) {
        int64_t eq = (pre_idx == s[i].idx);
        fo_weight pre = {pre_idx, pre_val}, dummy = {dummy_idx, 0.0f};
        s[i - 1] = u2w(o_mov(eq, w2u(pre), w2u(dummy)));
        fo_weight cur = s[i], acc = {pre_idx, pre_val + s[i].val};
        fo_weight nxt = u2w(o_mov(eq, w2u(cur), w2u(acc)));
        pre_idx = nxt.idx;
        pre_val = nxt.val;
        dummy_idx -= 1;
    }
    s[fold_len - 1].idx = pre_idx;
    s[fold_len - 1].val = pre_val;
}

/* advanced.rs:126-142 — pad with (u32::MAX, 0.0), sort, truncate */
static void oblivious_sort_idx(fo_weight *s, size_t len) {
    size_t m = fo_next_pow2(len);
    for (size_t i = len; i < m; ++i) { s[i].idx = UINT32_MAX; s[i].val = 0.0f; }
    fo_bitonic_sort_by_idx(s, m);
}

uint32_t fo_advanced_core(size_t k_req, size_t d, const fo_weight *w, size_t nw, size_t n,
                          fo_weight *scratch, size_t scratch_cap) {
    size_t len = nw + d;
    if (fo_next_pow2(len) > scratch_cap) return FO_ERROR_UNEXPECTED;
    memcpy(scratch, w, nw * sizeof(fo_weight));
    for (size_t i = 0; i < d; ++i) { scratch[nw + i].idx = (uint32_t)i; scratch[nw + i].val = 0.0f; } /* :116-123 */
    oblivious_sort_idx(scratch, len);                                                           /* :59 */
    size_t fold_len = n * k_req + d;                                                            /* :70 */
    if (fold_len > len || fold_len == 0) return FO_ERROR_ENCLAVE_CRASHED; /* Rust index panic */
    fo_fold(scratch, fold_len);
    oblivious_sort_idx(scratch, len);                                                           /* :109 */
    return FO_SUCCESS;
}

uint32_t fo_advanced(size_t k_req, float *g, size_t d, const fo_weight *w, size_t nw, size_t n,
                     fo_weight *scratch, size_t scratch_cap) {
    uint32_t st = fo_advanced_core(k_req, d, w, nw, n, scratch, scratch_cap);
    if (st != FO_SUCCESS) return st;
    for (size_t i = 0; i < d; ++i) g[i] = scratch[i].val; /* :32-34 */
    fo_average_params(g, d, n);
    return FO_SUCCESS;
}

/* lib.rs:498-573 + advanced.rs:10-21 (weights already decrypted, n*k entries) */
uint32_t fo_client_size_optimized(size_t batch, size_t k, float *g, size_t d, const fo_weight *w,
                                  size_t n, fo_weight *scratch, size_t scratch_cap) {
    if (batch == 0) return FO_ERROR_ENCLAVE_CRASHED; /* division by zero panic, lib.rs:499 */
    size_t cursor = 0, cursor_last = n / batch;
    while (cursor <= cursor_last) {
        if (cursor * batch >= n) break;
        size_t to = (cursor + 1) * batch < n ? (cursor + 1) * batch : n;
        size_t nb = to - cursor * batch;
        uint32_t st = fo_advanced_core(k, d, w + cursor * batch * k, nb * k, nb, scratch, scratch_cap);
        if (st != FO_SUCCESS) return st;
        for (size_t i = 0; i < d; ++i) g[i] += scratch[i].val;
        cursor += 1;
    }
    fo_average_params(g, d, n);
    return FO_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* nips19.rs + common.rs                                                      */
/* ------------------------------------------------------------------------ */

float fo_nips19_threshold(size_t d, size_t k, size_t n) {
    float epsilon = 100.0f;                   /* nips19.rs:25 */
    float delta = 1.0f / (float)n;            /* nips19.rs:26 */
    float l1 = 2.0f * (float)k;               /* common.rs:78 */
    return l1 / epsilon * logf((float)d / delta); /* common.rs:81 */
}

static inline float ln_f32(float x) { return (float)log((double)x); }

/* common.rs:77-98 (uniform from Philox instead of sgx_rand StdRng) and
 * common.rs:151-161 transform_to_random_int_vec */
void fo_laplace_r(size_t d, size_t k, size_t n, uint64_t seed, uint32_t *r, float *T_out) {
    float T = fo_nips19_threshold(d, k, n);
    float b = 2.0f * (float)k / 100.0f;
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (size_t i = 0; i < d; ++i) {
        uint32_t ctr[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), 0, STREAM_LAPLACE}, o[4];
        fo_philox4x32_10(ctr, key, o);
        float p = (float)(o[0] >> 8) * (1.0f / 16777216.0f);
        /* f32 ln as (float)ln((double)x): correctly rounded in practice and the same
         * bits on the GPU (k_nips19.hip), so the Laplace counts match exactly */
        float noise = p > 0.5f ? -b * ln_f32(2.0f - 2.0f * p) : b * ln_f32(2.0f * p);
        r[i] = fabsf(noise) > T ? f32_to_u32_sat(ceilf(T)) : f32_to_u32_sat(T + ceilf(noise));
    }
    if (T_out) *T_out = T;
}

/* common.rs:189-197 — d * floor(T) dummies, (r_i < j) ? i : u32::MAX */
size_t fo_oblivious_pad(const uint32_t *r, size_t d, float T, fo_weight *out) {
    size_t rmax = f32_to_usize_sat(T), o = 0;
    for (size_t i = 0; i < d; ++i) {
        size_t ri = r[i];
        for (size_t j = 0; j < rmax; ++j) {
            int flag = o_setb(ri, j);
            out[o].idx = (uint32_t)o_mov(flag, UINT32_MAX, (uint32_t)i);
            out[o].val = 0.0f;
            ++o;
        }
    }
    return o;
}

/* nips19.rs:66-105 with the comparator bit drawn from the product's keyed
 * mixer instead of a running FxHash of heap addresses. */
void fo_shuffle_keyed(fo_weight *s, size_t size, uint32_t seed) {
    size_t half = size >> 1;
    uint32_t ilog = 1;
    for (size_t i = 2; i <= size; i <<= 1, ++ilog) {
        uint32_t jlog = ilog - 1;
        for (size_t j = i >> 1; j > 0; j >>= 1, --jlog) {
            size_t ml = j - 1, mh = ~ml;
            uint32_t key = fo_shuffle_step_key(seed, ilog, jlog);
#pragma omp parallel for if (g_threads > 1 && half >= 65536) num_threads(g_threads) schedule(static)
            for (size_t k = 0; k < half; ++k) {
                size_t l = ((k & mh) << 1) | (k & ml);
                size_t m = l + j;
                int cond1 = o_equal(l & i, 0);
                int cond2 = (int)((((uint32_t)l ^ key) * 0x9E3779B1u) >> 31);
                o_swap((int64_t)(cond1 ^ cond2), (uint64_t *)&s[l], (uint64_t *)&s[m]);
            }
        }
    }
}

/* fxhash.rs:9-24 */
static inline uint64_t fx_add(uint64_t h, uint64_t i) {
    return (((h << 5) | (h >> 59)) ^ i) * 0x517cc1b727220a95ull;
}

/* nips19.rs:66-105 verbatim: cond2 = setb(h1, h2) of a running FxHash over
 * the ADDRESSES of source[l] and source[m]. */
void fo_shuffle_fxhash(fo_weight *s, size_t size) {
    size_t half = size >> 1;
    uint64_t h = fx_add(0, 100);
    for (size_t i = 2; i <= size; i <<= 1) {
        for (size_t j = i >> 1; j > 0; j >>= 1) {
            size_t ml = j - 1, mh = ~ml;
            for (size_t k = 0; k < half; ++k) {
                size_t l = ((k & mh) << 1) | (k & ml);
                size_t m = l + j;
                int cond1 = o_equal(l & i, 0);
                h = fx_add(h, (uint64_t)(uintptr_t)&s[l]);
                uint64_t h1 = h;
                h = fx_add(h, (uint64_t)(uintptr_t)&s[m]);
                uint64_t h2 = h;
                int cond2 = o_setb(h1, h2);
                o_swap((int64_t)(cond1 ^ cond2), (uint64_t *)&s[l], (uint64_t *)&s[m]);
            }
        }
    }
}

/* nips19.rs:18-63 */
uint32_t fo_nips19(size_t k, float *g, size_t d, const fo_weight *w, size_t nw, size_t n,
                   uint64_t seed, int reference_shuffle, fo_weight *scratch, size_t scratch_cap) {
    uint32_t *r = (uint32_t *)malloc((d ? d : 1) * sizeof(uint32_t));
    float T;
    fo_laplace_r(d, k, n, seed, r, &T);
    size_t npad = (size_t)d * f32_to_usize_sat(T);
    size_t len = nw + npad, m = fo_next_pow2(len);
    if (m > scratch_cap) { free(r); return FO_ERROR_UNEXPECTED; }
    memcpy(scratch, w, nw * sizeof(fo_weight));
    fo_oblivious_pad(r, d, T, scratch + nw);
    free(r);
    for (size_t i = len; i < m; ++i) { scratch[i].idx = UINT32_MAX; scratch[i].val = 0.0f; }
    if (reference_shuffle) fo_shuffle_fxhash(scratch, m);
    else fo_shuffle_keyed(scratch, m, (uint32_t)(seed ^ (seed >> 32)));
    fo_safe_aggregate(g, d, scratch, m, n);
    return FO_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* DP and clipping                                                            */
/* ------------------------------------------------------------------------ */

/* common.rs:56-72: g[i] += (N(0, clipping*sigma) as f64 / n) as f32 */
void fo_dp_noise(float *g, size_t d, float sigma, float clipping, size_t n, uint64_t seed) {
    double stddev = (double)(clipping * sigma);
    double nn = (double)n;
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (size_t i = 0; i < d; ++i) {
        uint32_t ctr[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), 0, STREAM_DP}, o[4];
        fo_philox4x32_10(ctr, key, o);
        double u1 = 1.0 - u53(o[0], o[1]);
        double u2 = u53(o[2], o[3]);
        double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        g[i] += (float)((0.0 + stddev * z) / nn);
    }
}

/* update.py:187-204 — coef = min(1, C / ||v||_2), v *= coef (fp32) */
void fo_l2_clip(float *vals, size_t k, float clipping) {
    double ss = 0.0;
    for (size_t i = 0; i < k; ++i) ss += (double)vals[i] * (double)vals[i];
    float norm = (float)sqrt(ss);
    float coef = clipping / norm;
    if (!(coef < 1.0f)) coef = 1.0f;
    for (size_t i = 0; i < k; ++i) vals[i] *= coef;
}

/* ------------------------------------------------------------------------ */
/* common.rs:101-105 — sgx_rand::sample (reservoir), Philox-driven           */
/* ------------------------------------------------------------------------ */
static uint64_t sample_draw(uint64_t seed, uint64_t *counter) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)*counter, (uint32_t)(*counter >> 32), 0, STREAM_SAMPLE}, o[4];
    fo_philox4x32_10(ctr, key, o);
    *counter += 1;
    return ((uint64_t)o[1] << 32) | o[0];
}

static uint64_t gen_range(uint64_t seed, uint64_t *counter, uint64_t range) {
    uint64_t zone = UINT64_MAX - UINT64_MAX % range;
    for (;;) {
        uint64_t v = sample_draw(seed, counter);
        if (v < zone) return v % range;
    }
}

void fo_sample_client_ids(const uint32_t *ids, size_t m, size_t amount, uint64_t seed,
                          uint32_t *out) {
    size_t take = amount < m ? amount : m;
    for (size_t i = 0; i < take; ++i) out[i] = ids[i];
    if (take != amount) return;
    uint64_t counter = 0;
    for (size_t i = 0; i + amount < m; ++i) {
        uint64_t k = gen_range(seed, &counter, (uint64_t)(i + 1 + amount));
        if (k < amount) out[k] = ids[amount + i];
    }
}

/* ------------------------------------------------------------------------ */
/* lib.rs — ECALL state machine (process-global like FL_CONFIG_MAP)          */
/* ------------------------------------------------------------------------ */
typedef struct {
    int used;
    uint32_t fl_id;
    uint32_t *client_ids;
    size_t client_size, d, k;
    float sigma, clipping, alpha, ratio;
    uint32_t alg, round;
    uint8_t verbose, dp;
    uint32_t *sampled; /* sorted copy of the current sample */
    size_t n_sampled;
} fo_cfg;

#define FO_MAX_CFG 64
static fo_cfg g_cfg[FO_MAX_CFG];
static uint32_t *g_keys; /* sorted set of client ids with a session key */
static size_t g_nkeys;
static int g_have_keys;
static uint64_t g_seed;
static int g_seeded;
static uint64_t g_calls;

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}
static int has_u32(const uint32_t *s, size_t n, uint32_t v) {
    return bsearch(&v, s, n, sizeof(uint32_t), cmp_u32) != NULL;
}
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static uint64_t next_seed(void) {
    if (g_seeded) return g_seed + 0x9E3779B97F4A7C15ull * (++g_calls);
    uint64_t s = 0;
    if (getrandom(&s, sizeof s, 0) != sizeof s) s = (uint64_t)time(NULL);
    return s;
}

void fo_reset(void) {
    for (int i = 0; i < FO_MAX_CFG; ++i) {
        free(g_cfg[i].client_ids);
        free(g_cfg[i].sampled);
        memset(&g_cfg[i], 0, sizeof g_cfg[i]);
    }
    free(g_keys);
    g_keys = NULL;
    g_nkeys = 0;
    g_have_keys = 0;
    g_seeded = 0;
    g_calls = 0;
}

void fo_set_seed(uint64_t seed) { g_seed = seed; g_seeded = 1; g_calls = 0; }

static fo_cfg *find_cfg(uint32_t fl_id) {
    for (int i = 0; i < FO_MAX_CFG; ++i)
        if (g_cfg[i].used && g_cfg[i].fl_id == fl_id) return &g_cfg[i];
    return NULL;
}

/* lib.rs:113-180 */
uint32_t fo_ecall_fl_init(uint32_t fl_id, const uint32_t *client_ids, size_t client_size,
                          size_t d, size_t k, float sigma, float clipping, float alpha,
                          float sampling_ratio, uint32_t alg, uint8_t verbose, uint8_t dp) {
    fo_cfg *c = find_cfg(fl_id);
    if (!c) {
        for (int i = 0; i < FO_MAX_CFG && !c; ++i)
            if (!g_cfg[i].used) c = &g_cfg[i];
        if (!c) return FO_ERROR_UNEXPECTED;
    }
    free(c->client_ids);
    free(c->sampled);
    memset(c, 0, sizeof *c);
    c->used = 1;
    c->fl_id = fl_id;
    c->client_ids = (uint32_t *)malloc((client_size ? client_size : 1) * 4);
    memcpy(c->client_ids, client_ids, client_size * 4);
    c->client_size = client_size;
    c->d = d; c->k = k; c->sigma = sigma; c->clipping = clipping; c->alpha = alpha;
    c->ratio = sampling_ratio; c->alg = alg; c->verbose = verbose; c->dp = dp;
    c->round = 0;
    /* mock_remote_attestation / SessionKeyStore::add (lib.rs:163-174) */
    size_t nk = g_nkeys + client_size;
    g_keys = (uint32_t *)realloc(g_keys, (nk ? nk : 1) * 4);
    for (size_t i = 0; i < client_size; ++i)
        if (!has_u32(g_keys, g_nkeys, client_ids[i])) g_keys[g_nkeys++] = client_ids[i];
    qsort(g_keys, g_nkeys, 4, cmp_u32);
    g_have_keys = 1;
    return FO_SUCCESS;
}

/* lib.rs:182-219 */
uint32_t fo_ecall_start_round(uint32_t fl_id, uint32_t round, size_t sample_size, uint32_t *out) {
    fo_cfg *c = find_cfg(fl_id);
    if (!c) return FO_ERROR_UNEXPECTED;
    if (c->round != round) return FO_ERROR_INVALID_PARAMETER;
    size_t calc = f32_to_usize_sat((float)c->client_size * c->ratio);
    if (calc != sample_size) return FO_ERROR_INVALID_PARAMETER;
    uint32_t *tmp = (uint32_t *)calloc(calc ? calc : 1, 4);
    fo_sample_client_ids(c->client_ids, c->client_size, calc, next_seed(), tmp);
    size_t got = calc < c->client_size ? calc : c->client_size;
    memcpy(out, tmp, got * 4);
    free(c->sampled);
    c->sampled = tmp;
    c->n_sampled = got;
    qsort(c->sampled, got, 4, cmp_u32);
    /* HashSet semantics: duplicates collapse (ids are distinct in practice) */
    size_t u = 0;
    for (size_t i = 0; i < got; ++i)
        if (u == 0 || c->sampled[u - 1] != c->sampled[i]) c->sampled[u++] = c->sampled[i];
    c->n_sampled = u;
    return FO_SUCCESS;
}

static uint32_t check_uploaded(fo_cfg *c, const uint32_t *ids, size_t n) {
    if (n != c->n_sampled) return FO_ERROR_INVALID_PARAMETER; /* lib.rs:269-272 */
    for (size_t i = 0; i < n; ++i)
        if (!has_u32(c->sampled, c->n_sampled, ids[i])) return FO_ERROR_INVALID_PARAMETER;
    return FO_SUCCESS;
}

/* lib.rs:221-423 */
uint32_t fo_ecall_secure_aggregation(uint32_t fl_id, uint32_t round, const uint32_t *client_ids,
                                     size_t client_size, const uint8_t *enc, size_t enc_len,
                                     size_t d, size_t k, uint32_t alg, float *out, float *times) {
    fo_cfg *c = find_cfg(fl_id);
    if (!c) return FO_ERROR_UNEXPECTED;
    if (c->round != round) return FO_ERROR_INVALID_PARAMETER;
    if (c->alg != alg) return FO_ERROR_INVALID_PARAMETER;
    memset(out, 0, d * sizeof(float)); /* Enclave_t.c:626 zero-fills [out] */
    memset(times, 0, 3 * sizeof(float));
    double t0 = now_s();
    if (client_size == 0) return FO_ERROR_INVALID_PARAMETER;
    uint32_t st = check_uploaded(c, client_ids, client_size);
    if (st) return st;
    uint8_t *copy = (uint8_t *)malloc(enc_len ? enc_len : 1); /* lib.rs:285-290 */
    memcpy(copy, enc, enc_len);
    times[0] = (float)(now_s() - t0);

    double t1 = now_s();
    for (size_t i = 0; i < client_size; ++i)
        if (!has_u32(g_keys, g_nkeys, client_ids[i])) { free(copy); return FO_ERROR_UNEXPECTED; }
    size_t given_k = (enc_len / client_size) / 8, nw = 0;
    fo_weight *w = (fo_weight *)malloc(((client_size * given_k) > 0 ? client_size * given_k : 1) * 8);
    if (fo_decrypt_and_parse(client_ids, client_size, copy, enc_len, w, &nw) != 0) {
        free(copy); free(w); return FO_ERROR_UNEXPECTED;
    }
    free(copy);
    times[1] = (float)(now_s() - t1);

    double t2 = now_s();
    size_t n = client_size;
    fo_weight *scratch = NULL;
    size_t cap = 0;
    switch (alg) {
    case 1:
        cap = fo_next_pow2(nw + d);
        scratch = (fo_weight *)malloc(cap * 8);
        st = fo_advanced(k, out, d, w, nw, n, scratch, cap);
        break;
    case 2: {
        float T = fo_nips19_threshold(d, k, n);
        cap = fo_next_pow2(nw + d * f32_to_usize_sat(T));
        scratch = (fo_weight *)malloc(cap * 8);
        st = fo_nips19(k, out, d, w, nw, n, next_seed(), 0, scratch, cap);
        break;
    }
    case 3: fo_baseline(out, d, w, nw, n); break;
    case 4: st = fo_non_oblivious(out, d, w, nw, n); break;
    case 5: st = fo_path_oram(out, d, w, nw, n); break;
    default: st = FO_ERROR_INVALID_PARAMETER; break; /* lib.rs:396 panics */
    }
    free(scratch);
    free(w);
    if (st) { /* a panic aborts the ECALL: the bridge never copies [out] back */
        memset(out, 0, d * sizeof(float));
        return st == FO_ERROR_ENCLAVE_CRASHED ? FO_ERROR_INVALID_PARAMETER : st;
    }
    if (c->dp) fo_dp_noise(out, d, c->sigma, c->clipping, n, next_seed());
    times[2] = (float)(now_s() - t2);
    c->round += 1; /* lib.rs:421 */
    return FO_SUCCESS;
}

/* lib.rs:425-592 */
uint32_t fo_ecall_client_size_optimized_secure_aggregation(
    uint32_t fl_id, uint32_t round, size_t batch, const uint32_t *client_ids, size_t client_size,
    const uint8_t *enc, size_t d, size_t k, uint32_t alg, float *out, float *times) {
    fo_cfg *c = find_cfg(fl_id);
    if (!c) return FO_ERROR_UNEXPECTED;
    if (c->round != round) return FO_ERROR_INVALID_PARAMETER;
    if (c->alg != alg) return FO_ERROR_INVALID_PARAMETER;
    memset(out, 0, d * sizeof(float));
    memset(times, 0, 3 * sizeof(float));
    if (client_size == 0 || batch == 0) return FO_ERROR_INVALID_PARAMETER;
    uint32_t st = check_uploaded(c, client_ids, client_size);
    if (st) return st;
    for (size_t i = 0; i < client_size; ++i)
        if (!has_u32(g_keys, g_nkeys, client_ids[i])) return FO_ERROR_UNEXPECTED;
    double t1 = now_s();
    size_t nw = 0;
    fo_weight *w = (fo_weight *)malloc(((client_size * k) > 0 ? client_size * k : 1) * 8);
    /* decrypting slice by slice is identical to decrypting the batches */
    if (fo_decrypt_and_parse(client_ids, client_size, enc, client_size * k * 8, w, &nw) != 0) {
        free(w); return FO_ERROR_UNEXPECTED;
    }
    size_t b = batch < client_size ? batch : client_size;
    size_t cap = fo_next_pow2(b * k + d);
    fo_weight *scratch = (fo_weight *)malloc(cap * 8);
    st = fo_client_size_optimized(batch, k, out, d, w, client_size, scratch, cap);
    free(scratch);
    free(w);
    if (st) { /* a panic aborts the ECALL: the bridge never copies [out] back */
        memset(out, 0, d * sizeof(float));
        return st == FO_ERROR_ENCLAVE_CRASHED ? FO_ERROR_INVALID_PARAMETER : st;
    }
    times[1] = (float)(now_s() - t1);
    if (c->dp) fo_dp_noise(out, d, c->sigma, c->clipping, client_size, next_seed());
    c->round += 1;
    return FO_SUCCESS;
}
