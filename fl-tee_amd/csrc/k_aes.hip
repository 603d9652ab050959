// k_aes.hip — AES-128-CTR decrypt of the uploaded client slices (gfx950).
//
// lib.rs:312-343: each client's slice is decrypted with rsgx_aes_ctr_decrypt
// under its session key (session_key_store.rs:17-32: 16 zero bytes with
// bytes[4..8] = client_id big-endian), a zero 16-byte counter block and
// ctr_inc_bits = 128, i.e. keystream block b = AES_k(BE128(b)).  The
// plaintext is the record stream [u32 LE idx][f32 LE val] (parameters.rs:53-67),
// which is also the in-HBM record layout: decrypt == parse.
//
// One lane per 16-byte block; T-tables (4 x 1 KB) and the S-box (1 KB) are
// staged in LDS per workgroup; round keys (44 words per client) are expanded on
// the host and read through L1.  Tables are generated at start-up from the
// GF(2^8) definition of the S-box (FIPS-197 §5.1.1), not typed in.
#include <mutex>

#include "common.h"

namespace fltee {

static uint8_t g_sbox[256];
static uint32_t g_te[5][256];  // Te0..Te3, S-box widened (Te4)
static std::once_flag g_tables_once;
static uint32_t *g_dev_tables[64];  // per device
static std::mutex g_dev_mu;

static inline uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return p;
}
static inline uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
static inline uint32_t rotr32(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }

static void build_tables() {
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) {  // x^254 = x^-1 in GF(2^8)
            uint8_t r = 1, b = (uint8_t)x;
            int e = 254;
            while (e) {
                if (e & 1) r = gmul(r, b);
                b = gmul(b, b);
                e >>= 1;
            }
            inv = r;
        }
        g_sbox[x] = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
    }
    for (int x = 0; x < 256; ++x) {
        const uint8_t s = g_sbox[x];
        const uint32_t t = ((uint32_t)gmul(s, 2) << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) |
                           (uint32_t)gmul(s, 3);
        g_te[0][x] = t;
        g_te[1][x] = rotr32(t, 8);
        g_te[2][x] = rotr32(t, 16);
        g_te[3][x] = rotr32(t, 24);
        g_te[4][x] = s;
    }
}

void aes128_expand_key(const uint8_t key[16], uint32_t rk[44]) {
    std::call_once(g_tables_once, build_tables);
    for (int i = 0; i < 4; ++i)
        rk[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
                ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
    uint8_t rc = 1;
    for (int i = 4; i < 44; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            t = (t << 8) | (t >> 24);  // RotWord
            t = ((uint32_t)g_sbox[t >> 24] << 24) | ((uint32_t)g_sbox[(t >> 16) & 0xff] << 16) |
                ((uint32_t)g_sbox[(t >> 8) & 0xff] << 8) | g_sbox[t & 0xff];
            t ^= (uint32_t)rc << 24;
            rc = xtime(rc);
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

// One AES-128 block encryption, big-endian word state (FIPS-197 / T-table form).
__host__ __device__ __forceinline__ void aes128_block(const uint32_t *T0, const uint32_t *T1,
                                                      const uint32_t *T2, const uint32_t *T3,
                                                      const uint32_t *S, const uint32_t *rk,
                                                      uint32_t s0, uint32_t s1, uint32_t s2,
                                                      uint32_t s3, uint32_t out[4]) {
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t t0 = T0[s0 >> 24] ^ T1[(s1 >> 16) & 0xff] ^ T2[(s2 >> 8) & 0xff] ^ T3[s3 & 0xff] ^ rk[4 * r];
        const uint32_t t1 = T0[s1 >> 24] ^ T1[(s2 >> 16) & 0xff] ^ T2[(s3 >> 8) & 0xff] ^ T3[s0 & 0xff] ^ rk[4 * r + 1];
        const uint32_t t2 = T0[s2 >> 24] ^ T1[(s3 >> 16) & 0xff] ^ T2[(s0 >> 8) & 0xff] ^ T3[s1 & 0xff] ^ rk[4 * r + 2];
        const uint32_t t3 = T0[s3 >> 24] ^ T1[(s0 >> 16) & 0xff] ^ T2[(s1 >> 8) & 0xff] ^ T3[s2 & 0xff] ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    out[0] = ((S[s0 >> 24] << 24) | (S[(s1 >> 16) & 0xff] << 16) | (S[(s2 >> 8) & 0xff] << 8) | S[s3 & 0xff]) ^ rk[40];
    out[1] = ((S[s1 >> 24] << 24) | (S[(s2 >> 16) & 0xff] << 16) | (S[(s3 >> 8) & 0xff] << 8) | S[s0 & 0xff]) ^ rk[41];
    out[2] = ((S[s2 >> 24] << 24) | (S[(s3 >> 16) & 0xff] << 16) | (S[(s0 >> 8) & 0xff] << 8) | S[s1 & 0xff]) ^ rk[42];
    out[3] = ((S[s3 >> 24] << 24) | (S[(s0 >> 16) & 0xff] << 16) | (S[(s1 >> 8) & 0xff] << 8) | S[s2 & 0xff]) ^ rk[43];
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// lane -> (client c, block b); blocks_per_client = ceil(rec_per_client * 8 / 16).
// ALIGNED: every slice starts on an 8-byte boundary (bpc % 8 == 0, the unchanged
// client).  Otherwise (enc_len % n != 0: lib.rs:305 floors bpc, so slice i starts
// at i*bpc) the ciphertext is read byte by byte; the output stays compact records.
__device__ __forceinline__ uint32_t ld_u32_bytes(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// block_off: the slices are the bytes [16 * block_off, ...) of each client's payload (a
// column slice of dense uploads, one GPU's parameter range): counter block b + block_off.
// idx_sub is subtracted from every record's idx (the slice's first parameter), so that
// the dense kernels' idx == position check runs on slice-local positions.
template <bool ALIGNED>
__global__ __launch_bounds__(256) void aes_ctr_kernel(const uint8_t *__restrict__ cipher,
                                                      size_t n, size_t bpc, size_t rpc,
                                                      const uint32_t *__restrict__ rks,
                                                      const uint32_t *__restrict__ tables,
                                                      uint8_t *__restrict__ plain,
                                                      uint64_t block_off, uint32_t idx_sub) {
    __shared__ uint32_t T[5 * 256];
    for (uint32_t e = threadIdx.x; e < 5 * 256; e += 256) T[e] = tables[e];
    __syncthreads();
    const size_t bpcl = (rpc + 1) / 2;  // 16-byte blocks per client
    const size_t total = n * bpcl;
    for (size_t g = (size_t)blockIdx.x * 256 + threadIdx.x; g < total;
         g += (size_t)gridDim.x * 256) {
        const size_t c = g / bpcl, b = g - c * bpcl;
        const uint64_t ctr = (uint64_t)b + block_off;
        uint32_t ks[4];
        aes128_block(T, T + 256, T + 512, T + 768, T + 1024, rks + c * 44, 0u, 0u,
                     (uint32_t)(ctr >> 32), (uint32_t)ctr, ks);
        uint2 *dst = reinterpret_cast<uint2 *>(plain + c * rpc * 8) + 2 * b;
        const bool two = 2 * b + 1 < rpc;
        uint2 x, y = make_uint2(0, 0);
        if (ALIGNED) {
            const uint2 *src = reinterpret_cast<const uint2 *>(cipher + c * bpc) + 2 * b;
            x = src[0];
            if (two) y = src[1];
        } else {
            const uint8_t *src = cipher + c * bpc + 16 * b;
            x = make_uint2(ld_u32_bytes(src), ld_u32_bytes(src + 4));
            if (two) y = make_uint2(ld_u32_bytes(src + 8), ld_u32_bytes(src + 12));
        }
        dst[0] = make_uint2((x.x ^ bswap32(ks[0])) - idx_sub, x.y ^ bswap32(ks[1]));
        if (two) dst[1] = make_uint2((y.x ^ bswap32(ks[2])) - idx_sub, y.y ^ bswap32(ks[3]));
    }
}

static uint32_t *device_tables(hipStream_t s) {
    std::call_once(g_tables_once, build_tables);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (!g_dev_tables[dev]) {
        uint32_t *p = nullptr;
        if (hipMalloc(&p, sizeof(g_te)) != hipSuccess) return nullptr;
        if (hipMemcpy(p, g_te, sizeof(g_te), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        g_dev_tables[dev] = p;
    }
    (void)s;
    return g_dev_tables[dev];
}

hipError_t launch_aes_ctr_slice(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                                size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                                uint64_t block_off, uint32_t idx_sub, hipStream_t s) {
    const size_t total = n * ((rec_per_client + 1) / 2);
    if (total == 0) return hipSuccess;
    uint32_t *tables = device_tables(s);
    if (!tables) return hipErrorOutOfMemory;
    size_t blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    if (bytes_per_client % 8 == 0 && (uintptr_t)cipher % 8 == 0)
        hipLaunchKernelGGL(aes_ctr_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, cipher, n,
                           bytes_per_client, rec_per_client, round_keys, tables, plain, block_off,
                           idx_sub);
    else
        hipLaunchKernelGGL(aes_ctr_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, cipher,
                           n, bytes_per_client, rec_per_client, round_keys, tables, plain,
                           block_off, idx_sub);
    return hipGetLastError();
}

hipError_t launch_aes_ctr(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                          size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                          hipStream_t s) {
    return launch_aes_ctr_slice(cipher, n, bytes_per_client, rec_per_client, round_keys, plain, 0,
                                0, s);
}

// host-side single block, for the CPU self-test (no GPU needed)
void aes128_encrypt_block_host(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    uint32_t rk[44], o[4];
    aes128_expand_key(key, rk);
    uint32_t w[4];
    for (int i = 0; i < 4; ++i)
        w[i] = ((uint32_t)in[4 * i] << 24) | ((uint32_t)in[4 * i + 1] << 16) |
               ((uint32_t)in[4 * i + 2] << 8) | in[4 * i + 3];
    aes128_block(g_te[0], g_te[1], g_te[2], g_te[3], g_te[4], rk, w[0], w[1], w[2], w[3], o);
    for (int i = 0; i < 4; ++i) {
        out[4 * i] = (uint8_t)(o[i] >> 24);
        out[4 * i + 1] = (uint8_t)(o[i] >> 16);
        out[4 * i + 2] = (uint8_t)(o[i] >> 8);
        out[4 * i + 3] = (uint8_t)o[i];
    }
}

}  // namespace fltee
