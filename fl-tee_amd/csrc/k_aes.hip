// k_aes.hip — AES-128-CTR decrypt of the uploaded client slices (gfx950), constant time.
//
// lib.rs:312-343: each client's slice is decrypted with rsgx_aes_ctr_decrypt
// under its session key (session_key_store.rs:17-32: 16 zero bytes with
// bytes[4..8] = client_id big-endian), a zero 16-byte counter block and
// ctr_inc_bits = 128, i.e. keystream block b = AES_k(BE128(b)).  The
// plaintext is the record stream [u32 LE idx][f32 LE val] (parameters.rs:53-67),
// which is also the in-HBM record layout: decrypt == parse.
//
// The enclave's sgx_tcrypto runs AES-NI: no memory address depends on the key or the
// data.  The kernel keeps that property by BITSLICING: state word s[r][i] holds bit i
// of one state byte of 32 counter blocks at once, and the S-box is a boolean circuit
// (aes_sbox_bs.h, generated and checked on all 256 inputs by scripts/gen_aes_sbox.py).
// A quad of lanes carries 32 blocks, lane c the state's column c: ShiftRows is a DPP
// quad_perm read of rows 1-3 from the neighbouring lanes, MixColumns XORs of planes,
// AddRoundKey XORs with the key bits sign-extended from the round-key word of the
// lane's column.  No table, no data-dependent branch or address.
//
// Quad g of a wave takes the counters W + g + 16 j (j = 0..31) of a 512-block window
// W: bits 0-3 of the counter are g, bits 4-8 are j (constant planes), the rest W's, so
// the counter planes cost nothing, and after one 32x32 bit transpose per lane, lane c of
// quad g holds keystream word c of blocks W + 16 j + g: each of the 32 loads/stores of
// the wave covers 256 B contiguously.
//
// The host key schedule and the CPU self-test block use the same circuit over 16-byte
// bitsliced states (no S-box table on the host either).  There is no table-based
// variant in the library (round 1's T-table kernel had key- and data-dependent LDS
// addresses; its last A/B is in profiles/r02/ab/aes_variants.jsonl).
#include <cstdlib>
#include <mutex>

#include "aes_sbox_bs.h"
#include "common.h"

namespace fltee {

// ------------------------------------------------------------ bitsliced AES core
// st[p][i]: bit i of state byte p (FIPS-197 column-major: p = 4 c + r) of every slice.
// rk: the 44 big-endian round-key words.  Constant-time on host and device.
__host__ __device__ __forceinline__ uint32_t key_plane(uint32_t w, int bit) {
    return 0u - ((w >> bit) & 1u);
}

template <bool FOLD63>
__host__ __device__ __forceinline__ void add_round_key_bs(uint32_t st[16][8], const uint32_t *rk) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        // the S-box circuit leaves out its 0x63; MixColumns and ShiftRows map the
        // all-0x63 state to itself, so the constant joins every later round key
        const uint32_t w = FOLD63 ? rk[c] ^ 0x63636363u : rk[c];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) st[4 * c + r][i] ^= key_plane(w, 24 - 8 * r + i);
    }
}

// SubBytes, ShiftRows, MixColumns (MIX) into ns
template <bool MIX>
__host__ __device__ __forceinline__ void round_bs(uint32_t st[16][8], uint32_t ns[16][8]) {
#pragma unroll
    for (int p = 0; p < 16; ++p) aes_sbox_bs(st[p]);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        // ShiftRows: row r of column c comes from column c + r
        const int q0 = 4 * ((c + 0) & 3) + 0, q1 = 4 * ((c + 1) & 3) + 1,
                  q2 = 4 * ((c + 2) & 3) + 2, q3 = 4 * ((c + 3) & 3) + 3;
        if (!MIX) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                ns[4 * c + 0][i] = st[q0][i];
                ns[4 * c + 1][i] = st[q1][i];
                ns[4 * c + 2][i] = st[q2][i];
                ns[4 * c + 3][i] = st[q3][i];
            }
            continue;
        }
        const int q[4] = {q0, q1, q2, q3};
        uint32_t t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = st[q0][i] ^ st[q1][i] ^ st[q2][i] ^ st[q3][i];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            // out_r = a_r ^ t ^ xtime(a_r ^ a_{r+1})  (2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3})
            uint32_t u[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) u[i] = st[q[r]][i] ^ st[q[(r + 1) & 3]][i];
            const uint32_t x[8] = {u[7], u[0] ^ u[7], u[1], u[2] ^ u[7], u[3] ^ u[7], u[4], u[5], u[6]};
#pragma unroll
            for (int i = 0; i < 8; ++i) ns[4 * c + r][i] = st[q[r]][i] ^ t[i] ^ x[i];
        }
    }
}

// The ten rounds after the input's AddRoundKey.
__host__ __device__ __forceinline__ void aes128_rounds_bs(uint32_t st[16][8], const uint32_t *rk) {
#pragma unroll 1
    for (int R = 1; R < 10; ++R) {
        uint32_t ns[16][8];
        round_bs<true>(st, ns);
        add_round_key_bs<true>(ns, rk + 4 * R);
#pragma unroll
        for (int p = 0; p < 16; ++p)
#pragma unroll
            for (int i = 0; i < 8; ++i) st[p][i] = ns[p][i];
    }
    uint32_t ns[16][8];
    round_bs<false>(st, ns);
    add_round_key_bs<true>(ns, rk + 40);
#pragma unroll
    for (int p = 0; p < 16; ++p)
#pragma unroll
        for (int i = 0; i < 8; ++i) st[p][i] = ns[p][i];
}

// The key schedule of up to 8 keys at once: SubWord's 4 bytes of key k are the slices
// 4 k .. 4 k + 3 of the planes (the AND/XOR form of the same S-box circuit).
static void expand_keys8(const uint8_t (*key)[16], int nk, uint32_t *rk) {
    for (int k = 0; k < nk; ++k)
        for (int i = 0; i < 4; ++i)
            rk[44 * k + i] = ((uint32_t)key[k][4 * i] << 24) | ((uint32_t)key[k][4 * i + 1] << 16) |
                             ((uint32_t)key[k][4 * i + 2] << 8) | key[k][4 * i + 3];
    uint32_t rc = 1;
    for (int i = 4; i < 44; ++i) {
        if (i % 4) {
            for (int k = 0; k < nk; ++k) rk[44 * k + i] = rk[44 * k + i - 4] ^ rk[44 * k + i - 1];
            continue;
        }
        uint32_t x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < nk; ++k) {
            const uint32_t t = rk[44 * k + i - 1], rot = (t << 8) | (t >> 24);  // RotWord
            for (int b = 0; b < 8; ++b)
                for (int q = 0; q < 4; ++q) x[b] |= ((rot >> (8 * q + b)) & 1u) << (4 * k + q);
        }
        aes_sbox_gates(x);
        for (int k = 0; k < nk; ++k) {
            uint32_t sw = 0;
            for (int b = 0; b < 8; ++b)
                for (int q = 0; q < 4; ++q) sw |= ((x[b] >> (4 * k + q)) & 1u) << (8 * q + b);
            rk[44 * k + i] = rk[44 * k + i - 4] ^ sw ^ 0x63636363u ^ (rc << 24);
        }
        rc = ((rc << 1) ^ (0x11bu & (0u - (rc >> 7)))) & 0xffu;  // public schedule
    }
}

// host_aesni.cpp: the same schedules with AES-NI (the ECALL's per-client key expansion)
bool host_has_aesni();
void aes128_expand_key_aesni(const uint8_t key[16], uint32_t rk[44]);
void aes128_session_round_keys_aesni(const uint32_t *ids, size_t n, uint32_t *rk);

void aes128_expand_key(const uint8_t key[16], uint32_t rk[44]) {
    if (host_has_aesni()) return aes128_expand_key_aesni(key, rk);
    expand_keys8(reinterpret_cast<const uint8_t (*)[16]>(key), 1, rk);
}

// session_key_store.rs:17-32: 16 zero bytes with bytes[4..8] = client_id big-endian
// (portable: the bitsliced circuit, 8 keys per pass)
void aes128_session_round_keys_portable(const uint32_t *ids, size_t n, uint32_t *rk) {
    for (size_t c0 = 0; c0 < n; c0 += 8) {
        const int nk = (int)(n - c0 < 8 ? n - c0 : 8);
        uint8_t key[8][16] = {};
        for (int k = 0; k < nk; ++k)
            for (int b = 0; b < 4; ++b) key[k][4 + b] = (uint8_t)(ids[c0 + k] >> (24 - 8 * b));
        expand_keys8(key, nk, rk + 44 * c0);
    }
}

void aes128_session_round_keys(const uint32_t *ids, size_t n, uint32_t *rk) {
    if (host_has_aesni()) return aes128_session_round_keys_aesni(ids, n, rk);
    aes128_session_round_keys_portable(ids, n, rk);
}

// host-side single block, for the CPU self-test (no GPU needed): slice 0 of the planes
void aes128_encrypt_block_host(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    uint32_t rk[44];
    aes128_expand_key(key, rk);
    uint32_t st[16][8];
    for (int p = 0; p < 16; ++p)
        for (int i = 0; i < 8; ++i) st[p][i] = (in[p] >> i) & 1u;
    add_round_key_bs<false>(st, rk);
    aes128_rounds_bs(st, rk);
    for (int p = 0; p < 16; ++p) {
        uint32_t b = 0;
        for (int i = 0; i < 8; ++i) b |= (st[p][i] & 1u) << i;
        out[p] = (uint8_t)b;
    }
}

// ------------------------------------------------------------- bitsliced kernel
__device__ __forceinline__ uint32_t ld_u32_bytes(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// In-place 32x32 bit transpose: afterwards m[j] bit r = (old m[r]) bit j.
__device__ __forceinline__ void transpose32(uint32_t m[32]) {
    constexpr uint32_t kMask[5] = {0x0000ffffu, 0x00ff00ffu, 0x0f0f0f0fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        const int s = 16 >> l;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & s) continue;
            const uint32_t t = ((m[r] >> s) ^ m[r + s]) & kMask[l];
            m[r + s] ^= t;
            m[r] ^= t << s;
        }
    }
}

// ------------------------------------------------ column-per-lane bitsliced kernel
// A quad of lanes holds 32 blocks: lane c of the quad keeps column c of the state (rows
// 0-3, 32 planes), ShiftRows reads rows 1-3 from the lanes c+1..c+3 of the quad (DPP
// quad_perm, no LDS), SubBytes and MixColumns stay in the lane.  96 VGPRs (5 waves per
// SIMD).  A/B (profiles/r02/ab/aes_variants.jsonl): one lane per 32 blocks with the
// whole state (452 VGPRs, one wave per SIMD) ran 2.04 ms on the 800 MB headline payload
// and this form 1.39 ms with two-input gates, 1.19 ms with the S-box as 119 bitop3s, 1.14
// ms with MixColumns + AddRoundKey as XOR3s too (the T-table kernel: 1.20 ms).
constexpr int kAesWindow4 = 512;  // counter blocks per wave: 16 quads x 32 slices

__device__ __forceinline__ uint32_t quad_rot(uint32_t v, int r) {
    // lane c of each quad reads lane (c + r) & 3
    switch (r) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x39, 0xf, 0xf, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);
    case 3: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x93, 0xf, 0xf, false);
    default: return v;
    }
}

__device__ __forceinline__ uint32_t sext_bit(uint32_t w, int pos) {
    return (uint32_t)((int32_t)(w << (31 - pos)) >> 31);  // v_bfe_i32 w, pos, 1
}

// SubBytes + ShiftRows of the lane's column
__device__ __forceinline__ void sub_shift_col(uint32_t s[4][8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) aes_sbox_bs(s[r]);
#pragma unroll
    for (int r = 1; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) s[r][i] = quad_rot(s[r][i], r);
}

__device__ __forceinline__ void ark_col(uint32_t s[4][8], uint32_t w) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) s[r][i] ^= sext_bit(w, 24 - 8 * r + i);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return lut3<0x96>(a, b, c);
}

// MixColumns and AddRoundKey (key word w of the lane's column) as three-input XORs:
// out_r = a_r ^ t ^ xtime(a_r ^ a_{r+1}) ^ k_r with t = a_0 ^ a_1 ^ a_2 ^ a_3, i.e.
// 2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3}; plane i of xtime(u) is u_{i-1}, plus u_7 for
// i = 1, 3, 4 (0x1b).  Two v_bitop3 per plane (three where u_7 enters).
__device__ __forceinline__ void mix_ark_col(uint32_t s[4][8], uint32_t w) {
    uint32_t t[8], ns[4][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = xor3(s[0][i], s[1][i], s[2][i]) ^ s[3][i];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t *a = s[r], *b = s[(r + 1) & 3];
        const uint32_t u7 = a[7] ^ b[7];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t k = sext_bit(w, 24 - 8 * r + i);
            if (i == 0) {
                ns[r][i] = xor3(xor3(a[0], t[0], a[7]), b[7], k);
            } else if (i == 1 || i == 3 || i == 4) {
                ns[r][i] = xor3(xor3(a[i], t[i], a[i - 1]), b[i - 1], u7) ^ k;
            } else {
                ns[r][i] = xor3(xor3(a[i], t[i], a[i - 1]), b[i - 1], k);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) s[r][i] = ns[r][i];
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void aes_ctr_bs4_kernel(const uint8_t *__restrict__ cipher,
                                                          size_t n, size_t bpc, size_t rpc,
                                                          const uint32_t *__restrict__ rks,
                                                          uint8_t *__restrict__ plain,
                                                          uint64_t block_off, uint32_t idx_sub,
                                                          uint64_t wpc, uint32_t *__restrict__ zero_word) {
    if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0u;
    const uint32_t lane = threadIdx.x & 63, col = lane & 3, g = lane >> 2;
    const uint64_t bpcl = (rpc + 1) / 2;  // 16-byte blocks per client
    const uint64_t waves = (uint64_t)n * wpc;
    const uint64_t w0 = block_off / kAesWindow4;
    for (uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); gw < waves;
         gw += (uint64_t)gridDim.x * 4) {
        const uint64_t gu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gw >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)gw);
        const uint64_t c = gu / wpc;
        const uint64_t W = (w0 + (gu - c * wpc)) * kAesWindow4;
        const uint32_t *rk = rks + c * 44 + col;  // this lane's column of every round key
        // all eleven round-key words up front, in one round trip (a load per round inside
        // the loop put ten dependent memory latencies on a small call's critical path)
        uint32_t rkw[11];
#pragma unroll
        for (int R = 0; R < 11; ++R) rkw[R] = rk[4 * R];
        const uint32_t wlo = (uint32_t)W, whi = (uint32_t)(W >> 32);
        // counter block BE128(W + g + 16 j): column 3 = counter bits 0-31, column 2 =
        // bits 32-63, columns 0-1 zero; bits 0-3 = g, 4-8 = j, the rest W's
        uint32_t s[4][8];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int t = 24 - 8 * r + i;
                const uint32_t v3 = t < 4 ? 0u - ((g >> t) & 1u)
                                  : t < 9 ? (t == 4 ? 0xaaaaaaaau : t == 5 ? 0xccccccccu
                                             : t == 6 ? 0xf0f0f0f0u : t == 7 ? 0xff00ff00u : 0xffff0000u)
                                          : 0u - ((wlo >> t) & 1u);
                const uint32_t v2 = 0u - ((whi >> t) & 1u);
                s[r][i] = col == 3 ? v3 : col == 2 ? v2 : 0u;
            }
        ark_col(s, rkw[0]);
#pragma unroll 1
        for (int R = 1; R < 10; ++R) {
            const uint32_t w = rkw[1] ^ 0x63636363u;  // the S-boxes' 0x63, folded
#pragma unroll
            for (int i = 1; i < 10; ++i) rkw[i] = rkw[i + 1];  // the next round's word first
            sub_shift_col(s);
            mix_ark_col(s, w);
        }
        sub_shift_col(s);
        ark_col(s, rkw[1] ^ 0x63636363u);
        // rows 8 r + i -> word j = keystream word `col` of block j
        transpose32(&s[0][0]);
        const uint8_t *cbase = cipher + c * bpc + 4 * col;
        uint8_t *dbase = plain + c * rpc * 8 + 4 * col;
        const uint32_t sub = (col & 1) ? 0u : idx_sub;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint64_t ctr = W + 16 * j + g;
            if (ctr < block_off || ctr - block_off >= bpcl) continue;
            const uint64_t b = ctr - block_off;
            if (2 * b + (col >> 1) >= rpc) continue;  // the half last block
            const uint32_t x = ALIGNED ? *reinterpret_cast<const uint32_t *>(cbase + 16 * b)
                                       : ld_u32_bytes(cbase + 16 * b);
            *reinterpret_cast<uint32_t *>(dbase + 16 * b) = (x ^ (&s[0][0])[j]) - sub;
        }
    }
}

// ------------------------------------------------- byte-per-lane bitsliced kernel
// For small payloads the quad kernel's latency is one wave's instruction stream: ~7k VALU
// per wave (four S-boxes per lane per round), ~20 us even for 12 KB, whatever the size
// below a chip's worth of waves.  This form spreads a 32-block slice over 16 lanes, one
// state byte per lane, so a lane runs one S-box per round (119 v_bitop3) and the round's
// stream is ~4x shorter; it costs ~1.4x the lane-instructions per block, so it only runs
// where the quad kernel leaves SIMDs idle (launch_aes_ctr_slice).
//   lane = 16 G + 4 r + p: G = slice group of the wave (0-3), r = AES row, p = physical
//   column.  ShiftRows is not applied to the data: after t of them, row r's logical
//   column c sits at p = (c + r t) mod 4, so MixColumns for (r, c) reads row r + D of the
//   same logical column from lane 4 (r + D) + (p + D t) mod 4 of its row: a DPP row
//   rotation by 4 D then a quad rotation by D t — uniform across lanes for fixed D, t.
//   Counter block of slice bit b in group G: W + 32 G + b (W: the wave's 128-block
//   window), so plane i of byte (r, c) is counter bit (15 - 4c - r) * 8 + i: bits 0-4 =
//   b (constant patterns), 5-6 = G, 7- = W.  The keystream goes through 2 KB of LDS per
//   wave (byte stores), each lane then XORs two whole 16-B blocks: 32 B contiguous per lane.
constexpr int kAesWindowR = 128;  // counter blocks per wave: 4 groups x 32 slices
constexpr uint64_t kAesRowBelowWaves = 1024;  // quad-kernel waves: one per SIMD

__device__ __forceinline__ uint32_t row_rot(uint32_t v, int quads) {
    // lane L of each 16-lane row reads lane (L + 4 quads) mod 16 (row_ror:16-4q)
    switch (quads & 3) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + 12, 0xf, 0xf, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + 8, 0xf, 0xf, false);
    case 3: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + 4, 0xf, 0xf, false);
    default: return v;
    }
}

// SubBytes, then MixColumns + AddRoundKey at ShiftRows count t (TM = t mod 4) on the
// lane's byte; wr = the lane's round-key word shifted so its row's byte is bits 24-31
template <int TM>
__device__ __forceinline__ void round_row(uint32_t x[8], uint32_t wr) {
    aes_sbox_bs(x);
    uint32_t a1[8], a2[8], a3[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a1[i] = quad_rot(row_rot(x[i], 1), (1 * TM) & 3);
        a2[i] = quad_rot(row_rot(x[i], 2), (2 * TM) & 3);
        a3[i] = quad_rot(row_rot(x[i], 3), (3 * TM) & 3);
    }
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) u[i] = x[i] ^ a1[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        // 2 a0 ^ 3 a1 ^ a2 ^ a3 = xtime(a0 ^ a1) ^ a1 ^ a2 ^ a3; xtime bit i = u_{i-1}
        // (+ u_7 for i = 0, 1, 3, 4: 0x1b)
        const uint32_t v = xor3(a1[i], a2[i], a3[i]);
        const uint32_t k = sext_bit(wr, 24 + i);
        if (i == 0) x[i] = xor3(v, u[7], k);
        else if (i == 1 || i == 3 || i == 4) x[i] = xor3(v, u[i - 1], u[7]) ^ k;
        else x[i] = xor3(v, u[i - 1], k);
    }
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void aes_ctr_row_kernel(const uint8_t *__restrict__ cipher,
                                                          size_t n, size_t bpc, size_t rpc,
                                                          const uint32_t *__restrict__ rks,
                                                          uint8_t *__restrict__ plain,
                                                          uint64_t block_off, uint32_t idx_sub,
                                                          uint64_t wpc, uint32_t *__restrict__ zero_word) {
    if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0u;
    __shared__ __attribute__((aligned(16))) uint8_t ks_lds[4][kAesWindowR * 16];
    uint8_t *ks = ks_lds[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63, G = lane >> 4, r = (lane >> 2) & 3, p = lane & 3;
    const uint64_t bpcl = (rpc + 1) / 2;  // 16-byte blocks per client
    const uint64_t waves = (uint64_t)n * wpc;
    const uint64_t w0 = block_off / kAesWindowR;
    for (uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); gw < waves;
         gw += (uint64_t)gridDim.x * 4) {
        const uint64_t gu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gw >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)gw);
        const uint64_t c = gu / wpc;
        const uint64_t W = (w0 + (gu - c * wpc)) * kAesWindowR;
        // this lane's two output blocks (window-local 2 lane, 2 lane + 1): their
        // ciphertext words first, so the loads overlap the rounds
        const uint8_t *cbase = cipher + c * bpc;
        uint32_t cw[8];
        bool ok[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t ctr = W + 2 * lane + h;
            const bool in = ctr >= block_off && ctr - block_off < bpcl;
            const uint64_t b = in ? ctr - block_off : 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                ok[4 * h + w] = in && 2 * b + (w >> 1) < rpc;  // the half last block
                const uint8_t *src = cbase + 16 * b + 4 * w;
                cw[4 * h + w] = !ok[4 * h + w] ? 0u
                                : ALIGNED      ? *reinterpret_cast<const uint32_t *>(src)
                                               : ld_u32_bytes(src);
            }
        }
        // round-key words: after R ShiftRows the lane's logical column is (p - r R) mod 4
        const uint32_t *rk = rks + c * 44;
        uint32_t rkw[11];
#pragma unroll
        for (int R = 0; R < 11; ++R) rkw[R] = rk[4 * R + ((p - r * (uint32_t)R) & 3u)] << (8 * r);
        // counter planes: byte (r, c = p) of block W + 32 G + b, b = slice bit
        uint32_t x[8];
        const uint32_t wlo = (uint32_t)W, whi = (uint32_t)(W >> 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int t = (int)((15 - 4 * p - r) * 8) + i;  // counter bit of this plane
            const uint32_t pat = t == 0 ? 0xaaaaaaaau : t == 1 ? 0xccccccccu : t == 2 ? 0xf0f0f0f0u
                               : t == 3 ? 0xff00ff00u : 0xffff0000u;
            const uint32_t wb = t < 32 ? (wlo >> (t & 31)) & 1u : t < 64 ? (whi >> (t & 31)) & 1u : 0u;
            x[i] = t < 5 ? pat : t < 7 ? 0u - ((G >> (t - 5)) & 1u) : 0u - wb;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] ^= sext_bit(rkw[0], 24 + i);
        // rounds 1-9 (t = R), MixColumns' rotations fixed per t mod 4: two passes of
        // rounds 4 i + 1 .. 4 i + 4 (t mod 4 = 1, 2, 3, 0), then round 9
#pragma unroll 1
        for (int it = 0; it < 2; ++it) {
            round_row<1>(x, rkw[1] ^ 0x63636363u);
            round_row<2>(x, rkw[2] ^ 0x63636363u);
            round_row<3>(x, rkw[3] ^ 0x63636363u);
            round_row<0>(x, rkw[4] ^ 0x63636363u);
#pragma unroll
            for (int i = 1; i < 7; ++i) rkw[i] = rkw[i + 4];  // the next four rounds' words
        }
        round_row<1>(x, rkw[1] ^ 0x63636363u);  // round 9; rkw[2] = round 10's word
        aes_sbox_bs(x);
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] ^= sext_bit(rkw[2] ^ 0x63636363u, 24 + i);
        // 8 x 32 bit transpose (three butterfly levels): byte q of x[i] = the keystream
        // byte of slice b = 8 q + i
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            const int sh = 1 << l;
            const uint32_t m = l == 0 ? 0x55555555u : l == 1 ? 0x33333333u : 0x0f0f0f0fu;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i & sh) continue;
                const uint32_t t = ((x[i] >> sh) ^ x[i + sh]) & m;
                x[i + sh] ^= t;
                x[i] ^= t << sh;
            }
        }
        // byte (r, c) of block 32 G + b at 16 (32 G + b) + 4 c + r; after ten ShiftRows
        // the lane's logical column is (p - 2 r) mod 4
        const uint32_t cfin = (p - 2 * r) & 3u;
        uint8_t *kb = ks + 16 * 32 * G + 4 * cfin + r;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) kb[16 * (8 * q + i)] = (uint8_t)(x[i] >> (8 * q));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint4 k0 = reinterpret_cast<const uint4 *>(ks)[2 * lane];
        const uint4 k1 = reinterpret_cast<const uint4 *>(ks)[2 * lane + 1];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next window's stores after every read
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t kw[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
        uint8_t *dbase = plain + c * rpc * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t ctr = W + 2 * lane + h;
            const uint64_t b = ctr >= block_off ? ctr - block_off : 0;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if (ok[4 * h + w])
                    *reinterpret_cast<uint32_t *>(dbase + 16 * b + 4 * w) =
                        (cw[4 * h + w] ^ kw[4 * h + w]) - ((w & 1) ? 0u : idx_sub);
        }
    }
}

static int g_aes_variant = 0;  // 0: by size, 1: the quad kernel, 2: the byte-per-lane kernel
void set_aes_variant(int v) { g_aes_variant = v; }

hipError_t launch_aes_ctr_slice(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                                size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                                uint64_t block_off, uint32_t idx_sub, hipStream_t s,
                                uint32_t *zero_word) {
    const size_t bpcl = (rec_per_client + 1) / 2;
    if (n == 0 || bpcl == 0)  // nothing to decrypt; the word still has to read 0
        return zero_word ? fl_memset_async(zero_word, 0, 4, s) : hipSuccess;
    const bool aligned = bytes_per_client % 8 == 0 && (uintptr_t)cipher % 8 == 0;
    // windows of 512 counter blocks (absolute counter space) touching each client's slice
    const uint64_t wpc = (block_off + bpcl - 1) / kAesWindow4 - block_off / kAesWindow4 + 1;
    const uint64_t waves = (uint64_t)n * wpc;
    // the byte-per-lane kernel while the quad kernel would leave SIMDs without a wave
    const bool row = g_aes_variant == 2 || (g_aes_variant == 0 && waves < kAesRowBelowWaves);
    if (row) {
        const uint64_t wpcr = (block_off + bpcl - 1) / kAesWindowR - block_off / kAesWindowR + 1;
        uint64_t rblocks = ((uint64_t)n * wpcr + 3) / 4;
        if (rblocks > 16384) rblocks = 16384;
        if (aligned)
            FLTEE_LAUNCH(aes_ctr_row_kernel<true>, dim3((unsigned)rblocks), dim3(256), 0, s,
                               cipher, n, bytes_per_client, rec_per_client, round_keys, plain,
                               block_off, idx_sub, wpcr, zero_word);
        else
            FLTEE_LAUNCH(aes_ctr_row_kernel<false>, dim3((unsigned)rblocks), dim3(256), 0, s,
                               cipher, n, bytes_per_client, rec_per_client, round_keys, plain,
                               block_off, idx_sub, wpcr, zero_word);
        return hipGetLastError();
    }
    uint64_t blocks = (waves + 3) / 4;
    if (blocks > 16384) blocks = 16384;  // grid-stride beyond 16 waves per SIMD
    if (aligned)
        FLTEE_LAUNCH(aes_ctr_bs4_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s,
                           cipher, n, bytes_per_client, rec_per_client, round_keys, plain,
                           block_off, idx_sub, wpc, zero_word);
    else
        FLTEE_LAUNCH(aes_ctr_bs4_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s,
                           cipher, n, bytes_per_client, rec_per_client, round_keys, plain,
                           block_off, idx_sub, wpc, zero_word);
    return hipGetLastError();
}

hipError_t launch_aes_ctr(const uint8_t *cipher, size_t n, size_t bytes_per_client,
                          size_t rec_per_client, const uint32_t *round_keys, uint8_t *plain,
                          hipStream_t s, uint32_t *zero_word) {
    return launch_aes_ctr_slice(cipher, n, bytes_per_client, rec_per_client, round_keys, plain, 0,
                                0, s, zero_word);
}

}  // namespace fltee
