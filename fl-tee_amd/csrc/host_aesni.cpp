// host_aesni.cpp — the clients' AES-128 key schedules on the host with AES-NI.
//
// ecall_secure_aggregation expands one session key per uploaded client (lib.rs:312-343:
// rsgx_aes_ctr_decrypt keys AES-128 with it); at n = 3000 clients the bitsliced portable
// schedule (k_aes.hip expand_keys8) took milliseconds of the host-inclusive ECALL.  With
// AES-NI (AESKEYGENASSIST: constant time, no table, like the enclave's own AES-NI) one
// schedule is a few tens of nanoseconds.  Plain host C++ (compiled by the system g++ with
// -maes only for these functions); the library falls back to the portable bitsliced
// schedule when the CPU lacks AES-NI.  Round-key words as k_aes.hip keeps them: rk[i] =
// big-endian word i of the FIPS-197 expansion.
#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>

namespace fltee {

bool host_has_aesni() {
    static const bool has = __builtin_cpu_supports("aes") && __builtin_cpu_supports("sse4.1");
    return has;
}

template <int RCON>
__attribute__((target("aes,sse4.1"))) static inline __m128i expand_step(__m128i k) {
    __m128i t = _mm_aeskeygenassist_si128(k, RCON);
    t = _mm_shuffle_epi32(t, 0xff);
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    return _mm_xor_si128(k, t);
}

__attribute__((target("aes,sse4.1"))) static inline void store_be_words(__m128i k, uint32_t *w) {
    // bytes b0..b15 of the round key -> words (b0 b1 b2 b3) ... big-endian
    const __m128i bswap = _mm_setr_epi8(3, 2, 1, 0, 7, 6, 5, 4, 11, 10, 9, 8, 15, 14, 13, 12);
    _mm_storeu_si128(reinterpret_cast<__m128i *>(w), _mm_shuffle_epi8(k, bswap));
}

__attribute__((target("aes,sse4.1"))) void aes128_expand_key_aesni(const uint8_t key[16], uint32_t rk[44]) {
    __m128i k = _mm_loadu_si128(reinterpret_cast<const __m128i *>(key));
    store_be_words(k, rk + 0);
    k = expand_step<0x01>(k); store_be_words(k, rk + 4);
    k = expand_step<0x02>(k); store_be_words(k, rk + 8);
    k = expand_step<0x04>(k); store_be_words(k, rk + 12);
    k = expand_step<0x08>(k); store_be_words(k, rk + 16);
    k = expand_step<0x10>(k); store_be_words(k, rk + 20);
    k = expand_step<0x20>(k); store_be_words(k, rk + 24);
    k = expand_step<0x40>(k); store_be_words(k, rk + 28);
    k = expand_step<0x80>(k); store_be_words(k, rk + 32);
    k = expand_step<0x1b>(k); store_be_words(k, rk + 36);
    k = expand_step<0x36>(k); store_be_words(k, rk + 40);
}

// session_key_store.rs:17-32: 16 zero bytes with bytes[4..8] = client_id big-endian
void aes128_session_round_keys_aesni(const uint32_t *ids, size_t n, uint32_t *rk) {
    for (size_t c = 0; c < n; ++c) {
        uint8_t key[16] = {};
        for (int b = 0; b < 4; ++b) key[4 + b] = (uint8_t)(ids[c] >> (24 - 8 * b));
        aes128_expand_key_aesni(key, rk + 44 * c);
    }
}

}  // namespace fltee
