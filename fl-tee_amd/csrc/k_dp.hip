// k_dp.hip — Gaussian DP noise (common.rs:56-72) and the per-client L2 clip
// (update.py:187-204) on gfx950.
//
// dp_noise   : g[i] += (N(0, clipping*sigma) as f64 / n) as f32, one Philox4x32-10
//              draw (2 x 53-bit uniforms, Box-Muller in f64) per parameter.
//              The enclave seeds sgx_rand from RDRAND and samples with a
//              ziggurat; parity is statistical (tests/test_dp.py).
// clip       : coef_c = min(1, C / ||v_c||_2) per client (f64 accumulation of the
//              client's k values; non-top-k entries are zero so the norm over the
//              payload equals torch.norm over the flattened model), then
//              v *= coef_c in f32 — either in place (sparse paths) or fused into
//              the dense accumulate as __fmul_rn before __fadd_rn.
#include "common.h"

namespace fltee {

__global__ void dp_noise_kernel(float *__restrict__ out, size_t d, double stddev, double n,
                                uint32_t k0, uint32_t k1) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    uint32_t c[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), 0u, FLTEE_STREAM_DP};
    philox4x32_10(c, k0, k1);
    const double u1 = 1.0 - ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) *
                                (1.0 / 9007199254740992.0);
    const double u2 = ((double)(c[2] >> 5) * 67108864.0 + (double)(c[3] >> 6)) *
                      (1.0 / 9007199254740992.0);
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    out[i] = __fadd_rn(out[i], (float)((0.0 + stddev * z) / n));
}

hipError_t launch_dp_noise(float *out, size_t d, float sigma, float clipping, size_t n,
                           uint64_t seed, hipStream_t s) {
    if (d == 0) return hipSuccess;
    const double stddev = (double)(clipping * sigma);  // (clipping * sigma) as f64
    FLTEE_LAUNCH(dp_noise_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, out,
                       d, stddev, (double)n, (uint32_t)seed, (uint32_t)(seed >> 32));
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void client_norm_kernel(const uint2 *__restrict__ rec, size_t k,
                                                          float clipping, float *__restrict__ coef) {
    __shared__ double part[4];
    const uint2 *src = rec + (size_t)blockIdx.x * k;
    double ss = 0.0;
    for (size_t e = threadIdx.x; e < k; e += 256) {
        const double v = (double)__uint_as_float(src[e].y);
        ss += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_down(ss, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = part[0] + part[1] + part[2] + part[3];
        const float norm = (float)sqrt(t);
        float cf = clipping / norm;
        if (!(cf < 1.0f)) cf = 1.0f;  // Python min(1, tensor): NaN / inf / >=1 -> 1
        coef[blockIdx.x] = cf;
    }
}

hipError_t launch_client_clip_coef(const void *rec, size_t n, size_t k, float clipping,
                                   float *coef, hipStream_t s) {
    if (n == 0) return hipSuccess;
    FLTEE_LAUNCH(client_norm_kernel, dim3((unsigned)n), dim3(256), 0, s, (const uint2 *)rec,
                       k, clipping, coef);
    return hipGetLastError();
}

__global__ void apply_clip_kernel(uint2 *__restrict__ rec, size_t n, size_t k,
                                  const float *__restrict__ coef) {
    const size_t total = n * k;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (size_t)gridDim.x * 256) {
        uint2 w = rec[e];
        w.y = __float_as_uint(__fmul_rn(__uint_as_float(w.y), coef[e / k]));
        rec[e] = w;
    }
}

hipError_t launch_apply_clip(void *rec, size_t n, size_t k, const float *coef, hipStream_t s) {
    const size_t total = n * k;
    if (total == 0) return hipSuccess;
    size_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    FLTEE_LAUNCH(apply_clip_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint2 *)rec, n,
                       k, coef);
    return hipGetLastError();
}

}  // namespace fltee
