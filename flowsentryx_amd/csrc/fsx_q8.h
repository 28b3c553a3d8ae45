// fsx_q8.h — the quantized scorer row (model/model.py:124-137), shared by the
// standalone scoring kernel (fsx_score.hip) and the fused per-source feature +
// scoring kernels (fsx_flows.hip). Arithmetic of torch 2.10's x86/fbgemm kernels,
// see fsx_score.hip and DESIGN.md §4.4.
#pragma once
#include <hip/hip_runtime.h>
#include <climits>
#include <stdint.h>

namespace fsx {

struct ScoreParams {
    int32_t w[8];
    float inv_in;
    int32_t zp_in;
    float bias_over_ats;
    float mult;
    int32_t zp_out;
    int32_t enabled;
    uint32_t lut[64];  // quantized sigmoid table, 256 u8 packed
};

// fbgemm QuantizeAvx2: t = min_ps(x*inv, 2147483520) (NaN -> 2147483520), cvtps_epi32,
// + zero point as a wrapping int32 add, clamp to [0, 255].
__device__ __forceinline__ int32_t quant_u8(float x, float inv, int32_t zp) {
    const float lim = 2147483520.0f;
    const float v = x * inv;
    const float t = v < lim ? v : lim;
    const int32_t c = (t >= -2147483648.0f) ? (int32_t)rintf(t) : INT_MIN;
    const int32_t r = (int32_t)((uint32_t)c + (uint32_t)zp);
    return r < 0 ? 0 : (r > 255 ? 255 : r);
}

// Requantized linear output lq in [0, 255].
__device__ __forceinline__ int32_t q8_linear(const float x[8], const ScoreParams &P) {
    int32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += (quant_u8(x[k], P.inv_in, P.zp_in) - P.zp_in) * P.w[k];
    const float raw = (float)acc + P.bias_over_ats;
    const float ab = raw * P.mult;
    const int32_t r = (ab >= -2147483648.0f && ab < 2147483648.0f) ? (int32_t)rintf(ab) : INT_MIN;
    int64_t lq = (int64_t)r + P.zp_out;
    return (int32_t)(lq < 0 ? 0 : (lq > 255 ? 255 : lq));
}

__device__ __forceinline__ uint32_t lut_get(const ScoreParams &P, int32_t q) {
    return (P.lut[q >> 2] >> (8 * (q & 3))) & 0xFFu;
}

}  // namespace fsx
