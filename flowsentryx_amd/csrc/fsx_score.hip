// fsx_score.hip — quantized scorer of model/model.py:124-137 on gfx950.
//
// QuantStub -> Linear(8,1) -> sigmoid -> DeQuantStub after torch.ao convert(), with
// the arithmetic of torch 2.10's x86/fbgemm kernels:
//   q_i  = clamp(cvt(min(x_i * fp32(1/s_in), 2147483520)) + zp_in, 0, 255)
//   acc  = sum_i (q_i - zp_in) * w_i                          (int32)
//   lq   = clamp(cvt(fp32(acc + bias/(s_in*s_w)) * (s_in*s_w)/s_out) + zp_out, 0, 255)
//          (cvt: round half even; NaN / out of int32 range -> INT32_MIN)
//   p    = sigmoid_q8[lq] / 256,   malicious = p > 0.5         (model/model.py:206)
// K = 8, N = 1 is 8 MACs per 32-byte row: the kernel is HBM-bound, so it runs on
// the VALU (an MFMA tile would be >98% padding). Algorithmic bytes: 32 B in,
// 4 B prob + 1 B decision out per flow.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>

#include "fsx_internal.h"

namespace fsx {

struct ScoreParams {
    int32_t w[8];
    float inv_in;
    int32_t zp_in;
    float bias_over_ats;
    float mult;
    int32_t zp_out;
    uint32_t lut[64];  // 256 u8 entries packed
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

__global__ __launch_bounds__(256) void k_score(const float4 *__restrict__ feat, uint64_t n,
                                               float *__restrict__ prob, uint8_t *__restrict__ dec,
                                               ScoreParams P) {
    __shared__ uint8_t s_lut[256];
    s_lut[threadIdx.x] = (uint8_t)(P.lut[threadIdx.x >> 2] >> (8 * (threadIdx.x & 3)));
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const float4 a = feat[2 * i], b = feat[2 * i + 1];
        const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        int32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += (quant_u8(x[k], P.inv_in, P.zp_in) - P.zp_in) * P.w[k];
        const float raw = (float)acc + P.bias_over_ats;
        const float ab = raw * P.mult;
        const int32_t r = (ab >= -2147483648.0f && ab < 2147483648.0f) ? (int32_t)rintf(ab) : INT_MIN;
        int64_t lq = (int64_t)r + P.zp_out;
        lq = lq < 0 ? 0 : (lq > 255 ? 255 : lq);
        const float p = (float)s_lut[lq] * 0.00390625f;
        prob[i] = p;
        dec[i] = p > 0.5f ? 1 : 0;
    }
}

hipError_t launch_score(const float *feat, size_t n, float *prob, uint8_t *dec, const int8_t w[8],
                        float inv_in, int32_t zp_in, float bias_over_ats, float mult, int32_t zp_out,
                        const uint8_t lut[256], hipStream_t st) {
    if (n == 0) return hipSuccess;
    ScoreParams P;
    for (int k = 0; k < 8; ++k) P.w[k] = w[k];
    P.inv_in = inv_in; P.zp_in = zp_in; P.bias_over_ats = bias_over_ats; P.mult = mult; P.zp_out = zp_out;
    for (int k = 0; k < 64; ++k)
        P.lut[k] = (uint32_t)lut[4 * k] | ((uint32_t)lut[4 * k + 1] << 8) |
                   ((uint32_t)lut[4 * k + 2] << 16) | ((uint32_t)lut[4 * k + 3] << 24);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(8192, (n + 255) / 256);
    k_score<<<grid, 256, 0, st>>>(reinterpret_cast<const float4 *>(feat), n, prob, dec, P);
    return hipGetLastError();
}

}  // namespace fsx
