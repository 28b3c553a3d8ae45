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

#include "fsx_internal.h"
#include "fsx_q8.h"

namespace fsx {

__global__ __launch_bounds__(256) void k_score(const float4 *__restrict__ feat, uint64_t n,
                                               float *__restrict__ prob, uint8_t *__restrict__ dec,
                                               ScoreParams P) {
    __shared__ uint8_t s_lut[256];
    s_lut[threadIdx.x] = (uint8_t)lut_get(P, (int32_t)threadIdx.x);
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const float4 a = feat[2 * i], b = feat[2 * i + 1];
        const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        const float p = (float)s_lut[q8_linear(x, P)] * 0.00390625f;
        prob[i] = p;
        dec[i] = p > 0.5f ? 1 : 0;
    }
}

ScoreParams make_score_params(const int8_t w[8], float inv_in, int32_t zp_in, float bias_over_ats,
                              float mult, int32_t zp_out, const uint8_t lut[256]) {
    ScoreParams P{};
    for (int k = 0; k < 8; ++k) P.w[k] = w[k];
    P.inv_in = inv_in; P.zp_in = zp_in; P.bias_over_ats = bias_over_ats; P.mult = mult; P.zp_out = zp_out;
    P.enabled = 1;
    for (int k = 0; k < 64; ++k)
        P.lut[k] = (uint32_t)lut[4 * k] | ((uint32_t)lut[4 * k + 1] << 8) |
                   ((uint32_t)lut[4 * k + 2] << 16) | ((uint32_t)lut[4 * k + 3] << 24);
    return P;
}

hipError_t launch_score(const float *feat, size_t n, float *prob, uint8_t *dec, const int8_t w[8],
                        float inv_in, int32_t zp_in, float bias_over_ats, float mult, int32_t zp_out,
                        const uint8_t lut[256], hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    if (n == 0) return hipSuccess;
    const ScoreParams P = make_score_params(w, inv_in, zp_in, bias_over_ats, mult, zp_out, lut);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(8192, (n + 255) / 256);
    k_score<<<grid, 256, 0, st>>>(reinterpret_cast<const float4 *>(feat), n, prob, dec, P);
    return hipGetLastError();
}

}  // namespace fsx
