// fsx_synth.hip — libfsx_synth.so: on-device synthetic packet streams for the
// benchmark and the parity tests (BASELINE.json configs; SURVEY.md §8 d).
// Every packet is a pure function of (params, index), shared with the CPU twin in
// oracle/fsx_oracle.c through fsx_synth_common.h. Not part of the verdict path.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fsx_synth_common.h"

namespace {

__global__ __launch_bounds__(256) void k_synth(fsx_synth_params P, const uint32_t *prob,
                                               const uint32_t *alias, uint64_t j0, uint64_t count,
                                               uint8_t *hdr, uint32_t *len, uint64_t *ts) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * 256u) {
        uint8_t rec[64];
        uint32_t L;
        uint64_t T;
        fsx_synth_packet(&P, prob, alias, j0 + i, rec, &L, &T);
        uint4 *dst = reinterpret_cast<uint4 *>(hdr + i * 64);
        const uint4 *src = reinterpret_cast<const uint4 *>(rec);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = src[k];
        len[i] = L;
        ts[i] = T;
    }
}

struct AliasCache {
    uint32_t n = 0;
    double s = 0;
    int device = -1;
    uint32_t *d_prob = nullptr, *d_alias = nullptr;
};
AliasCache g_cache;

}  // namespace

extern "C" {

// Generate packets [j0, j0+count) of the stream into device buffers.
int fsx_synth_generate(const fsx_synth_params *P, double zipf_s, uint64_t j0, uint64_t count,
                       uint8_t *d_hdr, uint32_t *d_len, uint64_t *d_ts, void *stream) {
    if (!P || (count && (!d_hdr || !d_len || !d_ts))) return -EINVAL;
    if (P->len_min > P->len_max) return -EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t *prob = nullptr, *alias = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -EIO;
    if (P->mode == FSX_SYNTH_ZIPF_V4) {
        if (P->n_ips == 0) return -EINVAL;
        if (g_cache.n != P->n_ips || g_cache.s != zipf_s || g_cache.device != dev) {
            (void)hipFree(g_cache.d_prob); (void)hipFree(g_cache.d_alias);
            g_cache = AliasCache{};
            std::vector<uint32_t> hp(P->n_ips), ha(P->n_ips);
            if (fsx_zipf_alias_build(P->n_ips, zipf_s, hp.data(), ha.data())) return -ENOMEM;
            if (hipMalloc(&g_cache.d_prob, (size_t)P->n_ips * 4) != hipSuccess) return -ENOMEM;
            if (hipMalloc(&g_cache.d_alias, (size_t)P->n_ips * 4) != hipSuccess) return -ENOMEM;
            if (hipMemcpy(g_cache.d_prob, hp.data(), (size_t)P->n_ips * 4, hipMemcpyHostToDevice) != hipSuccess) return -EIO;
            if (hipMemcpy(g_cache.d_alias, ha.data(), (size_t)P->n_ips * 4, hipMemcpyHostToDevice) != hipSuccess) return -EIO;
            g_cache.n = P->n_ips; g_cache.s = zipf_s; g_cache.device = dev;
        }
        prob = g_cache.d_prob;
        alias = g_cache.d_alias;
    }
    if (count == 0) return 0;
    const uint64_t blocks = (count + 255) / 256;
    const uint32_t grid = (uint32_t)(blocks < 16384 ? blocks : 16384);
    k_synth<<<grid, 256, 0, st>>>(*P, prob, alias, j0, count, d_hdr, d_len, d_ts);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // extern "C"
