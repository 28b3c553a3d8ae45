// Standalone micro-benchmark of the onesweep sort passes on the BASELINE config-2
// stream (64M IPv4 packets, 1M Zipf(1.1) sources): per-pass device time, a phase
// breakdown from s_memrealtime stamps (100 MHz), and streaming-copy baselines of the
// same byte counts. Build + run: scripts/micro/run_sort_micro.sh (GPU box).
#define FSX_MICRO_STAMPS 1
#include "../../flowsentryx_amd/csrc/fsx_device.hip"
#include "../../flowsentryx_amd/csrc/fsx_flows.hip"
#include "../../flowsentryx_amd/csrc/fsx_score.hip"
#include "../../flowsentryx_amd/csrc/fsx_synth.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void k_copy2(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
                        uint64_t *__restrict__ c, uint64_t *__restrict__ d, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        c[i] = a[i];
        d[i] = b[i];
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (64u << 20);
    fsx_synth_params P{};
    P.n = n; P.seed = 0xF5A0 + 2; P.t0_ns = 1000000000ull; P.duration_ns = 30000000000ull;
    P.n_ips = 1u << 20; P.mode = FSX_SYNTH_ZIPF_V4; P.len_min = 60; P.len_max = 1514;
    P.ip_salt = 0x5A17;
    uint8_t *hdr; uint32_t *len; uint64_t *ts;
    CK(hipMalloc(&hdr, (size_t)n * 64)); CK(hipMalloc(&len, (size_t)n * 4)); CK(hipMalloc(&ts, (size_t)n * 8));
    if (fsx_synth_generate(&P, 1.1, 0, n, hdr, len, ts, nullptr)) { fprintf(stderr, "synth failed\n"); return 1; }
    uint64_t *packed[2], *pay[2];
    for (int k = 0; k < 2; ++k) { CK(hipMalloc(&packed[k], (size_t)n * 8)); CK(hipMalloc(&pay[k], (size_t)n * 8)); }
    uint8_t *verdict; CK(hipMalloc(&verdict, n));
    fsx::BatchState *bs; CK(hipMalloc(&bs, sizeof(fsx::BatchState)));
    uint32_t *ctl, *gbase; CK(hipMalloc(&ctl, fsx::kSortCtlWords * 4)); CK(hipMalloc(&gbase, 1024 * 4));
    const uint32_t ntiles = (n + fsx::kSortTile - 1) / fsx::kSortTile;
    unsigned long long *status; CK(hipMalloc(&status, (size_t)(ntiles + 2) * 256 * 8));
    CK(hipMemset(status, 0, (size_t)(ntiles + 2) * 256 * 8));
    unsigned long long *stamps; CK(hipMalloc(&stamps, (size_t)ntiles * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fsx_stamps), &stamps, sizeof(stamps)));

    CK(hipMemset(bs, 0, sizeof(fsx::BatchState)));
    CK(hipMemset(ctl, 0, fsx::kSortCtlWords * 4));
    const uint32_t salt = 0x1234567u;
    fsx::k_parse<<<2048, 256>>>(hdr, len, ts, n, packed[0], verdict, bs, salt, 0x9E3779B97F4A7C15ull, 0, ctl);
    fsx::k_hist_prep<<<1, 256>>>(ctl, gbase, bs);
    CK(hipDeviceSynchronize());
    fsx::BatchState h;
    CK(hipMemcpy(&h, bs, sizeof(h), hipMemcpyDeviceToHost));
    printf("n=%u valid=%u pay_ok=%u tiles=%u\n", n, h.n_valid, h.pay_ok, ntiles);
    // keep the parsed keys: every repetition sorts the same input
    uint64_t *keys0; CK(hipMalloc(&keys0, (size_t)n * 8));
    CK(hipMemcpy(keys0, packed[0], (size_t)n * 8, hipMemcpyDeviceToDevice));

    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    uint32_t gen = 4;
    std::vector<unsigned long long> hs((size_t)ntiles * 8);
    // variants: 0 = tile histograms (default pipeline), 8 / 16 = onesweep look-back width
    const int lws[] = {0, 1, 8};  // 0: tile sort, early payload; 1: tile sort, late payload
    const uint32_t tcap = ntiles + 2;
    uint32_t *thist; CK(hipMalloc(&thist, (size_t)256 * tcap * 4));
    for (int rep = 0; rep < 6; ++rep) {
        const int lw = lws[rep / 2];
        CK(hipMemcpy(packed[0], keys0, (size_t)n * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(ctl + 1024, 0, 16));
        float ms[4];
        for (int pass = 0; pass < 4; ++pass) {
            CK(hipMemset(stamps, 0, (size_t)ntiles * 64));
            CK(hipEventRecord(e0));
#define OS_ARGS                                                                              \
    packed[pass & 1], packed[(pass + 1) & 1], n, pass == 0 ? nullptr : &bs->n_valid,          \
        32u + 8u * pass, gbase + 256 * pass, status, ctl + 1024 + pass, gen++, pass == 0, bs, \
        pass == 0 ? nullptr : pay[pass & 1], pay[(pass + 1) & 1], ts, len
            if (lw <= 1) {
                const uint32_t *Ld = pass == 0 ? nullptr : &bs->n_valid;
                fsx::k_tile_hist<<<ntiles, 256>>>(packed[pass & 1], n, Ld, 32u + 8u * pass, pass == 0, thist, tcap);
                CK(hipEventRecord(e3));
                fsx::k_tile_scan<<<256, 256>>>(thist, tcap, n, Ld, gbase + 256 * pass);
                CK(hipEventRecord(e2));
#define TS_ARGS                                                                             \
    packed[pass & 1], packed[(pass + 1) & 1], n, Ld, 32u + 8u * pass, pass == 0, thist, tcap, bs, \
        pass == 0 ? nullptr : pay[pass & 1], pay[(pass + 1) & 1], ts, len
                if (lw == 0) fsx::k_tile_scatter<false><<<ntiles, 256>>>(TS_ARGS);
                else fsx::k_tile_scatter<true><<<ntiles, 256>>>(TS_ARGS);
            } else fsx::k_onesweep<8><<<ntiles, 256>>>(OS_ARGS);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[pass], e0, e1));
            if (lw <= 1) {
                float mh, m3;
                CK(hipEventElapsedTime(&mh, e0, e2));
                CK(hipEventElapsedTime(&m3, e0, e3));
                printf("  tile sort pass %d: hist %.3f scan %.3f ms\n", pass, m3, mh - m3);
            }
            if (rep % 2 == 1) {
                CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
                unsigned long long t_min = ~0ull, t_max = 0;
                double ph[5] = {0, 0, 0, 0, 0};
                std::vector<double> lb;
                for (uint32_t t = 0; t < ntiles; ++t) {
                    const unsigned long long *s = &hs[(size_t)t * 8];
                    t_min = std::min(t_min, s[0]);
                    t_max = std::max(t_max, s[5]);
                    for (int k = 0; k < 5; ++k) ph[k] += (double)(s[k + 1] - s[k]);
                    lb.push_back((double)(s[2] - s[1]));
                }
                std::sort(lb.begin(), lb.end());
                printf("lw %d pass %d: %.3f ms  span %.1f us  per-tile us: load+rank %.2f lookback %.2f "
                       "scan+lds %.2f keys-out %.2f pay %.2f | lookback p50 %.2f p99 %.2f max %.2f\n",
                       lw, pass, ms[pass], (t_max - t_min) / 100.0, ph[0] / ntiles / 100, ph[1] / ntiles / 100,
                       ph[2] / ntiles / 100, ph[3] / ntiles / 100, ph[4] / ntiles / 100,
                       lb[lb.size() / 2] / 100, lb[lb.size() * 99 / 100] / 100, lb.back() / 100);
            }
        }
        printf("rep %d (%d): passes %.3f %.3f %.3f %.3f ms\n", rep, lw, ms[0], ms[1], ms[2], ms[3]);
        {
            std::vector<uint64_t> hk(h.n_valid);
            CK(hipMemcpy(hk.data(), packed[0], (size_t)h.n_valid * 8, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t q = 1; q < hk.size(); ++q) bad += (hk[q - 1] >> 31) > (hk[q] >> 31) ||
                ((hk[q - 1] >> 31) == (hk[q] >> 31) && (hk[q - 1] & 0x7FFFFFFF) >= (hk[q] & 0x7FFFFFFF));
            printf("  sorted+stable check: %zu violations\n", bad);
        }
    }
    CK(hipMemcpy(&h, bs, sizeof(h), hipMemcpyDeviceToHost));
    printf("err=%u\n", h.err);
    // streaming baseline: 2 x 8 B in, 2 x 8 B out per element
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        CK(hipEventRecord(e0));
        k_copy2<<<16384, 256>>>(packed[0], pay[0], packed[1], pay[1], n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy2 %.3f ms = %.2f TB/s\n", ms, 32.0 * n / ms / 1e9);
    }
    return 0;
}
