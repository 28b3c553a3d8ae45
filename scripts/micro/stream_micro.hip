// Streaming floors of k_parse's memory pattern (no parse logic): per packet the
// 64-byte header slot (16..64 bytes of it: every variant costs the same, the
// 64-byte slot is fetched whole), len (u32) and ts (u64) in, an 8-byte
// sort word and a 1-byte verdict out, with k_parse's grid (1024 blocks x 4 waves, one
// wave per 64-record step). Variants isolate what the bytes alone cost on MI355X.
// Build: scripts/micro/build_micro.sh; run on the GPU box: scripts/micro/run_micro.sh stream_micro
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

// kHdr: header uint4 chunks read per record (0..4); kOut: 0 none, 1 word only,
// 2 word + verdict; kLT: read len + ts.
template <int kHdr, int kOut, bool kLT, int kNT = 0, int kU = 1>
__global__ __launch_bounds__(256) void k_stream(const uint4 *__restrict__ hdr, const uint32_t *__restrict__ len,
                                                const uint64_t *__restrict__ ts, uint32_t n,
                                                uint64_t *__restrict__ word, uint8_t *__restrict__ verdict,
                                                uint64_t *__restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6), nw = gridDim.x * 4u;
    const uint32_t steps = (n + 63u) / 64u;
    uint64_t acc = 0;
    for (uint32_t s0 = wave * kU; s0 < steps; s0 += nw * kU) {
        uint4 hv[kU][kHdr > 0 ? kHdr : 1];
        uint32_t l[kU];
        uint64_t t[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t r0 = (s0 + u) * 64u;
#pragma unroll
            for (int k = 0; k < kHdr; ++k) {
                const uint32_t f = (uint32_t)k * 64u + lane;        // chunk f of the step
                constexpr uint32_t H = kHdr > 0 ? kHdr : 1;
                const uint32_t rec = r0 + f / H, c = f % H;
                const uint4 *a = hdr + (size_t)min(rec, n - 1) * 4u + c;
                if (kNT) {
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a));
                    hv[u][k] = make_uint4(q.x, q.y, q.z, q.w);
                } else {
                    hv[u][k] = *a;
                }
            }
            const uint32_t i = min(r0 + lane, n - 1);
            l[u] = 0; t[u] = 0;
            if (kLT) {
                if (kNT) { l[u] = __builtin_nontemporal_load(len + i); t[u] = __builtin_nontemporal_load(ts + i); }
                else { l[u] = len[i]; t[u] = ts[i]; }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t r0 = (s0 + u) * 64u;
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < kHdr; ++k) x ^= hv[u][k].x ^ hv[u][k].y ^ hv[u][k].z ^ hv[u][k].w;
            const uint64_t w = ((uint64_t)(x ^ l[u]) << 32) ^ t[u];
            if (kOut >= 1 && r0 + lane < n) word[r0 + lane] = w;
            if (kOut >= 2 && r0 + lane < n) verdict[r0 + lane] = (uint8_t)w;
            acc += w;
        }
    }
    if (kOut == 0 && acc == 0x123456789ull) sink[0] = acc;
}

template <int kHdr, int kOut, bool kLT, int kNT = 0, int kU = 1>
static void run(const char *name, const uint4 *hdr, const uint32_t *len, const uint64_t *ts, uint32_t n,
                uint64_t *word, uint8_t *verdict, uint64_t *sink, int grid) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)n * (kHdr * 16 + (kLT ? 12 : 0) + (kOut >= 1 ? 8 : 0) + (kOut >= 2 ? 1 : 0));
    float best = 1e9f, sum = 0.f;
    for (int rep = 0; rep < 8; ++rep) {
        CK(hipEventRecord(e0));
        k_stream<kHdr, kOut, kLT, kNT, kU><<<grid, 256>>>(hdr, len, ts, n, word, verdict, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 2) { sum += ms; best = ms < best ? ms : best; }
    }
    printf("%-34s grid %5d  mean %.4f ms  best %.4f ms  %.0f B/pkt  %.2f TB/s\n", name, grid, sum / 6, best,
           bytes / n, bytes / best / 1e9);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (64u << 20);
    uint4 *hdr; uint32_t *len; uint64_t *ts, *word, *sink; uint8_t *verdict;
    CK(hipMalloc(&hdr, (size_t)n * 64)); CK(hipMalloc(&len, (size_t)n * 4)); CK(hipMalloc(&ts, (size_t)n * 8));
    CK(hipMalloc(&word, (size_t)n * 8)); CK(hipMalloc(&verdict, n)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(hdr, 1, (size_t)n * 64)); CK(hipMemset(len, 2, (size_t)n * 4)); CK(hipMemset(ts, 3, (size_t)n * 8));
    for (int grid : {512, 1024, 2048}) {
        run<4, 2, true, 1, 1>("nt hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 2, true, 0, 2>("u2 hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 2, true, 1, 2>("nt u2 hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 2, true, 0, 4>("u4 hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 2, true, 1, 4>("nt u4 hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 0, true, 1, 2>("nt u2 hdr64+len+ts (read only)", hdr, len, ts, n, word, verdict, sink, grid);
        run<3, 2, true>("hdr48+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<4, 2, true>("hdr64+len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<3, 0, true>("hdr48+len+ts (read only)", hdr, len, ts, n, word, verdict, sink, grid);
        run<0, 2, true>("len+ts -> word+verdict", hdr, len, ts, n, word, verdict, sink, grid);
        run<0, 1, false>("word write only", hdr, len, ts, n, word, verdict, sink, grid);
    }
    return 0;
}
