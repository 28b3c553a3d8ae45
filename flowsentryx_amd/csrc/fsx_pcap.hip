// fsx_pcap.hip — ingest of captured traffic (SURVEY.md §8 f, row 2): classic pcap files
// (microsecond or nanosecond timestamps, either byte order, Ethernet link type) into the
// 64-byte header records + frame length + arrival time the batch entry points take.
//
//   fsx_pcap_index           host: one pass over the record headers (the only sequential
//                            step: each record's length gives the next offset)
//   k_pcap_records           device: the first min(caplen, 64) bytes of every record from
//                            an HBM copy of the file, zero padded — the record layout of
//                            include/fsx_hip.h (coalesced 16-byte stores)
// The reference reads packets from the NIC through XDP (src/fsx_kern.c:96-97), where
// data_end - data is the frame length; a capture's original length is that value.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

#include "../../include/fsx_hip.h"
#include "fsx_internal.h"

namespace fsx {

__global__ __launch_bounds__(256) void k_pcap_records(const uint8_t *__restrict__ buf,
                                                      const uint64_t *__restrict__ off,
                                                      const uint32_t *__restrict__ caplen, uint32_t n,
                                                      uint8_t *__restrict__ hdr) {
    // 4 lanes per record, 16 bytes each
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t total = (uint64_t)n * 4;
    for (uint64_t t = tid; t < total; t += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = (uint32_t)(t >> 2), part = (uint32_t)(t & 3u);
        const uint32_t cl = min(caplen[r], 64u);
        const uint8_t *src = buf + off[r];
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t pos = part * 16u + (uint32_t)k * 4u + (uint32_t)b;
                if (pos < cl) v |= (uint32_t)src[pos] << (8 * b);
            }
            w[k] = v;
        }
        *reinterpret_cast<uint4 *>(hdr + (size_t)r * 64 + part * 16u) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

hipError_t launch_pcap_records(const uint8_t *buf, const uint64_t *off, const uint32_t *caplen, uint32_t n,
                               uint8_t *hdr, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    if (n == 0) return hipSuccess;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, ((uint64_t)n * 4 + 255) / 256);
    k_pcap_records<<<grid, 256, 0, st>>>(buf, off, caplen, n, hdr);
    return hipGetLastError();
}

}  // namespace fsx

static inline uint32_t rd32(const uint8_t *p, bool swap) {
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

extern "C" int fsx_pcap_index(const uint8_t *buf, size_t size, uint32_t flags, uint64_t *data_off,
                              uint32_t *caplen, uint32_t *origlen, uint64_t *ts_ns, size_t cap,
                              size_t *n_out, size_t *consumed) {
    if (!n_out || !consumed || (size && !buf) || (cap && (!data_off || !caplen || !origlen || !ts_ns)))
        return -EINVAL;
    const bool ns = (flags & FSX_PCAP_NANOSECONDS) != 0, swap = (flags & FSX_PCAP_SWAPPED) != 0;
    size_t pos = 0, n = 0;
    while (n < cap && pos + 16 <= size) {
        const uint32_t sec = rd32(buf + pos, swap), frac = rd32(buf + pos + 4, swap);
        const uint32_t cl = rd32(buf + pos + 8, swap), ol = rd32(buf + pos + 12, swap);
        if (pos + 16 + (uint64_t)cl > size) break;   // incomplete record: stop before it
        data_off[n] = pos + 16;
        caplen[n] = cl;
        origlen[n] = ol;
        ts_ns[n] = (uint64_t)sec * 1000000000ull + (ns ? (uint64_t)frac : (uint64_t)frac * 1000ull);
        ++n;
        pos += 16 + (size_t)cl;
    }
    *n_out = n;
    *consumed = pos;
    return 0;
}
