// fsx_dev_common.h — device helpers shared by the hot-path kernels (wave scans,
// digit matching, key access on the packed sort words).
#pragma once
#include <hip/hip_runtime.h>

#include "fsx_internal.h"

namespace fsx {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Sorted positions a kernel covers: every IP packet, or (light_only 1) the light ones only
// — the heavy sources' verdicts come from their lists — or (2, the token bucket's heavy
// sources) the light ones only when the batch took the unsorted path (k_hmode), where the
// heavy sources never entered the sort.
__device__ __forceinline__ uint32_t cover_n(const BatchState *bs, uint32_t light_only) {
    return light_only == 1 || (light_only == 2 && bs->hfast) ? bs->n_light : bs->n_valid;
}

// Orders this wave's LDS accesses for the compiler (the hardware executes one wave's LDS
// operations in order). A wavefront-scope fence would also wait for every outstanding
// global load (s_waitcnt vmcnt(0)), draining software-pipelined prefetches each step.
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T x) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}

template <typename T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T y = __shfl_xor(x, o);
        x = y > x ? y : x;
    }
    return x;
}

// Sum over the 64 lanes, result in every lane.
template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// Exclusive prefix sum over the 256 threads of a block. s_tmp: >= 4 entries.
// Every thread of the block must call it. *total receives the block sum.
__device__ __forceinline__ uint32_t block256_excl(uint32_t x, uint32_t *s_tmp, uint32_t *total) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t incl = wave_incl_sum(x);
    if (lane == 63) s_tmp[w] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        uint32_t v = s_tmp[i];
        off += i < w ? v : 0u;
        tot += v;
    }
    __syncthreads();
    if (total) *total = tot;
    return off + incl - x;
}

// "Last non-zero" scan operator over encoded (position << 8 | mark) words: max.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x = y > x ? y : x;
    }
    return x;
}

// XCD-aware tile order (cdna_hip_programming.md §5.5 T1, bijective form): blocks are dealt
// round-robin over the 8 XCDs, so block b gets tile (b % 8)'s contiguous share — consecutive
// tiles (whose output runs meet in the same cache lines) land in one XCD's L2. Speed only.
#ifndef FSX_XCD_SWIZZLE
#define FSX_XCD_SWIZZLE 1   // (A/B: scripts/build_variant.sh)
#endif
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nwg) {
    if (!FSX_XCD_SWIZZLE || nwg <= 8u) return b;
    const uint32_t q = nwg >> 3, r = nwg & 7u, x = b & 7u;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + (b >> 3);
}

// A wave-uniform 64-bit value into scalar registers.
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    // (readfirstlane returns int: through uint32_t, or the low half sign-extends)
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32;
}

template <int kBits = 8>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t active) {
    uint64_t peers = active;
#pragma unroll
    for (int b = 0; b < kBits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// IPv6 source address of arrival index i (bytes 22..37 of the record).
__device__ __forceinline__ void load_key6(const uint8_t *hdr, uint32_t i, uint32_t k[4]) {
    const uint32_t *d = reinterpret_cast<const uint32_t *>(hdr + (size_t)i * 64);
    const uint32_t d5 = d[5], d6 = d[6], d7 = d[7], d8 = d[8], d9 = d[9];
    k[0] = (d5 >> 16) | (d6 << 16);
    k[1] = (d6 >> 16) | (d7 << 16);
    k[2] = (d7 >> 16) | (d8 << 16);
    k[3] = (d8 >> 16) | (d9 << 16);
}

// Full key (family tag 1/2 + address words) of a packed sort word, from its record (an IP
// packet's record: EtherType 0x86DD is IPv6, 0x0800 IPv4, as k_parse decided).
__device__ __forceinline__ uint32_t key_of(uint64_t v, const uint8_t *hdr, uint32_t salt,
                                           uint32_t k[4]) {
    (void)salt;
    const uint32_t *d = reinterpret_cast<const uint32_t *>(hdr + (size_t)pk_idx(v) * 64);
    if ((d[3] & 0xFFFFu) == 0xDD86u) {   // bytes 12..13 = 86 DD
        load_key6(hdr, pk_idx(v), k);
        return 2u;
    }
    k[0] = (d[6] >> 16) | (d[7] << 16);   // bytes 26..29
    k[1] = k[2] = k[3] = 0;
    return 1u;
}

// Total order on (family, address) used to group colliding IPv6 hash runs.
__device__ __forceinline__ int key_cmp(uint32_t ta, const uint32_t *a, uint32_t tb,
                                       const uint32_t *b) {
    if (ta != tb) return ta < tb ? -1 : 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return 0;
}

// Loads of data read exactly once per batch (packet records, lengths, timestamps):
// non-temporal, so the stream does not evict what is re-read from L2 (the source
// index). FSX_STREAM_NT=0 builds plain loads (A/B: scripts/build_variant.sh).
#ifndef FSX_STREAM_NT
#define FSX_STREAM_NT 1
#endif
template <class T>
__device__ __forceinline__ T stream_load(const T *p) {
    if constexpr (FSX_STREAM_NT) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ uint4 stream_load16(const uint8_t *p) {
    if constexpr (FSX_STREAM_NT) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p));
        return make_uint4(q.x, q.y, q.z, q.w);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

}  // namespace fsx
