// fsx_flow_common.h — per-source flow sums and their finish (features + q8 score, or
// the merge into the carried per-slot sums), shared by the flow tile kernels
// (fsx_flows.hip) and the fixed-window walkers that accumulate the features of the
// segments they replay (fsx_device.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>

#include "fsx_dev_common.h"
#include "fsx_internal.h"
#include "fsx_q8.h"
#include "fsx_shard.h"

namespace fsx {

typedef unsigned __int128 u128;

struct FlowAcc {
    uint64_t n, s1, dmax, pad;
    u128 s2, d1, d2;
};

__device__ __forceinline__ FlowAcc acc_zero() {
    FlowAcc a;
    a.n = a.s1 = a.dmax = a.pad = 0;
    a.s2 = a.d1 = a.d2 = 0;
    return a;
}
__device__ __forceinline__ void acc_add(FlowAcc &a, const FlowAcc &b) {
    a.n += b.n; a.s1 += b.s1; a.s2 += b.s2; a.d1 += b.d1; a.d2 += b.d2;
    a.dmax = b.dmax > a.dmax ? b.dmax : a.dmax;
}
__device__ __forceinline__ u128 shfl_up128(u128 v, int d) {
    const uint64_t lo = __shfl_up((uint64_t)v, d), hi = __shfl_up((uint64_t)(v >> 64), d);
    return ((u128)hi << 64) | lo;
}
__device__ __forceinline__ u128 shfl_xor128(u128 v, int d) {
    const uint64_t lo = __shfl_xor((uint64_t)v, d), hi = __shfl_xor((uint64_t)(v >> 64), d);
    return ((u128)hi << 64) | lo;
}
__device__ __forceinline__ FlowAcc shfl_up_acc(const FlowAcc &a, int d) {
    FlowAcc r;
    r.n = __shfl_up(a.n, d); r.s1 = __shfl_up(a.s1, d); r.dmax = __shfl_up(a.dmax, d); r.pad = 0;
    r.s2 = shfl_up128(a.s2, d); r.d1 = shfl_up128(a.d1, d); r.d2 = shfl_up128(a.d2, d);
    return r;
}
__device__ __forceinline__ FlowAcc wave_sum_acc(FlowAcc a) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        FlowAcc b;
        b.n = __shfl_xor(a.n, o); b.s1 = __shfl_xor(a.s1, o); b.dmax = __shfl_xor(a.dmax, o);
        b.s2 = shfl_xor128(a.s2, o); b.d1 = shfl_xor128(a.d1, o); b.d2 = shfl_xor128(a.d2, o);
        acc_add(a, b);
    }
    return a;
}

// Flow sums of positions [a, b) of the run that starts at rs <= a, one wave: 1024
// consecutive positions per round (16 loads in flight per lane), inter-arrival times
// across lanes by shuffles; the total in every lane.
template <class SV>
__device__ FlowAcc flow_wave_acc(const SV &sv, uint32_t rs, uint32_t a, uint32_t b) {
    const uint32_t lane = lane_id();
    FlowAcc A = acc_zero();
    uint64_t carry = a > rs ? sv.t(a - 1) : 0ull;   // timestamp of the position before the round
    for (uint32_t q0 = a; q0 < b; q0 += 1024) {
        uint64_t t[16];
        uint32_t L[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t q = q0 + 64u * (uint32_t)r + lane;
            if (q < b) sv.tl(q, t[r], L[r]);
            else { t[r] = 0; L[r] = 0; }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t q = q0 + 64u * (uint32_t)r + lane;
            uint64_t tp = __shfl_up(t[r], 1);
            if (lane == 0) tp = carry;
            if (q < b) {
                FlowAcc c = acc_zero();
                c.n = 1; c.s1 = L[r]; c.s2 = (u128)L[r] * L[r];
                if (q != rs) {
                    const uint64_t d = t[r] - tp;
                    c.d1 = d; c.d2 = (u128)d * d; c.dmax = d;
                }
                acc_add(A, c);
            }
            carry = __shfl(t[r], 63);
        }
    }
    return wave_sum_acc(A);
}

// A source's sums carried across the calls of one fsx_flows_begin .. fsx_flows_end
// epoch (the sharded owner receives a source's packets over several sub-batches, in
// global arrival order): merging call B after call A adds B's sums plus the gap
// d = first_t(B) - last_t(A) to the inter-arrival sums; dport is the first call's.
struct SlotAcc {
    uint64_t n, s1, dmax, last_t;
    u128 s2, d1, d2;
    uint32_t dport, epoch;
    uint32_t pad_[2];
};
static_assert(sizeof(SlotAcc) == 96, "SlotAcc layout");

struct FlowOut {
    FlowAcc *acc;  // per source: exact sums (finished by k_flow_finish)
    uint8_t *keys16;
    uint8_t *fam;
    float *feat;   // may be null
    float *prob;   // may be null
    uint8_t *dec;  // may be null
    uint32_t cap;
    SlotAcc *sacc;             // accumulate mode (else null)
    uint32_t epoch;
    const uint32_t *seg_slot;  // table slot of each source (accumulate mode)
    const uint64_t *ts;        // arrival timestamps (first / last packet of a source)
    // per source (may be null): low word of its first sort word (k_heads_write) and its first
    // frame length (k_flow_tile), so k_flow_finish gathers only the first header record
    const uint32_t *seg_lo;
    uint32_t *seg_len;
    PartialOut part;   // partials mode (buf non-null): raw sums per owner run, no row
};

// include/fsx_hip.h fsx_flow_partial (112 bytes).
struct FlowPartial {
    uint32_t key[4];
    uint32_t tag, dport;
    uint64_t n, s1, dmax, first_ts, last_ts;
    u128 s2, d1, d2;
};
static_assert(sizeof(FlowPartial) == 112 && offsetof(FlowPartial, s2) == 64, "fsx_flow_partial layout");

// Source (tag, k)'s partial into the run of its owner rank.
__device__ __forceinline__ void write_partial(const PartialOut &P, uint32_t tag, const uint32_t k[4], uint32_t dport,
                                              const FlowAcc &a, uint64_t t0, uint64_t t1) {
    const uint32_t o = shard_owner_of(tag, k, P.G);
    const unsigned long long j = atomicAdd(&P.cnt[o], 1ull);
    if (j >= P.cap) return;
    FlowPartial x;
    x.key[0] = k[0]; x.key[1] = k[1]; x.key[2] = k[2]; x.key[3] = k[3];
    x.tag = tag;
    x.dport = dport;
    x.n = a.n; x.s1 = a.s1; x.dmax = a.dmax;
    x.first_ts = t0;
    x.last_ts = t1;
    x.s2 = a.s2; x.d1 = a.d1; x.d2 = a.d2;
    reinterpret_cast<FlowPartial *>(P.buf)[(size_t)o * P.cap + j] = x;
}

// L4 destination port of the source's first packet (oracle fsxo_dst_port).
__device__ __forceinline__ uint32_t dst_port(const uint8_t *f, uint32_t len) {
    const uint32_t proto = ((uint32_t)f[12] << 8) | f[13];
    uint32_t off, l4;
    if (proto == 0x0800u) {
        if (len < 34) return 0;
        off = 14u + 4u * (f[14] & 0x0Fu);
        l4 = f[23];
    } else if (proto == 0x86DDu) {
        if (len < 54) return 0;
        off = 54;
        l4 = f[20];
    } else {
        return 0;
    }
    if (l4 != 6 && l4 != 17) return 0;
    if (off + 4 > len || off + 4 > 64) return 0;
    return ((uint32_t)f[off + 2] << 8) | f[off + 3];
}

// Family, key and L4 destination port of one 64-byte header record from four 16-byte loads
// (key_of + dst_port read the same bytes with up to eight scattered loads of a random
// record); identical results: the IPv4 port at byte off + 2 = 16 + 4 IHL is the low half
// of dword 4 + IHL, the IPv6 one at byte 56 that of dword 14.
__device__ __forceinline__ uint32_t record_src_port(const uint8_t *rec, uint32_t len, uint32_t k[4],
                                                   uint32_t &dport) {
    const uint4 *q = reinterpret_cast<const uint4 *>(rec);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    const uint32_t w[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    const uint32_t proto = ((w[3] & 0xFFu) << 8) | ((w[3] >> 8) & 0xFFu);
    uint32_t tag, off, l4;
    if (proto == 0x86DDu) {
        tag = 2;
        k[0] = (w[5] >> 16) | (w[6] << 16); k[1] = (w[6] >> 16) | (w[7] << 16);
        k[2] = (w[7] >> 16) | (w[8] << 16); k[3] = (w[8] >> 16) | (w[9] << 16);
        off = 54;
        l4 = w[5] & 0xFFu;   // byte 20: next header
        if (len < 54) { dport = 0; return tag; }
    } else {
        tag = 1;
        k[0] = (w[6] >> 16) | (w[7] << 16);   // bytes 26..29
        k[1] = k[2] = k[3] = 0;
        off = 14u + 4u * ((w[3] >> 16) & 0x0Fu);   // byte 14: IHL
        l4 = w[5] >> 24;                           // byte 23: protocol
        if (len < 34) { dport = 0; return tag; }
    }
    dport = 0;
    if ((l4 == 6 || l4 == 17) && off + 4 <= len && off + 4 <= 64) {
        // (IHL 0 .. 12: dword 4 .. 15, the port's first byte at the dword's start)
        const uint32_t wi = (off + 2) >> 2;
        uint32_t x = 0;
#pragma unroll
        for (uint32_t j = 4; j < 16; ++j) x = wi == j ? w[j] : x;
        dport = ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
    }
    return tag;
}

__device__ __forceinline__ void acc_store(const FlowOut &out, uint32_t g, const FlowAcc &a) {
    if (g < out.cap) out.acc[g] = a;
}

__device__ __forceinline__ void write_row(uint32_t g, const FlowAcc &a, uint32_t tag, const uint32_t k[4],
                                 uint32_t dport, const FlowOut &out, const ScoreParams &P);
__device__ __forceinline__ void flow_emit(uint32_t g, const FlowAcc &a, uint32_t tag, const uint32_t k[4],
                                          uint32_t dport, uint64_t t0, uint64_t t1, uint32_t slot,
                                          const FlowOut &out, const ScoreParams &P);

// Features of source g from its exact sums, then the q8 score (accumulate mode: the sums
// merge into the source's SlotAcc instead).
__device__ __forceinline__ void flow_finish(uint32_t g, const FlowAcc &a, const uint64_t *S,
                            const uint32_t *seg_start, const PacketIn &in, const uint32_t *len,
                            uint32_t salt, const FlowOut &out, const ScoreParams &P) {
    if (g >= out.cap) return;
    const uint32_t p0 = seg_start[g];
    const uint64_t v = out.seg_lo ? (uint64_t)out.seg_lo[g] : S[p0];   // (family, arrival index)
    uint32_t k[4];
    const uint32_t idx = pk_idx(v);
    uint32_t tag, dport;
    if (in.rec) {   // record mode: key and port travel in the exchange record
        uint32_t L;
        uint64_t T;
        tag = rec_read(in.rec, in.rec_bytes, idx, k, L, T, dport);
    } else {
        (void)salt;
        tag = record_src_port(in.hdr + (size_t)idx * 64, out.seg_len ? out.seg_len[g] : len[idx], k, dport);
    }
    const bool need_t = out.part.buf || out.sacc;
    flow_emit(g, a, tag, k, dport, need_t ? out.ts[idx] : 0ull,
              need_t ? out.ts[pk_idx(S[seg_start[g + 1] - 1])] : 0ull, out.sacc ? out.seg_slot[g] : 0u, out, P);
}

// Source g's finished sums (first / last timestamp t0 / t1, table slot for the accumulate
// mode): its flow partial, its merge into the carried per-slot sums, or its output row.
__device__ __forceinline__ void flow_emit(uint32_t g, const FlowAcc &a, uint32_t tag, const uint32_t k[4],
                                          uint32_t dport, uint64_t t0, uint64_t t1, uint32_t slot,
                                          const FlowOut &out, const ScoreParams &P) {
    if (g >= out.cap) return;
    if (out.part.buf) {   // partials mode: the raw sums with the run's first / last timestamp
        write_partial(out.part, tag, k, dport, a, t0, t1);
        return;
    }
    if (out.sacc) {
        SlotAcc &m = out.sacc[slot];
        if (m.epoch != out.epoch) {   // the source's first call of this epoch
            m.n = a.n; m.s1 = a.s1; m.s2 = a.s2; m.d1 = a.d1; m.d2 = a.d2; m.dmax = a.dmax;
            m.dport = dport;
            m.epoch = out.epoch;
        } else {
            const uint64_t d = t0 - m.last_t;
            m.n += a.n; m.s1 += a.s1; m.s2 += a.s2;
            m.d1 += a.d1 + (u128)d;
            m.d2 += a.d2 + (u128)d * d;
            const uint64_t mx = a.dmax > d ? a.dmax : d;
            m.dmax = mx > m.dmax ? mx : m.dmax;
        }
        m.last_t = t1;
        return;
    }
    write_row(g, a, tag, k, dport, out, P);
}

// Output row g: key, family, the eight features, q8 probability / decision.
__device__ __forceinline__ void write_row(uint32_t g, const FlowAcc &a, uint32_t tag, const uint32_t k[4],
                                 uint32_t dport, const FlowOut &out, const ScoreParams &P) {
    uint32_t *kw = reinterpret_cast<uint32_t *>(out.keys16 + (size_t)g * 16);
    kw[0] = k[0]; kw[1] = k[1]; kw[2] = k[2]; kw[3] = k[3];
    out.fam[g] = tag == 1 ? 4 : 6;
    const uint64_t n = a.n;
    const double dn = (double)n;
    const double mean = (double)a.s1 / dn;
    double var = 0.0;
    if (n >= 2) {
        const u128 num = (u128)n * a.s2 - (u128)a.s1 * (u128)a.s1;
        var = (double)num / (dn * (dn - 1.0));
    }
    double iat_mean = 0.0, iat_var = 0.0;
    if (n >= 2) iat_mean = (double)a.d1 / (double)(n - 1) / 1000.0;
    if (n >= 3) {
        const uint64_t m = n - 1;
        const u128 num = (u128)m * a.d2 - a.d1 * a.d1;
        iat_var = (double)num / ((double)m * ((double)m - 1.0)) / 1000000.0;
    }
    float x[8];
    x[0] = (float)dport;
    x[1] = (float)mean;
    x[2] = (float)sqrt(var);
    x[3] = (float)var;
    x[4] = (float)mean;
    x[5] = (float)iat_mean;
    x[6] = (float)sqrt(iat_var);
    x[7] = (float)((double)a.dmax / 1000.0);
    if (out.feat) {
        float4 *f4 = reinterpret_cast<float4 *>(out.feat + (size_t)g * 8);
        f4[0] = make_float4(x[0], x[1], x[2], x[3]);
        f4[1] = make_float4(x[4], x[5], x[6], x[7]);
    }
    if (P.enabled && out.prob) {
        const float p = (float)lut_get(P, q8_linear(x, P)) * 0.00390625f;
        out.prob[g] = p;
        out.dec[g] = p > 0.5f ? 1 : 0;
    }
}

}  // namespace fsx
