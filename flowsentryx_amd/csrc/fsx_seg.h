// fsx_seg.h — access to one source's run of sorted positions (its segment) for the
// limiter walkers: timestamps / lengths from the sort's payload words or gathered by
// arrival index, 64-wide cooperative and per-thread searches on non-decreasing
// timestamps, byte sums, and the verdict-change mark writer.
#pragma once
#include "fsx_dev_common.h"

namespace fsx {

#ifndef XDP_DROP
#define XDP_DROP 1
#define XDP_PASS 2
#endif

// Timestamp / length of sorted position q: from the payload words carried by the
// sort (kPay), else gathered through the arrival index.
template <bool kPay>
struct SegView {
    const uint64_t *S;
    const uint64_t *ts;
    const uint32_t *len;
    const uint64_t *pay;
    uint64_t tbase;
    __device__ __forceinline__ uint64_t t(uint32_t q) const {
        if constexpr (kPay) return tbase + (pay[q] >> kPayLenBits);
        else return ts[pk_idx(S[q])];
    }
    __device__ __forceinline__ uint32_t l(uint32_t q) const {
        if constexpr (kPay) return (uint32_t)pay[q] & ((1u << kPayLenBits) - 1u);
        else return len[pk_idx(S[q])];
    }
    // both from one payload word (or one arrival index)
    __device__ __forceinline__ void tl(uint32_t q, uint64_t &T, uint32_t &L) const {
        if constexpr (kPay) {
            const uint64_t w = pay[q];
            T = tbase + (w >> kPayLenBits);
            L = (uint32_t)w & ((1u << kPayLenBits) - 1u);
        } else {
            const uint32_t i = pk_idx(S[q]);
            T = ts[i];
            L = len[i];
        }
    }
    // Timestamps of positions q0 .. q0+15, q0 % 2 == 0, all < the valid count: 16-byte
    // vector loads of the payload words (one thread reads a whole 128-byte line).
    __device__ __forceinline__ void t16(uint32_t q0, uint64_t (&out)[16]) const {
        if constexpr (kPay) {
            const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(pay + q0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const ulonglong2 v = p[k];
                out[2 * k] = tbase + (v.x >> kPayLenBits);
                out[2 * k + 1] = tbase + (v.y >> kPayLenBits);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) out[k] = t(q0 + k);
        }
    }
};

// First q in [lo, hi) with t(q) > X (t non-decreasing on [lo, hi)); wave-uniform
// arguments, every lane calls. Round 0 probes 64 consecutive packets, round 1 64
// exponentially spaced ones, then 64-ary narrowing.
template <class SV>
__device__ uint32_t wave_gallop_gt(const SV &sv, uint32_t lo, uint32_t hi, uint64_t X) {
    const uint32_t lane = lane_id();
    if (lo >= hi) return hi;
    {
        const uint32_t q = lo + lane;
        const bool pr = q < hi && sv.t(q) > X;
        const uint64_t m = __ballot(pr);
        if (m) return lo + (uint32_t)__ffsll((unsigned long long)m) - 1u;
        if (hi - lo <= 64) return hi;
    }
    uint32_t good = lo + 63, bad = hi;  // t(good) <= X; answer in (good, bad]
    {
        const uint64_t q64 = (uint64_t)lo + (lane < 32 ? (64ull << lane) : (1ull << 40));
        const bool valid = q64 < hi;
        const bool pr = valid && sv.t((uint32_t)q64) > X;
        const uint64_t m = __ballot(pr);
        const uint64_t vm = __ballot(valid);
        if (m) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1u;
            bad = lo + (64u << f);
            if (f) good = lo + (64u << (f - 1));
        } else if (vm) {
            const uint32_t lv = 63u - (uint32_t)__clzll((long long)vm);
            good = lo + (64u << lv);
        }
    }
    while (bad - good > 64) {
        const uint32_t cnt = bad - good - 1;
        const uint32_t step = (cnt + 63) / 64;
        const uint32_t q = good + 1 + lane * step;
        const bool valid = q < bad;
        const bool pr = valid && sv.t(q) > X;
        const uint64_t m = __ballot(pr);
        if (m) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1u;
            const uint32_t nb = good + 1 + f * step;
            if (f) good = good + 1 + (f - 1) * step;
            bad = nb;
        } else {
            const uint64_t vm = __ballot(valid);
            good = good + 1 + (63u - (uint32_t)__clzll((long long)vm)) * step;
        }
    }
    const uint32_t q = good + 1 + lane;
    const bool pr = q < bad && sv.t(q) > X;
    const uint64_t m = __ballot(pr);
    return m ? good + (uint32_t)__ffsll((unsigned long long)m) : bad;
}

// Thread version: galloping from lo, O(log distance).
template <class SV>
__device__ __forceinline__ uint32_t gallop_gt(const SV &sv, uint32_t lo, uint32_t hi,
                                              uint64_t X) {
    if (lo >= hi) return hi;
    if (sv.t(lo) > X) return lo;
    uint32_t good = lo, bad = hi;
    uint32_t step = 1;
    for (;;) {
        const uint64_t cand = (uint64_t)good + step;
        if (cand >= hi) break;
        if (sv.t((uint32_t)cand) > X) { bad = (uint32_t)cand; break; }
        good = (uint32_t)cand;
        step <<= 1;
    }
    uint32_t l = good + 1, r = bad;
    while (l < r) {
        const uint32_t m = l + (r - l) / 2;
        if (sv.t(m) > X) r = m; else l = m + 1;
    }
    return l;
}

// Sum of frame lengths over [lo, hi): wave-strided (4 loads in flight per lane) or,
// for a thread, 16 independent gathers per step.
template <bool kWave, class SV>
__device__ __forceinline__ uint64_t sum_len(const SV &sv, uint32_t lo, uint32_t hi) {
    uint64_t s = 0;
    if constexpr (kWave) {
        const uint32_t lane = lane_id();
        uint32_t q = lo + lane;
        for (; q + 192 < hi; q += 256) {
            const uint32_t l0 = sv.l(q), l1 = sv.l(q + 64), l2 = sv.l(q + 128), l3 = sv.l(q + 192);
            s += (uint64_t)l0 + l1 + l2 + l3;
        }
        for (; q < hi; q += 64) s += sv.l(q);
        return wave_sum(s);
    } else {
        uint32_t q = lo;
        for (; q + 16 <= hi; q += 16) {
            uint32_t l[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) l[k] = sv.l(q + k);
#pragma unroll
            for (int k = 0; k < 16; ++k) s += l[k];
        }
        for (; q < hi; ++q) s += sv.l(q);
        return s;
    }
}

// First q in [from, lim) with acc0 + sum(L[from..q]) > B, else lim.
template <bool kWave, class SV>
__device__ uint32_t bytes_trigger(const SV &sv, uint32_t from, uint32_t lim, uint64_t acc0,
                                  uint64_t B) {
    uint64_t acc = acc0;
    if constexpr (kWave) {
        const uint32_t lane = lane_id();
        for (uint32_t q0 = from; q0 < lim; q0 += 64) {
            const uint32_t q = q0 + lane;
            const uint64_t L = q < lim ? sv.l(q) : 0;
            const uint64_t incl = wave_incl_sum(L);
            const uint64_t m = __ballot(q < lim && acc + incl > B);
            if (m) return q0 + (uint32_t)__ffsll((unsigned long long)m) - 1u;
            acc += __shfl(incl, 63);
        }
        return lim;
    } else {
        for (uint32_t q = from; q < lim; ++q) {
            acc += sv.l(q);
            if (acc > B) return q;
        }
        return lim;
    }
}

template <bool kWave, class SV>
__device__ __forceinline__ uint32_t search_gt(const SV &sv, uint32_t lo, uint32_t hi, uint64_t X) {
    if constexpr (kWave) return wave_gallop_gt(sv, lo, hi, X);
    else return gallop_gt(sv, lo, hi, X);
}

// Verdict-change marks of a segment: marks[pos] = the verdict from sorted position pos on
// (fill-forward by k_fill_*), or, in list mode (a heavy source's segment),
// an ordered list of {arrival index << 1 | DROP} of the packets where the verdict
// changes, stored over the segment's own positions, plus the PASS / DROP packet counts.
template <bool kWave, bool kList = false>
struct MarkWriter {
    uint8_t *marks;
    uint8_t last;
    uint32_t *list = nullptr;     // kList: entry e at list[e]
    const uint64_t *S = nullptr;  // sort words (arrival index of a position)
    uint32_t nl = 0, last_pos = 0;
    uint64_t npass = 0, ndrop = 0;
    __device__ __forceinline__ void emit(uint32_t pos, uint8_t v) {
        if (v != last) {
            if constexpr (kList) {
                count_run(pos);
                const uint32_t e = pk_idx(S[pos]) << 1 | (v == XDP_DROP ? 1u : 0u);
                if (!kWave || lane_id() == 0) list[nl] = e;
                ++nl;
                last_pos = pos;
            } else if (!kWave || lane_id() == 0) {
                marks[pos] = v;
            }
            last = v;
        }
    }
    // list mode: the run [last_pos, pos) of verdict `last` into the counts (selects, not a
    // branch: a branch between the two counters made the compiler keep them in scratch)
    __device__ __forceinline__ void count_run(uint32_t pos) {
        const uint64_t r = pos - last_pos;
        ndrop += last == XDP_DROP ? r : 0ull;
        npass += (last && last != XDP_DROP) ? r : 0ull;
    }
    // list mode: close the counts at the segment end b
    __device__ __forceinline__ void finish(uint32_t b) {
        count_run(b);
        last_pos = b;
    }
};

// Heavy verdict lists: a heavy source's segment (one run of sort pass 0, from
// n_light on) writes its verdict changes as an arrival-index list over its own positions in
// `list` instead of marks, and counts its PASS / DROP packets into stats_map here (k_fill_*
// cover the light positions only). Shared by the fixed-window and sliding-window walkers.
struct HeavyLists {
    uint32_t *list;   // nullptr: every segment writes marks
    HeavySet *hs;
    TableState *tstate;
    BatchState *bs;
};

template <bool kWave>
__device__ __forceinline__ void heavy_list_open(const HeavyLists &H, const uint64_t *S, uint32_t a,
                                                MarkWriter<kWave, true> &mw) {
    mw.list = H.list + 2u * a;   // bytes [8a, 8a + 4 * entries): inside the run's own 8-byte positions
    mw.S = S;
}

// heavy source h's list: its place and length for k_verdict_apply, its verdict counts
template <bool kWave>
__device__ __forceinline__ void heavy_list_close(const HeavyLists &H, int h, uint32_t a, uint32_t b,
                                                 MarkWriter<kWave, true> &mw) {
    mw.finish(b);
    if (kWave && lane_id() != 0) return;
    H.hs->lbase[h] = 2u * a;
    H.hs->lcnt[h] = mw.nl;
    unsigned long long *st = reinterpret_cast<unsigned long long *>(H.tstate->stats);
    if (mw.npass) {
        atomicAdd(st, (unsigned long long)mw.npass);
        atomicAdd(reinterpret_cast<unsigned long long *>(&H.bs->allowed), (unsigned long long)mw.npass);
    }
    if (mw.ndrop) {
        atomicAdd(st + 1, (unsigned long long)mw.ndrop);
        atomicAdd(reinterpret_cast<unsigned long long *>(&H.bs->dropped), (unsigned long long)mw.ndrop);
    }
}

}  // namespace fsx
