// fsx_walk.h — the fixed-window limiter of src/fsx_kern.c:150-346 over one source's run
// of packets in arrival order: the exact per-packet step, exact replays (one thread / one
// wave) and the epoch-jump evaluation, on any SegView-like accessor (sorted positions in
// HBM for the tile walkers, LDS positions for the light-bin tail, fsx_bins.hip).
#pragma once
#include "fsx_seg.h"

namespace fsx {

constexpr uint64_t kBig = 1ull << 62;

struct FwState {
    bool has_st, has_bl;
    uint64_t pps, bps, tt, till;
};

// One packet of src/fsx_kern.c:150-346 (exact, any timestamps, u64 wraparound).
template <class MW>
__device__ __forceinline__ void fw_step(FwState &s, uint64_t now, uint32_t L, uint32_t q,
                                        const Limits &lim, MW &mw) {
    if (s.has_bl && s.till > 0) {
        if (now > s.till) s.has_bl = false;                 // :193-204 delete
        else { mw.emit(q, XDP_DROP); return; }              // :205-215
    }
    uint64_t cp, cb;
    if (s.has_st) {
        if (now - s.tt > lim.window) { s.pps = 0; s.bps = 0; s.tt = now; cp = 0; cb = 0; }  // :245-250
        else { s.pps += 1; s.bps += L; cp = s.pps; cb = s.bps; }                            // :258-262
    } else {
        s.has_st = true; s.pps = 1; s.bps = L; s.tt = now; cp = 1; cb = L;                  // :265-284
    }
    if (cp > lim.pps || cb > lim.bps) {                     // :312
        s.till = now + lim.block; s.has_bl = true;          // :317-326
        mw.emit(q, XDP_DROP);
    } else {
        mw.emit(q, XDP_PASS);
    }
}

// Exact replay for one thread, 16 packets' loads in flight per step.
template <class SV, class MW>
__device__ void walk_fixed_exact_thread(const SV &sv, uint32_t a, uint32_t b,
                                        const Limits &lim, MW &mw, FwState &s) {
    for (uint32_t q0 = a; q0 < b; q0 += 16) {
        uint64_t t[16];
        uint32_t L[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (q0 + k < b) sv.tl(q0 + k, t[k], L[k]);
            else { t[k] = 0; L[k] = 0; }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (q0 + k < b) fw_step(s, t[k], L[k], q0 + k, lim, mw);
    }
}

// Exact replay for one wave: 64 packets loaded in parallel, then stepped uniformly
// (every lane keeps the same state; values broadcast by shuffles).
template <class SV, class MW>
__device__ void walk_fixed_exact_wave(const SV &sv, uint32_t a, uint32_t b, const Limits &lim,
                                      MW &mw, FwState &s) {
    const uint32_t lane = lane_id();
    for (uint32_t q0 = a; q0 < b; q0 += 64) {
        const uint32_t q = q0 + lane;
        const uint64_t tq = q < b ? sv.t(q) : 0ull;
        const uint32_t lq = q < b ? sv.l(q) : 0u;
        const uint32_t cnt = min(64u, b - q0);
        for (uint32_t k = 0; k < cnt; ++k)
            fw_step(s, __shfl(tq, (int)k), __shfl(lq, (int)k), q0 + k, lim, mw);
    }
}

// Epoch-jump evaluation (non-decreasing timestamps, no u64 overflow). An epoch
// starts where ip_stats (re)starts a window: the first-ever packet (count 1), a
// reset packet (count 0, not counted) or the carried window (continuation). With
// counts consecutive inside an epoch, the count trigger is at a closed-form
// position; the window end and the blacklist end are searches.
template <bool kWave, class SV, class MW>
__device__ __forceinline__ void walk_fixed_fast(const SV &sv, uint32_t a, uint32_t b, const Limits &lim,
                                uint32_t maxL, MW &mw, FwState &s) {
    const uint64_t P = lim.pps, B = lim.bps, W = lim.window, BLK = lim.block;
    uint32_t p = a;
    if (s.has_bl && s.till > 0) {
        const uint32_t j = search_gt<kWave>(sv, a, b, s.till);
        if (j > a) mw.emit(a, XDP_DROP);
        if (j < b) s.has_bl = false;
        p = j;
    }
    bool touched = false;
    uint32_t ep_lo = 0, ep_hi = 0;
    uint64_t bps_base = 0;
    while (p < b) {
        const uint64_t t = sv.t(p);
        uint64_t T0, pc, pb;
        uint32_t cs;
        if (s.has_st && !(t - s.tt > W)) { T0 = s.tt; pc = s.pps; pb = s.bps; cs = 1; }
        else if (s.has_st) { T0 = t; pc = 0; pb = 0; cs = 0; }
        else { T0 = t; pc = 0; pb = 0; cs = 1; }
        s.has_st = true;
        touched = true;
        const uint32_t e = search_gt<kWave>(sv, p + 1, b, T0 + W);
        const uint64_t c0 = pc + cs;
        uint64_t k64 = c0 > P ? (uint64_t)p : (uint64_t)p + (P + 1 - c0);
        if (k64 > e) k64 = e;
        // bytes: only scanned when bps could exceed B before the count does
        const bool bytes_possible = pb > B || (maxL && P + 1 > (B - pb) / maxL);
        if (bytes_possible) k64 = bytes_trigger<kWave>(sv, cs ? p : p + 1, (uint32_t)k64, pb, B);
        const uint32_t k = (uint32_t)k64;
        s.tt = T0;
        bps_base = pb;
        ep_lo = p + 1 - cs;
        if (k >= e) {   // window closes without a trigger
            mw.emit(p, XDP_PASS);
            s.pps = c0 + (uint64_t)(e - 1 - p);
            ep_hi = e;
            p = e;
            continue;
        }
        if (k > p) mw.emit(p, XDP_PASS);
        mw.emit(k, XDP_DROP);
        s.pps = c0 + (uint64_t)(k - p);
        ep_hi = k + 1;
        s.till = sv.t(k) + BLK;
        s.has_bl = true;
        uint32_t q = k + 1;
        for (;;) {
            const uint32_t j = search_gt<kWave>(sv, q, b, s.till);
            if (j >= b) { p = b; break; }
            s.has_bl = false;                    // expired: deleted at packet j
            const uint64_t tj = sv.t(j);
            if (tj - s.tt > W) { p = j; break; } // j resets the window: next epoch
            s.pps += 1;                          // re-trigger inside the window (block < window)
            bps_base += sv.l(j);
            s.till = tj + BLK;
            s.has_bl = true;
            q = j + 1;
        }
    }
    if (touched) s.bps = bps_base + sum_len<kWave>(sv, ep_lo, ep_hi);
}

// The whole slot line in four 16-byte loads: the walkers' state and the tag (0: a new
// source under lazy initialisation), one memory instruction per quarter instead of one per
// field (a flood's walker is bound by the per-segment memory operations).
struct SlotLine {
    uint4 q[4];
};
__device__ __forceinline__ SlotLine load_line(const Slot &sl) {
    const uint4 *p = reinterpret_cast<const uint4 *>(&sl);
    return SlotLine{{p[0], p[1], p[2], p[3]}};
}
__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)hi << 32 | lo; }
// field offsets: tag 0, flags 4, key 8..23, pps 24, bps 32, tt 40, till 48, aux 56
__device__ __forceinline__ FwState state_of(const SlotLine &L) {
    const uint32_t flags = L.q[0].y;
    return FwState{(flags & SLOT_HAS_ST) != 0, (flags & SLOT_HAS_BL) != 0, u64_of(L.q[1].z, L.q[1].w),
                   u64_of(L.q[2].x, L.q[2].y), u64_of(L.q[2].z, L.q[2].w), u64_of(L.q[3].x, L.q[3].y)};
}
__device__ __forceinline__ uint32_t tag_of(const SlotLine &L) { return L.q[0].x; }

__device__ __forceinline__ FwState load_state(const Slot &sl) {
    return FwState{(sl.flags & SLOT_HAS_ST) != 0, (sl.flags & SLOT_HAS_BL) != 0, sl.pps, sl.bps,
                   sl.tt, sl.till};
}
// A new source's Slot under lazy initialisation (IdTable::init = 0, the fixed window): k_parse
// claimed only its index head, so the walker that first stores its state also writes its
// family and key, from the head (IPv4 key word) and the IPv6 key words. Plain loads: the head
// was published by an earlier kernel (the parse, ordered before the tail by the stream or
// its front_done event), and no later writer changes it. heads null: k_parse initialised
// every slot. (Called after store_state, which leaves the tag alone: a tag still 0 is new.)
struct SlotKeys {
    const unsigned long long *heads;
    const uint32_t *k6;
    uint32_t fresh_bit = 0;   // sort words carry kFreshBit (fsx_internal.h)
    uint32_t tgen = 0;        // the table generation new lines are tagged with (Limits::tgen)
};

// h: the slot's head, loaded beside the slot's state (a load issued after the walk would
// add a memory round trip to every segment of a flood: config 5's walkers 11 -> 19.5 ms)
__device__ __forceinline__ void slot_adopt(Slot &sl, const SlotKeys &K, uint32_t i, unsigned long long h,
                                           uint32_t tgen) {
    const uint32_t tag = (uint32_t)(h >> 32) & 0xFFu;
    sl.key[0] = (uint32_t)h;
    sl.key[1] = tag == 2 ? K.k6[(size_t)i * 4 + 0] : 0u;
    sl.key[2] = tag == 2 ? K.k6[(size_t)i * 4 + 1] : 0u;
    sl.key[3] = tag == 2 ? K.k6[(size_t)i * 4 + 2] : 0u;
    sl.aux = 0;   // (a line of another table generation may hold its source's)
    sl.tag = slot_tag(tag, tgen);
}

// A new source's first state (lazy slots): the whole line in four 16-byte stores — family
// and key from its head h (and the IPv6 key words), the state, aux 0, no born stamp.
__device__ __forceinline__ void store_new_line(Slot &sl, const FwState &s, const SlotKeys &K, uint32_t i,
                                               unsigned long long h) {
    const uint32_t tag = (uint32_t)(h >> 32) & 0xFFu;
    uint32_t k1 = 0, k2 = 0, k3 = 0;
    if (tag == 2) { k1 = K.k6[(size_t)i * 4 + 0]; k2 = K.k6[(size_t)i * 4 + 1]; k3 = K.k6[(size_t)i * 4 + 2]; }
    const uint32_t flags = (s.has_st ? SLOT_HAS_ST : 0u) | (s.has_bl ? SLOT_HAS_BL : 0u);
    uint4 *p = reinterpret_cast<uint4 *>(&sl);
    p[0] = make_uint4(slot_tag(tag, K.tgen), flags, (uint32_t)h, k1);
    p[1] = make_uint4(k2, k3, (uint32_t)s.pps, (uint32_t)(s.pps >> 32));
    p[2] = make_uint4((uint32_t)s.bps, (uint32_t)(s.bps >> 32), (uint32_t)s.tt, (uint32_t)(s.tt >> 32));
    p[3] = make_uint4((uint32_t)s.till, (uint32_t)(s.till >> 32), 0u, 0u);
}

// store_state with the slot's flags as loaded (no re-read)
__device__ __forceinline__ void store_state_f(Slot &sl, const FwState &s, uint32_t flags0) {
    sl.flags = (flags0 & kFlagBits & ~(SLOT_HAS_ST | SLOT_HAS_BL)) | (s.has_st ? SLOT_HAS_ST : 0u) |
               (s.has_bl ? SLOT_HAS_BL : 0u);
    sl.pps = s.pps; sl.bps = s.bps; sl.tt = s.tt; sl.till = s.till;
}

__device__ __forceinline__ void store_state(Slot &sl, const FwState &s) {
    // (also clears the born stamp: the batch that inserted the slot got this far)
    sl.flags = (sl.flags & kFlagBits & ~(SLOT_HAS_ST | SLOT_HAS_BL)) | (s.has_st ? SLOT_HAS_ST : 0u) |
               (s.has_bl ? SLOT_HAS_BL : 0u);
    sl.pps = s.pps; sl.bps = s.bps; sl.tt = s.tt; sl.till = s.till;
}

__device__ __forceinline__ bool fast_ok(const BatchState *bs, const Limits &lim) {
    return !bs->nonmono && lim.block >= 1 && lim.pps < kBig && lim.bps < kBig && lim.window < kBig &&
           lim.block < kBig && bs->max_ts <= ~0ull - (lim.window > lim.block ? lim.window : lim.block);
}

}  // namespace fsx
