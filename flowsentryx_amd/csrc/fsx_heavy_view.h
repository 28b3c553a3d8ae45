// fsx_heavy_view.h — a heavy source's packets by rank in arrival order (DESIGN.md §3 "Heavy
// sources outside the sort"): the rank / select view the unsorted-path walkers run on (the
// fixed window's walk_fixed_fast in fsx_heavy.hip, the sliding window's rank walker in
// fsx_limiters.hip), its searches and byte sums, and its verdict-change list writer.
#pragma once
#include "fsx_dev_common.h"
#include "fsx_internal.h"
#include "fsx_search.h"
#include "fsx_seg.h"

namespace fsx {

// The 0x80-byte of every byte of x that equals b (exact: no borrow across bytes).
__device__ __forceinline__ uint32_t byte_eq_mask(uint32_t x, uint32_t pat) {
    const uint32_t y = x ^ pat;
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}

// Heavy source h's packets by rank (fsx_walk.h SegView interface; wave-cooperative: every
// lane calls with the same arguments).
struct HeavyView {
    const uint8_t *tags;          // verdict bytes: 0x80 | h for h's packets
    const uint64_t *ts;
    const uint32_t *len;
    const uint32_t *row;          // pass-0 tile offsets of bucket light_b + h (incl. base)
    const HeavyTileRec *rec;
    uint32_t base, cnt, ntiles, n, h;
    uint32_t pat;                 // (0x80 | h) in every byte
    uint32_t *err = nullptr;      // BatchState::err: ERR_HEAVY_VIEW on an inconsistent row / tags

    __device__ __forceinline__ uint32_t pre(uint32_t t) const { return row[t] - base; }

    // (a corrupted row or tag array fails the batch instead of hanging it)
    __device__ __forceinline__ void fail() const {
        if (err && lane_id() == 0) atomicOr(err, ERR_HEAVY_VIEW);
    }

    // the largest tile t with pre(t) <= r (bounded: ary64_step, fsx_search.h)
    __device__ __forceinline__ uint32_t tile_of(uint32_t r) const {
        const uint32_t lane = lane_id();
        uint32_t lo = 0, hi = ntiles;
        while (hi - lo > 1) {
            const uint32_t step = ary64_width(lo, hi);
            const uint32_t q = lo + lane * step;
            const uint64_t m = __ballot(q < hi && pre(q) <= r);   // lane 0 (q = lo) on a valid row
            if (!ary64_step(lo, hi, step, m)) fail();
        }
        return lo;
    }

    // lane's 64 verdict bytes of tile t as 16 words (0 beyond n)
    __device__ __forceinline__ void tile_words(uint32_t t, uint32_t (&w)[16]) const {
        const uint32_t lane = lane_id();
        const uint32_t p0 = t * (uint32_t)kSortTile + lane * 64u;
        if (p0 + 64u <= n) {
            const uint4 *q = reinterpret_cast<const uint4 *>(tags + p0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = q[k];
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                uint32_t x = 0;
                for (uint32_t b = 0; b < 4; ++b) {
                    const uint32_t p = p0 + (uint32_t)k * 4u + b;
                    if (p < n) x |= (uint32_t)tags[p] << (8 * b);
                }
                w[k] = x;
            }
        }
    }

    // arrival index of h's r-th packet (r < cnt)
    __device__ __forceinline__ uint32_t select(uint32_t r) const {
        const uint32_t lane = lane_id();
        const uint32_t t = tile_of(r);
        uint32_t k = r - pre(t);
        uint32_t w[16];
        tile_words(t, w);
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) c += (uint32_t)__popc(byte_eq_mask(w[j], pat));
        const uint32_t incl = wave_incl_sum(c);
        const uint32_t excl = incl - c;
        const bool mine = excl <= k && k < incl;
        uint32_t idx = 0;
        if (mine) {
            uint32_t kk = k - excl;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                uint32_t m = byte_eq_mask(w[j], pat);
                const uint32_t pc = (uint32_t)__popc(m);
                if (kk < pc && idx == 0) {
                    for (uint32_t s = 0; s < kk; ++s) m &= m - 1u;
                    idx = 1u + t * (uint32_t)kSortTile + lane * 64u + (uint32_t)j * 4u +
                          (uint32_t)(__ffs((int)m) - 1) / 8u;
                }
                kk = kk >= pc ? kk - pc : 0xFFFFFFFFu;
            }
        }
        const uint64_t bm = __ballot(mine);
        // (no lane: the tags do not hold r — a caller that rewrote the verdict buffer while the
        // batch was in flight, or a corrupted row; an index inside the batch rather than a
        // fault, and the batch fails)
        if (!bm) fail();
        return bm ? __shfl(idx, __ffsll((unsigned long long)bm) - 1) - 1u : n - 1u;
    }

    // h's packets at arrival indices < i (i <= n)
    __device__ __forceinline__ uint32_t rank(uint32_t i) const {
        if (i >= n) return cnt;
        const uint32_t lane = lane_id();
        const uint32_t t = i / (uint32_t)kSortTile;
        uint32_t w[16];
        tile_words(t, w);
        const uint32_t p0 = t * (uint32_t)kSortTile + lane * 64u;
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t m = byte_eq_mask(w[j], pat);
            const uint32_t pj = p0 + (uint32_t)j * 4u;   // byte b of word j: position pj + b
            if (pj + 4u <= i) c += (uint32_t)__popc(m);
            else if (pj < i) c += (uint32_t)__popc(m & ((1u << (8u * (i - pj))) - 1u));
        }
        return pre(t) + wave_sum(c);
    }

    // first arrival index with ts > X (the batch clock non-decreasing), n if none
    __device__ __forceinline__ uint32_t first_after(uint64_t X) const {
        const uint32_t lane = lane_id();
        uint32_t lo = 0, hi = n;   // ts <= X before lo, ts > X from hi on
        while (hi - lo > 64u) {
            const uint32_t step = (hi - lo + 63u) / 64u;
            const uint32_t q = lo + lane * step;
            const bool valid = q < hi;
            const uint64_t m = __ballot(valid && ts[q] > X);
            if (m) {
                const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1u;
                hi = lo + f * step;
                if (f) lo = lo + (f - 1u) * step + 1u;
            } else {
                const uint64_t vm = __ballot(valid);
                lo = lo + (63u - (uint32_t)__clzll((long long)vm)) * step + 1u;
            }
        }
        const uint32_t q = lo + lane;
        const uint64_t m = __ballot(q < hi && ts[q] > X);
        return m ? lo + (uint32_t)__ffsll((unsigned long long)m) - 1u : hi;
    }

    // The arrival index of h's rank R0 + lane in every lane (n for ranks >= cnt): the tile of
    // R0 by a search of the prefix row, then h's packets of that tile — and of the next ones
    // while lanes are left — ranked by scans of their verdict bytes. s_idx: 64 words of LDS
    // of this wave.
    __device__ __forceinline__ uint32_t block(uint32_t R0, uint32_t *s_idx) const {
        const uint32_t lane = lane_id();
        s_idx[lane] = n;
        wave_lds_order();
        if (R0 < cnt) {
            uint32_t t = tile_of(R0), k0 = R0 - pre(t), filled = 0;
            const uint32_t want = min(64u, cnt - R0);
            while (filled < want && t < ntiles) {
                uint32_t w[16];
                tile_words(t, w);
                uint32_t c = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) c += (uint32_t)__popc(byte_eq_mask(w[j], pat));
                const uint32_t incl = wave_incl_sum(c), excl = incl - c;
                const uint32_t tot = __shfl(incl, 63);
                const uint32_t room = want - filled;
                if (incl > k0 && excl < k0 + room) {   // some of this lane's packets are wanted
                    uint32_t r = excl;
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        uint32_t mm = byte_eq_mask(w[j], pat);
                        while (mm) {
                            const uint32_t bit = (uint32_t)__ffs((int)mm) - 1u;
                            if (r >= k0 && r < k0 + room)
                                s_idx[filled + r - k0] = t * (uint32_t)kSortTile + lane * 64u + (uint32_t)j * 4u + bit / 8u;
                            ++r;
                            mm &= mm - 1u;
                        }
                    }
                }
                filled += tot > k0 ? min(tot - k0, room) : 0u;
                k0 = 0;
                ++t;
                wave_lds_order();
            }
            if (filled < want) fail();   // (the tiles ran out before the ranks did)
        }
        wave_lds_order();
        return s_idx[lane];
    }

    __device__ __forceinline__ uint64_t t(uint32_t r) const { return ts[select(r)]; }
    __device__ __forceinline__ uint32_t l(uint32_t r) const { return len[select(r)]; }

    // sum of h's frame lengths at arrival positions [a, b] of tile t
    __device__ __forceinline__ uint64_t tile_len_sum(uint32_t t, uint32_t a, uint32_t b) const {
        const uint32_t lane = lane_id();
        uint64_t s = 0;
        const uint32_t p0 = t * (uint32_t)kSortTile;
#pragma unroll 4
        for (uint32_t j = 0; j < (uint32_t)kSortTile; j += 64u) {
            const uint32_t p = p0 + j + lane;
            if (p >= a && p <= b && p < n && tags[p] == (pat & 0xFFu)) s += len[p];
        }
        return wave_sum(s);
    }
};

// fsx_walk.h's accessors on the heavy view (found by argument-dependent lookup from
// walk_fixed_fast): ranks instead of sorted positions.
template <bool kWave>
__device__ __forceinline__ uint32_t search_gt(const HeavyView &sv, uint32_t lo, uint32_t hi, uint64_t X) {
    if (lo >= hi) return hi;
    const uint32_t r = sv.rank(sv.first_after(X));
    return r < lo ? lo : r > hi ? hi : r;
}

template <bool kWave>
__device__ __forceinline__ uint64_t sum_len(const HeavyView &sv, uint32_t lo, uint32_t hi) {
    if (lo >= hi) return 0;
    const uint32_t ia = sv.select(lo), ib = sv.select(hi - 1);
    const uint32_t ta = ia / (uint32_t)kSortTile, tb = ib / (uint32_t)kSortTile;
    if (ta == tb) return sv.tile_len_sum(ta, ia, ib);
    uint64_t s = sv.tile_len_sum(ta, ia, ~0u) + sv.tile_len_sum(tb, 0, ib);
    // the tiles in between from their sums, eight loads in flight per lane (a heavy source
    // spans up to every tile: one dependent load per 64 tiles made this the walker's long pole)
    uint64_t mid = 0;
    uint32_t t = ta + 1 + lane_id();
    for (; t + 7u * 64u < tb; t += 8u * 64u) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = sv.rec[t + (uint32_t)u * 64u].s1[sv.h];
#pragma unroll
        for (int u = 0; u < 8; ++u) mid += x[u];
    }
    for (; t < tb; t += 64u) mid += sv.rec[t].s1[sv.h];
    return s + wave_sum(mid);
}

// First rank q in [from, lim) where acc0 + the lengths of ranks from..q exceed B (else lim):
// a scan of h's packets in arrival order from select(from). k_hmode keeps the byte trigger
// out of reach (the batch takes the run path otherwise); this is its exact definition.
template <bool kWave>
__device__ __forceinline__ uint32_t bytes_trigger(const HeavyView &sv, uint32_t from, uint32_t lim, uint64_t acc0, uint64_t B) {
    if (from >= lim) return lim;
    const uint32_t lane = lane_id();
    uint64_t acc = acc0;
    uint32_t q = from;
    for (uint32_t p0 = sv.select(from); p0 < sv.n && q < lim; p0 += 64u) {
        const uint32_t p = p0 + lane;
        const bool mine = p < sv.n && sv.tags[p] == (sv.pat & 0xFFu);
        const uint64_t L = mine ? sv.len[p] : 0ull;
        const uint64_t bm = __ballot(mine);
        const uint64_t incl = wave_incl_sum(L);
        const uint32_t rk = q + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
        const uint64_t hit = __ballot(mine && rk < lim && acc + incl > B);
        if (hit) return q + (uint32_t)__popcll(bm & ((1ull << (__ffsll((unsigned long long)hit) - 1)) - 1ull));
        acc += __shfl(incl, 63);
        q += (uint32_t)__popcll(bm);
    }
    return lim;
}

// Verdict changes of heavy source h as its list {arrival index << 1 | DROP} (the
// MarkWriter<true, true> of the run path, positions = ranks).
struct HeavyMarkWriter {
    HeavyView hv;   // (by value: a pointer to it would put the view in scratch)
    uint32_t *list;
    uint8_t last = 0;
    uint32_t nl = 0, last_pos = 0;
    uint64_t npass = 0, ndrop = 0;
    __device__ __forceinline__ void count_run(uint32_t pos) {
        const uint64_t r = pos - last_pos;
        ndrop += last == XDP_DROP ? r : 0ull;
        npass += (last && last != XDP_DROP) ? r : 0ull;
    }
    __device__ __forceinline__ void emit(uint32_t pos, uint8_t v) {
        if (v != last) {
            count_run(pos);
            const uint32_t e = hv.select(pos) << 1 | (v == XDP_DROP ? 1u : 0u);
            if (lane_id() == 0) list[nl] = e;
            ++nl;
            last_pos = pos;
            last = v;
        }
    }
    __device__ __forceinline__ void finish(uint32_t b) {
        count_run(b);
        last_pos = b;
    }
};

// Sliding window: every timestamp so far non-decreasing in arrival order.
__device__ __forceinline__ bool sw_mono(const BatchState *bs, const TableState *ts) {
    return !bs->nonmono && !ts->ever_nonmono && ~bs->inv_min_ts >= ts->last_max_ts;
}

// The sliding window's epoch-style walkers hold when clocks are monotone, no byte trigger can
// come before the count trigger and till / window ends do not overflow u64.
__device__ __forceinline__ bool sw_fast(const BatchState *bs, const TableState *tst, const Limits &lim) {
    const uint32_t maxL = bs->max_len > tst->max_len_seen ? bs->max_len : tst->max_len_seen;
    const uint64_t lim_ts = lim.window > lim.block ? lim.window : lim.block;
    return sw_mono(bs, tst) && lim.pps * (uint64_t)maxL <= lim.bps && bs->max_ts <= ~0ull - lim_ts;
}

}  // namespace fsx
