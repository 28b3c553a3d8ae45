// fsx_limiters.hip — the build-defined limiters of DESIGN.md §4 on gfx950.
//
// The reference only names a token bucket and a sliding window (README.md:155-162,
// placeholder text copied from the fixed-window paragraph); their semantics are
// specified in DESIGN.md §4 and restated sequentially in oracle/fsx_oracle.c, which
// these kernels match bit-exactly (parity unpinned: no reference code exists).
// Both run after the shared front half of the pipeline (parse -> radix sort by source
// -> segment heads -> table lookup/insert) and leave one verdict mark per sorted
// position for the shared fill/scatter kernels.
//
// Token bucket. Per counted packet with refill s = sat(dt * rate):
//     y = min(C, x + s);  PASS iff y >= cost;  x' = max(0, y - cost)
// so x' = clamp(x + (s - cost), 0, C - cost): a clamp-add map x -> min(hi, max(lo, x+d)).
// Clamp-add maps are closed under composition, so the whole batch is ONE scan over the
// sorted positions (no per-source loop, heavy sources cost the same per packet as the
// tail): the first counted packet of every source is a constant map (its state comes
// from the table), which cuts the scan into independent segments by itself.
//   k_tb_seg      one thread per source: blacklist prefix (static rules still apply,
//                 src/fsx_kern.c:159-216 semantics), state after the first counted packet
//   k_tb_scan     per 4096-position tile, one pass: the tile's composed map, the state
//                 entering it by a decoupled look-back over the tiles before it (tiles in
//                 ticket order), then the replay from that state — verdict marks, the final
//                 {tokens, last} of every source ending in the tile
//   (FSX_TB_TWO_PASS=1, A/B: k_tb_tiles<0> maps per tile, k_tb_carry one block for the
//   entering states, k_tb_tiles<1> the replay — the timestamps read twice)
//
// Sliding window. Per counted packet: expire the source's log from the
// oldest entry while now - t_oldest >= W, append, count = |log|, bytes = sum of lengths;
// count > P or bytes > B -> blacklist until now + BLK, clear the log, DROP. The log of
// a source is a contiguous range of the virtual sequence "carried history, then the
// source's sorted positions from its first counted one", so a walker only moves two
// indices. With monotone clocks (and no byte trigger possible before the count one)
// packet q triggers iff t_q - t_{q-P} < W inside its phase: a wave tests 64 positions
// per step, then jumps over the blacklisted run with a search.
//   k_walk_sw / k_walk_sw_long  short segments one thread (exact), long ones one wave
//   k_sw_hist_count/scan/write  rebuild the carried logs, packed per source, in the
//                               other history buffer; with monotone clocks entries at
//                               least W behind the newest timestamp are dropped (they
//                               would be expired by any later packet)
//   k_sw_finish                 flip the buffers, clock facts for the next batch
#include <hip/hip_runtime.h>

#include "fsx_dev_common.h"
#include "fsx_internal.h"
#include "fsx_seg.h"
#include "fsx_heavy_view.h"

namespace fsx {

// ------------------------------------------------------------------ token bucket
constexpr uint64_t kTbCost = 1000000000ull;  // one token in nano-tokens
constexpr int64_t kTbSat = 1ll << 61;        // |d| saturation; capacity <= 2^61 (fsx_open)

// x -> min(hi, max(lo, x + d)) on the state domain [0, C - cost].
struct CMap {
    int64_t lo, hi, d;
};

__device__ __forceinline__ int64_t clamp64(int64_t v, int64_t a, int64_t b) {
    return v < a ? a : (v > b ? b : v);
}
// outer o inner. With lo, hi in [0, 2^61] and d in [-2^61, 2^61] nothing overflows; a
// saturated d decides the result alone on the domain, so saturation is exact.
__device__ __forceinline__ CMap cm_compose(const CMap &outer, const CMap &inner) {
    CMap r;
    r.d = clamp64(inner.d + outer.d, -kTbSat, kTbSat);
    r.lo = clamp64(inner.lo + outer.d, outer.lo, outer.hi);
    r.hi = clamp64(inner.hi + outer.d, outer.lo, outer.hi);
    return r;
}
__device__ __forceinline__ int64_t cm_apply(const CMap &f, int64_t x) { return clamp64(x + f.d, f.lo, f.hi); }

__device__ __forceinline__ CMap cm_shfl_up(const CMap &m, int o) {
    return CMap{__shfl_up(m.lo, o), __shfl_up(m.hi, o), __shfl_up(m.d, o)};
}

// Refill of a gap dt (u64 wraparound of now - last, as the oracle), saturated at 2^61.
// dt_sat = 2^61 / rate, hoisted (a 64-bit division is ~100 instructions on CDNA).
__device__ __forceinline__ uint64_t tb_dt_sat(uint64_t rate) { return rate ? (uint64_t)kTbSat / rate : 0; }
__device__ __forceinline__ int64_t tb_refill(uint64_t dt, uint64_t rate, uint64_t dt_sat) {
    if (rate == 0) return 0;
    if (dt > dt_sat) return kTbSat;
    return (int64_t)(dt * rate);
}

// One thread per source. seg_j[g] = first counted sorted position (end of the
// blacklisted prefix); seg_x[g] = tokens after it | PASS bit 63.
template <class SV>
__device__ __forceinline__ void tb_seg_body(const SV &sv, BatchState *bs, const uint32_t *seg_start,
                                            const uint32_t *seg_slot, Slot *table, const Limits &lim,
                                            uint32_t *seg_j, uint64_t *seg_x, uint32_t light_only) {
    // (light_only 2 on the unsorted path: the heavy segments k_heads_heavy appended hold no
    // sorted packets — launch_tb_heavy decides them)
    const uint32_t nseg = light_only == 2 && bs->hfast ? bs->nseg_light : bs->nseg;
    const bool mono = !bs->nonmono;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nseg; g += gridDim.x * 256u) {
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        Slot &sl = table[seg_slot[g]];
        const uint32_t flags = sl.flags & kFlagBits;   // (drops the born stamp)
        uint32_t j = a;
        if ((flags & SLOT_HAS_BL) && sl.till > 0) {   // src/fsx_kern.c:189
            const uint64_t till = sl.till;
            if (mono) j = gallop_gt(sv, a, b, till);
            else while (j < b && !(sv.t(j) > till)) ++j;
        }
        // blacklist entry deleted at j (src/fsx_kern.c:193-204); a source with a counted
        // packet gets its bucket state here (k_tb_tiles<1> then only stores, no read)
        uint32_t nf = j < b && (flags & SLOT_HAS_BL) && sl.till > 0 ? flags & ~SLOT_HAS_BL : flags;
        if (j < b) nf |= SLOT_HAS_TB;
        sl.flags = nf;
        seg_j[g] = j;
        if (j >= b) continue;
        const uint64_t C = lim.tb_cap;
        uint64_t y = C;                               // a new source starts full
        if (flags & SLOT_HAS_TB) {
            const uint64_t dt = sv.t(j) - sl.tt;
            uint64_t add;
            if (lim.tb_rate && dt > ~0ull / lim.tb_rate) add = ~0ull;
            else add = dt * lim.tb_rate;
            y = sl.aux + add;
            if (y < sl.aux) y = ~0ull;
            if (y > C) y = C;
        }
        const bool pass = y >= kTbCost;
        seg_x[g] = (pass ? y - kTbCost : 0ull) | (pass ? (1ull << 63) : 0ull);
    }
}

__global__ __launch_bounds__(256) void k_tb_seg(const uint64_t *__restrict__ S, BatchState *bs,
                                                const uint32_t *__restrict__ seg_start,
                                                const uint32_t *__restrict__ seg_slot,
                                                const uint64_t *__restrict__ ts,
                                                const uint32_t *__restrict__ len,
                                                const uint64_t *__restrict__ pay, Slot *table,
                                                Limits lim, uint32_t *__restrict__ seg_j,
                                                uint64_t *__restrict__ seg_x, uint32_t light_only) {
    if (bs->err) return;
    if (bs->pay_ok) tb_seg_body(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts}, bs, seg_start, seg_slot, table, lim, seg_j, seg_x, light_only);
    else tb_seg_body(SegView<false>{S, ts, len, pay, 0}, bs, seg_start, seg_slot, table, lim, seg_j, seg_x, light_only);
}

// Position kinds inside a tile.
enum : uint32_t { TB_BLOCKED = 0, TB_FIRST = 1, TB_NEXT = 2, TB_NONE = 3 };

// One-pass look-back state (k_tb_scan): three 64-bit words per tile, each its own flag (the
// words are memset to 0 per batch; relaxed agent-scope atomics, no fence: a word is valid
// alone, so no ordering between them is needed) —
//   A: 1 << 62 | lo of the tile's composed map, or 2 << 62 | x the state leaving the tile
//   B: 1 << 63 | hi,   C: 1 << 63 | (d + 2^61)      (lo, hi, x in [0, 2^61], |d| <= 2^61)
// Wave 0 of the tile looks back 64 tiles at a time: lane k reads tile j - k; the nearest
// inclusive state ends the walk, and the maps of the tiles after it are composed by an
// ordered tree over the lanes.
__device__ __forceinline__ CMap cm_shfl_down(const CMap &m, int o) {
    return CMap{__shfl_down(m.lo, o), __shfl_down(m.hi, o), __shfl_down(m.d, o)};
}

__device__ __forceinline__ void tb_put(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long tb_get(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int64_t tb_lookback(unsigned long long *status, uint32_t t, const CMap &agg,
                                               int64_t hi, uint32_t *err) {
    const uint32_t lane = lane_id();
    constexpr unsigned long long kM62 = (1ull << 62) - 1ull, kM63 = (1ull << 63) - 1ull;
    unsigned long long *my = status + 3ull * t;
    if (t == 0) {   // (tile 0 starts with a source head: the state entering it is irrelevant, 0)
        if (lane == 0) tb_put(my, (2ull << 62) | (unsigned long long)cm_apply(agg, 0));
        return 0;
    }
    if (lane == 0) {
        tb_put(my + 1, (1ull << 63) | (unsigned long long)agg.hi);
        tb_put(my + 2, (1ull << 63) | (unsigned long long)(agg.d + kTbSat));
        tb_put(my, (1ull << 62) | (unsigned long long)agg.lo);
    }
    const CMap id{0, hi, 0};
    CMap m = id;   // the maps of the tiles walked so far, composed (later tiles outer)
    int64_t x = 0;
    uint32_t spins = 0;
    for (int64_t j = (int64_t)t - 1;;) {
        const int64_t idx = j - (int64_t)lane;
        unsigned long long wa = 2ull << 62, wb = 0, wc = 0;   // (before tile 0: state 0)
        if (idx >= 0) {
            const unsigned long long *q = status + 3ull * (uint64_t)idx;
            wa = tb_get(q);
            if ((wa >> 62) == 1) {
                wb = tb_get(q + 1);
                wc = tb_get(q + 2);
                if (!(wb >> 63) || !(wc >> 63)) wa = 0;   // (its other words not seen yet)
            }
        }
        const uint32_t f = (uint32_t)(wa >> 62);
        const uint64_t b2 = __ballot(f == 2), b0 = __ballot(f == 0);
        const uint32_t l2 = b2 ? (uint32_t)__ffsll((unsigned long long)b2) - 1u : 64u;
        const uint32_t l0 = b0 ? (uint32_t)__ffsll((unsigned long long)b0) - 1u : 64u;
        if (l0 < l2) {   // a tile before the nearest state has published nothing yet: wait
            if (++spins > (1u << 22)) {   // (never expected: lower tickets are running)
                if (lane == 0 && err) atomicOr(err, ERR_SORT_HANG);   // the batch fails (-EIO)
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        CMap a = id;   // lanes before the nearest state: their maps
        if (lane < l2) a = CMap{(int64_t)(wa & kM62), (int64_t)(wb & kM63), (int64_t)(wc & kM63) - kTbSat};
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {   // lane 0: A_j o A_(j-1) o ... (ordered tree)
            const CMap y = cm_shfl_down(a, o);
            if ((lane & (2u * (uint32_t)o - 1u)) == 0 && lane + (uint32_t)o < 64u) a = cm_compose(a, y);
        }
        m = cm_compose(m, CMap{__shfl(a.lo, 0), __shfl(a.hi, 0), __shfl(a.d, 0)});
        if (l2 < 64u) {
            x = (int64_t)__shfl((long long)(wa & kM62), (int)l2);
            break;
        }
        j -= 64;
    }
    const int64_t xin = cm_apply(m, x);
    if (lane == 0) tb_put(my, (2ull << 62) | (unsigned long long)cm_apply(agg, xin));
    return xin;
}

// One 4096-position tile, 16 consecutive positions per thread. kMode 0: the tile's composed
// map to tile_map[t]; 1: replay from tile_x[t], marks and final source states; 2 (k_tb_scan):
// the map, the entering state by look-back (status), then the replay.
template <int kMode, class SV>
__device__ __forceinline__ void tb_tile(const SV &sv, uint32_t t, uint32_t M,
                                        const uint8_t *__restrict__ headf,
                                        const uint32_t *__restrict__ tile_off,
                                        const uint32_t *__restrict__ seg_j,
                                        const uint64_t *__restrict__ seg_x,
                                        const uint32_t *__restrict__ seg_slot, Slot *table,
                                        const Limits &lim, CMap *tile_map, const int64_t *tile_x,
                                        uint8_t *__restrict__ marks, CMap *s_w, uint32_t *s_tmp,
                                        unsigned long long *status = nullptr, int64_t *s_x = nullptr,
                                        uint32_t *err = nullptr) {
    constexpr bool kApply = kMode != 0;
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t p0 = t * kTile + tid * 16u;
    const int64_t hi = lim.tb_cap >= kTbCost ? (int64_t)(lim.tb_cap - kTbCost) : 0;
    const bool degen = lim.tb_cap < kTbCost;    // C < cost: every counted packet drops
    const uint64_t dt_sat = tb_dt_sat(lim.tb_rate);
    // head bits of positions p0 .. p0+16 (a position >= M ends the last segment)
    uint32_t hf = 0;
    if (p0 + 17 <= M) {
        const uint4 v = *reinterpret_cast<const uint4 *>(headf + p0);
        const uint32_t f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) hf |= ((f[k >> 2] >> (8 * (k & 3))) & 1u) << k;
        hf |= (uint32_t)(headf[p0 + 16] & 1u) << 16;
    } else {
        for (uint32_t k = 0; k <= 16; ++k) {
            const uint32_t p = p0 + k;
            if (p >= M || (headf[p] & 1u)) hf |= 1u << k;
        }
    }
    const uint32_t nh = p0 < M ? (uint32_t)__popc(hf & 0xFFFFu) : 0u;
    const uint32_t hb = tile_off[t] + block256_excl(nh, s_tmp, nullptr);
    // per-position kinds, and the thread's composed map folded on the fly (the apply
    // pass recomputes the per-position deltas from the 16 timestamps). Blocked / absent
    // positions are identity maps and skipped; a source's first counted packet is a
    // constant map.
    uint32_t kind = 0;  // 2 bits per position
    const uint64_t tprev0 = (p0 > 0 && p0 < M) ? sv.t(p0 - 1) : 0ull;
    auto delta = [&](uint64_t tp, uint64_t tprev) -> int64_t {
        return tb_refill(tp - tprev, lim.tb_rate, dt_sat) - (int64_t)kTbCost;
    };
    uint64_t tt[16];
    if (p0 + 16 <= M) sv.t16(p0, tt);
    else {
#pragma unroll
        for (int k = 0; k < 16; ++k) tt[k] = p0 + k < M ? sv.t(p0 + k) : 0ull;
    }
    CMap T{0, hi, 0};
    {
        uint64_t tprev = tprev0;
        int32_t cg = (int32_t)hb - 1;
        uint32_t cj = 0;
        uint64_t cx = 0;
        if (p0 < M && !(hf & 1u)) { cj = seg_j[cg]; cx = seg_x[cg]; }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t p = p0 + (uint32_t)k;
            uint32_t kd = TB_NONE;
            if (p < M) {
                if ((hf >> k) & 1u) { ++cg; cj = seg_j[cg]; cx = seg_x[cg]; }
                const uint64_t tp = tt[k];
                if (p < cj) {
                    kd = TB_BLOCKED;
                } else if (p == cj) {
                    kd = TB_FIRST;
                    const int64_t x = (int64_t)(cx & ~(1ull << 63));
                    T = CMap{x, x, 0};
                } else {
                    kd = TB_NEXT;
                    T = cm_compose(degen ? CMap{0, 0, 0} : CMap{0, hi, delta(tp, tprev)}, T);
                }
                tprev = tp;
            }
            kind |= kd << (2 * k);
        }
    }
    // block scan of the thread maps (in position order)
    CMap incl = T;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const CMap y = cm_shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl = cm_compose(incl, y);
    }
    CMap excl = cm_shfl_up(incl, 1);
    if (lane == 0) excl = CMap{0, hi, 0};
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    CMap pre{0, hi, 0};
    for (uint32_t k = 0; k < w; ++k) pre = cm_compose(s_w[k], pre);
    if constexpr (!kApply) {
        if (tid == 0) {
            CMap a = s_w[0];
            for (int k = 1; k < 4; ++k) a = cm_compose(s_w[k], a);
            tile_map[t] = a;
        }
    } else {
        int64_t xt;
        if constexpr (kMode == 2) {
            if (w == 0) {   // (wave 0 looks back)
                CMap a = s_w[0];
                for (int k = 1; k < 4; ++k) a = cm_compose(s_w[k], a);
                const int64_t xin = tb_lookback(status, t, a, hi, err);
                if (lane == 0) *s_x = xin;
            }
            __syncthreads();
            xt = *s_x;
        } else {
            xt = tile_x[t];
        }
        excl = cm_compose(excl, pre);
        int64_t x = cm_apply(excl, xt);
        uint32_t out[4] = {0, 0, 0, 0};
        int32_t g = (int32_t)hb - 1;
        uint64_t tprev = tprev0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t p = p0 + (uint32_t)k;
            const uint32_t kd = (kind >> (2 * k)) & 3u;
            if (kd == TB_NONE) continue;
            if ((hf >> k) & 1u) ++g;
            const uint64_t tp = tt[k];
            uint8_t v;
            if (kd == TB_BLOCKED) {
                v = XDP_DROP;
            } else if (kd == TB_FIRST) {
                const uint64_t cx = seg_x[g];
                v = (cx >> 63) ? XDP_PASS : XDP_DROP;
                x = (int64_t)(cx & ~(1ull << 63));
            } else if (degen) {
                v = XDP_DROP;
                x = 0;
            } else {
                const int64_t d = delta(tp, tprev);
                v = x + d >= 0 ? XDP_PASS : XDP_DROP;
                x = clamp64(x + d, 0, hi);
            }
            tprev = tp;
            out[k >> 2] |= (uint32_t)v << (8 * (k & 3));
            // last position of its source: the final {tokens, last} (counted packets only)
            if (kd != TB_BLOCKED && ((hf >> (k + 1)) & 1u)) {
                Slot &sl = table[seg_slot[g]];   // (SLOT_HAS_TB: set by k_tb_seg)
                sl.aux = (uint64_t)x;
                sl.tt = tp;
            }
        }
        if (p0 + 16 <= M) {
            *reinterpret_cast<uint4 *>(marks + p0) = make_uint4(out[0], out[1], out[2], out[3]);
        } else {
            for (uint32_t k = 0; p0 + k < M; ++k) marks[p0 + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
        }
    }
}

template <int kMode>
__global__ __launch_bounds__(256) void k_tb_tiles(const uint64_t *__restrict__ S, BatchState *bs,
                                                  const uint64_t *__restrict__ ts,
                                                  const uint32_t *__restrict__ len,
                                                  const uint64_t *__restrict__ pay,
                                                  const uint8_t *__restrict__ headf,
                                                  const uint32_t *__restrict__ tile_off,
                                                  const uint32_t *__restrict__ seg_j,
                                                  const uint64_t *__restrict__ seg_x,
                                                  const uint32_t *__restrict__ seg_slot, Slot *table,
                                                  Limits lim, CMap *tile_map, const int64_t *tile_x,
                                                  uint8_t *__restrict__ marks, uint32_t light_only) {
    __shared__ CMap s_w[4];
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const bool pay_ok = bs->pay_ok != 0;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (pay_ok)
            tb_tile<kMode>(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts}, t, M, headf, tile_off, seg_j,
                           seg_x, seg_slot, table, lim, tile_map, tile_x, marks, s_w, s_tmp);
        else
            tb_tile<kMode>(SegView<false>{S, ts, len, pay, 0}, t, M, headf, tile_off, seg_j, seg_x,
                           seg_slot, table, lim, tile_map, tile_x, marks, s_w, s_tmp);
        __syncthreads();
    }
}

// One pass (see the file header): a block per tile, tiles in ticket order.
#ifndef FSX_TB_SCAN_MINB
#define FSX_TB_SCAN_MINB 1   // waves/SIMD bound (A/B: scripts/build_variant.sh)
#endif
__global__ __launch_bounds__(256, FSX_TB_SCAN_MINB) void k_tb_scan(const uint64_t *__restrict__ S, BatchState *bs,
                                                 const uint64_t *__restrict__ ts,
                                                 const uint32_t *__restrict__ len,
                                                 const uint64_t *__restrict__ pay,
                                                 const uint8_t *__restrict__ headf,
                                                 const uint32_t *__restrict__ tile_off,
                                                 const uint32_t *__restrict__ seg_j,
                                                 const uint64_t *__restrict__ seg_x,
                                                 const uint32_t *__restrict__ seg_slot, Slot *table,
                                                 Limits lim, CMap *tile_map, unsigned long long *status,
                                                 uint32_t *ticket, uint8_t *__restrict__ marks, uint32_t light_only) {
    __shared__ CMap s_w[4];
    __shared__ uint32_t s_tmp[4];
    __shared__ uint32_t s_t;
    __shared__ int64_t s_x;
    if (bs->err) return;
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t t = s_t;
    if (t >= ntiles) return;
    if (bs->pay_ok)
        tb_tile<2>(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts}, t, M, headf, tile_off, seg_j, seg_x, seg_slot,
                   table, lim, tile_map, nullptr, marks, s_w, s_tmp, status, &s_x, &bs->err);
    else
        tb_tile<2>(SegView<false>{S, ts, len, pay, 0}, t, M, headf, tile_off, seg_j, seg_x, seg_slot, table, lim,
                   tile_map, nullptr, marks, s_w, s_tmp, status, &s_x, &bs->err);
}

// One block: the state entering every tile (tile 0 starts with a source head, so its
// entering state is irrelevant and taken as 0).
__global__ __launch_bounds__(1024) void k_tb_carry(BatchState *bs, const CMap *__restrict__ tile_map,
                                                   int64_t *__restrict__ tile_x, Limits lim, uint32_t light_only) {
    __shared__ CMap s_w[16];
    if (bs->err) return;
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const int64_t hi = lim.tb_cap >= kTbCost ? (int64_t)(lim.tb_cap - kTbCost) : 0;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t per = (ntiles + 1023) / 1024;
    const uint32_t t0 = min(ntiles, threadIdx.x * per), t1 = min(ntiles, t0 + per);
    CMap run{0, hi, 0};
    for (uint32_t t = t0; t < t1; ++t) run = cm_compose(tile_map[t], run);
    CMap incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const CMap y = cm_shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl = cm_compose(incl, y);
    }
    CMap excl = cm_shfl_up(incl, 1);
    if (lane == 0) excl = CMap{0, hi, 0};
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    CMap pre{0, hi, 0};
    for (uint32_t k = 0; k < w; ++k) pre = cm_compose(s_w[k], pre);
    int64_t x = cm_apply(cm_compose(excl, pre), 0);
    for (uint32_t t = t0; t < t1; ++t) {
        tile_x[t] = x;
        x = cm_apply(tile_map[t], x);
    }
}

hipError_t launch_token_bucket(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                               const Scratch &sc, Slot *table, const Limits &lim, uint32_t n,
                               hipStream_t st, const Marker &mark, uint32_t light_only) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t gridSeg = std::min<uint32_t>(2048, std::max<uint32_t>(1, (n + 255) / 256));
    const uint32_t gridTiles = std::min<uint32_t>(4096, std::max<uint32_t>(1, (n + kTile - 1) / kTile));
    uint32_t *seg_j = sc.seg_order;
    uint64_t *seg_x = sc.packed[1];
    CMap *tile_map = reinterpret_cast<CMap *>(sc.lim_tiles);
    int64_t *tile_x = reinterpret_cast<int64_t *>(sc.lim_tiles + 3 * sc.lim_tiles_n);
    k_tb_seg<<<gridSeg, 256, 0, st>>>(S, bs, sc.seg_start, sc.seg_slot, ts, len, sc.pay[0], table, lim,
                                      seg_j, seg_x, light_only);
    mark("k_tb_seg");
    static const bool two_pass = getenv("FSX_TB_TWO_PASS") != nullptr;
    if (!two_pass) {
        // (three status words per tile over the map and carry region; the ticket in its last
        // word, past every tile: 3 * tiles < 4 * lim_tiles_n - 1)
        unsigned long long *status = reinterpret_cast<unsigned long long *>(sc.lim_tiles);
        uint32_t *ticket = reinterpret_cast<uint32_t *>(sc.lim_tiles + 4 * sc.lim_tiles_n - 1);
        hipError_t e = hipMemsetAsync(sc.lim_tiles, 0, sc.lim_tiles_n * 4 * 8, st);
        if (e != hipSuccess) return e;
        const uint32_t grid = std::max<uint32_t>(1, (n + kTile - 1) / kTile);   // (>= the valid tiles)
        // Unused dynamic LDS caps the blocks in flight at three per CU (four fit the VGPRs): a
        // tile's look-back walks back over the tiles still in flight, and fewer of them beside
        // the front measured 3.85-3.96 vs 3.92-3.93 ms per step (two per CU 4.02-4.05, one
        // 4.52; profiles/r06/ab_r06ts*). FSX_TB_SCAN_LDS=<bytes> overrides (0: uncapped).
        static const uint32_t scan_lds = getenv("FSX_TB_SCAN_LDS") ? (uint32_t)atoi(getenv("FSX_TB_SCAN_LDS")) : 42000u;
        k_tb_scan<<<grid, 256, scan_lds, st>>>(S, bs, ts, len, sc.pay[0], sc.headf, sc.tile_aux, seg_j, seg_x,
                                        sc.seg_slot, table, lim, tile_map, status, ticket, sc.marks, light_only);
        mark("k_tb_scan");
        return hipGetLastError();
    }
    k_tb_tiles<0><<<gridTiles, 256, 0, st>>>(S, bs, ts, len, sc.pay[0], sc.headf, sc.tile_aux, seg_j,
                                             seg_x, sc.seg_slot, table, lim, tile_map, tile_x,
                                             sc.marks, light_only);
    mark("k_tb_tiles_reduce");
    k_tb_carry<<<1, 1024, 0, st>>>(bs, tile_map, tile_x, lim, light_only);
    k_tb_tiles<1><<<gridTiles, 256, 0, st>>>(S, bs, ts, len, sc.pay[0], sc.headf, sc.tile_aux, seg_j,
                                             seg_x, sc.seg_slot, table, lim, tile_map, tile_x,
                                             sc.marks, light_only);
    mark("k_tb_tiles_apply");
    return hipGetLastError();
}

// ------------------------------------------------------------------ token bucket, heavy sources unsorted
// (DESIGN.md §4.2 "Heavy sources outside the sort") As for the fixed
// window, k_parse tags a heavy source's packets 0x80 | h and writes no sort word for them, so
// the sort carries the light entries only. A heavy source's packets are decided in arrival
// order by clamp-add maps (its refill between consecutive packets is a map, and maps compose):
//   k_tb_heavy_tiles<0>  per sort tile: for every heavy source, the map of its packets of the
//                        tile after the first one, composed in arrival order (the tile's heavy
//                        packets listed by source in LDS, a segmented scan over the lists)
//   k_tb_heavy_scan      one wave per heavy source: the tiles in order, 64 at a time — the
//                        map of a tile's first packet from the previous tile's last timestamp
//                        (HeavyTileRec t1), an ordered scan of the tile maps from the carried
//                        {tokens, last} (a new source starts full) — the state after each
//                        tile's first packet with its verdict, and the source's final state
//   k_tb_heavy_tiles<1>  per sort tile again: the replay from those states, every heavy
//                        packet's verdict byte written over its tag, PASS / DROP counted
// A heavy source with a live blacklist entry (a user rule: the token bucket inserts none)
// sends the batch to the run path (k_hmode_state), as do the clock facts k_hmode checks.
constexpr unsigned long long kTbNone = ~0ull;

__device__ __forceinline__ CMap cm_shfl(const CMap &m, uint32_t src) {
    return CMap{__shfl(m.lo, (int)src), __shfl(m.hi, (int)src), __shfl(m.d, (int)src)};
}

struct TbHeavyOut {
    CMap *map;      // [tile][kHeavyMax]: h's packets of the tile after its first, composed
    uint64_t *x1;   // [tile][kHeavyMax]: the state after the tile's first packet of h | PASS << 63
};

// Per sort tile (one block): the tile's heavy packets listed by source in arrival order (a
// stable counting sort in LDS: per-wave counts, their offsets, then each 64-packet row's
// same-source lanes placed in order), the timestamps staged in LDS, and a segmented scan of
// the packets' maps over the lists (a segment per source, 16 entries per thread) — kApply
// false: the maps of a source's packets after its first composed (-> o.map); true: the replay
// from the state after the tile's first packet (o.x1), every packet's verdict byte written over
// its tag, PASS / DROP counted.
// (Measured, maps + replay per 64M packets, DESIGN.md §4.2: per-row pointer jumping over
// same-source lanes 0.6-0.75 + 1.25-1.43 ms; one thread walking each list 2.6-3.6 + 1.9 ms;
// one wave per source scanning its list 1.75-3.0 + 1.6-1.9 ms — 2M (tile, source) pairs each a
// dependent scan; this segmented scan 1.0 (beside the light scan) + 0.57 ms.)
template <bool kApply>
__global__ __launch_bounds__(256) void k_tb_heavy_tiles(BatchState *bs, uint8_t *__restrict__ verdict,
                                                        const uint64_t *__restrict__ ts, uint32_t n,
                                                        const HeavySet *__restrict__ hs, Limits lim, TbHeavyOut o,
                                                        TableState *tstate) {
    __shared__ unsigned long long s_ts[kSortTile];
    __shared__ __attribute__((aligned(16))) uint16_t s_list[kSortTile];
    __shared__ uint32_t s_wc[4][kHeavyMax];   // per wave: its count of h, then its next place
    __shared__ uint32_t s_off[kHeavyMax + 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_hsrc[kSortTile];   // the source of each entry
    __shared__ unsigned long long s_x1[kHeavyMax];
    __shared__ CMap s_wagg[4];
    __shared__ uint32_t s_wflag[4];
    __shared__ unsigned long long s_cnt[2];
    if (bs->err || !bs->hfast) return;
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    if (blockIdx.x >= ntiles) return;
    const uint32_t t = xcd_swizzle(blockIdx.x, ntiles);
    const uint32_t t0 = t * kSortTile;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint32_t nh = hs->n;
    const int64_t H = (int64_t)(lim.tb_cap - kTbCost);   // (k_hmode: C >= cost on this path)
    const uint64_t dt_sat = tb_dt_sat(lim.tb_rate);
    for (uint32_t j = tid; j < 4 * kHeavyMax; j += 256) (&s_wc[0][0])[j] = 0;
    if (tid < 2) s_cnt[tid] = 0;
    __syncthreads();
    // 1. the chunk's rows: tags, timestamps to LDS, per-wave counts of every heavy source
    uint32_t Gr[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t p = w * 1024u + r * 64u + lane, i = t0 + p;
        const bool live = i < n;
        const uint32_t g = live ? verdict[i] : 0u;
        Gr[r] = g >= 0x80u && (g & 0x7Fu) < nh ? (g & 0x7Fu) : 0xFFu;
        s_ts[p] = ts[live ? i : 0u];
    }
    // (LDS atomics: a ballot match here would be kept alive by the compiler for step 3's —
    // 320 VGPRs)
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
        if (Gr[r] != 0xFFu) atomicAdd(&s_wc[w][Gr[r]], 1u);
    __syncthreads();
    // 2. the lists' offsets: sources in order, waves in order within a source (a scan over the
    //    128 sources by two waves; one thread's serial pass over them cost ~50 us per tile)
    static_assert(kHeavyMax == 128, "two waves scan the sources");
    __shared__ uint32_t s_w0;
    uint32_t c4[4] = {0, 0, 0, 0}, tot = 0;
    if (tid < kHeavyMax) {
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww) { c4[ww] = s_wc[ww][tid]; tot += c4[ww]; }
    }
    const uint32_t incl = tid < kHeavyMax ? wave_incl_sum(tot) : 0u;
    if (tid == 63) s_w0 = incl;
    __syncthreads();
    if (tid < kHeavyMax) {
        uint32_t a = incl - tot + (tid >= 64 ? s_w0 : 0u);
        s_off[tid] = a;
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww) { s_wc[ww][tid] = a; a += c4[ww]; }
        if (tid == kHeavyMax - 1) s_off[kHeavyMax] = a;
        if constexpr (kApply) {   // the tile's first packet of h: from k_tb_heavy_scan
            if (tid < nh && tot) s_x1[tid] = o.x1[(size_t)t * kHeavyMax + tid];
        }
    }
    __syncthreads();
    // 3. every heavy packet's place in its source's list (rows in order: stable)
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t g = Gr[r];
        const uint64_t act = __ballot(g != 0xFFu);
        if (!act) continue;
        const uint64_t peers = match_digit(g, act);
        if (g != 0xFFu) {
            const uint32_t base = s_wc[w][g];
            const uint32_t e = base + (uint32_t)__popcll(peers & lt_mask);
            s_list[e] = (uint16_t)(w * 1024u + r * 64u + lane);
            s_hsrc[e] = (uint8_t)g;
        }
        wave_lds_order();
        if (g != 0xFFu && (peers >> lane) == 1ull) s_wc[w][g] += (uint32_t)__popcll(peers);   // (the last lane)
        wave_lds_order();
    }
    __syncthreads();
    // 4. a segmented scan over the lists (one segment per source, its first entry the identity):
    //    each thread composes 16 consecutive entries, the 256 thread aggregates are scanned
    //    across the block, then each thread replays its entries from its exclusive prefix
    //    (kApply false: a source's last entry writes its map; true: every entry's verdict from
    //    the state after the source's first packet, o.x1, staged in LDS)
    const uint32_t total = s_off[kHeavyMax];
    const uint32_t j0 = tid * 16u;
    const CMap id{0, H, 0};
    uint32_t hp = 0xFFu;   // the source and timestamp of the entry before j0
    uint64_t Tp = 0;
    if (j0 > 0 && j0 - 1u < total) {
        hp = s_hsrc[j0 - 1u];
        Tp = s_ts[s_list[j0 - 1u]];
    }
    // the thread's 16 entries in registers (vector LDS reads; the timestamps gathered at once)
    uint32_t hw[4], pw[8];
    *reinterpret_cast<uint4 *>(hw) = *reinterpret_cast<const uint4 *>(&s_hsrc[j0]);
    *reinterpret_cast<uint4 *>(pw) = *reinterpret_cast<const uint4 *>(&s_list[j0]);
    *reinterpret_cast<uint4 *>(pw + 4) = *reinterpret_cast<const uint4 *>(&s_list[j0 + 8u]);
    const uint32_t hnext = j0 + 16u < total ? s_hsrc[j0 + 16u] : 0xFFu;
    const uint32_t nv = total > j0 ? min(total - j0, 16u) : 0u;
    uint64_t Tv[16];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t P = (pw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
        Tv[k] = s_ts[k < nv ? P : 0u];
    }
    int64_t dv[16];
    uint32_t firstm = 0;
    CMap agg = id;
    bool fl = false;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t h = (hw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t hq = k == 0 ? hp : (hw[(k - 1) >> 2] >> (8 * ((k - 1) & 3))) & 0xFFu;
        const uint64_t Tq = k == 0 ? Tp : Tv[k - 1];
        const bool first = h != hq;
        dv[k] = first ? 0 : tb_refill(Tv[k] - Tq, lim.tb_rate, dt_sat) - (int64_t)kTbCost;
        if (k < nv) {
            firstm |= (uint32_t)first << k;
            agg = first ? id : cm_compose(CMap{0, H, dv[k]}, agg);
            fl = fl || first;
        }
    }
    CMap inc = agg;
    bool ifl = fl;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const CMap y = cm_shfl_up(inc, k);
        const bool yf = __shfl_up((int)ifl, k) != 0;
        if (lane >= (uint32_t)k) {
            if (!ifl) inc = cm_compose(inc, y);
            ifl = ifl || yf;
        }
    }
    if (lane == 63) {
        s_wagg[w] = inc;
        s_wflag[w] = ifl;
    }
    __syncthreads();
    CMap run = id;   // the block's entries before the wave
    for (uint32_t ww = 0; ww < w; ++ww) run = s_wflag[ww] ? s_wagg[ww] : cm_compose(s_wagg[ww], run);
    {
        const CMap y = cm_shfl_up(inc, 1);
        const bool yf = __shfl_up((int)ifl, 1) != 0;
        if (lane > 0) run = yf ? y : cm_compose(y, run);
    }
    uint32_t np = 0, nd = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        if (k < nv) {
            const uint32_t h = (hw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            const bool first = (firstm >> k) & 1u;
            if constexpr (kApply) {
                const uint32_t P = (pw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                const uint64_t x1 = s_x1[h];
                const bool pass = first ? (x1 >> 63) != 0
                                        : cm_apply(run, (int64_t)(x1 & ~(1ull << 63))) + dv[k] >= 0;
                verdict[t0 + P] = pass ? XDP_PASS : XDP_DROP;
                np += pass;
                nd += !pass;
            }
            run = first ? id : cm_compose(CMap{0, H, dv[k]}, run);
            if constexpr (!kApply) {
                const uint32_t hn = k == 15 ? hnext : (k + 1 < nv ? (hw[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu : 0xFFu);
                if (hn != h) o.map[(size_t)t * kHeavyMax + h] = run;
            }
        }
    }
    if constexpr (kApply) {
        np = wave_sum(np);
        nd = wave_sum(nd);
        if (lane == 0) {
            if (np) atomicAdd(&s_cnt[0], (unsigned long long)np);
            if (nd) atomicAdd(&s_cnt[1], (unsigned long long)nd);
        }
        __syncthreads();
        if (tid == 0) {
            unsigned long long *sp = reinterpret_cast<unsigned long long *>(tstate->stats);
            if (s_cnt[0]) {
                atomicAdd(sp, s_cnt[0]);
                atomicAdd(reinterpret_cast<unsigned long long *>(&bs->allowed), s_cnt[0]);
            }
            if (s_cnt[1]) {
                atomicAdd(sp + 1, s_cnt[1]);
                atomicAdd(reinterpret_cast<unsigned long long *>(&bs->dropped), s_cnt[1]);
            }
        }
    }
}

// The scan over a heavy source's tiles, in groups of kTbGroup tiles so that 128 sources fill
// the device (one wave per source took 0.8-1.1 ms per 64M packets: 256 dependent steps of 64
// tiles): k_tb_heavy_gmap composes each group's tiles into one map, k_tb_heavy_scan applies
// the groups before its own to the carried state and replays the group's tiles. A tile's count
// comes from pass 0's prefix row, its first / last timestamp from the tile records, its map
// after the first packet from k_tb_heavy_tiles<0>; a group's first tile takes its previous
// timestamp from the tile of the source's packet before the group (a search of the prefix row).
constexpr uint32_t kTbGroup = 1024;   // tiles per group: 16 steps of 64

struct TbHeavyCtx {
    const uint32_t *row;    // pass-0 prefix row of bucket light_b + h (h's packets before tile t, + base)
    uint32_t base, end, ntiles, h;
    const HeavyTileRec *rec;
    TbHeavyOut o;
    int64_t H;
    uint64_t rate, dt_sat;
};

// h's last timestamp before tile t0 (its carried one when it has no packet before t0)
__device__ __forceinline__ uint64_t tb_prev_ts(const TbHeavyCtx &C, uint32_t t0, uint64_t carried_last) {
    const uint32_t before = C.row[t0] - C.base;
    if (before == 0) return carried_last;
    const uint32_t r = before - 1, lane = lane_id();
    uint32_t lo = 0, hi = t0;   // the largest tile t < t0 with pre(t) <= r (fsx_search.h)
    while (hi - lo > 1) {
        const uint32_t step = ary64_width(lo, hi);
        const uint32_t q = lo + lane * step;
        const uint64_t m = __ballot(q < hi && C.row[q] - C.base <= r);
        ary64_step(lo, hi, step, m);
    }
    return C.rec[lo].t1[C.h];
}

// Tiles [t0, t1) of h from the state x (previous timestamp `last`): kWrite stores every present
// tile's state after its first packet with that packet's verdict; returns the composed map of
// the range (and leaves `last` at the range's last timestamp).
template <bool kWrite>
__device__ CMap tb_heavy_range(const TbHeavyCtx &C, uint32_t t0, uint32_t t1, int64_t x, uint64_t &last) {
    const uint32_t lane = lane_id();
    const CMap id{0, C.H, 0};
    CMap acc = id;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t tb = t0; tb < t1; tb += 64) {
        const uint32_t t = tb + lane;
        uint32_t cnt = 0;
        if (t < t1) cnt = (t + 1 < C.ntiles ? C.row[t + 1] : C.end) - C.row[t];
        const bool present = cnt != 0;
        const uint64_t pm = __ballot(present);
        if (!pm) continue;
        uint64_t f = 0, l = 0;
        CMap M = id;
        if (present) {
            f = C.rec[t].t0[C.h];
            l = C.rec[t].t1[C.h];
            M = C.o.map[(size_t)t * kHeavyMax + C.h];
        }
        const uint64_t below = pm & lt;
        const uint32_t pl = below ? 63u - (uint32_t)__clzll((long long)below) : lane;
        const uint64_t lpl = __shfl(l, (int)pl);
        const uint64_t prev = below ? lpl : last;
        // the tile's first packet: a refill from the source's previous packet, or (a new
        // source) a full bucket
        const CMap F = prev != kTbNone ? CMap{0, C.H, tb_refill(f - prev, C.rate, C.dt_sat) - (int64_t)kTbCost}
                                       : CMap{C.H, C.H, 0};
        const CMap T = present ? cm_compose(M, F) : id;
        CMap incl = T;
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const CMap y = cm_shfl_up(incl, k);
            if (lane >= (uint32_t)k) incl = cm_compose(incl, y);
        }
        if constexpr (kWrite) {
            CMap excl = cm_shfl_up(incl, 1);
            if (lane == 0) excl = id;
            const int64_t xin = cm_apply(cm_compose(excl, acc), x);
            if (present) {
                const bool pass = prev == kTbNone || xin + F.d >= 0;
                const int64_t x1 = cm_apply(F, xin);
                C.o.x1[(size_t)t * kHeavyMax + C.h] = (uint64_t)x1 | (pass ? (1ull << 63) : 0ull);
            }
        }
        acc = cm_compose(cm_shfl(incl, 63), acc);
        last = __shfl(l, 63 - __clzll((long long)pm));
    }
    return acc;
}

__device__ __forceinline__ bool tb_heavy_ctx(const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0,
                                             const uint32_t *offs, uint32_t tcap, uint32_t n,
                                             const HeavyTileRec *rec, const TbHeavyOut &o, const Limits &lim,
                                             const HeavySet *hs, uint32_t h, TbHeavyCtx &C) {
    if (h >= hs->n) return false;
    const uint32_t lb = bs->light_b;
    const uint32_t c = cnt0[lb + h];
    if (c == 0) return false;
    C.row = offs + (size_t)(lb + h) * tcap;
    C.base = base0[lb + h];
    C.end = C.base + c;
    C.ntiles = (n + kSortTile - 1) / kSortTile;
    C.h = h;
    C.rec = rec;
    C.o = o;
    C.H = (int64_t)(lim.tb_cap - kTbCost);
    C.rate = lim.tb_rate;
    C.dt_sat = tb_dt_sat(lim.tb_rate);
    return true;
}

// the carried {tokens, last} of h's slot (a stored token count above the capacity — a map
// update may write one — clamps as the first packet's min(C, ...) does: 2^62 is past every
// state the maps reach)
__device__ __forceinline__ void tb_carried(const Slot &sl, int64_t &x, uint64_t &last) {
    const bool carried = ((sl.flags & kFlagBits) & SLOT_HAS_TB) != 0;
    x = carried ? (int64_t)(sl.aux < (1ull << 62) ? sl.aux : (1ull << 62)) : 0;
    last = carried ? sl.tt : kTbNone;
}

struct TbCarried {
    int64_t x;        // tokens after the previous batch (clamped, tb_carried)
    uint64_t last;    // its last packet's timestamp (kTbNone: a new source)
    uint32_t flags, pad_[3];
};

// one wave per (heavy source, group): the group's composed map -> gmap[h][g]; group 0's wave
// also copies the carried state (k_tb_heavy_scan's last group rewrites the slot)
__global__ __launch_bounds__(256) void k_tb_heavy_gmap(const BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                       const uint32_t *__restrict__ base0,
                                                       const uint32_t *__restrict__ offs, uint32_t tcap, uint32_t n,
                                                       const HeavyTileRec *__restrict__ rec, TbHeavyOut o,
                                                       const Slot *table, Limits lim, const HeavySet *__restrict__ hs,
                                                       CMap *gmap, TbCarried *carried, uint32_t ngroups) {
    if (bs->err || !bs->hfast) return;
    const uint32_t wv = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t h = wv / ngroups, g = wv % ngroups;
    TbHeavyCtx C;
    if (!tb_heavy_ctx(bs, cnt0, base0, offs, tcap, n, rec, o, lim, hs, h, C)) return;
    const uint32_t t0 = g * kTbGroup, t1 = min(C.ntiles, t0 + kTbGroup);
    if (t0 >= t1) return;
    const Slot &sl = table[hs->slot[h]];
    int64_t x;
    uint64_t last;
    tb_carried(sl, x, last);
    if (g == 0 && lane_id() == 0) carried[h] = TbCarried{x, last, sl.flags & kFlagBits, {0, 0, 0}};
    last = tb_prev_ts(C, t0, last);
    const CMap M = tb_heavy_range<false>(C, t0, t1, 0, last);
    if (lane_id() == 0) gmap[(size_t)h * ngroups + g] = M;
}

// one wave per (heavy source, group): the state entering the group (the groups before it
// applied to the carried state), the replay of its tiles; the last group stores the source's
// state after the batch
__global__ __launch_bounds__(256) void k_tb_heavy_scan(const BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                       const uint32_t *__restrict__ base0,
                                                       const uint32_t *__restrict__ offs, uint32_t tcap, uint32_t n,
                                                       const HeavyTileRec *__restrict__ rec, TbHeavyOut o,
                                                       Slot *table, Limits lim, const HeavySet *__restrict__ hs,
                                                       const CMap *gmap, const TbCarried *carried, uint32_t ngroups) {
    if (bs->err || !bs->hfast) return;
    const uint32_t wv = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t h = wv / ngroups, g = wv % ngroups;
    TbHeavyCtx C;
    if (!tb_heavy_ctx(bs, cnt0, base0, offs, tcap, n, rec, o, lim, hs, h, C)) return;
    const uint32_t t0 = g * kTbGroup, t1 = min(C.ntiles, t0 + kTbGroup);
    if (t0 >= t1) return;
    const TbCarried cs = carried[h];
    int64_t x = cs.x;
    for (uint32_t k = 0; k < g; ++k) x = cm_apply(gmap[(size_t)h * ngroups + k], x);
    uint64_t last = tb_prev_ts(C, t0, cs.last);
    const CMap M = tb_heavy_range<true>(C, t0, t1, x, last);
    if (t1 == C.ntiles && lane_id() == 0) {
        Slot &sl = table[hs->slot[h]];
        sl.aux = (uint64_t)cm_apply(M, x);
        sl.tt = last;
        sl.flags = cs.flags | SLOT_HAS_TB;   // (drops the born stamp, as k_tb_seg)
    }
}

static uint32_t tb_groups(uint64_t tiles) { return (uint32_t)std::max<uint64_t>(1, (tiles + kTbGroup - 1) / kTbGroup); }

hipError_t launch_tb_heavy(BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, const uint32_t *offs,
                           uint32_t tcap, uint8_t *verdict, const uint64_t *ts, uint32_t n, const void *rec,
                           void *tbh, Slot *table, const Limits &lim, const HeavySet *hs, TableState *tstate,
                           hipStream_t st) {
    const uint32_t ntiles = std::max<uint32_t>(1, (n + kSortTile - 1) / kSortTile);
    const uint64_t tiles_cap = tcap;   // (tcap >= ntiles: the rows' pitch)
    CMap *maps = static_cast<CMap *>(tbh);
    uint64_t *x1 = reinterpret_cast<uint64_t *>(maps + tiles_cap * kHeavyMax);
    CMap *gmap = reinterpret_cast<CMap *>(x1 + tiles_cap * kHeavyMax);
    TbCarried *carried = reinterpret_cast<TbCarried *>(gmap + (size_t)kHeavyMax * tb_groups(tiles_cap));
    const TbHeavyOut o{maps, x1};
    const uint32_t ng = tb_groups(ntiles);
    const HeavyTileRec *R = static_cast<const HeavyTileRec *>(rec);
    const uint32_t gw = (kHeavyMax * ng + 3) / 4;   // (4 waves per block)
    k_tb_heavy_tiles<false><<<ntiles, 256, 0, st>>>(bs, verdict, ts, n, hs, lim, o, tstate);
    k_tb_heavy_gmap<<<gw, 256, 0, st>>>(bs, cnt0, base0, offs, tcap, n, R, o, table, lim, hs, gmap, carried, ng);
    k_tb_heavy_scan<<<gw, 256, 0, st>>>(bs, cnt0, base0, offs, tcap, n, R, o, table, lim, hs, gmap, carried, ng);
    k_tb_heavy_tiles<true><<<ntiles, 256, 0, st>>>(bs, verdict, ts, n, hs, lim, o, tstate);
    return hipGetLastError();
}

size_t tb_heavy_bytes(uint64_t cap) {
    const uint64_t tiles = cap / kSortTile + 2;
    return (size_t)tiles * kHeavyMax * (sizeof(CMap) + 8) + (size_t)kHeavyMax * tb_groups(tiles) * sizeof(CMap) +
           kHeavyMax * sizeof(TbCarried);
}

// The run path of a token-bucket batch with tagged heavy packets (k_hmode_state refused the
// unsorted path): k_heavy_gather built the heavy runs at [n_light, n_valid), whose heads
// (k_heads_heavy's segments) the light heads kernels did not flag; after the fill stored the
// DROPs, a heavy packet still tagged passed.
__global__ __launch_bounds__(256) void k_tb_run_heads(const BatchState *bs, const uint32_t *__restrict__ seg_start,
                                                      uint8_t *__restrict__ headf, uint32_t *__restrict__ tile_off) {
    __shared__ uint32_t s_st[kHeavyMax];
    if (bs->err || bs->hfast) return;
    const uint32_t L = bs->nseg_light, nhs = bs->nseg - L;
    for (uint32_t k = threadIdx.x; k < nhs && k < kHeavyMax; k += 256) s_st[k] = seg_start[L + k];
    __syncthreads();
    const uint32_t a = bs->n_light, b = bs->n_valid;
    for (uint32_t p = a + blockIdx.x * 256u + threadIdx.x; p < b; p += gridDim.x * 256u) {
        uint32_t lo = 0, hi = nhs;   // (the run starts are increasing)
        while (lo < hi) {
            const uint32_t md = (lo + hi) >> 1;
            if (s_st[md] < p) lo = md + 1; else hi = md;
        }
        headf[p] = lo < nhs && s_st[lo] == p ? 1u : 0u;
    }
    // the scan's per-tile segment offsets past the light tiles (heads before the tile's first
    // position: every light segment and the heavy runs that start before it)
    const uint32_t t0 = (a + kTile - 1) / kTile, t1 = (b + kTile - 1) / kTile;
    for (uint32_t t = t0 + blockIdx.x * 256u + threadIdx.x; t < t1; t += gridDim.x * 256u) {
        const uint32_t p = t * kTile;
        uint32_t lo = 0, hi = nhs;   // heavy runs starting before p
        while (lo < hi) {
            const uint32_t md = (lo + hi) >> 1;
            if (s_st[md] < p) lo = md + 1; else hi = md;
        }
        tile_off[t] = L + lo;
    }
}

__global__ __launch_bounds__(256) void k_tb_untag(const BatchState *bs, uint8_t *__restrict__ verdict, uint32_t n) {
    if (bs->err || bs->hfast) return;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        if (verdict[i] >= 0x80u) verdict[i] = XDP_PASS;
}

hipError_t launch_tb_run_heads(const BatchState *bs, const uint32_t *seg_start, uint8_t *headf, uint32_t *tile_off,
                               uint32_t n, hipStream_t st) {
    const uint32_t grid = std::min<uint32_t>(2048, std::max<uint32_t>(1, (n + 255) / 256));
    k_tb_run_heads<<<grid, 256, 0, st>>>(bs, seg_start, headf, tile_off);
    return hipGetLastError();
}

hipError_t launch_tb_untag(const BatchState *bs, uint8_t *verdict, uint32_t n, hipStream_t st) {
    const uint32_t grid = std::min<uint32_t>(2048, std::max<uint32_t>(1, (n + 255) / 256));
    k_tb_untag<<<grid, 256, 0, st>>>(bs, verdict, n);
    return hipGetLastError();
}

// ------------------------------------------------------------------ sliding window
// The virtual sequence of one source: its carried log (hoff, m) then its sorted
// positions j0, j0+1, ...
template <class SV>
struct VView {
    SV sv;
    const uint64_t *ht;
    const uint32_t *hl;
    uint64_t hoff;
    uint32_t m, j0;
    __device__ __forceinline__ uint64_t t(uint32_t v) const { return v < m ? ht[hoff + v] : sv.t(j0 + (v - m)); }
    __device__ __forceinline__ uint32_t l(uint32_t v) const { return v < m ? hl[hoff + v] : sv.l(j0 + (v - m)); }
};

struct SwState {
    bool has_st, has_bl;
    uint64_t pps, bps, tt, till;
};

__device__ __forceinline__ SwState sw_load(const Slot &sl) {
    return SwState{(sl.flags & SLOT_HAS_ST) != 0, (sl.flags & SLOT_HAS_BL) != 0, sl.pps, sl.bps, sl.tt, sl.till};
}
__device__ __forceinline__ void sw_store(Slot &sl, const SwState &s, uint32_t g) {
    sl.flags = (sl.flags & kFlagBits & ~(SLOT_HAS_ST | SLOT_HAS_BL)) | (s.has_st ? SLOT_HAS_ST : 0u) |
               (s.has_bl ? SLOT_HAS_BL : 0u);
    sl.pps = s.pps; sl.bps = s.bps; sl.tt = s.tt; sl.till = s.till;
    sl.aux = kAuxWalked | g;
}
__device__ __forceinline__ void sw_hist_of(uint64_t aux, uint64_t &hoff, uint32_t &m) {
    hoff = aux >> kHistCntBits;
    m = (uint32_t)(aux & ((1ull << kHistCntBits) - 1));
}

// Exact sequential replay (any clock, u64 wraparound as the oracle).
template <class SV, class MW>
__device__ void sw_walk_exact(const SV &sv, uint32_t a, uint32_t b, const Limits &lim,
                              const uint64_t *ht, const uint32_t *hl, uint64_t hoff, uint32_t m,
                              MW &mw, SwState &s, SwSeg &rec) {
    uint32_t q = a;
    if (s.has_bl && s.till > 0) {                           // src/fsx_kern.c:189-215 semantics
        while (q < b && !(sv.t(q) > s.till)) { mw.emit(q, XDP_DROP); ++q; }
        if (q < b) s.has_bl = false;
    }
    const uint32_t j0 = q;
    const VView<SV> vv{sv, ht, hl, hoff, m, j0};
    uint32_t lo = 0;
    uint64_t bytes = 0;
    for (uint32_t v = 0; v < m; ++v) bytes += hl[hoff + v];
    bool cleared = false;
    for (; q < b; ++q) {
        const uint64_t now = sv.t(q);
        if (s.has_bl && s.till > 0) {
            if (now > s.till) s.has_bl = false;
            else { mw.emit(q, XDP_DROP); continue; }
        }
        const uint32_t v = m + (q - j0);
        if (cleared) { lo = v; bytes = 0; cleared = false; }
        while (lo < v && now - vv.t(lo) >= lim.window) { bytes -= vv.l(lo); ++lo; }
        bytes += sv.l(q);
        const uint64_t cnt = (uint64_t)(v - lo) + 1;
        s.has_st = true; s.pps = cnt; s.bps = bytes; s.tt = vv.t(lo);
        if (cnt > lim.pps || bytes > lim.bps) {
            s.till = now + lim.block; s.has_bl = true;
            cleared = true;
            mw.emit(q, XDP_DROP);
        } else {
            mw.emit(q, XDP_PASS);
        }
    }
    rec.hoff = hoff; rec.m = m; rec.j0 = j0;
    if (cleared) { rec.lo = 0; rec.hi = 0; }
    else { rec.lo = lo; rec.hi = m + (b - j0); }
}

// Stats of the log [lo, v] (wave): {count, bytes, oldest timestamp}.
template <class VV>
__device__ __forceinline__ void sw_stats_wave(const VV &vv, uint32_t lo, uint32_t v, SwState &s) {
    s.has_st = true;
    s.pps = (uint64_t)(v - lo) + 1;
    s.bps = sum_len<true>(vv, lo, v + 1);
    s.tt = vv.t(lo);
}

// Oldest log entry at packet time tq: first v in [f, vq] with tq - t(v) < W (monotone).
template <class VV>
__device__ __forceinline__ uint32_t sw_log_start(const VV &vv, uint32_t f, uint32_t vq, uint64_t tq, uint64_t W) {
    if (tq < W) return f;
    const uint32_t lo = wave_gallop_gt(vv, f, vq + 1, tq - W);
    return lo < vq ? lo : vq;
}

// Monotone clocks, no byte trigger possible before the count trigger, no u64 overflow.
template <class SV, class MW>
__device__ void sw_walk_fast_wave(const SV &sv, uint32_t a, uint32_t b, const Limits &lim,
                                  const uint64_t *ht, const uint32_t *hl, uint64_t hoff, uint32_t m,
                                  MW &mw, SwState &s, SwSeg &rec) {
    const uint32_t lane = lane_id();
    const uint64_t P = lim.pps, W = lim.window;
    uint32_t p = a;
    if (s.has_bl && s.till > 0) {
        p = wave_gallop_gt(sv, a, b, s.till);
        if (p > a) mw.emit(a, XDP_DROP);
        if (p < b) s.has_bl = false;
    }
    const uint32_t j0 = p;
    const VView<SV> vv{sv, ht, hl, hoff, m, j0};
    rec.hoff = hoff; rec.m = m; rec.j0 = j0;
    rec.lo = 0; rec.hi = m;                 // no counted packet: the log is unchanged
    uint32_t f = 0;                         // first virtual index of the current log
    while (p < b) {
        uint32_t k = b;                     // first count trigger at or after p
        // no trigger before v = f + P (the count cannot exceed P earlier in the phase)
        uint32_t qs = p;
        if (P > 0) {
            const uint64_t need = (uint64_t)f + P, vp = (uint64_t)m + (p - j0);
            if (need > vp) qs = (uint32_t)min((uint64_t)b, (uint64_t)j0 + (need - m));
        }
        for (uint32_t q0 = qs; q0 < b; q0 += 64) {
            const uint32_t q = q0 + lane;
            bool pr = false;
            if (q < b) {
                const uint32_t v = m + (q - j0);
                if (P == 0) pr = true;
                else if ((uint64_t)v >= (uint64_t)f + P) pr = sv.t(q) - vv.t(v - (uint32_t)P) < W;
            }
            const uint64_t bal = __ballot(pr);
            if (bal) { k = q0 + (uint32_t)__ffsll((unsigned long long)bal) - 1u; break; }
        }
        if (k >= b) {                       // the phase runs to the end of the batch
            mw.emit(p, XDP_PASS);
            const uint32_t vl = m + (b - 1 - j0);
            const uint32_t lo = sw_log_start(vv, f, vl, sv.t(b - 1), W);
            sw_stats_wave(vv, lo, vl, s);
            rec.lo = lo; rec.hi = vl + 1;
            break;
        }
        if (k > p) mw.emit(p, XDP_PASS);
        mw.emit(k, XDP_DROP);
        const uint32_t vk = m + (k - j0);
        const uint64_t tk = sv.t(k);
        sw_stats_wave(vv, sw_log_start(vv, f, vk, tk, W), vk, s);
        s.till = tk + lim.block;
        s.has_bl = true;
        rec.lo = 0; rec.hi = 0;             // log cleared
        const uint32_t j = wave_gallop_gt(sv, k + 1, b, s.till);
        if (j >= b) break;                  // blacklisted to the end of the batch
        s.has_bl = false;                   // deleted at packet j
        f = m + (j - j0);
        p = j;
    }
}

// Thread version of sw_walk_fast_wave for short segments: the count trigger of a phase
// starting at virtual index f cannot fire before v = f + P, so the scan starts there
// (a segment shorter than P - m has no trigger to look for: O(log) per segment).
template <class SV>
__device__ void sw_walk_fast_thread(const SV &sv, uint32_t a, uint32_t b, const Limits &lim,
                                    const uint64_t *ht, const uint32_t *hl, uint64_t hoff, uint32_t m,
                                    MarkWriter<false> &mw, SwState &s, SwSeg &rec) {
    const uint64_t P = lim.pps, W = lim.window;
    uint32_t p = a;
    if (s.has_bl && s.till > 0) {
        p = gallop_gt(sv, a, b, s.till);
        if (p > a) mw.emit(a, XDP_DROP);
        if (p < b) s.has_bl = false;
    }
    const uint32_t j0 = p;
    const VView<SV> vv{sv, ht, hl, hoff, m, j0};
    rec.hoff = hoff; rec.m = m; rec.j0 = j0;
    rec.lo = 0; rec.hi = m;
    uint32_t f = 0;
    auto log_start = [&](uint32_t vq, uint64_t tq) -> uint32_t {
        if (tq < W) return f;
        const uint32_t lo = gallop_gt(vv, f, vq + 1, tq - W);
        return lo < vq ? lo : vq;
    };
    auto stats = [&](uint32_t lo, uint32_t v) {
        s.has_st = true;
        s.pps = (uint64_t)(v - lo) + 1;
        s.bps = sum_len<false>(vv, lo, v + 1);
        s.tt = vv.t(lo);
    };
    while (p < b) {
        uint32_t k = b;
        if (P == 0) {
            k = p;
        } else {
            const uint64_t need = (uint64_t)f + P;                 // first v that can trigger
            const uint64_t vp = (uint64_t)m + (p - j0);
            const uint64_t q0 = need <= vp ? p : (uint64_t)j0 + (need - m);
            for (uint64_t q = q0; q < b; ++q) {
                const uint32_t v = m + ((uint32_t)q - j0);
                if (sv.t((uint32_t)q) - vv.t(v - (uint32_t)P) < W) { k = (uint32_t)q; break; }
            }
        }
        if (k >= b) {
            mw.emit(p, XDP_PASS);
            const uint32_t vl = m + (b - 1 - j0);
            const uint32_t lo = log_start(vl, sv.t(b - 1));
            stats(lo, vl);
            rec.lo = lo; rec.hi = vl + 1;
            break;
        }
        if (k > p) mw.emit(p, XDP_PASS);
        mw.emit(k, XDP_DROP);
        const uint32_t vk = m + (k - j0);
        const uint64_t tk = sv.t(k);
        stats(log_start(vk, tk), vk);
        s.till = tk + lim.block;
        s.has_bl = true;
        rec.lo = 0; rec.hi = 0;
        const uint32_t j = gallop_gt(sv, k + 1, b, s.till);
        if (j >= b) break;
        s.has_bl = false;
        f = m + (j - j0);
        p = j;
    }
}

template <class SV>
__device__ __forceinline__ void sw_short_body(const SV &sv, const BatchState *bs, const TableState *tst,
                                              const uint32_t *seg_start,
                                              const uint32_t *seg_slot, const uint32_t *order,
                                              const uint32_t *cls, uint8_t *marks, Slot *table,
                                              const Limits &lim, const uint64_t *ht, const uint32_t *hl,
                                              SwSeg *segs, bool lists) {
    const uint32_t nshort = bs->nseg - cls[kSegClasses - 1];
    const bool fast = sw_fast(bs, tst, lim);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nshort; i += gridDim.x * 256u) {
        const uint32_t g = order[i];
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        if (lists && a >= bs->n_light) continue;   // a heavy source: k_walk_sw_heavy
        Slot &sl = table[seg_slot[g]];
        SwState st = sw_load(sl);
        uint64_t hoff;
        uint32_t m;
        sw_hist_of(sl.aux, hoff, m);
        MarkWriter<false> mw{marks, 0};
        SwSeg rec{};
        if (fast) sw_walk_fast_thread(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
        else sw_walk_exact(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
        segs[g] = rec;
        sw_store(sl, st, g);
    }
}

template <class SV>
__device__ __forceinline__ void sw_long_body(const SV &sv, const BatchState *bs, const TableState *tst,
                                             const uint32_t *seg_start, const uint32_t *seg_slot,
                                             const uint32_t *order, const uint32_t *cls, uint8_t *marks,
                                             Slot *table, const Limits &lim, const uint64_t *ht,
                                             const uint32_t *hl, SwSeg *segs, bool lists) {
    const uint32_t nl = cls[kSegClasses - 1], first = bs->nseg - nl;
    const bool fast = sw_fast(bs, tst, lim);
    const uint32_t lane = lane_id();
    for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < nl; i += gridDim.x * 4u) {
        const uint32_t g = order[first + i];
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        if (lists && a >= bs->n_light) continue;   // a heavy source: k_walk_sw_heavy
        Slot &sl = table[seg_slot[g]];
        SwState st = sw_load(sl);
        uint64_t hoff;
        uint32_t m;
        sw_hist_of(sl.aux, hoff, m);
        SwSeg rec{};
        if (fast) {
            MarkWriter<true> mw{marks, 0};
            sw_walk_fast_wave(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
        } else if (lane == 0) {
            MarkWriter<false> mw{marks, 0};
            sw_walk_exact(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
        }
        if (lane == 0) {
            segs[g] = rec;
            sw_store(sl, st, g);
        }
    }
}

template <bool kLong>
__global__ __launch_bounds__(256) void k_walk_sw(const uint64_t *__restrict__ S, BatchState *bs,
                                                 const TableState *tst,
                                                 const uint32_t *__restrict__ seg_start,
                                                 const uint32_t *__restrict__ seg_slot,
                                                 const uint64_t *__restrict__ ts,
                                                 const uint32_t *__restrict__ len,
                                                 const uint64_t *__restrict__ pay,
                                                 const uint32_t *__restrict__ order,
                                                 const uint32_t *__restrict__ cls,
                                                 uint8_t *__restrict__ marks, Slot *table, Limits lim,
                                                 HistBufs hb, SwSeg *__restrict__ segs, uint32_t lists) {
    if (bs->err) return;
    const uint32_t cur = tst->hist_cur;
    const uint64_t *ht = hb.t[cur];
    const uint32_t *hl = hb.l[cur];
    if (bs->pay_ok) {
        const SegView<true> sv{S, ts, len, pay, ~bs->inv_min_ts};
        if constexpr (kLong) sw_long_body(sv, bs, tst, seg_start, seg_slot, order, cls, marks, table, lim, ht, hl, segs, lists != 0);
        else sw_short_body(sv, bs, tst, seg_start, seg_slot, order, cls, marks, table, lim, ht, hl, segs, lists != 0);
    } else {
        const SegView<false> sv{S, ts, len, pay, 0};
        if constexpr (kLong) sw_long_body(sv, bs, tst, seg_start, seg_slot, order, cls, marks, table, lim, ht, hl, segs, lists != 0);
        else sw_short_body(sv, bs, tst, seg_start, seg_slot, order, cls, marks, table, lim, ht, hl, segs, lists != 0);
    }
}

// Heavy verdict lists (fixed window's scheme): one wave per heavy source, its
// pass-0 run [base0, + cnt0) walked like a long segment, its verdict changes as the list
// k_verdict_apply reads; its segment id (nseg_light + rank among the non-empty buckets, as
// k_heads_heavy numbered them) keys its log record for the history rebuild.
__global__ __launch_bounds__(256) void k_walk_sw_heavy(const uint64_t *__restrict__ S, BatchState *bs,
                                                       const TableState *tst, const uint32_t *__restrict__ cnt0,
                                                       const uint32_t *__restrict__ base0,
                                                       const uint32_t *__restrict__ seg_slot,
                                                       const uint64_t *__restrict__ ts,
                                                       const uint32_t *__restrict__ len,
                                                       const uint64_t *__restrict__ pay, Slot *table, Limits lim,
                                                       HistBufs hb, SwSeg *__restrict__ segs, HeavyLists H) {
    if (bs->err || (bs->hfast && !H.hs->nrun)) return;   // (hfast: k_walk_sw_heavy_sel, but sparse ones)
    const uint32_t h = blockIdx.x * 4u + (threadIdx.x >> 6), lane = lane_id();
    const uint32_t lb = bs->light_b;
    const bool live0 = lane < kHeavyMax && cnt0[lb + lane] > 0;
    const bool live1 = lane + 64u < kHeavyMax && cnt0[lb + 64u + lane] > 0;
    const uint64_t m0 = __ballot(live0), m1 = __ballot(live1);
    if (h >= H.hs->n) return;
    if (bs->hfast && !((H.hs->srun[h >> 6] >> (h & 63u)) & 1u)) return;
    const uint32_t c = cnt0[lb + h];
    if (c == 0) return;
    const uint32_t rk = h < 64 ? (uint32_t)__popcll(m0 & ((1ull << h) - 1ull))
                               : (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1 & ((1ull << (h - 64)) - 1ull));
    const uint32_t g = bs->nseg_light + rk;
    const uint32_t a = base0[lb + h], b = a + c;
    const uint32_t cur = tst->hist_cur;
    const uint64_t *ht = hb.t[cur];
    const uint32_t *hl = hb.l[cur];
    Slot &sl = table[seg_slot[g]];
    SwState st = sw_load(sl);
    uint64_t hoff;
    uint32_t m;
    sw_hist_of(sl.aux, hoff, m);
    SwSeg rec{};
    auto walk = [&](const auto &sv) {
        if (sw_fast(bs, tst, lim)) {
            MarkWriter<true, true> mw{nullptr, 0};
            heavy_list_open(H, S, a, mw);
            sw_walk_fast_wave(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
            heavy_list_close(H, (int)h, a, b, mw);
        } else if (lane == 0) {
            MarkWriter<false, true> mw{nullptr, 0};
            heavy_list_open(H, S, a, mw);
            sw_walk_exact(sv, a, b, lim, ht, hl, hoff, m, mw, st, rec);
            heavy_list_close(H, (int)h, a, b, mw);
        }
    };
    if (bs->pay_ok) walk(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts});
    else walk(SegView<false>{S, ts, len, pay, 0});
    if (lane == 0) {
        segs[g] = rec;
        sw_store(sl, st, g);
    }
}

// A carried log as a plain timestamp array (wave_gallop_gt over its entries).
struct LogView {
    const uint64_t *t_;
    __device__ __forceinline__ uint64_t t(uint32_t v) const { return t_[v]; }
};

// Heavy sources outside the sort: one wave per heavy source, sw_walk_fast_wave's
// phases over its carried log (hoff, m) followed by its packets by rank (HeavyView: select /
// rank over the verdict tags, block() for 64 consecutive ranks). Monotone clocks only
// (k_hmode_state: sw_fast); the final log — at most pps_threshold <= kSwHeavyMaxP entries —
// is staged past the history's capacity (hist_cap + h * kSwHeavyMaxP of the current buffer)
// so that k_sw_hist copies it like any carried log.
__global__ __launch_bounds__(256) void k_walk_sw_heavy_sel(BatchState *bs, const TableState *tst,
                                                           const uint32_t *__restrict__ cnt0,
                                                           const uint32_t *__restrict__ base0,
                                                           const uint32_t *__restrict__ offs, uint32_t tcap,
                                                           const uint8_t *__restrict__ tags,
                                                           const uint64_t *__restrict__ ts,
                                                           const uint32_t *__restrict__ len, uint32_t n,
                                                           const HeavyTileRec *__restrict__ hrec, Slot *table,
                                                           Limits lim, HistBufs hb, SwSeg *__restrict__ segs,
                                                           HeavySet *hs, uint32_t *list, TableState *tstate) {
    __shared__ uint32_t s_idx[4][64];
    if (bs->err || !bs->hfast) return;
    const uint32_t wv = threadIdx.x >> 6, h = blockIdx.x * 4u + wv, lane = lane_id();
    const uint32_t lb = bs->light_b;
    const bool live0 = lane < kHeavyMax && cnt0[lb + lane] > 0;
    const bool live1 = lane + 64u < kHeavyMax && cnt0[lb + 64u + lane] > 0;
    const uint64_t m0 = __ballot(live0), m1 = __ballot(live1);
    if (h >= hs->n || ((hs->srun[h >> 6] >> (h & 63u)) & 1u)) return;   // (sparse: k_walk_sw_heavy)
    const uint32_t c = cnt0[lb + h];
    if (c == 0) return;
    const uint32_t rk = h < 64 ? (uint32_t)__popcll(m0 & ((1ull << h) - 1ull))
                               : (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1 & ((1ull << (h - 64)) - 1ull));
    const uint32_t g = bs->nseg_light + rk;   // (k_heads_heavy's numbering)
    const uint32_t a = base0[lb + h];
    uint32_t *sx = s_idx[wv];
    const HeavyView hv{tags, ts, len, offs + (size_t)(lb + h) * tcap, hrec, a, c, (n + kSortTile - 1) / kSortTile,
                       n, h, (0x80u | h) * 0x01010101u, &bs->err};
    const uint32_t cur = tst->hist_cur;
    uint64_t *ht = hb.t[cur];
    uint32_t *hl = hb.l[cur];
    Slot &sl = table[hs->slot[h]];
    SwState s = sw_load(sl);
    uint64_t hoff;
    uint32_t m;
    sw_hist_of(sl.aux, hoff, m);
    HeavyMarkWriter mw{hv, list + 2u * a};
    const uint64_t P = lim.pps, W = lim.window;
    uint32_t p = 0;   // ranks
    if (s.has_bl && s.till > 0) {
        p = search_gt<true>(hv, 0, c, s.till);
        if (p > 0) mw.emit(0, XDP_DROP);
        if (p < c) s.has_bl = false;
    }
    const uint32_t j0 = p;   // virtual index v: the log's entry v < m, else rank j0 + v - m
    const LogView lv{ht + hoff};
    auto vt = [&](uint32_t v) __attribute__((always_inline)) -> uint64_t { return v < m ? ht[hoff + v] : hv.t(j0 + v - m); };
    auto vgt = [&](uint32_t lo, uint32_t hi, uint64_t X) __attribute__((always_inline)) -> uint32_t {   // first v in [lo, hi): t(v) > X
        if (lo >= hi) return hi;
        if (lo < m) {
            const uint32_t e = min(hi, m);
            const uint32_t r = wave_gallop_gt(lv, lo, e, X);
            if (r < e || e == hi) return r;
            lo = m;
        }
        return m + search_gt<true>(hv, j0 + lo - m, j0 + hi - m, X) - j0;
    };
    auto vsum = [&](uint32_t lo, uint32_t hi) __attribute__((always_inline)) -> uint64_t {
        uint64_t x = 0;
        for (uint32_t v = lo + lane; v < min(hi, m); v += 64) x += hl[hoff + v];
        x = wave_sum(x);
        const uint32_t l2 = max(lo, m);
        if (hi > l2) x += sum_len<true>(hv, j0 + l2 - m, j0 + hi - m);
        return x;
    };
    auto log_start = [&](uint32_t f, uint32_t vq, uint64_t tq) __attribute__((always_inline)) -> uint32_t {
        if (tq < W) return f;
        const uint32_t lo = vgt(f, vq + 1, tq - W);
        return lo < vq ? lo : vq;
    };
    auto stats = [&](uint32_t lo, uint32_t v) __attribute__((always_inline)) {
        s.has_st = true;
        s.pps = (uint64_t)(v - lo) + 1;
        s.bps = vsum(lo, v + 1);
        s.tt = vt(lo);
    };
    SwSeg rec{};
    rec.hoff = hoff; rec.m = m; rec.j0 = j0;
    rec.lo = 0; rec.hi = m;   // no counted packet: the log is unchanged
    uint32_t f = 0;
    while (p < c) {
        uint32_t k = c;   // first count trigger at or after p (not before v = f + P)
        uint32_t qs = p;
        if (P > 0) {
            const uint64_t need = (uint64_t)f + P, vp = (uint64_t)m + (p - j0);
            if (need > vp) qs = (uint32_t)min((uint64_t)c, (uint64_t)j0 + (need - m));
        }
        for (uint32_t q0 = qs; q0 < c; q0 += 64) {
            const uint32_t q = q0 + lane;
            const uint32_t iq = hv.block(q0, sx);
            const uint64_t tq = iq < n ? ts[iq] : 0ull;
            bool pr;
            if (P == 0) {
                pr = q < c;
            } else {
                // the entry P before each lane's packet: u = v - P >= f (q0 >= qs), from the log
                // below m, else rank j0 + u - m — one block from the first such rank, shifted
                const uint32_t u0 = m + (q0 - j0) - (uint32_t)P;
                const uint32_t u = u0 + lane;
                uint64_t tu = 0;
                if (u0 + 63u >= m) {
                    const uint32_t b0 = max(u0, m), sft = b0 - u0;
                    const uint32_t iu = hv.block(j0 + b0 - m, sx);
                    const uint64_t tb = iu < n ? ts[iu] : 0ull;
                    tu = __shfl(tb, (int)(lane >= sft ? lane - sft : 0u));
                }
                if (u < m) tu = ht[hoff + u];
                pr = q < c && tq - tu < W;
            }
            const uint64_t bal = __ballot(pr);
            if (bal) { k = q0 + (uint32_t)__ffsll((unsigned long long)bal) - 1u; break; }
        }
        if (k >= c) {   // the phase runs to the end of the batch
            mw.emit(p, XDP_PASS);
            const uint32_t vl = m + (c - 1 - j0);
            const uint32_t lo = log_start(f, vl, hv.t(c - 1));
            stats(lo, vl);
            rec.lo = lo; rec.hi = vl + 1;
            break;
        }
        if (k > p) mw.emit(p, XDP_PASS);
        mw.emit(k, XDP_DROP);
        const uint32_t vk = m + (k - j0);
        const uint64_t tk = hv.t(k);
        stats(log_start(f, vk, tk), vk);
        s.till = tk + lim.block;
        s.has_bl = true;
        rec.lo = 0; rec.hi = 0;   // log cleared
        const uint32_t j = search_gt<true>(hv, k + 1, c, s.till);
        if (j >= c) break;        // blacklisted to the end of the batch
        s.has_bl = false;
        f = m + (j - j0);
        p = j;
    }
    mw.finish(c);
    if (rec.hi > m) {   // the log holds packets of this batch: stage it (<= P entries)
        const uint64_t so = hb.cap + (uint64_t)h * kSwHeavyMaxP;
        const uint32_t lo = rec.lo, hi = rec.hi;
        for (uint32_t v = lo + lane; v < min(hi, m); v += 64) {
            ht[so + (v - lo)] = ht[hoff + v];
            hl[so + (v - lo)] = hl[hoff + v];
        }
        const uint32_t l2 = max(lo, m);
        const uint32_t r1 = j0 + hi - m;
        for (uint32_t r0 = j0 + l2 - m; r0 < r1; r0 += 64) {
            const uint32_t i = hv.block(r0, sx);
            const uint32_t r = r0 + lane;
            if (r < r1) {
                const uint64_t o = so + (m + r - j0 - lo);
                ht[o] = ts[i];
                hl[o] = len[i];
            }
        }
        rec.hoff = so; rec.m = hi - lo; rec.j0 = 0; rec.lo = 0; rec.hi = hi - lo;
    }
    if (lane != 0) return;
    segs[g] = rec;
    sw_store(sl, s, g);
    hs->lbase[h] = 2u * a;
    hs->lcnt[h] = mw.nl;
    unsigned long long *sp = reinterpret_cast<unsigned long long *>(tstate->stats);
    if (mw.npass) {
        atomicAdd(sp, (unsigned long long)mw.npass);
        atomicAdd(reinterpret_cast<unsigned long long *>(&bs->allowed), (unsigned long long)mw.npass);
    }
    if (mw.ndrop) {
        atomicAdd(sp + 1, (unsigned long long)mw.ndrop);
        atomicAdd(reinterpret_cast<unsigned long long *>(&bs->dropped), (unsigned long long)mw.ndrop);
    }
}

// The surviving carried log of table slot i as a virtual range [lo, hi) (pruned), and
// its view parameters. Returns false for an empty slot / no log.
template <class SV>
__device__ __forceinline__ uint32_t sw_slot_log(const SV &sv, const Slot &sl, const SwSeg *segs,
                                                const uint64_t *ht, const uint32_t *hl, bool prune,
                                                uint64_t cutoff, SwSeg &r, uint32_t tgen) {
    if (slot_fam(sl.tag, tgen) == 0 || sl.aux == 0) return 0;
    if (sl.aux & kAuxWalked) {
        r = segs[(uint32_t)(sl.aux & 0xFFFFFFFFull)];
    } else {
        sw_hist_of(sl.aux, r.hoff, r.m);
        r.j0 = 0; r.lo = 0; r.hi = r.m;
    }
    if (r.lo >= r.hi) return 0;
    if (prune) {   // drop entries with t <= cutoff (= newest timestamp - W): a prefix
        const VView<SV> vv{sv, ht, hl, r.hoff, r.m, r.j0};
        r.lo = gallop_gt(vv, r.lo, r.hi, cutoff);
    }
    return r.hi - r.lo;
}

constexpr uint32_t kSlotTile = 4096;   // table slots per block in the history rebuild
constexpr uint32_t kCoopLog = 32;      // longer carried logs are copied by the whole wave

struct SwClock {
    bool prune;
    uint64_t cutoff;
};

__device__ __forceinline__ SwClock sw_clock(const BatchState *bs, const TableState *tst, const Limits &lim) {
    const uint64_t T = bs->max_ts > tst->last_max_ts ? bs->max_ts : tst->last_max_ts;
    return SwClock{sw_mono(bs, tst) && T >= lim.window, T - lim.window};
}

// The history rebuild's tile offsets in one pass (kMode 2, k_sw_hist_scan not needed): tiles in
// ticket order, per tile one status word — 1 << 62 | its entries, or 2 << 62 | the entries of
// every tile up to it (the word is the data) — and wave 0 looks back 64 tiles at a time.
__device__ __forceinline__ uint64_t hist_lookback(unsigned long long *status, uint32_t t, uint64_t cnt,
                                                  uint32_t *err) {
    const uint32_t lane = lane_id();
    constexpr unsigned long long kM = (1ull << 62) - 1ull;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(status, (2ull << 62) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(status + t, (1ull << 62) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    uint32_t spins = 0;
    for (int64_t j = (int64_t)t - 1;;) {
        const int64_t idx = j - (int64_t)lane;
        const unsigned long long w = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT)
                                              : (2ull << 62);
        const uint32_t f = (uint32_t)(w >> 62);
        const uint64_t b2 = __ballot(f == 2), b0 = __ballot(f == 0);
        const uint32_t l2 = b2 ? (uint32_t)__ffsll((unsigned long long)b2) - 1u : 64u;
        const uint32_t l0 = b0 ? (uint32_t)__ffsll((unsigned long long)b0) - 1u : 64u;
        if (l0 < l2) {   // a tile before the nearest prefix has published nothing yet
            if (++spins > (1u << 22)) {   // (never expected: lower tickets are running)
                if (lane == 0) atomicOr(err, ERR_SORT_HANG);   // the batch fails (-EIO)
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        // (lanes before the nearest prefix: their tiles' counts; lane l2: that prefix)
        excl += wave_sum(lane <= l2 ? (uint64_t)(w & kM) : 0ull);
        if (l2 < 64u) break;
        j -= 64;
    }
    if (lane == 0) __hip_atomic_store(status + t, (2ull << 62) | (excl + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

template <int kMode>
__global__ __launch_bounds__(256) void k_sw_hist(const uint64_t *__restrict__ S, const BatchState *bs,
                                                 const TableState *tst, const uint64_t *__restrict__ ts,
                                                 const uint32_t *__restrict__ len,
                                                 const uint64_t *__restrict__ pay, Slot *table,
                                                 Limits lim, HistBufs hb, const SwSeg *__restrict__ segs) {
    constexpr bool kWrite = kMode != 0;
    __shared__ uint32_t s_tmp[4];
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_t;
    if (bs->err) return;
    const uint64_t nslots = lim.table_mask + 1;
    const uint64_t ntiles = (nslots + kSlotTile - 1) / kSlotTile;
    const uint32_t cur = tst->hist_cur;
    const uint64_t *ht = hb.t[cur];
    const uint32_t *hl = hb.l[cur];
    uint64_t *nt = hb.t[cur ^ 1u];
    uint32_t *nl = hb.l[cur ^ 1u];
    const SwClock ck = sw_clock(bs, tst, lim);
    const bool pay_ok = bs->pay_ok != 0;
    const SegView<true> svp{S, ts, len, pay, ~bs->inv_min_ts};
    const SegView<false> svg{S, ts, len, pay, 0};
    uint32_t *tile_cnt = hb.tile_cnt;
    uint64_t t0 = blockIdx.x;
    if constexpr (kMode == 2) {   // (one tile per block, in ticket order: the ticket in tile_cnt[0])
        if (threadIdx.x == 0) s_t = atomicAdd(tile_cnt, 1u);
        __syncthreads();
        t0 = s_t;
    }
    for (uint64_t t = t0; t < ntiles; t += kMode == 2 ? ntiles : gridDim.x) {
        // thread x owns slots i0 + 256 k (coalesced slot reads); its logs are stored
        // contiguously in k order (any order works: the slot's aux holds the offset)
        const uint64_t i0 = t * kSlotTile + threadIdx.x;
        auto slot_log = [&](uint64_t i, SwSeg &r) -> uint32_t {
            if (i >= nslots) return 0;
            return pay_ok ? sw_slot_log(svp, table[i], segs, ht, hl, ck.prune, ck.cutoff, r, lim.tgen)
                          : sw_slot_log(svg, table[i], segs, ht, hl, ck.prune, ck.cutoff, r, lim.tgen);
        };
        uint32_t cnt = 0;
        for (int k = 0; k < 16; ++k) {
            SwSeg r;
            cnt += slot_log(i0 + 256u * k, r);
        }
        if constexpr (!kWrite) {
            uint32_t tot;
            block256_excl(cnt, s_tmp, &tot);
            if (threadIdx.x == 0) tile_cnt[t] = tot;
        } else {
            uint64_t off;
            if constexpr (kMode == 2) {
                uint32_t tot;
                const uint32_t ex = block256_excl(cnt, s_tmp, &tot);
                if (threadIdx.x < 64) {   // (wave 0)
                    const uint64_t b = hist_lookback(reinterpret_cast<unsigned long long *>(hb.tile_off),
                                                     (uint32_t)t, tot, const_cast<uint32_t *>(&bs->err));
                    if (threadIdx.x == 0) {
                        s_base = b;
                        if (t == ntiles - 1) *hb.total = b + tot;
                    }
                }
                __syncthreads();
                off = s_base + ex;
            } else {
                off = hb.tile_off[t] + block256_excl(cnt, s_tmp, nullptr);
            }
            // copy log entries [lo + first, hi) step `step` of r to off + (v - lo)
            auto copy = [&](const SwSeg &r, uint64_t o0, uint32_t first, uint32_t step) {
                if (pay_ok) {
                    const VView<SegView<true>> vv{svp, ht, hl, r.hoff, r.m, r.j0};
                    for (uint32_t v = r.lo + first; v < r.hi; v += step) {
                        nt[o0 + (v - r.lo)] = vv.t(v); nl[o0 + (v - r.lo)] = vv.l(v);
                    }
                } else {
                    const VView<SegView<false>> vv{svg, ht, hl, r.hoff, r.m, r.j0};
                    for (uint32_t v = r.lo + first; v < r.hi; v += step) {
                        nt[o0 + (v - r.lo)] = vv.t(v); nl[o0 + (v - r.lo)] = vv.l(v);
                    }
                }
            };
            const uint32_t lane = lane_id();
            for (int k = 0; k < 16; ++k) {   // wave-uniform trip count (no early exit)
                SwSeg r{};
                const uint64_t i = i0 + 256u * k;
                const uint32_t c = slot_log(i, r);
                if (i < nslots) {
                    Slot &sl = table[i];
                    if (slot_fam(sl.tag, lim.tgen) != 0) {
                        if (c == 0) sl.aux = 0;
                        else {
                            if (c <= kCoopLog) copy(r, off, 0, 1);
                            sl.aux = (off << kHistCntBits) | c;
                        }
                    }
                }
                // long logs (a heavy source keeps up to P entries): the whole wave copies
                uint64_t big = __ballot(c > kCoopLog);
                while (big) {
                    const int src = __ffsll((unsigned long long)big) - 1;
                    big &= big - 1;
                    SwSeg rb;
                    rb.hoff = __shfl(r.hoff, src);
                    rb.m = __shfl(r.m, src);
                    rb.j0 = __shfl(r.j0, src);
                    rb.lo = __shfl(r.lo, src);
                    rb.hi = __shfl(r.hi, src);
                    copy(rb, __shfl(off, src), lane, 64);
                }
                off += c;
            }
        }
        __syncthreads();
    }
}

// One block: exclusive scan of the per-tile log counts into 64-bit offsets, total to *total.
__global__ __launch_bounds__(1024) void k_sw_hist_scan(const BatchState *bs, const uint32_t *__restrict__ cnt,
                                                       uint64_t *__restrict__ offs, uint64_t ntiles,
                                                       uint64_t *total) {
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_carry;
    if (bs->err) return;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint64_t i = c0 + threadIdx.x;
        const uint64_t x = i < ntiles ? cnt[i] : 0u;
        const uint64_t incl = wave_incl_sum(x);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint64_t off = s_carry, tot = 0;
        for (uint32_t k = 0; k < 16; ++k) {
            off += k < w ? s_w[k] : 0u;
            tot += s_w[k];
        }
        if (i < ntiles) offs[i] = off + incl - x;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = s_carry;
}

// Flip the history buffers and record the clock facts of this batch.
__global__ void k_sw_finish(const BatchState *bs, TableState *tst, const uint64_t *total) {
    if (bs->err) return;
    const bool mono = sw_mono(bs, tst);
    tst->hist_cur ^= 1u;
    tst->hist_total = *total;
    if (!mono) tst->ever_nonmono = 1;
    if (bs->max_ts > tst->last_max_ts) tst->last_max_ts = bs->max_ts;
    if (bs->max_len > tst->max_len_seen) tst->max_len_seen = bs->max_len;
}

// The heavy sources' walkers (heavy verdict lists): by rank on the unsorted path (tags), the
// pass-0 runs otherwise and for the sparse ones; each returns at once on the other path.
hipError_t launch_sw_heavy(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                           const Scratch &sc, Slot *table, TableState *tstate, const HistBufs &hb,
                           const Limits &lim, uint32_t n, const HeavyLists &H, const uint8_t *tags,
                           hipStream_t st) {
    if (tags) {
        const uint32_t tcap = (uint32_t)(sc.cap / kSortTile + 2);
        k_walk_sw_heavy_sel<<<kHeavyMax / 4, 256, 0, st>>>(
            bs, tstate, sc.sort_ctl, sc.gbase, sc.hist, tcap, tags, ts, len, n,
            static_cast<const HeavyTileRec *>(sc.hrec), table, lim, hb, sc.sw_seg, sc.heavy, H.list, tstate);
    }
    k_walk_sw_heavy<<<kHeavyMax / 4, 256, 0, st>>>(S, bs, tstate, sc.sort_ctl, sc.gbase, sc.seg_slot, ts, len,
                                                   sc.pay[0], table, lim, hb, sc.sw_seg, H);
    return hipGetLastError();
}

hipError_t launch_sliding_window(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                                 const Scratch &sc, Slot *table, TableState *tstate, const HistBufs &hb,
                                 const Limits &lim, uint32_t n, hipStream_t st, const Marker &mark,
                                 hipStream_t st3, hipEvent_t fork_ev, hipEvent_t join_ev, const HeavyLists *H,
                                 const uint8_t *tags, hipEvent_t heavy_done) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t lists = H && H->list ? 1u : 0u;
    const uint32_t gridSeg = std::min<uint32_t>(2048, std::max<uint32_t>(1, (n + 255) / 256));
    const uint32_t *cls = sc.sort_ctl + 1028;
    // short and long segments are disjoint (marks, slots, log records): the wave walker
    // runs on its own stream beside the thread walker when one is given
    const bool fork = st3 && fork_ev && join_ev;
    hipError_t e;
    if (fork) {
        if ((e = hipEventRecord(fork_ev, st)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(st3, fork_ev, 0)) != hipSuccess) return e;
    }
    // heavy verdict lists: the heavy sources' runs (pass 0's buffer, which with 3 passes is
    // also the light entries' final one: S, pay[0]) first on the side stream, latency-bound
    // (heavy_done: the caller launched them on another stream)
    if (lists && !heavy_done) {
        if ((e = launch_sw_heavy(S, ts, len, bs, sc, table, tstate, hb, lim, n, *H, tags, fork ? st3 : st)) !=
            hipSuccess)
            return e;
        mark("k_walk_sw_heavy");
    }
    k_walk_sw<true><<<1024, 256, 0, fork && !lists ? st3 : st>>>(S, bs, tstate, sc.seg_start, sc.seg_slot, ts, len,
                                                                 sc.pay[0], sc.seg_order, cls, sc.marks, table, lim,
                                                                 hb, sc.sw_seg, lists);
    if (fork && (e = hipEventRecord(join_ev, st3)) != hipSuccess) return e;
    k_walk_sw<false><<<gridSeg, 256, 0, st>>>(S, bs, tstate, sc.seg_start, sc.seg_slot, ts, len, sc.pay[0],
                                              sc.seg_order, cls, sc.marks, table, lim, hb, sc.sw_seg, lists);
    mark("k_walk_sw_short");
    if (fork && (e = hipStreamWaitEvent(st, join_ev, 0)) != hipSuccess) return e;
    mark("k_walk_sw_long_join");
    if (lists && heavy_done && (e = hipStreamWaitEvent(st, heavy_done, 0)) != hipSuccess) return e;
    const uint64_t nslots = lim.table_mask + 1;
    const uint64_t ntiles = (nslots + kSlotTile - 1) / kSlotTile;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, ntiles);
    static const bool two_pass = getenv("FSX_SW_HIST_TWO_PASS") != nullptr;   // A/B: count, scan, write
    if (!two_pass && ntiles < (1ull << 31)) {
        // one pass: each tile's offset by a look-back (status words in tile_off, the ticket in
        // tile_cnt[0]); the last tile writes the total
        if ((e = hipMemsetAsync(hb.tile_off, 0, ntiles * 8, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(hb.tile_cnt, 0, 4, st)) != hipSuccess) return e;
        // (A/B: FSX_SW_HIST_LDS bytes of unused dynamic LDS per block cap the blocks in flight,
        // hence the look-back's depth, as for k_tb_scan)
        static const uint32_t hist_lds = getenv("FSX_SW_HIST_LDS") ? (uint32_t)atoi(getenv("FSX_SW_HIST_LDS")) : 0u;
        k_sw_hist<2><<<(uint32_t)ntiles, 256, hist_lds, st>>>(S, bs, tstate, ts, len, sc.pay[0], table, lim, hb, sc.sw_seg);
    } else {
        k_sw_hist<0><<<grid, 256, 0, st>>>(S, bs, tstate, ts, len, sc.pay[0], table, lim, hb, sc.sw_seg);
        k_sw_hist_scan<<<1, 1024, 0, st>>>(bs, hb.tile_cnt, hb.tile_off, ntiles, hb.total);
        mark("k_sw_hist_count");
        k_sw_hist<1><<<grid, 256, 0, st>>>(S, bs, tstate, ts, len, sc.pay[0], table, lim, hb, sc.sw_seg);
    }
    k_sw_finish<<<1, 1, 0, st>>>(bs, tstate, hb.total);
    mark("k_sw_hist_write");
    return hipGetLastError();
}

}  // namespace fsx
