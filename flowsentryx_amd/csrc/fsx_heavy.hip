// fsx_heavy.hip — heavy sources outside the sort (fixed window with heavy verdict lists,
// DESIGN.md §3 "Heavy sources outside the sort").
//
// A Zipf flood puts half of a batch's packets in its 128 heaviest sources. k_parse tags
// their verdict bytes 0x80 | h and counts them per sort tile (pass 0's digit counts, whose
// scan gives "h's packets before tile t"); it writes no sort word for them, and k_pass0h
// reduces each tile's packets of every heavy source to a HeavyTileRec (flow sums). The
// heavy source's packets are then addressed by rank in arrival order:
//   select(h, r)  the arrival index of h's r-th packet: a 64-wide search of the tile
//                 prefix row, then a scan of that tile's 4096 verdict bytes;
//   rank(h, i)    h's packets before arrival index i: prefix row + one tile scan;
// and, with the batch clock non-decreasing, "h's first packet later than X" is rank(h, the
// first arrival index later than X) — one search over the timestamps. The epoch-jump
// walker of src/fsx_kern.c:150-346 (fsx_walk.h walk_fixed_fast) runs unchanged on that view.
//
// k_hmode decides per batch (on the device) whether this holds: clock non-decreasing,
// payloads exact, frames < 2^16 B, tiles < 2^32 ns, every heavy source's carried state on
// the epoch-jump path. Otherwise k_heavy_gather builds the runs pass 0 used to build and
// the run-based kernels (k_walk_heavy, k_flow_heavy) take over; every kernel of the other
// path returns at once.
#include <hip/hip_runtime.h>

#include "fsx_dev_common.h"
#include "fsx_flow_common.h"
#include "fsx_internal.h"
#include "fsx_seg.h"
#include "fsx_walk.h"
#include "fsx_heavy_view.h"

namespace fsx {

// ------------------------------------------------------------------ k_hmode
// After k_pass0h (one thread): the payload words' validity and the batch's path for its
// heavy sources from the batch's own facts. The heavy sources' carried state is checked at
// the start of the batch's tail (k_hmode_state), after the previous batch's walkers stored
// it: a pipelined front runs beside the previous tail.
__global__ void k_hmode(BatchState *bs, const uint64_t *__restrict__ ts, uint32_t n, Limits lim) {
    const uint64_t t0 = n ? ts[0] : 0ull;
    const uint32_t maxL = bs->max_len;
    const uint64_t P = lim.pps, B = lim.bps;
    const uint64_t mn = ~bs->inv_min_ts;
    const bool pay = maxL < (1u << kPayLenBits) && mn == t0 && bs->max_ts - t0 < kPayTsRange;
    bs->pay_ok = pay ? 1u : 0u;
    // (fixed window: walk_fixed_fast's preconditions; sliding window: its final logs fit their
    // staging, the clock facts across batches in k_hmode_state)
    // (token bucket: its heavy maps assume a capacity of at least one token, C >= cost)
    const bool lim_ok = lim.limiter == 2   ? lim.tb_cap >= 1000000000ull
                        : lim.limiter == 1 ? P <= kSwHeavyMaxP
                                           : fast_ok(bs, lim) && !(maxL && P + 1 > B / maxL);
    const bool fast = !bs->err && pay && !bs->nonmono && !bs->span_big && maxL < (1u << 16) && lim_ok;
    bs->hfast = fast ? 1u : 0u;
}

// First kernel of the tail (one block of 128 threads, a thread per heavy source): every
// heavy source's carried state on the epoch-jump path, or the batch takes the run path.
// Sliding window: a heavy source with fewer than 1/kSwDenseDiv of the batch's packets (on
// average < 32 per sort tile, where a block of 64 ranks costs a tile scan per packet or two)
// takes the run path alone (HeavySet::srun). Counts the path taken (TableState::n_hfast /
// n_hrun, fsx_last_batch_info [16] / [17]).
constexpr uint32_t kSwDenseDiv = 128;
__global__ __launch_bounds__(128) void k_hmode_state(const uint32_t *__restrict__ cnt0, uint32_t n, BatchState *bs,
                                                     HeavySet *__restrict__ hs,
                                                     const Slot *__restrict__ table, Limits lim,
                                                     TableState *tstate) {
    __shared__ uint32_t s_bad, s_nrun[2];
    if (threadIdx.x == 0) s_bad = 0;
    const bool fast0 = bs->hfast != 0;
    {   // (every batch: the fixed window and the run path leave the mask empty)
        const uint32_t h = threadIdx.x;
        const bool sparse = fast0 && lim.limiter == 1 && h < hs->n &&
                            (uint64_t)cnt0[bs->light_b + h] * kSwDenseDiv < n;
        const uint64_t b = __ballot(sparse);
        if (lane_id() == 0) {
            hs->srun[h >> 6] = b;
            s_nrun[h >> 6] = (uint32_t)__popcll(b);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) hs->nrun = s_nrun[0] + s_nrun[1];
    if (fast0) {
        const uint32_t h = threadIdx.x;
        const uint32_t maxL = bs->max_len;
        const uint64_t P = lim.pps, B = lim.bps, W = lim.window;
        bool ok = true;
        if (lim.limiter == 2) {   // token bucket: no live blacklist entry (a user rule) on a heavy source
            if (h < hs->n && hs->resolved && hs->slot[h] != kNoSlot) {
                const Slot &sl = table[hs->slot[h]];
                ok = !((sl.flags & SLOT_HAS_BL) && sl.till > 0);
            } else if (h < hs->n) {
                ok = false;
            }
        } else if (lim.limiter == 1) {   // sliding window: sw_walk_fast_wave's facts; carried logs fit
            ok = sw_fast(bs, tstate, lim);
            if (h < hs->n && hs->resolved && hs->slot[h] != kNoSlot) {
                const uint64_t aux = table[hs->slot[h]].aux;
                ok = ok && (aux & ((1ull << kHistCntBits) - 1)) <= kSwHeavyMaxP;
            } else if (h < hs->n) {
                ok = false;
            }
        } else if (h < hs->n && hs->resolved && hs->slot[h] != kNoSlot) {
            const FwState st = load_state(table[hs->slot[h]]);
            ok = !st.has_st || (st.tt <= ~0ull - W && st.pps < kBig && st.bps < kBig);
            if (st.has_st && (st.bps > B || (maxL && P + 1 > (B - st.bps) / maxL))) ok = false;
        } else if (h < hs->n) {
            ok = false;
        }
        if (!ok) s_bad = 1;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const bool fast = fast0 && !s_bad;
    if (fast0 && !fast) bs->hfast = 0;
    if (!bs->err) atomicAdd(fast ? &tstate->n_hfast : &tstate->n_hrun, 1u);
}

// ------------------------------------------------------------------ k_heavy_recs
// (FSX_PARSE_PAY) Every sort tile's sums of every heavy source (HeavyTileRec), at the start of
// the tail beside the next batch's light passes: one block per tile, wave w = the tile's
// 1024-packet chunk w. Lengths, squared lengths, first / last timestamp, first arrival offset,
// and the squared gaps and the largest gap between consecutive packets of a source — a
// packet's predecessor is the last lane below it with the same source (eight ballots), else
// the wave's last packet of it in an earlier row; the waves' chunks are joined at the end.
// Only on the unsorted path (k_hmode / k_hmode_state decided it before the fork).
__global__ __launch_bounds__(256) void k_heavy_recs(const BatchState *bs, const uint64_t *__restrict__ ts,
                                                    const uint32_t *__restrict__ len,
                                                    const uint8_t *__restrict__ tags, uint32_t n,
                                                    const HeavySet *__restrict__ hs,
                                                    HeavyTileRec *__restrict__ rec) {
    __shared__ uint32_t h_s1[kHeavyMax], h_dmax[kHeavyMax], h_fo[kHeavyMax];
    __shared__ unsigned long long h_s2[kHeavyMax], h_d2[kHeavyMax];
    __shared__ unsigned long long h_first[4][kHeavyMax], h_last[4][kHeavyMax];
    if (bs->err || !bs->hfast) return;
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    if (blockIdx.x >= ntiles) return;
    const uint32_t t = xcd_swizzle(blockIdx.x, ntiles);
    const uint32_t t0 = t * kSortTile, c0 = t0 + w * 1024u;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint32_t nh = hs->n;
    constexpr unsigned long long kNone = ~0ull;
    if (tid < kHeavyMax) {
        h_s1[tid] = 0; h_dmax[tid] = 0; h_fo[tid] = 0xFFFFFFFFu;
        h_s2[tid] = 0; h_d2[tid] = 0;
    }
    for (uint32_t j = tid; j < 4 * kHeavyMax; j += 256) {
        (&h_first[0][0])[j] = kNone;
        (&h_last[0][0])[j] = kNone;
    }
    __syncthreads();
    // the chunk's 16 rows loaded up front (the LDS ordering below is a compiler barrier)
    uint64_t Tr[16];
    uint32_t Lr[16], Gr[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t i = c0 + r * 64u + lane;
        const bool live = i < n;
        Gr[r] = live ? tags[i] : 0u;
        Tr[r] = ts[live ? i : 0u];
        Lr[r] = len[live ? i : 0u];
    }
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t i = c0 + r * 64u + lane;
        const uint64_t T = Tr[r];
        const uint32_t L = Lr[r], g = Gr[r];
        const bool hv = g >= 0x80u && (g & 0x7Fu) < nh;
        const uint64_t act = __ballot(hv);
        if (!act) continue;
        const uint32_t h = g & 0x7Fu;
        const uint64_t peers = match_digit(h, act);
        const uint64_t below = peers & lt_mask;
        const uint32_t pl = below ? 63u - (uint32_t)__clzll((long long)below) : lane;
        const uint64_t tpl = __shfl(T, (int)pl);
        if (hv) {
            uint64_t tp = tpl;
            bool gap = below != 0;
            if (!gap) {   // first of h in this row: the wave's last packet of h so far
                tp = h_last[w][h];
                gap = tp != kNone;
                if (!gap) {
                    h_first[w][h] = T;
                    atomicMin(&h_fo[h], i - t0);
                }
            }
            atomicAdd(&h_s1[h], L);
            atomicAdd(&h_s2[h], (unsigned long long)L * L);
            if (gap) {
                const uint64_t d = T - tp;
                atomicAdd(&h_d2[h], (unsigned long long)(d * d));
                atomicMax(&h_dmax[h], d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d);
            }
            if ((peers >> lane) == 1ull) h_last[w][h] = T;   // the row's last of h
        }
        wave_lds_order();
    }
    __syncthreads();
    if (tid >= kHeavyMax) return;
    const uint32_t h = tid;   // join the waves' chunks: the gaps across chunk boundaries
    uint64_t d2 = h_d2[h], first = kNone, last = kNone;
    uint32_t dm = h_dmax[h];
#pragma unroll
    for (uint32_t ww = 0; ww < 4; ++ww) {
        const uint64_t f = h_first[ww][h];
        if (f == kNone) continue;
        if (last != kNone) {
            const uint64_t d = f - last;
            d2 += d * d;
            const uint32_t d32 = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
            dm = d32 > dm ? d32 : dm;
        } else {
            first = f;
        }
        last = h_last[ww][h];
    }
    HeavyTileRec &R = rec[t];
    R.s1[h] = h_s1[h]; R.dmax[h] = dm; R.fo[h] = h_fo[h];
    R.s2[h] = h_s2[h]; R.t0[h] = first; R.t1[h] = last; R.d2[h] = d2;
}

// ------------------------------------------------------------------ k_heavy_gather
// The run path's input when k_hmode refused the batch: every heavy packet's sort word and
// payload word at its place in its source's run (pass 0's layout: bucket light_b + h from
// its base), stable in arrival order — on the unsorted path, of the sliding window's sparse
// heavy sources only (HeavySet::srun). One wave per sort tile.
__global__ __launch_bounds__(256) void k_heavy_gather(const BatchState *bs, const uint8_t *__restrict__ tags,
                                                      const uint64_t *__restrict__ ts, const uint32_t *__restrict__ len,
                                                      uint32_t n, const uint32_t *__restrict__ offs, uint32_t tcap,
                                                      const HeavySet *__restrict__ hs, uint32_t shift0,
                                                      uint64_t id_mask, uint64_t *__restrict__ out,
                                                      uint64_t *__restrict__ pout) {
    __shared__ uint32_t s_cnt[4][kHeavyMax];
    if (bs->err || (bs->hfast && !hs->nrun)) return;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t lb = bs->light_b, nh = hs->n;
    const uint64_t r0m = bs->hfast ? hs->srun[0] : ~0ull, r1m = bs->hfast ? hs->srun[1] : ~0ull;
    const uint64_t tb = n ? ts[0] : 0ull;
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t t = blockIdx.x * 4u + w; t < ntiles; t += gridDim.x * 4u) {
        // each heavy source's next place in its run: its pass-0 tile offset, then advanced by
        // the rows (a global load of the offset per row and lane, waited on inside the row
        // loop, made this kernel take ~1 ms per 64M packets)
        for (uint32_t h = lane; h < kHeavyMax; h += 64) s_cnt[w][h] = h < nh ? offs[(size_t)(lb + h) * tcap + t] : 0u;
        wave_lds_order();
        // 16 rows' tags, then their heavy packets' timestamps and lengths, in flight at once
        for (uint32_t r0 = 0; r0 < (uint32_t)kSortTile / 64u; r0 += 16) {
            uint32_t G[16], L[16];
            uint64_t T[16];
#pragma unroll
            for (uint32_t r = 0; r < 16; ++r) {
                const uint32_t i = t * (uint32_t)kSortTile + (r0 + r) * 64u + lane;
                G[r] = i < n ? tags[i] : 0u;
            }
#pragma unroll
            for (uint32_t r = 0; r < 16; ++r) {
                const uint32_t i = t * (uint32_t)kSortTile + (r0 + r) * 64u + lane;
                const uint32_t hg = G[r] & 0x7Fu;
                const bool hv = G[r] >= 0x80u && hg < nh && (((hg < 64 ? r0m : r1m) >> (hg & 63u)) & 1u);
                G[r] = hv ? hg : 0xFFu;
                // (unconditional loads, all in flight — a load under hv waited for the one
                // before it; a lane not gathering reads element 0, so only the gathered packets'
                // lines are fetched: the sliding window gathers its sparse heavy sources alone)
                T[r] = ts[hv ? i : 0u];
                L[r] = len[hv ? i : 0u];
            }
#pragma unroll
            for (uint32_t r = 0; r < 16; ++r) {
                const uint32_t i = t * (uint32_t)kSortTile + (r0 + r) * 64u + lane;
                const bool hv = G[r] != 0xFFu;
                const uint64_t act = __ballot(hv);
                if (!act) continue;
                const uint32_t h = G[r] & 0x7Fu;
                const uint64_t peers = match_digit(h, act);
                const uint32_t lead = (uint32_t)__ffsll((unsigned long long)peers) - 1u;
                uint32_t base = 0;
                if (hv && lane == lead) base = s_cnt[w][h];
                base = __shfl(base, (int)lead);
                wave_lds_order();
                if (hv) {
                    const uint32_t pos = base + (uint32_t)__popcll(peers & lt);
                    out[pos] = ((uint64_t)(lb + h) << shift0) | ((uint64_t)(hs->slot[h] & id_mask) << kIdShift) | i;
                    pout[pos] = ((T[r] - tb) << kPayLenBits) | L[r];
                    if ((peers >> lane) == 1ull) s_cnt[w][h] = base + (uint32_t)__popcll(peers);
                }
                wave_lds_order();
            }
        }
    }
}

// ------------------------------------------------------------------ k_walk_heavy_sel
// One wave per heavy source: the epoch-jump walker (fsx_walk.h) over its packets by rank.
__global__ __launch_bounds__(256) void k_walk_heavy_sel(BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                        const uint32_t *__restrict__ base0,
                                                        const uint32_t *__restrict__ offs, uint32_t tcap,
                                                        const uint8_t *__restrict__ tags,
                                                        const uint64_t *__restrict__ ts,
                                                        const uint32_t *__restrict__ len, uint32_t n,
                                                        const HeavyTileRec *__restrict__ rec, Slot *table,
                                                        Limits lim, HeavySet *hs, uint32_t *list,
                                                        TableState *tstate) {
    if (bs->err || !bs->hfast) return;
    const uint32_t h = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (h >= hs->n) return;
    const uint32_t lb = bs->light_b;
    const uint32_t c = cnt0[lb + h];
    if (c == 0) return;
    const uint32_t a = base0[lb + h];
    HeavyView hv{tags, ts, len, offs + (size_t)(lb + h) * tcap, rec, a, c, (n + kSortTile - 1) / kSortTile, n, h,
                 (0x80u | h) * 0x01010101u, &bs->err};
    Slot &sl = table[hs->slot[h]];
    FwState st = load_state(sl);
    HeavyMarkWriter mw{hv, list + 2u * a};
    walk_fixed_fast<true>(hv, 0, c, lim, bs->max_len, mw, st);
    mw.finish(c);
    if (lane_id() != 0) return;
    store_state(sl, st);
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

// ------------------------------------------------------------------ heavy flow rows
// Per (group of kHGroupTiles tiles, heavy source): the group's sums over h's packets.
struct HFlowPart {
    FlowAcc a;
    uint64_t t0, t1;    // first / last timestamp
    uint32_t fi, has;   // arrival index of the first packet; any packet
    uint32_t pad_[2];
};

__device__ __forceinline__ void hpart_merge(HFlowPart &x, const HFlowPart &y) {
    if (!y.has) return;
    if (!x.has) { x = y; return; }
    const uint64_t d = y.t0 - x.t1;
    acc_add(x.a, y.a);
    x.a.d1 += (u128)d;
    x.a.d2 += (u128)d * d;
    x.a.dmax = d > x.a.dmax ? d : x.a.dmax;
    x.t1 = y.t1;
}

// group g = blockIdx.x, thread h: the group's tiles in order
__global__ __launch_bounds__(128) void k_hflow_combine(const BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                       const uint32_t *__restrict__ base0,
                                                       const uint32_t *__restrict__ offs, uint32_t tcap, uint32_t n,
                                                       const HeavyTileRec *__restrict__ rec, HFlowPart *part) {
    if (bs->err || !bs->hfast) return;
    const uint32_t h = threadIdx.x;
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    const uint32_t g = blockIdx.x;
    const uint32_t lb = bs->light_b;
    const uint32_t *row = offs + (size_t)(lb + h) * tcap;
    const uint32_t end = base0[lb + h] + cnt0[lb + h];
    HFlowPart x;
    x.a = acc_zero();
    x.t0 = x.t1 = 0;
    x.fi = 0;
    x.has = 0;
    x.pad_[0] = x.pad_[1] = 0;
    const uint32_t t1 = min(ntiles, (g + 1) * kHGroupTiles);
    // eight tiles' loads in flight at a time, merged in order
    constexpr int kU = 8;
    for (uint32_t tb = g * kHGroupTiles; tb < t1; tb += kU) {
        uint32_t c[kU], s1[kU], dm[kU], fo[kU];
        uint64_t s2[kU], a0[kU], a1[kU], d2[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t t = tb + (uint32_t)u;
            const uint32_t tc = t < t1 ? t : tb;
            const HeavyTileRec &R = rec[tc];
            c[u] = t < t1 ? (t + 1 < ntiles ? row[t + 1] : end) - row[t] : 0u;
            s1[u] = R.s1[h]; dm[u] = R.dmax[h]; fo[u] = R.fo[h];
            s2[u] = R.s2[h]; a0[u] = R.t0[h]; a1[u] = R.t1[h]; d2[u] = R.d2[h];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (c[u] == 0) continue;
            HFlowPart y;
            y.a = acc_zero();
            y.a.n = c[u];
            y.a.s1 = s1[u];
            y.a.s2 = s2[u];
            y.a.d1 = a1[u] - a0[u];   // (consecutive gaps of a non-decreasing clock)
            y.a.d2 = d2[u];
            y.a.dmax = dm[u];
            y.t0 = a0[u];
            y.t1 = a1[u];
            y.fi = (tb + (uint32_t)u) * (uint32_t)kSortTile + fo[u];
            y.has = 1;
            y.pad_[0] = y.pad_[1] = 0;
            hpart_merge(x, y);
        }
    }
    part[(size_t)g * kHeavyMax + h] = x;
}

__device__ __forceinline__ HFlowPart shfl_down_part(const HFlowPart &x, uint32_t o) {
    HFlowPart y;
    y.a.n = __shfl_down(x.a.n, o); y.a.s1 = __shfl_down(x.a.s1, o); y.a.dmax = __shfl_down(x.a.dmax, o);
    y.a.pad = 0;
    const uint64_t s2l = __shfl_down((uint64_t)x.a.s2, o), s2h = __shfl_down((uint64_t)(x.a.s2 >> 64), o);
    const uint64_t d1l = __shfl_down((uint64_t)x.a.d1, o), d1h = __shfl_down((uint64_t)(x.a.d1 >> 64), o);
    const uint64_t d2l = __shfl_down((uint64_t)x.a.d2, o), d2h = __shfl_down((uint64_t)(x.a.d2 >> 64), o);
    y.a.s2 = ((u128)s2h << 64) | s2l;
    y.a.d1 = ((u128)d1h << 64) | d1l;
    y.a.d2 = ((u128)d2h << 64) | d2l;
    y.t0 = __shfl_down(x.t0, o); y.t1 = __shfl_down(x.t1, o);
    y.fi = __shfl_down(x.fi, o); y.has = __shfl_down(x.has, o);
    y.pad_[0] = y.pad_[1] = 0;
    return y;
}

// After the heads (k_heads_heavy numbered the heavy segments): heavy source h's row is
// segment nseg_light + (its rank among the non-empty ones), as on the run path. One wave
// per heavy source: lane j merges a contiguous run of the groups' partials in order, then
// an ordered tree over the lanes (the merge is associative, not commutative).
__global__ __launch_bounds__(256) void k_hflow_finish(const BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                      const HeavySet *__restrict__ hs,
                                                      const HFlowPart *__restrict__ part, uint32_t ngroups,
                                                      PacketIn in, const uint32_t *__restrict__ len, FlowOut out,
                                                      ScoreParams P) {
    if (bs->err || !bs->hfast) return;
    const uint32_t h = blockIdx.x * 4u + (threadIdx.x >> 6), lane = lane_id();
    const uint32_t lb = bs->light_b;
    const bool live0 = lane < kHeavyMax && lane < hs->n && cnt0[lb + lane] > 0;
    const bool live1 = lane + 64u < kHeavyMax && lane + 64u < hs->n && cnt0[lb + 64u + lane] > 0;
    const uint64_t m0 = __ballot(live0), m1 = __ballot(live1);
    if (h >= hs->n || cnt0[lb + h] == 0) return;
    const uint32_t r = h < 64 ? (uint32_t)__popcll(m0 & ((1ull << h) - 1ull))
                              : (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1 & ((1ull << (h - 64)) - 1ull));
    const uint32_t per = (ngroups + 63u) / 64u;
    const uint32_t g0 = min(ngroups, lane * per), g1 = min(ngroups, g0 + per);
    HFlowPart x;
    x.a = acc_zero();
    x.t0 = x.t1 = 0;
    x.fi = 0;
    x.has = 0;
    x.pad_[0] = x.pad_[1] = 0;
    for (uint32_t g = g0; g < g1; g += 4) {   // four groups' loads in flight
        HFlowPart y[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t gg = g + (uint32_t)u;
            y[u] = part[(size_t)(gg < g1 ? gg : g0) * kHeavyMax + h];
            if (gg >= g1) y[u].has = 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) hpart_merge(x, y[u]);
    }
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {   // lane k (multiple of 2o) merges lane k + o's run
        const HFlowPart y = shfl_down_part(x, o);
        if ((lane & (2u * o - 1u)) == 0) hpart_merge(x, y);
    }
    if (lane != 0) return;
    const uint32_t row = bs->nseg_light + r;
    uint32_t k[4] = {hs->key[h][0], hs->key[h][1], hs->key[h][2], hs->key[h][3]};
    uint32_t dport;
    if (in.rec) {   // record mode: the port travels in the exchange record
        uint32_t kr[4], L;
        uint64_t T;
        rec_read(in.rec, in.rec_bytes, x.fi, kr, L, T, dport);
    } else {
        dport = dst_port(in.hdr + (size_t)x.fi * 64, len[x.fi]);
    }
    flow_emit(row, x.a, hs->tag[h], k, dport, x.t0, x.t1, hs->slot[h], out, P);
}

size_t hflow_bytes(uint64_t cap) {
    return ((cap / kSortTile + 2) / kHGroupTiles + 1) * kHeavyMax * sizeof(HFlowPart);
}

// ------------------------------------------------------------------ launchers
hipError_t launch_hmode(BatchState *bs, const uint64_t *ts, uint32_t n, const Limits &lim, hipStream_t st) {
    // (A/B: FSX_TB_RUNS=1 sends every token-bucket batch of the unsorted path to its run path —
    // the heavy runs gathered in the tail and scanned with the light entries; read per batch)
    if (lim.limiter == 2 && getenv("FSX_TB_RUNS")) {
        Limits l = lim;
        l.tb_cap = 0;   // (k_hmode's decision only)
        k_hmode<<<1, 1, 0, st>>>(bs, ts, n, l);
        return hipGetLastError();
    }
    k_hmode<<<1, 1, 0, st>>>(bs, ts, n, lim);
    return hipGetLastError();
}

hipError_t launch_heavy_recs(const BatchState *bs, const uint64_t *ts, const uint32_t *len, const uint8_t *tags,
                             uint32_t n, const HeavySet *hs, void *rec, hipStream_t st) {
    const uint32_t ntiles = std::max<uint32_t>(1, (n + kSortTile - 1) / kSortTile);
    k_heavy_recs<<<ntiles, 256, 0, st>>>(bs, ts, len, tags, n, hs, static_cast<HeavyTileRec *>(rec));
    return hipGetLastError();
}

hipError_t launch_hmode_state(const uint32_t *cnt0, uint32_t n, BatchState *bs, HeavySet *hs, const Slot *table,
                              const Limits &lim, TableState *tstate, hipStream_t st) {
    k_hmode_state<<<1, 128, 0, st>>>(cnt0, n, bs, hs, table, lim, tstate);
    return hipGetLastError();
}

hipError_t launch_heavy_gather(const BatchState *bs, const uint8_t *tags, const uint64_t *ts, const uint32_t *len,
                               uint32_t n, const uint32_t *offs, uint32_t tcap, const HeavySet *hs, uint32_t shift0,
                               uint64_t id_mask, uint64_t *out, uint64_t *pout, hipStream_t st) {
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(1024, (ntiles + 3) / 4));
    k_heavy_gather<<<grid, 256, 0, st>>>(bs, tags, ts, len, n, offs, tcap, hs, shift0, id_mask, out, pout);
    return hipGetLastError();
}

// Test hook (FSX_TEST_HEAVY_ROW_CORRUPT, tests/test_gpu_heavy.py): every heavy source's prefix
// row is overwritten past its count — what round 5's aliasing did (ff010e0) — so the walker's
// searches meet an inconsistent row; the batch must fail with -EIO instead of hanging.
__global__ void k_test_corrupt_rows(const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0,
                                    uint32_t *offs, uint32_t tcap, uint32_t n, const HeavySet *hs) {
    if (bs->err || !bs->hfast) return;
    const uint32_t lb = bs->light_b, ntiles = (n + kSortTile - 1) / kSortTile;
    for (uint32_t h = blockIdx.x; h < hs->n; h += gridDim.x) {
        uint32_t *row = offs + (size_t)(lb + h) * tcap;
        const uint32_t bad = base0[lb + h] + cnt0[lb + h] + 7u;
        for (uint32_t t = threadIdx.x; t < ntiles; t += blockDim.x) row[t] = bad;
    }
}

hipError_t launch_walk_heavy_sel(BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, const uint32_t *offs,
                                 uint32_t tcap, const uint8_t *tags, const uint64_t *ts, const uint32_t *len,
                                 uint32_t n, const void *rec, Slot *table, const Limits &lim, HeavySet *hs,
                                 uint32_t *list, TableState *tstate, hipStream_t st) {
    const bool corrupt = getenv("FSX_TEST_HEAVY_ROW_CORRUPT") != nullptr;   // (per call: tests set it)
    if (corrupt) k_test_corrupt_rows<<<kHeavyMax, 256, 0, st>>>(bs, cnt0, base0, const_cast<uint32_t *>(offs), tcap,
                                                                n, hs);
    k_walk_heavy_sel<<<kHeavyMax / 4, 256, 0, st>>>(bs, cnt0, base0, offs, tcap, tags, ts, len, n,
                                                     static_cast<const HeavyTileRec *>(rec), table, lim, hs, list,
                                                     tstate);
    return hipGetLastError();
}

hipError_t launch_hflow_combine(const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0,
                                const uint32_t *offs, uint32_t tcap, uint32_t n, const void *rec, void *part,
                                hipStream_t st) {
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    const uint32_t ng = std::max<uint32_t>(1, (ntiles + kHGroupTiles - 1) / kHGroupTiles);
    k_hflow_combine<<<ng, 128, 0, st>>>(bs, cnt0, base0, offs, tcap, n, static_cast<const HeavyTileRec *>(rec),
                                         static_cast<HFlowPart *>(part));
    return hipGetLastError();
}

hipError_t launch_hflow_finish(const BatchState *bs, const uint32_t *cnt0, const HeavySet *hs, const void *part,
                               uint32_t n, const PacketIn &in, const uint32_t *len, const uint64_t *ts,
                               uint8_t *keys16, uint8_t *fam, float *feat, float *prob, uint8_t *dec,
                               uint32_t rows_cap, const ScoreParams &P, void *sacc, uint32_t epoch,
                               const PartialOut &partial, hipStream_t st) {
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    const uint32_t ng = std::max<uint32_t>(1, (ntiles + kHGroupTiles - 1) / kHGroupTiles);
    FlowOut out{nullptr, keys16, fam, feat, prob, dec, rows_cap, (SlotAcc *)sacc, epoch, nullptr, ts,
                nullptr, nullptr, partial};
    k_hflow_finish<<<kHeavyMax / 4, 256, 0, st>>>(bs, cnt0, hs, static_cast<const HFlowPart *>(part), ng, in, len,
                                                  out, P);
    return hipGetLastError();
}

}  // namespace fsx
