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
//   k_tb_tiles<0> per 4096-position tile: composed map of the tile
//   k_tb_carry    one block: state entering every tile
//   k_tb_tiles<1> per tile: replay the tile from its entering state, verdict marks, the
//                 final {tokens, last} of every source ending in the tile
#include <hip/hip_runtime.h>

#include "fsx_dev_common.h"
#include "fsx_internal.h"
#include "fsx_seg.h"

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
__device__ __forceinline__ int64_t tb_refill(uint64_t dt, uint64_t rate) {
    if (rate == 0) return 0;
    if (dt > (uint64_t)kTbSat / rate) return kTbSat;
    return (int64_t)(dt * rate);
}

// One thread per source. seg_j[g] = first counted sorted position (end of the
// blacklisted prefix); seg_x[g] = tokens after it | PASS bit 63.
template <class SV>
__device__ __forceinline__ void tb_seg_body(const SV &sv, BatchState *bs, const uint32_t *seg_start,
                                            const uint32_t *seg_slot, Slot *table, const Limits &lim,
                                            uint32_t *seg_j, uint64_t *seg_x) {
    const uint32_t nseg = bs->nseg;
    const bool mono = !bs->nonmono;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nseg; g += gridDim.x * 256u) {
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        Slot &sl = table[seg_slot[g]];
        uint32_t flags = sl.flags;
        uint32_t j = a;
        if ((flags & SLOT_HAS_BL) && sl.till > 0) {   // src/fsx_kern.c:189
            const uint64_t till = sl.till;
            if (mono) j = gallop_gt(sv, a, b, till);
            else while (j < b && !(sv.t(j) > till)) ++j;
            if (j < b) sl.flags = flags & ~SLOT_HAS_BL;  // deleted at packet j (:193-204)
        }
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
                                                uint64_t *__restrict__ seg_x) {
    if (bs->err) return;
    if (bs->pay_ok) tb_seg_body(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts}, bs, seg_start, seg_slot, table, lim, seg_j, seg_x);
    else tb_seg_body(SegView<false>{S, ts, len, pay, 0}, bs, seg_start, seg_slot, table, lim, seg_j, seg_x);
}

// Position kinds inside a tile.
enum : uint32_t { TB_BLOCKED = 0, TB_FIRST = 1, TB_NEXT = 2, TB_NONE = 3 };

// One 4096-position tile, 16 consecutive positions per thread. kApply = false: the
// tile's composed map to tile_map[t]; true: replay from tile_x[t], marks and final
// source states.
template <bool kApply, class SV>
__device__ __forceinline__ void tb_tile(const SV &sv, uint32_t t, uint32_t M,
                                        const uint8_t *__restrict__ headf,
                                        const uint32_t *__restrict__ tile_off,
                                        const uint32_t *__restrict__ seg_j,
                                        const uint64_t *__restrict__ seg_x,
                                        const uint32_t *__restrict__ seg_slot, Slot *table,
                                        const Limits &lim, CMap *tile_map, const int64_t *tile_x,
                                        uint8_t *__restrict__ marks, CMap *s_w, uint32_t *s_tmp) {
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t p0 = t * kTile + tid * 16u;
    const int64_t hi = lim.tb_cap >= kTbCost ? (int64_t)(lim.tb_cap - kTbCost) : 0;
    const bool degen = lim.tb_cap < kTbCost;    // C < cost: every counted packet drops
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
    // per-position maps
    int64_t D[16];
    uint32_t kind = 0;  // 2 bits per position
    uint64_t tprev = (p0 > 0 && p0 < M) ? sv.t(p0 - 1) : 0ull;
    int32_t cg = (int32_t)hb - 1;
    uint32_t cj = 0;
    uint64_t cx = 0;
    if (p0 < M && !(hf & 1u)) { cj = seg_j[cg]; cx = seg_x[cg]; }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t p = p0 + (uint32_t)k;
        uint32_t kd = TB_NONE;
        D[k] = 0;
        if (p < M) {
            if ((hf >> k) & 1u) { ++cg; cj = seg_j[cg]; cx = seg_x[cg]; }
            const uint64_t tp = sv.t(p);
            if (p < cj) kd = TB_BLOCKED;
            else if (p == cj) { kd = TB_FIRST; D[k] = (int64_t)cx; }
            else { kd = TB_NEXT; D[k] = tb_refill(tp - tprev, lim.tb_rate) - (int64_t)kTbCost; }
            tprev = tp;
        }
        kind |= kd << (2 * k);
    }
    auto map_of = [&](int k) -> CMap {
        const uint32_t kd = (kind >> (2 * k)) & 3u;
        if (kd == TB_FIRST) {
            const int64_t x = D[k] & (int64_t)~(1ull << 63);
            return CMap{x, x, 0};
        }
        if (kd == TB_NEXT) return degen ? CMap{0, 0, 0} : CMap{0, hi, D[k]};
        return CMap{0, hi, 0};
    };
    CMap T{0, hi, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) T = cm_compose(map_of(k), T);
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
        excl = cm_compose(excl, pre);
        int64_t x = cm_apply(excl, tile_x[t]);
        uint32_t out[4] = {0, 0, 0, 0};
        int32_t g = (int32_t)hb - 1;
        uint64_t tp = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t p = p0 + (uint32_t)k;
            const uint32_t kd = (kind >> (2 * k)) & 3u;
            if (kd == TB_NONE) continue;
            if ((hf >> k) & 1u) ++g;
            uint8_t v;
            if (kd == TB_BLOCKED) {
                v = XDP_DROP;
            } else if (kd == TB_FIRST) {
                v = ((uint64_t)D[k] >> 63) ? XDP_PASS : XDP_DROP;
                x = D[k] & (int64_t)~(1ull << 63);
            } else if (degen) {
                v = XDP_DROP;
                x = 0;
            } else {
                v = x + D[k] >= 0 ? XDP_PASS : XDP_DROP;
                x = clamp64(x + D[k], 0, hi);
            }
            out[k >> 2] |= (uint32_t)v << (8 * (k & 3));
            // last position of its source: the final {tokens, last} (counted packets only)
            if (kd != TB_BLOCKED && ((hf >> (k + 1)) & 1u)) {
                Slot &sl = table[seg_slot[g]];
                sl.aux = (uint64_t)x;
                sl.tt = sv.t(p);
                sl.flags |= SLOT_HAS_TB;
            }
        }
        if (p0 + 16 <= M) {
            *reinterpret_cast<uint4 *>(marks + p0) = make_uint4(out[0], out[1], out[2], out[3]);
        } else {
            for (uint32_t k = 0; p0 + k < M; ++k) marks[p0 + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
        }
    }
}

template <bool kApply>
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
                                                  uint8_t *__restrict__ marks) {
    __shared__ CMap s_w[4];
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t M = bs->n_valid;
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const bool pay_ok = bs->pay_ok != 0;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (pay_ok)
            tb_tile<kApply>(SegView<true>{S, ts, len, pay, ~bs->inv_min_ts}, t, M, headf, tile_off, seg_j,
                            seg_x, seg_slot, table, lim, tile_map, tile_x, marks, s_w, s_tmp);
        else
            tb_tile<kApply>(SegView<false>{S, ts, len, pay, 0}, t, M, headf, tile_off, seg_j, seg_x,
                            seg_slot, table, lim, tile_map, tile_x, marks, s_w, s_tmp);
        __syncthreads();
    }
}

// One block: the state entering every tile (tile 0 starts with a source head, so its
// entering state is irrelevant and taken as 0).
__global__ __launch_bounds__(1024) void k_tb_carry(BatchState *bs, const CMap *__restrict__ tile_map,
                                                   int64_t *__restrict__ tile_x, Limits lim) {
    __shared__ CMap s_w[16];
    if (bs->err) return;
    const uint32_t M = bs->n_valid;
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
                               hipStream_t st) {
    const uint32_t gridSeg = std::min<uint32_t>(2048, std::max<uint32_t>(1, (n + 255) / 256));
    const uint32_t gridTiles = std::min<uint32_t>(4096, std::max<uint32_t>(1, (n + kTile - 1) / kTile));
    uint32_t *seg_j = sc.seg_order;
    uint64_t *seg_x = sc.packed[1];
    CMap *tile_map = reinterpret_cast<CMap *>(sc.lim_tiles);
    int64_t *tile_x = reinterpret_cast<int64_t *>(sc.lim_tiles + 3 * sc.lim_tiles_n);
    k_tb_seg<<<gridSeg, 256, 0, st>>>(S, bs, sc.seg_start, sc.seg_slot, ts, len, sc.pay[0], table, lim,
                                      seg_j, seg_x);
    k_tb_tiles<false><<<gridTiles, 256, 0, st>>>(S, bs, ts, len, sc.pay[0], sc.headf, sc.tile_aux, seg_j,
                                                 seg_x, sc.seg_slot, table, lim, tile_map, tile_x,
                                                 sc.marks);
    k_tb_carry<<<1, 1024, 0, st>>>(bs, tile_map, tile_x, lim);
    k_tb_tiles<true><<<gridTiles, 256, 0, st>>>(S, bs, ts, len, sc.pay[0], sc.headf, sc.tile_aux, seg_j,
                                                seg_x, sc.seg_slot, table, lim, tile_map, tile_x,
                                                sc.marks);
    return hipGetLastError();
}

}  // namespace fsx
