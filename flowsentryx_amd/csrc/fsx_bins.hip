// fsx_bins.hip — the third sort pass of the heavy-source sort as a per-bin local sort
// (DESIGN.md §3 "Bin sort").
//
// With the heavy-source sort, sort pass 0 buckets the light entries by slot bits
// [8, 15) and pass 1 by bits [15, id bits): the pass-1 output is ordered by slot >> 8, so
// a bin — the run of one value of slot >> 8, in arrival order — holds the 256 consecutive
// slots b * 256 + k. Instead of a third global LSD pass (per-tile digit counts, a scan, a
// scatter over the whole light array), each bin is ordered by k inside its own range:
//   k_bin_bounds  bin starts in the pass-1 output (one compare per position)
//   k_bin_order   bins of more than one chunk first (they are the kernel's long poles)
//   k_bin_sort    one block per bin: a stable counting sort by k (ballot matching per wave
//                 round, rounds and waves in order), entries written from registers to
//                 their place in the bin's range; the segment heads and their per-tile
//                 counts come out with them (no k_heads_count)
// The result is the order the global third pass gives (sources by slot, each in arrival
// order), so everything after it is unchanged.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fsx_bins.h"
#include "fsx_dev_common.h"

namespace fsx {

#ifndef FSX_BIN_CAP
#define FSX_BIN_CAP 4096   // entries per chunk of a bin (A/B: scripts/build_variant.sh)
#endif
constexpr uint32_t kBinCap = FSX_BIN_CAP;
static_assert(kBinCap % 256 == 0, "whole block rounds");


// bin of a light sort word: its source slot without the low kBinSlotBits bits
__device__ __forceinline__ uint32_t bin_of(uint64_t v, uint32_t idm) {
    return ((uint32_t)(v >> 32) & idm) >> kBinSlotBits;
}

// bin starts: bin_start[b] = first light position whose bin is >= b (b <= nbins). Thread
// t of the grid-stride loop covers 8 consecutive positions (four 16-byte loads), the
// position before them through the lane below.
__global__ __launch_bounds__(256) void k_bin_bounds(const uint64_t *__restrict__ S, const BatchState *bs,
                                                    uint32_t *__restrict__ bin_start, uint32_t idm,
                                                    uint32_t nbins) {
    if (bs->err) return;
    const uint32_t M = bs->n_light;
    const uint32_t lane = lane_id();
    const uint32_t ngroups = M / 8u + 1u;   // (the last group holds the end position M)
    for (uint32_t g0 = blockIdx.x * 256u; g0 < ngroups; g0 += gridDim.x * 256u) {
        const uint32_t g = g0 + threadIdx.x;
        const uint32_t p0 = g * 8u;
        uint32_t bn[8];
        if (p0 + 8u <= M) {
            const ulonglong2 *q = reinterpret_cast<const ulonglong2 *>(S + p0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const ulonglong2 x = q[k];
                bn[2 * k] = bin_of(x.x, idm);
                bn[2 * k + 1] = bin_of(x.y, idm);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) bn[k] = p0 + k < M ? bin_of(S[p0 + k], idm) : nbins;
        }
        int64_t prev = (int64_t)__shfl_up(bn[7], 1);
        if (lane == 0) prev = p0 == 0 ? -1 : (p0 - 1 < M ? (int64_t)bin_of(S[p0 - 1], idm) : (int64_t)nbins);
        if (p0 == 0) prev = -1;
        if (g >= ngroups) continue;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t p = p0 + k;
            if (p > M) break;
            const uint32_t cur = p < M ? bn[k] : nbins;
            for (int64_t b = prev + 1; b <= (int64_t)cur; ++b) bin_start[b] = p;
            prev = cur;
        }
    }
}

// Bins of more than one chunk first (a bin's chunks run in order in one block: started
// last, a large bin would be the kernel's tail), then the others (any order: the results
// do not depend on it).
__global__ __launch_bounds__(1024) void k_bin_order(const uint32_t *__restrict__ bin_start, uint32_t nbins,
                                                    uint32_t *__restrict__ bin_order, const BatchState *bs) {
    __shared__ uint32_t s_big, s_nb, s_ns;
    if (bs->err) return;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) { s_big = 0; s_nb = 0; s_ns = 0; }
    __syncthreads();
    uint32_t big = 0;
    for (uint32_t b = tid; b < nbins; b += 1024) big += bin_start[b + 1] - bin_start[b] > kBinCap;
    if (big) atomicAdd(&s_big, big);
    __syncthreads();
    const uint32_t nbig = s_big;
    for (uint32_t b0 = 0; b0 < nbins; b0 += 1024) {
        const uint32_t b = b0 + tid;
        const bool live = b < nbins;
        const bool g = live && bin_start[b + 1] - bin_start[b] > kBinCap;
        const uint32_t lane = lane_id();
        const uint64_t mg = __ballot(g), ml = __ballot(live && !g);
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t bb = 0, bs_ = 0;
        if (lane == 0) {
            if (mg) bb = atomicAdd(&s_nb, (uint32_t)__popcll(mg));
            if (ml) bs_ = atomicAdd(&s_ns, (uint32_t)__popcll(ml));
        }
        bb = __shfl(bb, 0);
        bs_ = __shfl(bs_, 0);
        if (g) bin_order[bb + (uint32_t)__popcll(mg & lt)] = b;
        else if (live) bin_order[nbig + bs_ + (uint32_t)__popcll(ml & lt)] = b;
    }
}

// The segment-head flag of output position p (what k_heads_count would write): every
// source's first position is a head; heads are counted per kTile tile and per 1024-position
// flow sub-tile.
// The heads of a bin are counted per 1024-position sub-tile in LDS (relative to the bin's
// first sub-tile; kBinSubs of them) and added to the global counters once per sub-tile at
// the end; a bin spanning more sub-tiles counts its heads past them directly.
constexpr uint32_t kBinSubs = 256;
__device__ __forceinline__ void head_out(const BinSort &A, uint32_t p, bool h, uint32_t sub0, uint32_t *s_sub) {
    A.headf[p] = h ? 1u : 0u;
    if (h) {
        const uint32_t s = p / 1024u - sub0;
        if (s < kBinSubs) {
            atomicAdd(&s_sub[s], 1u);
        } else {
            atomicAdd(&A.tile_cnt[p / (uint32_t)kTile], 1u);
            atomicAdd(&A.sub_cnt[p / 1024u], 1u);
        }
    }
}

// One block per bin (a run of the pass-1 output in arrival order, <= 256 sources): a
// stable counting sort by the slot's low 8 bits k, each entry written from registers
// straight to its position inside the bin's range (runs of equal k from consecutive
// lanes). Per chunk of kBinCap entries: every wave counts its quarter per k (one LDS add
// for a round of one source), the bin's running base of k plus the waves before give each
// wave's cursor, then each round is ranked by ballot matching and placed. Bins of more
// than one chunk take their per-k totals first.
template <bool kPay>
__device__ __forceinline__ void bin_sort(const BinSort &A, uint32_t (*wc)[256], uint32_t *base, uint32_t *head,
                                         uint32_t *s_tmp, uint32_t *s_sub) {
    const uint32_t b = A.bin_order[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const uint32_t lo = A.bin_start[b], hi = A.bin_start[b + 1];
    if (lo >= hi) return;
    const uint32_t idm = (uint32_t)A.table_mask;
    const uint64_t lt = (1ull << lane) - 1ull;
    auto kof = [&](uint64_t v) { return (uint32_t)(v >> 32) & 255u; };
    constexpr uint32_t kQ = kBinCap / 4, kR = kQ / 64;
    (void)idm;
    const uint32_t sub0 = lo / 1024u;
    s_sub[tid] = 0;   // (kBinSubs == 256 threads; ordered by the barriers below)
    // per-wave counts of k over [c0, c0 + m): thread tid owns k = tid afterwards
    auto count = [&](uint32_t c0, uint32_t m, const uint64_t *v) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) wc[wv][lane + 64u * i] = 0;   // (each wave its own row)
        wave_lds_order();
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = wv * kQ + r * 64u + lane;
            const bool ok = j < m;
            const uint64_t act = __ballot(ok);
            if (!act) break;
            const uint32_t k = kof(v[r]);
            const uint32_t kl = __builtin_amdgcn_readfirstlane(k);
            if (__ballot(ok && k == kl) == act) {
                if (lane == 0) atomicAdd(&wc[wv][kl], (uint32_t)__popcll(act));
            } else if (ok) {
                atomicAdd(&wc[wv][k], 1u);
            }
        }
        (void)c0;
    };
    const bool multi = hi - lo > kBinCap;
    if (multi) {   // the bin's totals per k -> running bases
        base[tid] = 0;
        __syncthreads();
        constexpr uint32_t kPre = 16;   // loads in flight per thread
        for (uint32_t q0 = lo; q0 < hi; q0 += 256 * kPre) {
            uint32_t kk[kPre];
#pragma unroll
            for (uint32_t r = 0; r < kPre; ++r) {
                const uint32_t q = q0 + r * 256u + tid;
                kk[r] = q < hi ? kof(A.S[q]) : 256u;
            }
#pragma unroll
            for (uint32_t r = 0; r < kPre; ++r) {
                const bool ok = kk[r] < 256u;
                const uint64_t act = __ballot(ok);
                if (!act) break;
                const uint32_t kl = __builtin_amdgcn_readfirstlane(kk[r]);
                if (__ballot(ok && kk[r] == kl) == act) {
                    if (lane == 0) atomicAdd(&base[kl], (uint32_t)__popcll(act));
                } else if (ok) {
                    atomicAdd(&base[kk[r]], 1u);
                }
            }
        }
        __syncthreads();
        uint32_t tot;
        const uint32_t c = base[tid];
        const uint32_t ex = block256_excl(c, s_tmp, &tot);
        base[tid] = ex;
        head[tid] = c ? ex : ~0u;
        __syncthreads();
    }
    for (uint32_t c0 = lo; c0 < hi; c0 += kBinCap) {
        const uint32_t m = min(kBinCap, hi - c0);
        uint64_t v[kR], pw[kR];
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = wv * kQ + r * 64u + lane;
            v[r] = j < m ? A.S[c0 + j] : 0ull;
        }
        if constexpr (kPay) {
#pragma unroll
            for (uint32_t r = 0; r < kR; ++r) {
                const uint32_t j = wv * kQ + r * 64u + lane;
                pw[r] = j < m ? A.pay[c0 + j] : 0ull;
            }
        }
        count(c0, m, v);
        __syncthreads();
        // thread tid = k: the chunk's count of k, per wave; cursors of the four waves
        const uint32_t c_0 = wc[0][tid], c_1 = wc[1][tid], c_2 = wc[2][tid], c_3 = wc[3][tid];
        const uint32_t cnt = c_0 + c_1 + c_2 + c_3;
        uint32_t b0;
        if (multi) {
            b0 = base[tid];
        } else {
            uint32_t tot;
            b0 = block256_excl(cnt, s_tmp, &tot);
            head[tid] = cnt ? b0 : ~0u;
        }
        __syncthreads();
        wc[0][tid] = b0;
        wc[1][tid] = b0 + c_0;
        wc[2][tid] = b0 + c_0 + c_1;
        wc[3][tid] = b0 + c_0 + c_1 + c_2;
        if (multi) base[tid] = b0 + cnt;
        __syncthreads();
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = wv * kQ + r * 64u + lane;
            const bool ok = j < m;
            const uint64_t act = __ballot(ok);
            if (!act) break;
            const uint32_t k = kof(v[r]);
            const uint32_t kl = __builtin_amdgcn_readfirstlane(k);
            const uint64_t peers = __ballot(ok && k == kl) == act ? act : match_digit(k, act);
            const uint32_t below = (uint32_t)__popcll(peers & lt);
            const uint32_t cur = wc[wv][k];
            wave_lds_order();
            if (ok && below == 0) wc[wv][k] = cur + (uint32_t)__popcll(peers);
            wave_lds_order();
            if (ok) {
                const uint32_t p = cur + below;   // bin-relative output position
                A.out[lo + p] = v[r];
                if constexpr (kPay) A.pout[lo + p] = pw[r];
                if (A.headf) head_out(A, lo + p, p == head[k], sub0, s_sub);
            }
        }
        __syncthreads();
    }
    if (A.headf) {   // the bin's head counts per sub-tile and tile, one add each
        const uint32_t c = s_sub[tid];
        if (c) atomicAdd(&A.sub_cnt[sub0 + tid], c);
        // tile t = sub-tiles 4t .. 4t + 3: the thread of each tile's first sub-tile in range adds them
        const uint32_t sub = sub0 + tid;
        if (tid < kBinSubs && (sub % 4u == 0u || tid == 0)) {
            uint32_t tc = 0;
            for (uint32_t s = sub; s < (sub / 4u + 1u) * 4u && s - sub0 < kBinSubs; ++s) tc += s_sub[s - sub0];
            if (tc) atomicAdd(&A.tile_cnt[sub / 4u], tc);
        }
    }
}

__global__ __launch_bounds__(256) void k_bin_sort(BinSort A) {
    __shared__ uint32_t wc[4][256], base[256], head[256], s_tmp[4], s_sub[kBinSubs];
    static_assert(kBinSubs == 256, "one sub-tile counter per thread");
    if (A.bs->err) return;
    if (A.bs->pay_ok) bin_sort<true>(A, wc, base, head, s_tmp, s_sub);
    else bin_sort<false>(A, wc, base, head, s_tmp, s_sub);
}

static inline uint32_t cdiv32(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_bin_sort(const BinSort &A, uint32_t n, hipStream_t st) {
    (void)hipGetLastError();
    const uint32_t nbins = (uint32_t)((A.table_mask + 1) >> kBinSlotBits);
    k_bin_bounds<<<std::max<uint32_t>(1, std::min<uint32_t>(4096, cdiv32((uint64_t)n + 1, 256 * 8))), 256, 0, st>>>(
        A.S, A.bs, A.bin_start, (uint32_t)A.table_mask, nbins);
    k_bin_order<<<1, 1024, 0, st>>>(A.bin_start, nbins, A.bin_order, A.bs);
    k_bin_sort<<<nbins, 256, 0, st>>>(A);
    return hipGetLastError();
}

}  // namespace fsx
