// fsx_flows.hip — per-source flow features fused with the quantized scorer.
//
// The reference has no feature code (src/fsx_kern_ml.c:1-16 is a comment); the
// eight model inputs are the CICFlowMeter columns of model/model.py:117. Their
// build-defined semantics (restated in oracle/fsx_oracle.c
// fsxo_flow_features) are computed here per source IP over one batch:
//   n, S1 = sum L, S2 = sum L^2, D1 = sum d, D2 = sum d^2, Dmax = max d
// (L frame length, d inter-arrival time of consecutive packets of the source) as
// exact integers (u64 / u128), then the features in fp64, rounded to fp32, then the
// q8 scorer of model/model.py:132-137 -> probability and decision per source.
//
// Work layout: the sources are the segments of the sorted packet array. One wave
// owns a 1024-position tile (16 consecutive positions per lane): lane-level
// accumulation, a segmented wave scan to join lanes, and every source that starts
// and ends inside the tile is finished by the lane holding its last packet. A source
// crossing tile boundaries leaves one partial per tile (first/last piece) and is
// finished by k_flow_combine (one wave per such source, lanes striding its tiles).
// Per packet: 8 B sort word + 12 B gathered (len, ts) in; per source: 8 x fp32
// features + prob + decision out.
//
// light_only (the fixed window with heavy verdict lists): these kernels cover the light
// positions [0, n_light) and segments [0, nseg_light); each heavy source is one run of
// sort pass 0, summed right after that pass in kHeavyChunk-position chunks (k_flow_heavy,
// beside sort passes 1-2) and finished after the heads (k_flow_heavy_finish).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "fsx_flow_common.h"
#include "fsx_seg.h"

namespace fsx {

constexpr uint32_t kFT = 1024;  // flow tile: one wave, 16 positions per lane

// kPay: (ts, len) of sorted positions come from the sort's payload words (relative
// timestamps suffice: only differences are used); else gathered by arrival index.
template <bool kPay>
__device__ __forceinline__ void flow_tiles(const uint64_t *__restrict__ S,
                                           const uint64_t *__restrict__ pay, BatchState *bs,
                                           const uint8_t *__restrict__ headf,
                                           const uint32_t *__restrict__ len,
                                           const uint64_t *__restrict__ ts,
                                           const PacketIn &in,
                                           const uint32_t *__restrict__ tile_off,
                                           const uint32_t *__restrict__ sub_cnt,
                                           const uint32_t *__restrict__ seg_start,
                                           FlowAcc *__restrict__ firstp, FlowAcc *__restrict__ lastp,
                                           uint32_t *__restrict__ span_list, const FlowOut &out,
                                           const ScoreParams &P, uint32_t salt,
                                           unsigned long long (*s_S)[64 * 17], uint32_t light_only) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t M = light_only ? bs->n_light : bs->n_valid;
    const uint32_t nsub = (M + kFT - 1) / kFT;
    unsigned long long *sS = s_S[w];
    for (uint32_t sub = blockIdx.x * 4u + w; sub < nsub; sub += gridDim.x * 4u) {
        const uint32_t base = sub * kFT;
        const uint32_t p0 = base + lane * 16u;
        // heads before this tile
        const uint32_t t4 = sub >> 2, j4 = sub & 3u;
        uint32_t hb = tile_off[t4];
        for (uint32_t j = 0; j < j4; ++j) hb += sub_cnt[t4 * 4 + j];
        // stage the tile's payload (or sort) words through LDS (coalesced load,
        // 17-word row pitch)
        // (element r * 64 + lane lands in row 4r + lane / 16: one LDS base, constant offsets)
        const uint64_t *src = kPay ? pay : S;
        unsigned long long *sdst = sS + (lane >> 4) * 17u + (lane & 15u);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t p = base + (uint32_t)r * 64u + lane;
            sdst[r * 68] = p < M ? src[p] : 0ull;
        }
        wave_lds_order();
        uint32_t hf[4] = {0, 0, 0, 0};
        if (p0 + 16 <= M) {
            const uint4 h4 = *reinterpret_cast<const uint4 *>(headf + p0);
            hf[0] = h4.x; hf[1] = h4.y; hf[2] = h4.z; hf[3] = h4.w;
        } else {
            for (uint32_t k = 0; k < 16 && p0 + k < M; ++k) hf[k >> 2] |= (uint32_t)headf[p0 + k] << (8 * (k & 3));
        }
        // (len, ts) of the lane's position k, read from the LDS row when needed (holding
        // all 16 in registers halved the occupancy)
        auto LT = [&](int k, uint32_t &Lk, uint64_t &Tk) {
            const uint64_t v = sS[lane * 17u + (uint32_t)k];
            const bool ok = p0 + (uint32_t)k < M;
            if constexpr (kPay) {
                Lk = ok ? (uint32_t)v & ((1u << kPayLenBits) - 1u) : 0u;
                Tk = ok ? v >> kPayLenBits : 0ull;
            } else {
                const uint32_t idx = pk_idx(v);
                Lk = ok ? len[idx] : 0u;
                Tk = ok ? ts[idx] : 0ull;
            }
        };
        uint32_t L15;
        uint64_t T15;
        LT(15, L15, T15);
        uint64_t tprev = __shfl_up(T15, 1);
        if (lane == 0) {
            if constexpr (kPay) tprev = (p0 > 0 && p0 < M) ? pay[p0 - 1] >> kPayLenBits : 0ull;
            else tprev = (p0 > 0 && p0 < M) ? ts[pk_idx(S[p0 - 1])] : 0ull;
        }
        // head flag of the position after this lane (end of array counts as a head)
        const uint32_t h_first = hf[0] & 1u;
        uint32_t next_head = __shfl_down(h_first, 1);
        if (lane == 63) next_head = (base + kFT >= M) ? 1u : headf[base + kFT];
        if (p0 + 16 >= M) next_head = 1;
        uint32_t nh = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) nh += __popc(hf[k] & 0x01010101u);
        const uint32_t hoff = wave_incl_sum(nh) - nh;
        uint32_t g = hb + hoff;  // id of this lane's first head
        FlowAcc A = acc_zero(), F = acc_zero();
        uint32_t seen = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (p0 + k < M) {
                uint32_t Lk;
                uint64_t Tk;
                LT(k, Lk, Tk);
                const bool h = (hf[k >> 2] >> (8 * (k & 3))) & 1u;
                if (h) {
                    if (seen == 0) F = A;
                    else acc_store(out, g + seen - 1, A);
                    if (out.seg_len && g + seen < out.cap) out.seg_len[g + seen] = Lk;   // its first frame
                    ++seen;
                    A = acc_zero();
                }
                FlowAcc c = acc_zero();
                c.n = 1; c.s1 = Lk; c.s2 = (u128)Lk * Lk;
                if (!h) {
                    const uint64_t d = Tk - tprev;
                    c.d1 = d; c.d2 = (u128)d * d; c.dmax = d;
                }
                acc_add(A, c);
                tprev = Tk;
            }
        }
        if (nh == 0) F = A;
        // segmented inclusive scan over lanes of (has_head, piece open at lane end)
        uint32_t fl = nh > 0;
        FlowAcc val = nh > 0 ? A : F;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t ofl = __shfl_up(fl, o);
            const FlowAcc ov = shfl_up_acc(val, o);
            if (lane >= (uint32_t)o) {
                if (!fl) acc_add(val, ov);
                fl |= ofl;
            }
        }
        uint32_t in_fl = __shfl_up(fl, 1);
        FlowAcc in = shfl_up_acc(val, 1);
        if (lane == 0) { in_fl = 0; in = acc_zero(); }
        // the source open at this lane's start ends at its first head
        if (nh > 0 && p0 > 0) {
            FlowAcc tot = in;
            acc_add(tot, F);
            if (in_fl) acc_store(out, g - 1, tot);
            else firstp[sub] = tot;   // started in an earlier tile
        }
        // ... and the source open at the lane end finishes here if the next packet
        // starts another source (inside the tile: the next lane handles it)
        if (lane == 63) {
            const uint32_t g_last = hb + hoff + nh - 1;
            if (fl) {
                if (next_head) acc_store(out, g_last, val);
                else {
                    lastp[sub] = val;
                    span_list[atomicAdd(&bs->n_span, 1u)] = g_last;
                }
            } else {
                firstp[sub] = val;    // no head in the tile: a middle / final piece
            }
        }
    }
}

#ifndef FSX_FLOW_TILE_BLOCKS
#define FSX_FLOW_TILE_BLOCKS 1024   // k_flow_tile grid cap: leaves CU slots to the walkers and classes beside it (2048: profiles/r04/ab_r04z.txt)
#endif
#ifndef FSX_FLOW_MINB
#define FSX_FLOW_MINB 4   // waves/SIMD bound of k_flow_tile (A/B: scripts/build_variant.sh)
#endif
__global__ __launch_bounds__(256, FSX_FLOW_MINB) void k_flow_tile(const uint64_t *__restrict__ S,
                                                   const uint64_t *__restrict__ pay, BatchState *bs,
                                                   const uint8_t *__restrict__ headf,
                                                   const uint32_t *__restrict__ len,
                                                   const uint64_t *__restrict__ ts,
                                                   PacketIn in,
                                                   const uint32_t *__restrict__ tile_off,
                                                   const uint32_t *__restrict__ sub_cnt,
                                                   const uint32_t *__restrict__ seg_start,
                                                   FlowAcc *__restrict__ firstp,
                                                   FlowAcc *__restrict__ lastp,
                                                   uint32_t *__restrict__ span_list, FlowOut out,
                                                   ScoreParams P, uint32_t salt, uint32_t light_only) {
    __shared__ unsigned long long s_S[4][64 * 17];
    if (bs->pay_ok)
        flow_tiles<true>(S, pay, bs, headf, len, ts, in, tile_off, sub_cnt, seg_start, firstp,
                         lastp, span_list, out, P, salt, s_S, light_only);
    else
        flow_tiles<false>(S, pay, bs, headf, len, ts, in, tile_off, sub_cnt, seg_start, firstp,
                          lastp, span_list, out, P, salt, s_S, light_only);
}

__global__ __launch_bounds__(256) void k_flow_combine(const uint64_t *__restrict__ S, BatchState *bs,
                                                      const uint32_t *__restrict__ seg_start,
                                                      const FlowAcc *__restrict__ firstp,
                                                      const FlowAcc *__restrict__ lastp,
                                                      const uint32_t *__restrict__ span_list,
                                                      PacketIn in,
                                                      const uint32_t *__restrict__ len, FlowOut out,
                                                      ScoreParams P, uint32_t salt) {
    const uint32_t lane = lane_id();
    const uint32_t ns = bs->n_span;
    for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < ns; i += gridDim.x * 4u) {
        const uint32_t g = span_list[i];
        const uint32_t s = seg_start[g], e = seg_start[g + 1];
        const uint32_t t0 = s / kFT, t1 = (e - 1) / kFT;
        // a heavy source spans thousands of tiles: four partials in flight per lane
        // (integer sums and max: any grouping gives the same result)
        FlowAcc a = acc_zero();
        uint32_t t = t0 + 1 + lane;
        for (; t + 192u <= t1; t += 256u) {
            FlowAcc b0 = firstp[t], b1 = firstp[t + 64u];
            const FlowAcc b2 = firstp[t + 128u], b3 = firstp[t + 192u];
            acc_add(b0, b2);
            acc_add(b1, b3);
            acc_add(a, b0);
            acc_add(a, b1);
        }
        for (; t <= t1; t += 64u) acc_add(a, firstp[t]);
        a = wave_sum_acc(a);
        if (lane == 0) {
            FlowAcc tot = lastp[t0];
            acc_add(tot, a);
            acc_store(out, g, tot);
        }
    }
}

// One thread per source: features from the exact sums, then the q8 score (kept out
// of the tile loop, where a source's end lands on arbitrary lanes).
__global__ __launch_bounds__(256) void k_flow_finish(const uint64_t *__restrict__ S, BatchState *bs,
                                                     const uint32_t *__restrict__ seg_start,
                                                     PacketIn in,
                                                     const uint32_t *__restrict__ len, FlowOut out,
                                                     ScoreParams P, uint32_t salt, uint32_t light_only) {
    const uint32_t ns = min(light_only ? bs->nseg_light : bs->nseg, out.cap);
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < ns; g += gridDim.x * 256u)
        flow_finish(g, out.acc[g], S, seg_start, in, len, salt, out, P);
}

hipError_t launch_flows(const uint64_t *S, const uint64_t *pay, BatchState *bs, const uint8_t *headf, const uint32_t *len,
                        const uint64_t *ts, const PacketIn &in, const uint32_t *tile_off,
                        const uint32_t *sub_cnt, const uint32_t *seg_start, void *firstp, void *lastp,
                        uint32_t *span_list, void *acc, uint8_t *keys16, uint8_t *fam, float *feat,
                        float *prob, uint8_t *dec, uint32_t cap, const ScoreParams &P, uint32_t salt,
                        uint32_t n, void *sacc, uint32_t epoch, const uint32_t *seg_slot, bool light_only,
                        const uint32_t *seg_lo, uint32_t *seg_len, const PartialOut &part, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const FlowOut out{(FlowAcc *)acc, keys16, fam, feat, prob, dec, cap, (SlotAcc *)sacc, epoch, seg_slot, ts,
                      seg_lo, seg_len, part};
    const uint32_t nsub = (n + kFT - 1) / kFT;
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(FSX_FLOW_TILE_BLOCKS, (nsub + 3) / 4));
    k_flow_tile<<<grid, 256, 0, st>>>(S, pay, bs, headf, len, ts, in, tile_off, sub_cnt, seg_start,
                                      (FlowAcc *)firstp, (FlowAcc *)lastp, span_list, out, P, salt,
                                      light_only ? 1u : 0u);
    k_flow_combine<<<256, 256, 0, st>>>(S, bs, seg_start, (const FlowAcc *)firstp,
                                        (const FlowAcc *)lastp, span_list, in, len, out, P, salt);
    const uint32_t gf = std::max<uint32_t>(1, std::min<uint32_t>(4096, (std::min(n, cap) + 255) / 256));
    k_flow_finish<<<gf, 256, 0, st>>>(S, bs, seg_start, in, len, out, P, salt, light_only ? 1u : 0u);
    return hipGetLastError();
}

// ------------------------------------------------------------------ heavy sources
// Heavy bucket h of pass 0 holds heavy source h's packets as one run [base0, +cnt0) of the
// final sorted arrays (passes >= 1 write only [0, n_light)). Chunk j of run h is item
// pre[h] + j; pre (computed by every block, written by block 0) and the per-chunk
// partials live in the context's heavy-flow scratch.
#ifndef FSX_HEAVY_CHUNK
#define FSX_HEAVY_CHUNK 8192   // positions per k_flow_heavy wave (A/B: scripts/build_variant.sh)
#endif
#ifndef FSX_HEAVY_FLOW_BLOCKS
#define FSX_HEAVY_FLOW_BLOCKS 1024
#endif
constexpr uint32_t kHeavyChunk = FSX_HEAVY_CHUNK;

__device__ __forceinline__ void heavy_chunk_prefix(const uint32_t *cnt0, uint32_t lb, uint32_t *s_pre,
                                                   uint32_t *s_tmp) {
    const uint32_t h = threadIdx.x;
    const uint32_t c = h < kHeavyMax ? (cnt0[lb + h] + kHeavyChunk - 1) / kHeavyChunk : 0u;
    uint32_t tot;
    const uint32_t e = block256_excl(c, s_tmp, &tot);
    if (h < kHeavyMax) s_pre[h] = e;
    if (h == 0) s_pre[kHeavyMax] = tot;
    __syncthreads();
}

template <class SV>
__device__ __forceinline__ void flow_heavy_body(const SV &sv, const uint32_t *cnt0, const uint32_t *base0,
                                                uint32_t lb, const uint32_t *s_pre, FlowAcc *part) {
    const uint32_t items = s_pre[kHeavyMax];
    for (uint32_t it = blockIdx.x * 4u + (threadIdx.x >> 6); it < items; it += gridDim.x * 4u) {
        uint32_t lo = 0, hi = kHeavyMax;   // the bucket h with pre[h] <= it < pre[h + 1]
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (s_pre[m] <= it) lo = m; else hi = m;
        }
        const uint32_t rs = base0[lb + lo], e = rs + cnt0[lb + lo];
        const uint32_t a = rs + (it - s_pre[lo]) * kHeavyChunk, b = min(e, a + kHeavyChunk);
        const FlowAcc A = flow_wave_acc(sv, rs, a, b);
        if (lane_id() == 0) part[it] = A;
    }
}

__global__ __launch_bounds__(256) void k_flow_heavy(const uint64_t *__restrict__ S, const uint64_t *__restrict__ pay,
                                                    const uint64_t *__restrict__ ts, const uint32_t *__restrict__ len,
                                                    const BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                    const uint32_t *__restrict__ base0, uint32_t *__restrict__ pre,
                                                    FlowAcc *__restrict__ part) {
    __shared__ uint32_t s_pre[kHeavyMax + 1];
    __shared__ uint32_t s_tmp[4];
    if (bs->err || bs->hfast) return;   // (hfast: k_hflow_combine)
    heavy_chunk_prefix(cnt0, bs->light_b, s_pre, s_tmp);
    if (blockIdx.x == 0 && threadIdx.x <= kHeavyMax) pre[threadIdx.x] = s_pre[threadIdx.x];
    if (bs->pay_ok) {
        const SegView<true> sv{S, ts, len, pay, ~bs->inv_min_ts};
        flow_heavy_body(sv, cnt0, base0, bs->light_b, s_pre, part);
    } else {
        const SegView<false> sv{S, ts, len, pay, 0};
        flow_heavy_body(sv, cnt0, base0, bs->light_b, s_pre, part);
    }
}

// One wave per heavy bucket: the sum of its chunks.
__global__ __launch_bounds__(256) void k_flow_heavy_sum(const BatchState *bs, const uint32_t *__restrict__ pre,
                                                        const FlowAcc *__restrict__ part, FlowAcc *__restrict__ hacc) {
    if (bs->err || bs->hfast) return;
    const uint32_t h = blockIdx.x * 4u + (threadIdx.x >> 6), lane = lane_id();
    if (h >= kHeavyMax) return;
    FlowAcc A = acc_zero();
    for (uint32_t it = pre[h] + lane; it < pre[h + 1]; it += 64) acc_add(A, part[it]);
    A = wave_sum_acc(A);
    if (lane == 0) hacc[h] = A;
}

// After the heads: heavy bucket h's row is segment nseg_light + (rank among the non-empty
// buckets), as k_heads_heavy numbered them.
__global__ __launch_bounds__(256) void k_flow_heavy_finish(const uint64_t *__restrict__ S, const BatchState *bs,
                                                           const uint32_t *__restrict__ cnt0,
                                                           const uint32_t *__restrict__ seg_start,
                                                           const FlowAcc *__restrict__ hacc, PacketIn in,
                                                           const uint32_t *__restrict__ len, FlowOut out,
                                                           ScoreParams P, uint32_t salt) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err || bs->hfast) return;   // (hfast: k_hflow_finish)
    const uint32_t h = threadIdx.x;
    const bool live = h < kHeavyMax && cnt0[bs->light_b + h] > 0;
    const uint32_t r = block256_excl(live ? 1u : 0u, s_tmp, nullptr);
    if (live) flow_finish(bs->nseg_light + r, hacc[h], S, seg_start, in, len, salt, out, P);
}

size_t heavy_flow_bytes(uint64_t cap) {
    return (cap / kHeavyChunk + kHeavyMax + 1) * sizeof(FlowAcc) + kHeavyMax * sizeof(FlowAcc) +
           (kHeavyMax + 1) * 4;
}

// The heavy runs' sums (right after sort pass 0): part = scratch of heavy_flow_bytes(cap).
hipError_t launch_flows_heavy(const uint64_t *S, const uint64_t *pay, const uint64_t *ts, const uint32_t *len,
                              const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, void *scratch,
                              uint64_t cap, hipStream_t st) {
    (void)hipGetLastError();
    FlowAcc *part = reinterpret_cast<FlowAcc *>(scratch);
    FlowAcc *hacc = part + (cap / kHeavyChunk + kHeavyMax + 1);
    uint32_t *pre = reinterpret_cast<uint32_t *>(hacc + kHeavyMax);
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(FSX_HEAVY_FLOW_BLOCKS, (cap / kHeavyChunk + kHeavyMax + 3) / 4));
    k_flow_heavy<<<grid, 256, 0, st>>>(S, pay, ts, len, bs, cnt0, base0, pre, part);
    k_flow_heavy_sum<<<kHeavyMax / 4, 256, 0, st>>>(bs, pre, part, hacc);
    return hipGetLastError();
}

// The heavy sources' rows (after k_heads_heavy).
hipError_t launch_flows_heavy_finish(const uint64_t *S, const BatchState *bs, const uint32_t *cnt0,
                                     const uint32_t *seg_start, const PacketIn &in, const uint32_t *len,
                                     const uint64_t *ts, void *scratch, uint64_t cap, uint8_t *keys16, uint8_t *fam,
                                     float *feat, float *prob, uint8_t *dec, uint32_t rows_cap,
                                     const ScoreParams &P, uint32_t salt, void *sacc, uint32_t epoch,
                                     const uint32_t *seg_slot, hipStream_t st) {
    (void)hipGetLastError();
    const FlowAcc *hacc = reinterpret_cast<const FlowAcc *>(scratch) + (cap / kHeavyChunk + kHeavyMax + 1);
    const FlowOut out{nullptr, keys16, fam, feat, prob, dec, rows_cap, (SlotAcc *)sacc, epoch, seg_slot, ts,
                      nullptr, nullptr};
    k_flow_heavy_finish<<<1, 256, 0, st>>>(S, bs, cnt0, seg_start, hacc, in, len, out, P, salt);
    return hipGetLastError();
}

size_t flow_acc_bytes() { return sizeof(FlowAcc); }
size_t slot_acc_bytes() { return sizeof(SlotAcc); }

// The rows of an accumulation epoch: every live slot merged in it, features + score from the
// carried sums. Rows are unordered (a row counter): when cap < rows, which rows are kept is
// unspecified (include/fsx_hip.h fsx_flows_end).
__global__ __launch_bounds__(256) void k_flows_end(const SlotAcc *__restrict__ sacc, uint32_t epoch,
                                                   const Slot *__restrict__ table, uint64_t slots, uint32_t tgen,
                                                   FlowOut out, ScoreParams P,
                                                   unsigned long long *count) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256u + threadIdx.x; s < slots; s += (uint64_t)gridDim.x * 256u) {
        const SlotAcc &m = sacc[s];
        if (m.epoch != epoch) continue;
        const uint32_t fam = slot_fam(table[s].tag, tgen);
        if (fam == 0) continue;   // emptied by a rolled-back sub-batch
        const unsigned long long g = atomicAdd(count, 1ull);
        if (g >= out.cap) continue;
        FlowAcc a = acc_zero();
        a.n = m.n; a.s1 = m.s1; a.s2 = m.s2; a.d1 = m.d1; a.d2 = m.d2; a.dmax = m.dmax;
        const Slot &sl = table[s];
        write_row((uint32_t)g, a, fam, sl.key, m.dport, out, P);
    }
}

// Accumulate mode: partial i of m (distinct sources) merges into its source's SlotAcc of the
// epoch as the call after everything merged so far (the flow_finish merge, with the partial's
// own first / last timestamps); a source absent from the table is skipped.
__global__ __launch_bounds__(256) void k_flows_merge(const FlowPartial *__restrict__ part, uint32_t m0,
                                                     const unsigned long long *__restrict__ d_m,
                                                     const Slot *__restrict__ table, Limits lim, SlotAcc *sacc,
                                                     uint32_t epoch) {
    // (d_m: the count on the device, at most m0: a fixed-capacity exchange block)
    const uint32_t m = d_m ? (uint32_t)(*d_m < m0 ? *d_m : m0) : m0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < m; i += gridDim.x * 256u) {
        const FlowPartial p = part[i];
        const uint32_t s = table_find(table, lim, p.tag, p.key);
        if (s == kNoSlot || p.n == 0) continue;
        SlotAcc &a = sacc[s];
        if (a.epoch != epoch) {
            a.n = p.n; a.s1 = p.s1; a.s2 = p.s2; a.d1 = p.d1; a.d2 = p.d2; a.dmax = p.dmax;
            a.dport = p.dport;
            a.epoch = epoch;
        } else {
            const uint64_t d = p.first_ts - a.last_t;
            a.n += p.n; a.s1 += p.s1; a.s2 += p.s2;
            a.d1 += p.d1 + (u128)d;
            a.d2 += p.d2 + (u128)d * d;
            const uint64_t mx = p.dmax > d ? p.dmax : d;
            a.dmax = mx > a.dmax ? mx : a.dmax;
        }
        a.last_t = p.last_ts;
    }
}

hipError_t launch_flows_merge(const void *partials, uint32_t m, const Slot *table, const Limits &lim, void *sacc,
                              uint32_t epoch, hipStream_t st, const uint64_t *d_m) {
    (void)hipGetLastError();
    if (m == 0) return hipSuccess;
    k_flows_merge<<<std::min<uint32_t>(1024, (m + 255) / 256), 256, 0, st>>>(
        static_cast<const FlowPartial *>(partials), m, reinterpret_cast<const unsigned long long *>(d_m), table, lim,
        static_cast<SlotAcc *>(sacc), epoch);
    return hipGetLastError();
}

hipError_t launch_flows_end(const void *sacc, uint32_t epoch, const Slot *table, uint64_t slots, uint32_t tgen,
                            uint8_t *keys16, uint8_t *fam, float *feat, float *prob, uint8_t *dec,
                            uint32_t cap, const ScoreParams &P, unsigned long long *d_count,
                            hipStream_t st) {
    (void)hipGetLastError();
    const FlowOut out{nullptr, keys16, fam, feat, prob, dec, cap, nullptr, epoch, nullptr, nullptr};
    hipError_t e = hipMemsetAsync(d_count, 0, 8, st);
    if (e != hipSuccess) return e;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, (slots + 255) / 256);
    k_flows_end<<<grid, 256, 0, st>>>((const SlotAcc *)sacc, epoch, table, slots, tgen, out, P, d_count);
    return hipGetLastError();
}

}  // namespace fsx
