// fsx_bins.hip — the light sources' tail of a fixed-window batch, one pass over slot bins
// (DESIGN.md §3 "Light bins").
//
// With the heavy-source sort (tables of 2^17..2^21 slots) sort passes 0 and 1 leave the
// light entries ordered by the low `binbits` bits of their source's table slot: a bin is
// the run of one value of those bits, in arrival order, and holds at most 64 sources (the
// slots bin + k * 2^binbits, k < 64). One wave per bin then does what the third sort pass,
// the segment heads, the walkers, the flow tiles and the verdict fill did over the whole
// light array:
//   k_bin_bounds  bin starts in the pass-1 output (one compare per position)
//   k_bin_order   bins of more than one chunk first
//   k_bin_tail    per bin, one block of four waves, in LDS chunks of kBinCap entries: a
//                 stable counting sort by k (lane k owns slot bin + k * 2^binbits), the fixed
//                 window of src/fsx_kern.c:150-346 (lane k replays its source, or walks it by
//                 epoch jumps when it is long), the flow sums on another wave;
//                 DROP bytes go straight to the verdict array, the final state to the table
//                 slot, the sums to a per-slot stage (rows) or the epoch's SlotAcc
//                 (accumulate mode)
//   k_bin_scan    row numbering: sources per bin, exclusive scan -> bs->nseg (light)
//   k_bin_rows    features + q8 score of every light source, rows in (bin, k) order
// The walkers and the flow sums are the same functions as the tile kernels' (fsx_walk.h,
// fsx_flow_common.h) on an LDS accessor, so the results are those of the sequential
// program whatever the binning.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fsx_bins.h"
#include "fsx_dev_common.h"
#include "fsx_flow_common.h"
#include "fsx_walk.h"

namespace fsx {

#ifndef FSX_BIN_CAP
#define FSX_BIN_CAP 2048   // entries per LDS chunk of a bin (A/B: scripts/build_variant.sh)
#endif
#ifndef FSX_BIN_EXACT
#define FSX_BIN_EXACT 32       // a source with more entries in a chunk is walked by epoch jumps
#endif
#ifndef FSX_BIN_FLOW_LONG
#define FSX_BIN_FLOW_LONG 64   // ... and its flow sums taken by a whole wave
#endif
constexpr uint32_t kBinCap = FSX_BIN_CAP;
constexpr uint32_t kBinItems = kBinCap / 64;   // entries per lane and chunk
constexpr uint32_t kBinExact = FSX_BIN_EXACT;
constexpr uint32_t kBinFlowLong = FSX_BIN_FLOW_LONG;
static_assert(kBinCap % 64 == 0, "whole wave rounds");

// Per-bin phase times for scripts/bin_profile.py (a measurement build, -DFSX_BIN_PROFILE:
// never the product): {bin, entries, start, count, place, walk, long, end} per block, in
// s_memrealtime ticks (100 MHz), appended to $FSX_BIN_PROFILE_OUT after each batch.
#ifdef FSX_BIN_PROFILE
__device__ unsigned long long *g_bin_prof;
#define BIN_T() __builtin_amdgcn_s_memrealtime()
#endif

// The chunk's entries in LDS, ordered by k (stable): the payload word (kPay: relative ts
// << kPayLenBits | len; else the absolute timestamp, the length gathered by arrival index)
// and the low sort word (family << 31 | arrival index).
template <bool kPay>
struct BinSV {
    const uint64_t *w;
    const uint32_t *lo;
    const uint32_t *len;
    uint64_t tbase;
    __device__ __forceinline__ uint64_t t(uint32_t q) const {
        if constexpr (kPay) return tbase + (w[q] >> kPayLenBits);
        else return w[q];
    }
    __device__ __forceinline__ uint32_t l(uint32_t q) const {
        if constexpr (kPay) return (uint32_t)w[q] & ((1u << kPayLenBits) - 1u);
        else return len[pk_idx(lo[q])];
    }
    __device__ __forceinline__ void tl(uint32_t q, uint64_t &T, uint32_t &L) const {
        T = t(q);
        L = l(q);
    }
};

// Lanes of `act` whose 6-bit value equals mine.
__device__ __forceinline__ uint64_t match6(uint32_t k, uint64_t act) {
    uint64_t peers = act;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        const bool bit = (k >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// bin starts: bin_start[b] = first light position whose bin is >= b (b <= nbins). Thread
// t of the grid-stride loop covers 8 consecutive positions (two 32-byte loads), the
// position before them through the lane below.
__global__ __launch_bounds__(256) void k_bin_bounds(const uint64_t *__restrict__ S, const BatchState *bs,
                                                    uint32_t *__restrict__ bin_start, uint32_t bmask,
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
                bn[2 * k] = (uint32_t)(x.x >> 32) & bmask;
                bn[2 * k + 1] = (uint32_t)(x.y >> 32) & bmask;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) bn[k] = p0 + k < M ? (uint32_t)(S[p0 + k] >> 32) & bmask : nbins;
        }
        int64_t prev = (int64_t)__shfl_up(bn[7], 1);
        if (lane == 0) prev = p0 == 0 ? -1 : (p0 - 1 < M ? (int64_t)((uint32_t)(S[p0 - 1] >> 32) & bmask) : nbins);
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

// Bins of more than one chunk first (a bin's chunks run in order on one wave: started
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
    for (uint32_t b = tid; b < nbins; b += 1024) {
        const bool g = bin_start[b + 1] - bin_start[b] > kBinCap;
        const uint64_t m = __ballot(g);
        const uint32_t lane = lane_id(), below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint32_t nbg = (uint32_t)__popcll(m), nsm = (uint32_t)__popcll(__ballot(true)) - nbg;
        uint32_t bb = 0, bs_ = 0;
        if (lane == 0) {
            if (nbg) bb = atomicAdd(&s_nb, nbg);
            if (nsm) bs_ = atomicAdd(&s_ns, nsm);
        }
        bb = __shfl(bb, 0);
        bs_ = __shfl(bs_, 0);
        if (g) bin_order[bb + below] = b;
        else bin_order[nbig + bs_ + (lane - below)] = b;
    }
}

// The verdicts of a lane's own source, straight from the exact replay (one emit per
// packet): DROP bytes to the arrival index, PASS / DROP counts.
struct DirectWriter {
    uint8_t *verdict;
    const uint32_t *lo;   // LDS: low sort word per sorted position
    uint64_t npass, ndrop;
    __device__ __forceinline__ void emit(uint32_t q, uint8_t v) {
        if (v == XDP_DROP) {
            ++ndrop;
            verdict[pk_idx(lo[q])] = XDP_DROP;
        } else {
            ++npass;
        }
    }
};

// The verdicts of an epoch-jump walk from its verdict-change emits: a DROP run's bytes are
// stored when the run closes (by the whole wave for a wave walk), PASS runs are only
// counted (no marks, no fill pass).
template <bool kWave>
struct RunWriter {
    uint8_t *verdict;
    const uint32_t *lo;   // LDS: low sort word per sorted position
    uint8_t last;
    uint32_t last_pos;
    uint64_t npass, ndrop;   // a wave walk: counted in lane 0
    __device__ __forceinline__ void close(uint32_t end) {
        const uint32_t n = end - last_pos;
        if (last == XDP_DROP) {
            for (uint32_t q = last_pos + (kWave ? lane_id() : 0u); q < end; q += kWave ? 64u : 1u)
                verdict[pk_idx(lo[q])] = XDP_DROP;
        }
        if (!kWave || lane_id() == 0) {
            ndrop += last == XDP_DROP ? n : 0u;
            npass += last == XDP_PASS ? n : 0u;
        }
        last_pos = end;
    }
    __device__ __forceinline__ void emit(uint32_t pos, uint8_t v) {
        if (v == last) return;
        close(pos);
        last = v;
    }
};

// Per-bin LDS of k_bin_tail: the chunk sorted by k, the per-wave digit counts / cursors.
struct BinLds {
    uint64_t w[kBinCap];      // payload word (kPay) or absolute timestamp
    uint32_t lo[kBinCap];     // low sort word: family << 31 | arrival index
    uint32_t wc[4][64];       // entries per (wave, k), then the wave's cursors
    FlowAcc fl[64];           // flow sums of source k's long run in the chunk (waves 1-3)
    uint64_t fl_t[64][2];     // its first / last timestamp
};

// One block of four waves per bin (DESIGN.md §3 "Light bins"). Per chunk of kBinCap
// entries: wave w loads and ranks its quarter (all loads in flight at once), the chunk is
// placed in LDS ordered by k (stable: waves in order, rounds in order, lanes in order);
// then wave 0 walks the fixed window (lane k: source k of the bin; exact replay, or epoch
// jumps for more than kBinExact entries) while wave 1 sums the flow features of the same
// sources (runs of more than kBinFlowLong entries: one of waves 1-3 each). Lane k of wave 0 carries source k's limiter state
// and verdict counts across chunks, lane k of wave 1 its flow sums.
template <bool kPay, bool kFlows>
__device__ __forceinline__ void bin_tail(const BinTail &A, BinLds &L) {
    BatchState *bs = A.bs;
    const uint32_t b = A.bin_order[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const uint32_t lo = A.bin_start[b], hi = A.bin_start[b + 1];
    if (lo >= hi) {
        if (tid == 0) A.bin_mask[b] = 0;
        return;
    }
    const Limits &lim = A.lim;
    const uint32_t idm = (uint32_t)lim.table_mask, bb = A.binbits;
    const uint32_t slot = b | (lane << bb);
    const uint64_t tbase = ~bs->inv_min_ts;
    const uint64_t lt = (1ull << lane) - 1ull;
    const BinSV<kPay> sv{L.w, L.lo, A.len, tbase};
    const uint64_t *__restrict__ S = A.S;
    const uint64_t *__restrict__ pay = A.pay;
    auto kof = [&](uint64_t v) { return ((uint32_t)(v >> 32) & idm) >> bb; };
    constexpr uint32_t kQ = kBinCap / 4, kR = kQ / 64;   // entries / rounds per wave and chunk
    // wave 0: limiter state + verdict counts; wave 1: flow sums (lane k: source k)
    bool present = false;
    FwState st{};
    DirectWriter dw{A.verdict, L.lo, 0, 0};
    FlowAcc fa = acc_zero();
    uint64_t first_t = 0, last_t = 0;
    uint32_t first_lo = 0;
    const bool glob_fast = fast_ok(bs, lim);
    const uint32_t maxL = bs->max_len;
#ifdef FSX_BIN_PROFILE
    uint64_t pt[6] = {BIN_T(), 0, 0, 0, 0, 0};
    uint64_t tp = pt[0];
    auto ph = [&](int i) { const uint64_t t = BIN_T(); pt[i] += t - tp; tp = t; };
#else
    auto ph = [](int) {};
#endif
    for (uint32_t c0 = lo; c0 < hi; c0 += kBinCap) {
        const uint32_t m = min(kBinCap, hi - c0);
        const uint32_t q0 = wv * kQ;   // this wave's quarter of the chunk: [q0, q0 + kQ)
        uint64_t v[kR], pw[kR];
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = q0 + r * 64u + lane;
            v[r] = j < m ? S[c0 + j] : 0ull;
        }
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = q0 + r * 64u + lane;
            if constexpr (kPay) pw[r] = j < m ? pay[c0 + j] : 0ull;
            else pw[r] = j < m ? A.ts[pk_idx(v[r])] : 0ull;
        }
        // entries per (wave, k) (a round of one source: one add)
        L.wc[wv][lane] = 0;
        wave_lds_order();
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = q0 + r * 64u + lane;
            const bool ok = j < m;
            const uint64_t act = __ballot(ok);
            if (!act) break;
            const uint32_t k = kof(v[r]);
            const uint32_t kl = __builtin_amdgcn_readfirstlane(k);
            if (__ballot(ok && k == kl) == act) {
                if (lane == 0) atomicAdd(&L.wc[wv][kl], (uint32_t)__popcll(act));
            } else if (ok) {
                atomicAdd(&L.wc[wv][k], 1u);
            }
        }
        __syncthreads();
        // k's entries of the chunk and of the waves before mine -> my cursor for k = lane
        const uint32_t c_0 = L.wc[0][lane], c_1 = L.wc[1][lane], c_2 = L.wc[2][lane], c_3 = L.wc[3][lane];
        const uint32_t cnt = c_0 + c_1 + c_2 + c_3;
        const uint32_t a = wave_incl_sum(cnt) - cnt;   // source k's entries: [a, a + cnt)
        const uint32_t before = (wv > 0 ? c_0 : 0u) + (wv > 1 ? c_1 : 0u) + (wv > 2 ? c_2 : 0u);
        __syncthreads();
        L.wc[wv][lane] = a + before;
        wave_lds_order();
        ph(1);
        // stable placement by k: my rounds in order, lanes in order inside a round
#pragma unroll
        for (uint32_t r = 0; r < kR; ++r) {
            const uint32_t j = q0 + r * 64u + lane;
            const bool ok = j < m;
            const uint64_t act = __ballot(ok);
            if (!act) break;
            const uint32_t k = kof(v[r]);
            const uint32_t kl = __builtin_amdgcn_readfirstlane(k);
            const uint64_t peers = __ballot(ok && k == kl) == act ? act : match6(k, act);
            const uint32_t below = (uint32_t)__popcll(peers & lt);
            const uint32_t base = L.wc[wv][k];
            wave_lds_order();
            if (ok && below == 0) L.wc[wv][k] = base + (uint32_t)__popcll(peers);
            wave_lds_order();
            if (ok) {
                const uint32_t p = base + below;
                L.w[p] = pw[r];
                L.lo[p] = (uint32_t)v[r];
            }
        }
        __syncthreads();
        ph(2);
        if (wv == 0) {
            // fixed window, lane k: source k of the bin. Up to kBinExact entries (or clocks
            // the epoch jumps cannot take): exact replay, 4 entries' LDS reads ahead; longer
            // runs: epoch jumps on the lane (a light source's windows, not its packets)
            if (cnt && !present) {   // the source's first entry of the batch
                present = true;
                st = load_state(A.table[slot]);
            }
            const bool fast = cnt > kBinExact && glob_fast &&
                              (!st.has_st || (st.tt <= ~0ull - lim.window && st.pps < kBig && st.bps < kBig));
            if (fast) {
                RunWriter<false> rw{A.verdict, L.lo, 0, a, 0, 0};
                walk_fixed_fast<false>(sv, a, a + cnt, lim, maxL, rw, st);
                rw.close(a + cnt);
                dw.npass += rw.npass;
                dw.ndrop += rw.ndrop;
            } else if (cnt) {
                const uint32_t e = a + cnt;
                for (uint32_t q = a; q < e; q += 4) {
                    uint64_t T[4];
                    uint32_t Ln[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (q + i < e) sv.tl(q + i, T[i], Ln[i]);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (q + i < e) fw_step(st, T[i], Ln[i], q + i, lim, dw);
                }
            }
        } else if (kFlows) {
            // flow sums. Wave 1, lane k: source k's run when it is short (sequential); the
            // runs longer than kBinFlowLong: one wave each among waves 1-3 (their parts go
            // through LDS to lane k of wave 1 after the barrier)
            if (wv == 1) {
                if (cnt && !present) {
                    present = true;
                    first_lo = L.lo[a];
                    first_t = sv.t(a);
                }
                if (cnt && cnt <= kBinFlowLong) {
                    const uint32_t e = a + cnt;
                    for (uint32_t q = a; q < e; q += 4) {
                        uint64_t T[4];
                        uint32_t Ln[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (q + i < e) sv.tl(q + i, T[i], Ln[i]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            if (q + i >= e) continue;
                            fa.s1 += Ln[i];
                            fa.s2 += (u128)Ln[i] * Ln[i];
                            if (fa.n) {
                                const uint64_t d = T[i] - last_t;
                                fa.d1 += d;
                                fa.d2 += (u128)d * d;
                                fa.dmax = d > fa.dmax ? d : fa.dmax;
                            }
                            fa.n += 1;
                            last_t = T[i];
                        }
                    }
                }
            }
            uint32_t i = 0;
            for (uint64_t lm = __ballot(cnt > kBinFlowLong); lm; lm &= lm - 1, ++i) {
                if (i % 3u != wv - 1u) continue;
                const int src = __ffsll((unsigned long long)lm) - 1;
                const uint32_t la = __builtin_amdgcn_readlane(a, src), lc = __builtin_amdgcn_readlane(cnt, src);
                const FlowAcc wa = flow_wave_acc(sv, la, la, la + lc);
                if (lane == 0) {
                    L.fl[src] = wa;
                    L.fl_t[src][0] = sv.t(la);
                    L.fl_t[src][1] = sv.t(la + lc - 1);
                }
            }
        }
        ph(3);
        __syncthreads();
        if (kFlows && wv == 1 && cnt > kBinFlowLong) {   // the long runs' parts, in order
            FlowAcc wa = L.fl[lane];
            if (fa.n) {
                const uint64_t d = L.fl_t[lane][0] - last_t;
                wa.d1 += d;
                wa.d2 += (u128)d * d;
                wa.dmax = d > wa.dmax ? d : wa.dmax;
            }
            acc_add(fa, wa);
            last_t = L.fl_t[lane][1];
        }
        ph(4);
    }
    if (wv == 0) {
        if (present) store_state(A.table[slot], st);
        const uint64_t pm = __ballot(present);
        const uint64_t npass = wave_sum(dw.npass), ndrop = wave_sum(dw.ndrop);
#ifdef FSX_BIN_PROFILE
        if (lane == 0 && g_bin_prof) {
            unsigned long long *o = g_bin_prof + (size_t)blockIdx.x * 8;
            o[0] = b; o[1] = hi - lo; o[2] = pt[0]; o[3] = pt[1]; o[4] = pt[2]; o[5] = pt[3]; o[6] = pt[4];
            o[7] = BIN_T();
        }
#endif
        if (lane == 0) {
            A.bin_mask[b] = pm;
            unsigned long long *stt = reinterpret_cast<unsigned long long *>(A.tstate->stats);
            if (npass) {
                atomicAdd(stt, (unsigned long long)npass);
                atomicAdd(reinterpret_cast<unsigned long long *>(&bs->allowed), (unsigned long long)npass);
            }
            if (ndrop) {
                atomicAdd(stt + 1, (unsigned long long)ndrop);
                atomicAdd(reinterpret_cast<unsigned long long *>(&bs->dropped), (unsigned long long)ndrop);
            }
        }
    } else if (kFlows && wv == 1 && present) {
        fa.pad = first_lo;
        if (A.sacc) {   // accumulate mode: merge into the epoch's per-slot sums (as flow_finish)
            const uint32_t idx = pk_idx(first_lo);
            uint32_t dport;
            if (A.in.rec) {
                uint32_t k[4], Lr;
                uint64_t Tr;
                rec_read(A.in.rec, A.in.rec_bytes, idx, k, Lr, Tr, dport);
            } else {
                dport = dst_port(A.in.hdr + (size_t)idx * 64, A.len[idx]);
            }
            SlotAcc &mm = static_cast<SlotAcc *>(A.sacc)[slot];
            if (mm.epoch != A.epoch) {
                mm.n = fa.n; mm.s1 = fa.s1; mm.s2 = fa.s2; mm.d1 = fa.d1; mm.d2 = fa.d2; mm.dmax = fa.dmax;
                mm.dport = dport;
                mm.epoch = A.epoch;
            } else {
                const uint64_t d = first_t - mm.last_t;
                mm.n += fa.n; mm.s1 += fa.s1; mm.s2 += fa.s2;
                mm.d1 += fa.d1 + (u128)d;
                mm.d2 += fa.d2 + (u128)d * d;
                const uint64_t mx = fa.dmax > d ? fa.dmax : d;
                mm.dmax = mx > mm.dmax ? mx : mm.dmax;
            }
            mm.last_t = last_t;
        } else {
            static_cast<FlowAcc *>(A.stage)[slot] = fa;
        }
    }
}

template <bool kFlows>
__global__ __launch_bounds__(256) void k_bin_tail(BinTail A) {
    __shared__ BinLds L;
    if (A.bs->err) return;
    if (A.bs->pay_ok) bin_tail<true, kFlows>(A, L);
    else bin_tail<false, kFlows>(A, L);
}

// Sources per bin -> exclusive row bases; bs->nseg = light sources (k_heads_heavy appends
// the heavy ones after them).
__global__ __launch_bounds__(256) void k_bin_scan(const uint64_t *__restrict__ bin_mask, uint32_t *__restrict__ bin_row,
                                                  uint32_t nbins, BatchState *bs) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nbins; c0 += 1024) {
        const uint32_t i = c0 + threadIdx.x * 4u;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = i + k < nbins ? (uint32_t)__popcll(bin_mask[i + k]) : 0u;
        uint32_t tot;
        uint32_t off = carry + block256_excl(x[0] + x[1] + x[2] + x[3], s_tmp, &tot);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < nbins) { bin_row[i + k] = off; off += x[k]; }
        carry += tot;
    }
    if (threadIdx.x == 0) bs->nseg = carry;
}

// One wave per bin, lane k: the row of source bin + k * 2^binbits (features + q8 score).
__global__ __launch_bounds__(256) void k_bin_rows(const uint64_t *__restrict__ bin_mask,
                                                  const uint32_t *__restrict__ bin_row,
                                                  const FlowAcc *__restrict__ stage, uint32_t nbins,
                                                  uint32_t binbits, PacketIn in, const uint32_t *__restrict__ len,
                                                  FlowOut out, ScoreParams P, uint32_t salt, const BatchState *bs) {
    if (bs->err) return;
    const uint32_t lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t b = blockIdx.x * 4u + (threadIdx.x >> 6); b < nbins; b += gridDim.x * 4u) {
        const uint64_t mask = bin_mask[b];
        if (!((mask >> lane) & 1ull)) continue;
        const uint32_t g = bin_row[b] + (uint32_t)__popcll(mask & lt);
        if (g >= out.cap) continue;
        const FlowAcc a = stage[b | (lane << binbits)];
        const uint32_t lo = (uint32_t)a.pad, idx = pk_idx(lo);
        uint32_t k[4], tag, dport;
        if (in.rec) {
            uint32_t L;
            uint64_t T;
            tag = rec_read(in.rec, in.rec_bytes, idx, k, L, T, dport);
        } else {
            tag = key_of((uint64_t)lo, in.hdr, salt, k);
            dport = dst_port(in.hdr + (size_t)idx * 64, len[idx]);
        }
        write_row(g, a, tag, k, dport, out, P);
    }
}

static inline uint32_t cdiv32(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_bins(const BinTail &A, uint32_t n, const FlowRequest *fq, uint32_t salt, hipStream_t st,
                       const Marker &mark) {
    (void)hipGetLastError();
    const uint32_t nbins = 1u << A.binbits;
    k_bin_bounds<<<std::max<uint32_t>(1, std::min<uint32_t>(4096, cdiv32((uint64_t)n + 1, 256))), 256, 0, st>>>(
        A.S, A.bs, A.bin_start, nbins - 1u, nbins);
    k_bin_order<<<1, 1024, 0, st>>>(A.bin_start, nbins, A.bin_order, A.bs);
    mark("k_bin_bounds");
#ifdef FSX_BIN_PROFILE
    static unsigned long long *d_prof = nullptr;
    if (!d_prof) {
        (void)hipMalloc(&d_prof, (size_t)nbins * 64);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bin_prof), &d_prof, sizeof(d_prof));
    }
    (void)hipMemsetAsync(d_prof, 0, (size_t)nbins * 64, st);
#endif
    if (fq) k_bin_tail<true><<<nbins, 256, 0, st>>>(A);
    else k_bin_tail<false><<<nbins, 256, 0, st>>>(A);
    mark("k_bin_tail");
#ifdef FSX_BIN_PROFILE
    if (const char *path = getenv("FSX_BIN_PROFILE_OUT")) {
        std::vector<unsigned long long> h((size_t)nbins * 8);
        (void)hipStreamSynchronize(st);
        (void)hipMemcpy(h.data(), d_prof, h.size() * 8, hipMemcpyDeviceToHost);
        if (FILE *fp = fopen(path, "ab")) {
            fwrite(h.data(), 8, h.size(), fp);
            fclose(fp);
        }
    }
#endif
    k_bin_scan<<<1, 256, 0, st>>>(A.bin_mask, A.bin_row, nbins, A.bs);
    mark("k_bin_scan");
    if (fq && !A.sacc) {
        const FlowOut out{nullptr, fq->keys16, fq->fam, fq->feat, fq->prob, fq->dec, fq->cap, nullptr, 0,
                          nullptr, A.ts, nullptr, nullptr};
        k_bin_rows<<<std::min<uint32_t>(4096, cdiv32(nbins, 4)), 256, 0, st>>>(
            A.bin_mask, A.bin_row, static_cast<const FlowAcc *>(A.stage), nbins, A.binbits, A.in, A.len, out,
            fq->score, salt, A.bs);
        mark("k_bin_rows");
    }
    return hipGetLastError();
}

size_t bin_stage_bytes(uint64_t slots) { return slots * sizeof(FlowAcc); }

}  // namespace fsx
