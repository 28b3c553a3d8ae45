// fsx_device.hip — gfx950 kernels of the packet-verdict hot path.
//
// Pipeline for one batch of n packets, all on one HIP stream:
//   k_parse          header records -> packed sort word per IP packet
//                    (src/parsing_helper.h:49-136 + src/fsx_kern.c:123-148)
//   k_sort_* x4      stable LSD radix sort (8-bit digits) of the packed words by
//                    the 32-bit source key: per-source segments in arrival order
//   k_v6_mixed/fixup exact separation of IPv6 hash collisions (IPv4 keys are a
//                    bijection of the address and never collide)
//   k_heads_*        ordered compaction of segment starts
//   k_batch_check    new sources must fit max_entries (else the batch is rolled back)
//   k_walk_fixed     the fixed-window limiter + blacklist of src/fsx_kern.c:150-346
//                    evaluated per segment by epoch jumps (binary searches on the
//                    segment's timestamps), writing verdict change marks
//   k_fill_*         fill-forward of the marks, scatter of verdicts to arrival
//                    order, stats_map counters (src/fsx_kern.c:210,332,342)
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "fsx_dev_common.h"
#include "fsx_plan.h"
#include "fsx_internal.h"
#include "fsx_seg.h"
#include "fsx_walk.h"
#include "fsx_shard.h"

#define XDP_DROP 1
#define XDP_PASS 2

// Phase timestamps for the standalone micro-benchmarks (scripts/micro/): compiled in
// only when the including translation unit defines FSX_MICRO_STAMPS.
#ifdef FSX_MICRO_STAMPS
__device__ unsigned long long *g_fsx_stamps;
#define FSX_STAMP(tile, k)                                                                 \
    do {                                                                                   \
        if (threadIdx.x == 0) g_fsx_stamps[(size_t)(tile) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define FSX_STAMP(tile, k) \
    do {                   \
    } while (0)
#endif

namespace fsx {

// ------------------------------------------------------------------ per-batch source ids
// Every IP source of a batch gets a dense id: its slot in an open-addressing table of
// table_mask + 1 slots: a 64-bit head {generation 16 | state 8 | tag 8 | key word 0}
// (8 bytes: IPv4 probes stay dense in L2) and, in a parallel array, IPv6 key words
// 1..3. Slots of older generations are empty, so the table is never cleared. IPv4 keys are published by one 64-bit CAS; IPv6 slots are claimed
// BUSY, their key words stored at agent scope, then published READY (release). Other
// XCDs' L2s are not coherent with each other, so every head and IPv6 key word is read
// with an agent-scope (coherent) load; a stale line would otherwise force a CAS on
// every packet of a hot source until it is evicted.
constexpr uint64_t kIdBusy = 1, kIdReady = 2;
constexpr uint32_t kIdSpin = 1u << 22;

__device__ __forceinline__ uint64_t id_head(uint32_t gen, uint64_t state, uint32_t tag, uint32_t k0) {
    return ((uint64_t)gen << 48) | (state << 40) | ((uint64_t)tag << 32) | k0;
}

struct IdTable {
    unsigned long long *head;   // [slots]
    uint32_t *k6;               // [slots][4]: IPv6 key words 1..3
    uint64_t mask;
    uint64_t seed;              // probe_start() seed (the table's, for the persistent index)
    uint32_t gen;               // generation (per batch) or epoch (persistent index)
    uint32_t test_flags;
    Slot *slots;                // persistent index: a new source also gets its Slot here
    uint32_t born;              // ... stamped with this batch generation (rollback)
    uint32_t coherent;          // first probe with an agent-scope load (A/B: FSX_ID_COHERENT)
    void *mir = nullptr;        // persistent index: IPv4 mirror (mir_entry), null when off
    uint32_t mir_shift = 0;     // log2(slots)
    // 0: a new source's Slot is left to its walker (the fixed window's k_parse: one random
    // line per insert, the head's; SlotKeys)
    uint32_t init = 1;
    uint32_t tgen = 0;          // the table generation its new slots are tagged with (Limits::tgen)
};

__device__ __forceinline__ uint64_t id_start(const IdTable &T, uint32_t tag, const uint32_t k[4]) {
    return probe_start(tag, k, T.seed, T.mask, T.test_flags);
}

// Slot of (tag, key), inserted if absent (*fresh = true); kNoSlot when the table is full
// or a publication never completes (reported as a full table). h = id_start(...),
// hint0 = a plain load of T.head[h] issued earlier.
// kMirPub false: the caller knows the table has no mirror (k_parse's head-probe variant).
template <bool kMirPub = true>
__device__ __forceinline__ uint32_t id_resolve(const IdTable &T, uint32_t tag, const uint32_t k[4],
                                               uint64_t h, uint64_t hint0, bool *fresh) {
    const uint64_t ready = id_head(T.gen, kIdReady, tag, k[0]);
    for (uint64_t probes = 0; probes <= T.mask; ++probes, h = (h + 1) & T.mask) {
        unsigned long long *hp = T.head + h;
        uint64_t cur = probes == 0 ? hint0 : *hp;   // hint
        for (;;) {
            if ((uint32_t)(cur >> 48) != T.gen) {   // empty in this generation: claim it
                const uint64_t want = tag == 2 ? id_head(T.gen, kIdBusy, tag, k[0]) : ready;
                const uint64_t prev = atomicCAS(hp, (unsigned long long)cur, (unsigned long long)want);
                if (prev == cur) {
                    *fresh = true;
                    if (T.slots && T.init) {   // a new source of the persistent index: its map state
                        Slot &sl = T.slots[h];
                        sl.flags = T.born << kBornShift;
                        sl.key[0] = k[0]; sl.key[1] = k[1]; sl.key[2] = k[2]; sl.key[3] = k[3];
                        sl.pps = sl.bps = sl.tt = sl.till = sl.aux = 0;
                        sl.tag = slot_tag(tag, T.tgen);
                    }
                    // (a reader that misses the new entry, 0 in a stale line, defers to this
                    // full protocol; no other value can be seen in this epoch)
                    if (kMirPub && tag == 1) mir_publish(T.mir, T.mir_shift, T.mask, T.seed, h, k[0]);
                    if (tag == 2) {
                        // Publication without release / acquire fences: on gfx950 an
                        // agent-scope release is a whole-L2 writeback (buffer_wbl2) and an
                        // acquire a whole-L2 invalidate (buffer_inv), per new IPv6 source.
                        // The key words go out as returning agent-scope exchanges (performed
                        // at the coherence point before they return); READY is stored only
                        // after all three returned (the asm consumes their results), and
                        // readers load the words with agent-scope (L2-bypassing) loads issued
                        // after they saw READY.
                        uint32_t *kw = T.k6 + h * 4;
                        const uint32_t r1 = __hip_atomic_exchange(kw + 0, k[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t r2 = __hip_atomic_exchange(kw + 1, k[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t r3 = __hip_atomic_exchange(kw + 2, k[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("" ::"v"(r1), "v"(r2), "v"(r3) : "memory");
                        __hip_atomic_store(hp, (unsigned long long)ready, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                    return (uint32_t)h;
                }
                cur = prev;       // lost a race, or the hint was stale: decide on the truth
                continue;
            }
            uint32_t spins = 0;
            while (((cur >> 40) & 0xFFu) == kIdBusy) {
                if (++spins > kIdSpin) return kNoSlot;
                __builtin_amdgcn_s_sleep(1);
                cur = __hip_atomic_load(hp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
        if (((cur >> 32) & 0xFFu) != tag || (uint32_t)cur != k[0]) continue;
        if (tag == 1) return (uint32_t)h;
        asm volatile("" ::"v"((uint32_t)(cur >> 40)) : "memory");   // the words after READY
        const uint32_t *kw = T.k6 + h * 4;
        if (__hip_atomic_load(kw + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k[1] &&
            __hip_atomic_load(kw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k[2] &&
            __hip_atomic_load(kw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k[3])
            return (uint32_t)h;
    }
    return kNoSlot;
}

// ------------------------------------------------------------------ parse
// Radix digits of the sort: pass p uses (word >> shift[p]) & mask[p]. Plain: equal
// digits of the source id. Heavy-source sort: pass 0 uses the 8-bit bucket (bits
// 56..63: light digit 0, or the heavy index above it), passes 1.. the remaining id
// digits of the light entries only.
struct DigitPlan {
    uint32_t shift[4], mask[4];
    uint32_t npass;
    uint32_t light_b;   // heavy sort: buckets below light_b are light (id digit 0); 0 = plain
    uint32_t nhist;     // digits k_parse counts (the 9-bit light passes take their bases from
                        // the tile scan: k_digit_base)
};

// parse_ethhdr / parse_ip6hdr / parse_ip4hdr (src/parsing_helper.h:49-136, dispatch
// src/fsx_kern.c:123-148) on a record's dwords 3 and 5..9: family tag 1 (IPv4) / 2
// (IPv6) with the raw source address in k, or 0 with the verdict of a packet that
// never reaches the limiter (short frame: DROP; not IPv4/IPv6: PASS, uncounted).
__device__ __forceinline__ uint32_t parse_src(uint32_t L, uint32_t d3, uint32_t d5, uint32_t d6,
                                              uint32_t d7, uint32_t d8, uint32_t d9, uint32_t k[4],
                                              uint8_t &v) {
    v = XDP_PASS;
    k[0] = k[1] = k[2] = k[3] = 0;
    // parse_ethhdr (14-byte bound; raw h_proto, no VLAN)
    const uint32_t proto = ((d3 & 0xFFu) << 8) | ((d3 >> 8) & 0xFFu);
    if (L < 14u) {
        v = XDP_DROP;                // src/fsx_kern.c:124-127
        return 0;
    }
    if (proto == 0x86DDu) {
        if (L < 54u) { v = XDP_DROP; return 0; }   // parse_ip6hdr bound, src/fsx_kern.c:139-140
        k[0] = (d5 >> 16) | (d6 << 16); k[1] = (d6 >> 16) | (d7 << 16);
        k[2] = (d7 >> 16) | (d8 << 16); k[3] = (d8 >> 16) | (d9 << 16);
        return 2;
    }
    if (proto == 0x0800u) {
        if (L < 34u) { v = XDP_DROP; return 0; }   // parse_ip4hdr fixed 20-byte bound, :146-147
        k[0] = (d6 >> 16) | (d7 << 16);            // bytes 26..29 raw
        return 1;
    }
    return 0;
}

// Count sketch of a strided sample of the batch (kHeavySample packets spread over all
// of it): per-block LDS counts, then one add per bucket; the candidate of a bucket is
// one sampled packet that hashed there (the heavy source when one dominates it).
// Sketch and map hash of a source: its probe start in the id table (already computed by
// k_parse for every packet; tables of heavy-sort size have >= 2^17 slots).
// Source of packet i (tag 0: not an IP packet) in either input mode.
__device__ __forceinline__ uint32_t packet_src(const PacketIn &in, const uint32_t *len, uint32_t i,
                                               uint32_t k[4]) {
    if (in.rec) {
        uint32_t L, dp;
        uint64_t T;
        return rec_read(in.rec, in.rec_bytes, i, k, L, T, dp);
    }
    const uint32_t *d = reinterpret_cast<const uint32_t *>(in.hdr + (size_t)i * 64);
    uint8_t v;
    return parse_src(len[i], d[3], d[5], d[6], d[7], d[8], d[9], k, v);
}

// Second sketch hash of a source (independent bits of its 64-bit table hash): two heavy
// sources that share a bucket of the first sketch rarely share one of the second.
__device__ __forceinline__ uint32_t sketch2_of(uint32_t tag, const uint32_t k[4], uint64_t seed) {
    return (uint32_t)(slot_hash(tag, k, seed) >> 40) & (kSketch - 1);
}

__global__ __launch_bounds__(256) void k_heavy_sample(PacketIn in, const uint32_t *__restrict__ len,
                                                      uint32_t n, uint32_t *__restrict__ sketch,
                                                      uint64_t seed, uint64_t mask, uint32_t test_flags) {
    __shared__ uint32_t s_cnt[2][kSketch], s_cand[2][kSketch];
    for (uint32_t c = threadIdx.x; c < kSketch; c += 256) s_cnt[0][c] = s_cnt[1][c] = 0;
    __syncthreads();
    const uint32_t S = n < kHeavySample ? n : kHeavySample;
    const uint32_t per = (S + gridDim.x - 1) / gridDim.x;
    const uint32_t s0 = blockIdx.x * per, s1 = min(S, s0 + per);
    for (uint32_t q = s0 + threadIdx.x; q < s1; q += 256) {
        const uint32_t i = (uint32_t)((uint64_t)q * n / S);
        uint32_t k[4];
        const uint32_t tag = packet_src(in, len, i, k);
        if (!tag) continue;
        const uint32_t h = (uint32_t)probe_start(tag, k, seed, mask, test_flags) & (kSketch - 1);
        const uint32_t h2 = sketch2_of(tag, k, seed);
        atomicAdd(&s_cnt[0][h], 1u);
        s_cand[0][h] = i;
        atomicAdd(&s_cnt[1][h2], 1u);
        s_cand[1][h2] = i;
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < kSketch; c += 256) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const uint32_t x = s_cnt[s][c];
            if (x >= 2) {
                atomicAdd(&sketch[2 * s * kSketch + c], x);
                sketch[(2 * s + 1) * kSketch + c] = s_cand[s][c];
            }
        }
    }
}

// Block-wide selection of at most nmax values (the largest, by log2 bins: every value of
// the bins above the cut bin, then values of the bin below it while room is left) among
// the threads' candidates x[0..4) (0: none). sel[k]: candidate k selected.
template <int kPer>
__device__ __forceinline__ void select_top(const uint32_t (&x)[kPer], uint32_t nmax, bool (&sel)[kPer],
                                           uint32_t *s_bin, uint32_t *s_scal) {
    const uint32_t tid = threadIdx.x;
    if (tid < 32) s_bin[tid] = 0;
    if (tid == 0) s_scal[2] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (x[k]) atomicAdd(&s_bin[31 - __clz((int)x[k])], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0, B = 32;
        for (int b = 31; b >= 0; --b) {
            if (acc + s_bin[b] > nmax) break;
            acc += s_bin[b];
            B = (uint32_t)b;
        }
        s_scal[0] = B;
        s_scal[1] = nmax - acc;
    }
    __syncthreads();
    const uint32_t cut = s_scal[0], room = s_scal[1];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        sel[k] = false;
        if (!x[k]) continue;
        const uint32_t b = 31u - (uint32_t)__clz((int)x[k]);
        sel[k] = b >= cut || (b + 1 == cut && atomicAdd(&s_scal[2], 1u) < room);
    }
    __syncthreads();
}

// A rule may cover the address: its /24 filter bit is set (rules of any length set the bits
// of every /24 they touch); false without rules.
__device__ __forceinline__ bool rule_maybe(const RuleSet &R, uint32_t tag, const uint32_t k[4]) {
    if (!R.slot) return false;
    const uint32_t p24 = (k[0] & 0xFFu) << 16 | (k[0] & 0xFF00u) | ((k[0] >> 16) & 0xFFu);
    return (R.filter[(tag - 1u) << (kRuleFilterBits - 5) | p24 >> 5] >> (p24 & 31u)) & 1u;
}

// One block: the heavy set of the batch from the two sketches. Candidates: the sampled
// source of each of the (at most 2 nmax) buckets of highest count >= floor per sketch; a
// candidate's estimate is the smaller of its two buckets' counts (a count-min estimate:
// a source sharing a bucket of one sketch with a heavier one is still found through the
// other), duplicates dropped; the nmax highest estimates become the heavy set, with an
// open-addressing map of them. Zeroes the counts.
// With `resolve`, every heavy source is also found in (or inserted into) the id table
// here, once, so k_parse takes its slot from LDS instead of probing per packet (not with
// prefix rules: a rule may drop every packet of the source, which must then never be
// inserted).
__global__ __launch_bounds__(1024) void k_heavy_pick(PacketIn in, const uint32_t *__restrict__ len,
                                                     uint32_t *__restrict__ sketch, HeavySet *hs,
                                                     uint32_t nmax, uint32_t floor_cnt, uint64_t seed,
                                                     uint64_t mask, uint32_t test_flags, IdTable idt,
                                                     uint32_t resolve, BatchState *bs, RuleSet rules) {
    constexpr uint32_t kMap = 1u << kHeavyMapBits;
    constexpr uint32_t kCand = 2 * 2 * kHeavyMax;   // candidate buckets over both sketches
    __shared__ uint32_t s_n, s_nc;
    __shared__ uint32_t s_cb[kCand];                // candidate: sketch << 16 | bucket
    __shared__ uint32_t s_ctag[kCand], s_ckey[kCand][4], s_cest[kCand];
    __shared__ uint32_t s_sel[kHeavyMax];
    __shared__ uint32_t s_tag[kHeavyMax], s_key[kHeavyMax][4];
    __shared__ uint8_t s_map[kMap];
    __shared__ uint32_t s_bin[32], s_scal[4];
    __shared__ uint16_t s_b2c[kSketch];             // first-sketch bucket -> candidate + 1
    const uint32_t tid = threadIdx.x;
    static_assert(kSketch == 4 * 1024, "4 buckets per thread");
    for (uint32_t c = tid; c < kSketch; c += 1024) s_b2c[c] = 0;
    const uint32_t *cnt1 = sketch, *cand1 = sketch + kSketch;
    const uint32_t *cnt2 = sketch + 2 * kSketch, *cand2 = sketch + 3 * kSketch;
    if (tid == 0) { s_n = 0; s_nc = 0; }
    s_map[tid] = 0;
    // 1. per sketch, the 2 nmax buckets of highest count >= floor
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const uint32_t *cs = s ? cnt2 : cnt1;
        uint32_t x[4];
        bool sel[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = cs[tid * 4 + k];
            x[k] = c >= floor_cnt ? c : 0u;
        }
        select_top<4>(x, 2 * nmax, sel, s_bin, s_scal);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (sel[k]) s_cb[atomicAdd(&s_nc, 1u)] = (uint32_t)s << 16 | (tid * 4 + k);
        __syncthreads();
    }
    // 2. the candidates' sources and their count-min estimates
    const uint32_t nc = s_nc;
    if (tid < nc) {
        const uint32_t s = s_cb[tid] >> 16, bk = s_cb[tid] & 0xFFFFu;
        const uint32_t i = (s ? cand2 : cand1)[bk];
        uint32_t k[4];
        const uint32_t tag = packet_src(in, len, i, k);
        const uint32_t h1 = (uint32_t)probe_start(tag, k, seed, mask, test_flags) & (kSketch - 1);
        const uint32_t a = cnt1[h1], b = cnt2[sketch2_of(tag, k, seed)];
        s_ctag[tid] = tag;
        for (int j = 0; j < 4; ++j) s_ckey[tid][j] = k[j];
        // (prefix rules: a source whose /24 some rule touches stays light — the parse decides
        // its packets one by one — so a heavy source is never rule-dropped and is inserted here)
        s_cest[tid] = tag && !rule_maybe(rules, tag, k) ? (a < b ? a : b) : 0u;
    }
    __syncthreads();
    // 3. duplicates (a source found through both sketches): a second-sketch candidate whose
    // first-sketch bucket is a candidate of the same source is dropped
    if (tid < nc && s_cb[tid] < (1u << 16)) s_b2c[s_cb[tid]] = (uint16_t)(tid + 1);
    __syncthreads();
    uint32_t est[1] = {0};
    if (tid < nc) {
        est[0] = s_cest[tid] >= floor_cnt ? s_cest[tid] : 0u;
        if (s_cb[tid] >> 16) {
            const uint32_t h1 = (uint32_t)probe_start(s_ctag[tid], s_ckey[tid], seed, mask, test_flags) & (kSketch - 1);
            const uint32_t u = s_b2c[h1];
            if (u && s_ctag[u - 1] == s_ctag[tid] && s_ckey[u - 1][0] == s_ckey[tid][0] &&
                s_ckey[u - 1][1] == s_ckey[tid][1] && s_ckey[u - 1][2] == s_ckey[tid][2] &&
                s_ckey[u - 1][3] == s_ckey[tid][3])
                est[0] = 0;
        }
    }
    // the counts are read: zero them for the next batch
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        sketch[tid * 4 + k] = 0;
        sketch[2 * kSketch + tid * 4 + k] = 0;
    }
    // 4. the nmax highest estimates
    bool pick[1];
    select_top<1>(est, nmax, pick, s_bin, s_scal);
    if (pick[0]) {
        const uint32_t e = atomicAdd(&s_n, 1u);
        s_tag[e] = s_ctag[tid];
        for (int j = 0; j < 4; ++j) s_key[e][j] = s_ckey[tid][j];
    }
    __syncthreads();
    const uint32_t n = s_n;
    if (tid == 0) {
        for (uint32_t e = 0; e < n; ++e) {
            uint32_t h = (uint32_t)probe_start(s_tag[e], s_key[e], seed, mask, test_flags) & (kMap - 1);
            while (s_map[h]) h = (h + 1) & (kMap - 1);
            s_map[h] = (uint8_t)(e + 1);
        }
        hs->n = n;
    }
    __syncthreads();
    if (tid < n) {
        hs->tag[tid] = s_tag[tid];
        for (int j = 0; j < 4; ++j) hs->key[tid][j] = s_key[tid][j];
        uint32_t slot = kNoSlot;
        if (resolve) {
            const uint64_t h = id_start(idt, s_tag[tid], s_key[tid]);
            const uint64_t hint = __hip_atomic_load(idt.head + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool fresh = false;
            slot = id_resolve(idt, s_tag[tid], s_key[tid], h, hint, &fresh);
            if (slot == kNoSlot) atomicOr(&bs->err, ERR_TABLE_FULL);
            if (fresh && idt.slots) atomicAdd(&bs->n_new, 1u);
        }
        hs->slot[tid] = slot;
    }
    if (tid == 0) hs->resolved = resolve;
    hs->map[tid] = s_map[tid];
}

// Prefix blocklist: a packet whose /24 filter bit is clear matches no
// rule (one load); otherwise the family's distinct rule lengths are probed longest first
// (the first slots of four lengths at a time loaded together); the first rule found is
// the longest match and drops the packet when 0 < now <= till (till 0 or expired: the
// packet goes on, an exception inside a shorter blocked prefix).
// (the filter word is loaded by the caller, rule_filter_word, ahead of the work that does
// not depend on it)
__device__ __forceinline__ uint32_t rule_filter_word(const RuleSet &R, uint32_t tag, const uint32_t k[4]) {
    const uint32_t p24 = (k[0] & 0xFFu) << 16 | (k[0] & 0xFF00u) | ((k[0] >> 16) & 0xFFu);
    return R.filter[(tag - 1u) << (kRuleFilterBits - 5) | p24 >> 5];
}
__device__ __forceinline__ bool rule_drop(const RuleSet &R, uint32_t tag, const uint32_t k[4], uint64_t now,
                                          uint32_t fw) {
    const uint32_t p24 = (k[0] & 0xFFu) << 16 | (k[0] & 0xFF00u) | ((k[0] >> 16) & 0xFFu);
    if (!((fw >> (p24 & 31u)) & 1u)) return false;
    const uint32_t nl = tag == 1 ? R.nlen4 : R.nlen6;
    const uint8_t *lens = R.lens + (tag == 1 ? 0u : kRuleLens6);
    const uint4 *slot = reinterpret_cast<const uint4 *>(R.slot);   // 2 uint4 per slot
    // first probe slot of length index q (q >= nl: an empty dummy)
    auto first = [&](uint32_t q, uint32_t &sq) -> uint4 {
        sq = 0;
        if (q >= nl) return make_uint4(0, 0, 0, 0);
        const uint32_t L = lens[q];
        uint32_t a[4];
        rule_mask(k, L, a);
        sq = rule_hash(tag << 8 | L, a) & R.mask;
        return slot[2 * sq];
    };
    // the chain of length index q from its loaded first slot (a load factor <= 1/4 keeps
    // it short): -1 no rule of this length, else the rule's verdict (1 drop). An IPv4
    // fingerprint is the address itself; an IPv6 one is confirmed on the words.
    auto walk = [&](uint32_t q, uint4 e, uint32_t sq) -> int {
        if (q >= nl) return -1;
        const uint32_t L = lens[q], rt = tag << 8 | L;
        uint32_t a[4];
        rule_mask(k, L, a);
        const uint32_t fp = rule_fp(a);
        for (; e.x != 0; sq = (sq + 1) & R.mask, e = slot[2 * sq]) {
            if (e.x != rt || e.y != fp) continue;
            if (tag == 2) {
                const uint4 w = slot[2 * sq + 1];
                if (w.x != a[0] || w.y != a[1] || w.z != a[2] || w.w != a[3]) continue;
            }
            const uint64_t till = (uint64_t)e.z | ((uint64_t)e.w << 32);
            return till > 0 && now <= till ? 1 : 0;
        }
        return -1;
    };
    for (uint32_t q = 0; q < nl; q += 4) {   // four lengths' first slots loaded together
        uint32_t s0, s1, s2, s3;
        const uint4 e0 = first(q, s0), e1 = first(q + 1, s1), e2 = first(q + 2, s2), e3 = first(q + 3, s3);
        int r;
        if ((r = walk(q, e0, s0)) >= 0) return r == 1;
        if ((r = walk(q + 1, e1, s1)) >= 0) return r == 1;
        if ((r = walk(q + 2, e2, s2)) >= 0) return r == 1;
        if ((r = walk(q + 3, e3, s3)) >= 0) return r == 1;
    }
    return false;
}

// One wave handles 64 consecutive records per step: the 4 KiB tile is loaded with
// four fully coalesced 1 KiB wave loads and staged through LDS (13-dword record
// pitch: conflict-free 32-bit reads), then each lane parses its own record.
// Record mode (kRec = 16 / 32): every lane loads its own exchange record (coalesced, no
// LDS staging), all of them IP packets; their len / ts go out to in.rec_len / rec_ts.
// FSX_PARSE_PAY (A/B, default 0; DESIGN.md §3 "Pass 0 in the parse, measured"): with the heavy
// sources outside the sort, k_parse also reads the timestamps, computes the clock facts (and
// each sort tile's span) and writes every light packet's payload word beside its sort word,
// so pass 0 (k_pass0h<false>) only ranks and scatters the light words; the heavy tile records
// come from k_heavy_recs at the start of the tail. Bit-exact, slower: 3.09-3.19 vs 2.95-2.96
// ms per step (profiles/r05/ab_r05d_parse_pay.txt). 0 (the product): k_parse reads no
// timestamps and k_pass0h<true> reads ts / len / verdicts once for the records, the clock facts
// and the payload words.
#ifndef FSX_PARSE_PAY
#define FSX_PARSE_PAY 0
#endif
constexpr uint32_t kRecPitch = 13;   // LDS staging pitch of a record (12 dwords used; odd: conflict-free reads)
// kOrd (home-ordered inserts): no index probe at all — an IP packet's sort word
// is its home-ordered key hash (ord_hkey) << kIdShift | arrival index, bit 63 set for IPv6; the
// segment heads find / insert their slots after the sort (k_ord_resolve).
template <uint32_t kRec, bool kRules, bool kMir, bool kHf, bool kOrd = false>
#ifndef FSX_PARSE_MINB
#define FSX_PARSE_MINB 4   // waves/SIMD bound of k_parse (A/B: scripts/build_variant.sh)
#endif
#ifndef FSX_PARSE_DEFCAP   // deferred probes per wave before k_parse resolves them (CAS inserts)
#define FSX_PARSE_DEFCAP 128u
#endif
#ifndef FSX_PARSE_GRID   // persistent blocks of k_parse (256 CUs x its blocks per CU)
#define FSX_PARSE_GRID (256u * FSX_PARSE_MINB)
#endif
__global__ __launch_bounds__(256, FSX_PARSE_MINB) void k_parse(PacketIn in,
                                               const uint32_t *__restrict__ len,
                                               const uint64_t *__restrict__ ts, uint32_t n,
                                               uint64_t *__restrict__ packed,
                                               uint8_t *__restrict__ verdict, BatchState *bs,
                                               IdTable idt, uint32_t *__restrict__ ghist,
                                               uint32_t *__restrict__ thist, uint32_t tcap,
                                               DigitPlan dp, const HeavySet *__restrict__ heavy,
                                               RuleSet rules, uint32_t tagh,
                                               uint32_t *__restrict__ chunk_cnt,
                                               uint64_t *__restrict__ lmask) {
    // kHf (unsorted heavy sources): no sort word for a heavy source's packet (its
    // verdict byte carries 0x80 | h), the light sort words compacted per 1024-packet chunk
    // (wave) with their count in chunk_cnt, and
    //   FSX_PARSE_PAY: each light packet's payload word at the same compacted position of
    //   lmask (the payload array), the clock facts and the sort tiles' span;
    //   else: no timestamp loads, the light-packet mask of every 64-packet step in lmask
    //   (k_pass0h<true> reads ts / len / verdicts for the records and the payloads)
    static_assert(!kOrd || (!kHf && !kMir && kRec == 0), "home-ordered inserts: header records, no heavy sources");
    const uint32_t ord_s = kOrd ? (uint32_t)__popcll(idt.mask) : 0u;   // log2(slots)
    constexpr bool kHr = kHf && FSX_PARSE_PAY;   // (the payload words from the parse)
    __shared__ uint32_t s_rec[4][64 * kRecPitch];
    __shared__ uint32_t s_red[4][3];
    __shared__ unsigned long long s_ts[4], s_its[4];
    __shared__ uint32_t s_hist[4][256];     // the radix digits of every sort key (per pass)
    __shared__ uint32_t s_t0[256];          // pass-0 digit of the current sort tile
    __shared__ uint32_t s_hkey[kHeavyMax][4];
    __shared__ uint32_t s_htag[kHeavyMax];
    __shared__ uint32_t s_hmap4[(1u << kHeavyMapBits) / 4];   // HeavySet::map
    __shared__ uint32_t s_hslot[kHeavyMax];
    // per wave: deferred probes {i, tag | hidx, key word 0, probe hint (not with kMir + kHf),
    // light position (kHf)}
    constexpr uint32_t kDefW = kHf ? (kMir ? 4 : 6) : 5;   // words per deferred packet
    constexpr uint32_t kDefPos = kDefW - 1;                 // (kHf) its light position
    __shared__ uint32_t s_def[4][FSX_PARSE_DEFCAP * kDefW];
    __shared__ unsigned long long s_cb[4], s_cz[4];   // kHr: each chunk's first / last timestamp
    const uint8_t *s_hmap = reinterpret_cast<const uint8_t *>(s_hmap4);
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 0; d < 4; ++d) s_hist[d][threadIdx.x] = 0;
    s_t0[threadIdx.x] = 0;
    const uint32_t nh = heavy ? heavy->n : 0u;
    const bool hres = heavy && heavy->resolved;   // heavy slots known: no probe for them
    if (heavy) {
        s_hmap4[threadIdx.x] = reinterpret_cast<const uint32_t *>(heavy->map)[threadIdx.x];
        if (threadIdx.x < nh) {
            s_htag[threadIdx.x] = heavy->tag[threadIdx.x];
            for (int j = 0; j < 4; ++j) s_hkey[threadIdx.x][j] = heavy->key[threadIdx.x][j];
            s_hslot[threadIdx.x] = heavy->slot[threadIdx.x];
        }
    }
    __syncthreads();
    uint32_t *rec = s_rec[w];
    uint32_t any6 = 0, nonmono = 0, maxlen = 0, nfresh = 0, nrule = 0;
    // the high word's kFreshBit for an inserting packet (lazy slots; without the heavy-source
    // sort, or kHf: a light word's bucket is below 128 and k_pass0h ranks it without the bit)
    const uint32_t fresh_hi = __builtin_amdgcn_readfirstlane(!idt.init && (!dp.light_b || kHf) ? 0x80000000u : 0u);
    uint64_t maxts = 0, inv_mints = 0;  // ~min ts, max-reduced
    // a block owns whole 4096-record sort tiles (so it can emit pass 0's per-tile digit
    // counts: no k_tile_hist for pass 0); wave w parses records [w*1024, +1024) of the
    // tile in 64-record steps
    const uint32_t ntiles = (n + 63u) >> 6;
    const uint32_t nsort = (n + kSortTile - 1) / kSortTile;
    constexpr uint32_t kSteps = kSortTile / 256;   // 64-record steps per wave and sort tile
    auto step_of = [&](uint32_t st, uint32_t j) { return st * (kSortTile / 64) + w * kSteps + j; };
    // software pipeline: the next tile's loads are in flight while this one is parsed.
    // Header records: only their first 48 bytes (the parse reads bytes 12..39), as 3 x 16 B
    // per lane: flat chunk f = k * 64 + lane is chunk f % 3 of record f / 3
    constexpr int kHv = kRec == 0 ? 3 : (int)(kRec / 16);   // uint4 registers per lane and step
    // Unconditional loads (out-of-range lanes read record / packet 0 and are discarded by
    // the parse's `live`), so every step issues the same loads and s_waitcnt counts stay
    // exact: a conditional load would make the compiler wait for everything in flight.
    auto load = [&](uint32_t tt, uint4 (&h)[kHv], uint32_t &L_, uint64_t &T_, uint64_t &P_) {
        const uint32_t base = tt << 6;
        const bool tv = tt < ntiles;
        const uint32_t i = base + lane;
        const bool live = tv && i < n;
        const uint32_t ic = live ? i : 0u;
        if constexpr (kRec == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t f = (uint32_t)k * 64u + lane, r = f / 3u, c = f - 3u * r;
                const uint32_t rr = tv && base + r < n ? base + r : 0u;
                h[k] = stream_load16(in.hdr + (size_t)rr * 64u + c * 16u);
            }
            L_ = stream_load(len + ic);
            if constexpr (kHf && !kHr) {   // (prefix rules: a rule's till is checked against ts)
                T_ = kRules ? stream_load(ts + ic) : 0ull;
                P_ = 0ull;
            } else if constexpr (kHr) {   // (the record before a step: c_prev, see parse_step)
                T_ = stream_load(ts + ic);
                P_ = 0ull;
            } else {
                T_ = stream_load(ts + ic);
                // the record before the step, for lane 0 only (one address instead of 64: the
                // same s_waitcnt count, a quarter of the cache-line lookups of a full ts load)
                P_ = lane == 0 ? ts[ic > 0 ? ic - 1 : 0] : 0ull;
            }
        } else {
            const uint4 *r = reinterpret_cast<const uint4 *>(in.rec);
            constexpr uint32_t kW = kRec / 16;   // uint4 words per record
            h[0] = r[(size_t)ic * kW];
            if constexpr (kW == 2) h[1] = r[(size_t)ic * kW + 1];
            L_ = 0u;
            T_ = 0ull;
            // timestamp of the record before the step (lane 0)
            const uint4 pr = r[(size_t)(ic > 0 ? ic - 1 : 0) * kW + (kW - 1)];
            P_ = kW == 1 ? ((uint64_t)pr.z | ((uint64_t)pr.w << 32)) : ((uint64_t)pr.x | ((uint64_t)pr.y << 32));
        }
    };
    // Software pipeline, per wave: iteration j parses step j + 1 (its
    // records were loaded two iterations earlier) and issues that step's source-index
    // probes, then issues the record loads of step j + 3, then resolves step j from the
    // probes issued one iteration earlier. vmcnt drains in issue order, so a probe read
    // issued after a prefetch would wait for the prefetch; issued one iteration ahead,
    // before it, the probes never stall the stream. A probe that does not find its
    // source READY in the first two slots (new source, longer probe chain, IPv6) is
    // deferred: the wave resolves its deferred packets together (CAS inserts) at the end
    // of the sort tile, or earlier when the LDS list fills.
    // the parsed step awaiting resolution: tag, key word 0, probe start, heavy index, the
    // two probe reads
    // (one step's worth of these awaits its resolution: ProbeSet)
    // kHr: the wave's chunk's first timestamp and the last one so far (wave-uniform): the clock
    // check of a step's first record against the step before it, the tile's span and the
    // check across its chunks at the tile's end (across tiles: k_pass0h<false>)
    uint64_t c_base = 0, c_prev = 0;
    uint64_t tb = 0;   // kHr: the batch's first timestamp (payload words: ts - tb)
    if constexpr (kHr) {
        if (n) {
            if constexpr (kRec == 0) {
                tb = ts[0];
            } else {
                const uint4 *r0 = reinterpret_cast<const uint4 *>(in.rec);
                tb = kRec == 16 ? ((uint64_t)r0[0].z | ((uint64_t)r0[0].w << 32))
                                : ((uint64_t)r0[1].x | ((uint64_t)r0[1].y << 32));
            }
        }
    }
    // kMir: the two mirror entries as the halves of one register (two 16-bit loads that
    // stay in flight until the resolve)
    typedef unsigned short mir2_t __attribute__((ext_vector_type(2)));
    struct ProbeSet {
        uint32_t tag = 0, k0 = 0, h = 0;
        int hidx = -1;
        uint64_t hint0 = 0, hint1 = 0;
        mir2_t m = {0, 0};
    };
    constexpr uint32_t kDefCap = FSX_PARSE_DEFCAP;   // deferred packets per wave (LDS)
    uint32_t crun = 0;                  // kHf: light words of the wave's current chunk so far
    uint32_t *dq = s_def[w];
    uint32_t ndef = 0;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    // radix histograms of the key digits: block LDS counters (a heavy source repeats in
    // few lanes of one 64-packet step, so same-address serialization stays short)
    // (FSX_MEASURE_NO_PROBE: a cost-attribution build for scripts/ab.sh only — every
    // IPv4 source takes its first probe slot, wrong ids but in range; never the product)
    auto count_digits = [&](uint64_t out, int hidx) {
        if (!ghist) return;
        const uint32_t d0 = (uint32_t)(out >> dp.shift[0]) & dp.mask[0];
        atomicAdd(&s_t0[d0], 1u);   // (the block's digit-0 totals from s_t0 per sort tile)
        if (hidx < 0)   // heavy entries are final after pass 0
            for (uint32_t dg = 1; dg < dp.nhist; ++dg)
                atomicAdd(&s_hist[dg][(uint32_t)(out >> dp.shift[dg]) & dp.mask[dg]], 1u);
    };
    auto word_of = [&](uint32_t id, uint32_t tag, uint32_t i, int hidx) -> uint64_t {
        (void)tag;
        uint64_t out = ((uint64_t)(id & idt.mask) << kIdShift) | i;
        if (dp.light_b)   // heavy-source sort: the first pass's bucket in bits [shift[0], 64)
            out |= (uint64_t)(hidx >= 0 ? dp.light_b + (uint32_t)hidx
                                        : (uint32_t)(out >> kIdShift) & (dp.light_b - 1u)) << dp.shift[0];
        return out;
    };
    // the deferred packets of this wave: full probes (CAS inserts), 64 at a time
    auto flush = [&]() {
        for (uint32_t e0 = 0; e0 < ndef; e0 += 64) {
            const uint32_t e = e0 + lane;
            bool fresh = false;
            if (e < ndef) {
                const uint32_t *q = dq + e * kDefW;
                const uint32_t i = q[0], tag = q[1] & 0xFFu;
                const int hidx = (int)(q[1] >> 8) - 1;
                uint32_t k[4] = {q[2], 0, 0, 0};
                if (tag == 2) packet_src(in, len, i, k);   // IPv6: the key again from the record
                const uint64_t h = id_start(idt, tag, k);
                // IPv4: the first probe slot's head as the probe read it (a stale value only
                // costs the CAS one retry); IPv6 (and IPv4 probed on the mirror) had no head read
                const uint64_t hint = tag == 1 && kDefW >= 5 && !kMir ? ((uint64_t)q[kDefW >= 5 ? 4 : 0] << 32 | q[3])
                                               : __hip_atomic_load(idt.head + h, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t id = id_resolve<kMir>(idt, tag, k, h, hint, &fresh);
                if (id == kNoSlot) atomicOr(&bs->err, ERR_TABLE_FULL);
                const uint64_t out = word_of(id, tag, i, hidx);
                const uint64_t outf = out | (uint64_t)(fresh ? fresh_hi : 0u) << 32;
                if constexpr (kHf) {
                    if (hidx < 0) packed[q[kDefPos]] = outf;
                } else {
                    packed[i] = outf;
                }
                count_digits(out, hidx);
            }
            nfresh += (uint32_t)__popcll(__ballot(fresh));   // new sources (persistent index)
        }
        ndef = 0;
        wave_lds_order();
    };
    // parse one step (its records in hv / Lc / Tc / Pc): verdict bytes, clock facts, and
    // the probes of its IP packets into the c_* registers
    auto parse_step = [&](ProbeSet &c, uint32_t t, const uint4 (&hv)[kHv], uint32_t Lc, uint64_t Tc, uint64_t Pc) {
        const uint32_t base = t << 6;
        const uint32_t i = base + lane;
        const bool live = t < ntiles && i < n;
        uint32_t L = Lc;
        uint64_t T = Tc;
        uint8_t v = XDP_PASS;  // non-IP: PASS, not counted (src/fsx_kern.c:128-131)
        uint32_t k[4] = {0, 0, 0, 0};
        uint32_t tag = 0;
        if constexpr (kRec == 0) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const uint32_t f = (uint32_t)q * 64u + lane, r = f / 3u, c = f - 3u * r;
                uint32_t *d = rec + r * kRecPitch + c * 4u;
                d[0] = hv[q].x; d[1] = hv[q].y; d[2] = hv[q].z; d[3] = hv[q].w;
            }
            wave_lds_order();
            const uint32_t *my = rec + lane * kRecPitch;
            const uint32_t d3 = my[3], d5 = my[5], d6 = my[6], d7 = my[7], d8 = my[8], d9 = my[9];
            tag = live ? parse_src(L, d3, d5, d6, d7, d8, d9, k, v) : 0u;
        } else if (live) {   // ShardRecord16 {key, len | dport << 16, ts} / ShardRecord
            if constexpr (kRec == 16) {
                k[0] = hv[0].x;
                L = hv[0].y & 0xFFFFu;
                T = (uint64_t)hv[0].z | ((uint64_t)hv[0].w << 32);
                tag = 1;
            } else {
                k[0] = hv[0].x; k[1] = hv[0].y; k[2] = hv[0].z; k[3] = hv[0].w;
                T = (uint64_t)hv[1].x | ((uint64_t)hv[1].y << 32);
                L = hv[1].z;
                tag = ((hv[1].w >> 16) & 0xFFu) == 6 ? 2u : 1u;
            }
            in.rec_len[i] = L;
            in.rec_ts[i] = T;
        }
        // prefix blocklist, kHf: the /24 filter word loaded first, its latency under the
        // source's hash and heavy-map lookup; a heavy source needs no rule check (the pick
        // leaves every source whose filter bit is set light, rule_maybe). (Without kHf the rule
        // decides first: the early word spills in those instantiations.)
        uint32_t rfw = 0;
        if constexpr (kRules && kHf) {
            if (tag) rfw = rule_filter_word(rules, tag, k);
        }
        if constexpr (kRules && !kHf) {
            if (tag && rule_drop(rules, tag, k, T, rule_filter_word(rules, tag, k))) {
                tag = 0;              // never reaches the per-source path
                v = XDP_DROP;
                ++nrule;
            }
        }
        uint64_t prev = __shfl_up(T, 1);
        if constexpr (kHr) {
            (void)Pc;
            if (lane == 0) prev = (t & 15u) ? c_prev : T;
        } else {
            if (lane == 0) prev = (live && i > 0) ? Pc : T;
        }
        uint64_t h = 0;
        if (tag) h = id_start(idt, tag, k);
        // heavy source? (LDS map of the batch's heavy set)
        int hidx = -1;
        if (tag && nh) {
            constexpr uint32_t kMapMask = (1u << kHeavyMapBits) - 1u;
            uint32_t hh = (uint32_t)h & kMapMask;
            for (uint32_t e; (e = s_hmap[hh]) != 0; hh = (hh + 1) & kMapMask) {
                --e;
                if (s_htag[e] == tag && s_hkey[e][0] == k[0] &&
                    (tag == 1 || (s_hkey[e][1] == k[1] && s_hkey[e][2] == k[2] && s_hkey[e][3] == k[3]))) {
                    hidx = (int)e;
                    break;
                }
            }
        }
        if constexpr (kRules && kHf) {   // the longest matching rule decides
            if (tag && hidx < 0 && rule_drop(rules, tag, k, T, rfw)) {
                tag = 0;              // never reaches the per-source path
                v = XDP_DROP;
                ++nrule;
                h = 0;
            }
        }
        const bool ip = tag != 0;
        if (tag == 2) any6 = 1;
        // the fast path reads the first two slots of an IPv4 source's probe chain (IPv6
        // sources are always resolved by the full protocol, which reads their key words
        // only after the head shows READY)
        c.hint0 = c.hint1 = 0;
        if constexpr (kMir) c.m = mir2_t{0, 0};
        if constexpr (kOrd) {   // (no probe: the key hash, resolve_step writes the word)
            c.tag = live ? tag : 0u;
            c.h = ip ? ord_hkey(tag, k, h, idt.seed, ord_s) : 0u;
            c.hidx = -1;
        }
#ifdef FSX_MEASURE_NO_PROBE
        if (false) {
#else
        if (!kOrd && tag == 1 && !(hres && hidx >= 0)) {
#endif
            // (coherent=1 reads past the XCD's L2, which may hold the head of an older
            // epoch: a stale head can only fail the match, never fake one)
            const uint64_t h1 = (h + 1) & idt.mask;
            if constexpr (kMir) {   // the 2-byte mirror entries of the two slots (exact: mir_entry)
                const unsigned short *mp = static_cast<const unsigned short *>(idt.mir);
                c.m.x = mp[h];
                c.m.y = mp[h1];
            } else if (idt.coherent) {
                c.hint0 = __hip_atomic_load(idt.head + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                c.hint1 = __hip_atomic_load(idt.head + h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                c.hint0 = idt.head[h];
                c.hint1 = idt.head[h1];
            }
        }
        if constexpr (!kOrd) {
            c.tag = live ? tag : 0u;
            c.k0 = k[0];
            c.h = (uint32_t)h;
            c.hidx = hidx;
        }
        if constexpr (kHr) {
            {   // the light packets' positions in the chunk (arrival order) and payload words
                const bool lt = live && tag != 0 && hidx < 0;
                const uint64_t lm = __ballot(lt);
                // (ts - tb) << kPayLenBits | len (k_hmode: pay_ok), at the light word's compacted
                // position (lmask is the payload array); resolve_step recomputes the position
                if (lt) lmask[((t >> 4) << 10) + crun + (uint32_t)__popcll(lm & lt_mask)] = ((T - tb) << kPayLenBits) | L;
                crun += (uint32_t)__popcll(lm);
            }
            // the chunk's first and last timestamp (a step past n: its lane 63 is no packet, but
            // then no later chunk of the tile holds one either)
            if ((t & 15u) == 0) c_base = uni64(__shfl(T, 0));
            c_prev = uni64(__shfl(T, 63));
        }
        if (live) {
            // IP packets default to PASS here (coalesced); the fill pass writes only
            // the DROP verdicts, which cluster in the heavy sources' segments
            // (tagh: a heavy source's packet carries 0x80 | its index until k_verdict_apply)
            if (verdict) verdict[i] = !ip ? v : (tagh && hidx >= 0) ? (uint8_t)(0x80u | (uint32_t)hidx)
                                                                  : (uint8_t)XDP_PASS;
            maxlen = L > maxlen ? L : maxlen;
            if constexpr (!kHf || kHr) {   // (kHf && !kHr: k_pass0h<true> has the clock facts)
                if (!kHf && !ip) packed[i] = kSentinel;
                nonmono |= T < prev ? 1u : 0u;
                maxts = T > maxts ? T : maxts;
                inv_mints = ~T > inv_mints ? ~T : inv_mints;
            }
        }
    };
    // resolve step t ("cur"): heavy slot from LDS, the fast-path probe match, or defer
    auto resolve_step = [&](ProbeSet &c, uint32_t t) {
        const uint32_t i = (t << 6) + lane;
        if constexpr (kOrd) {
            if (c.tag) {
                const uint64_t out = ((uint64_t)c.h << kIdShift) | i | (c.tag == 2 ? kFreshBit : 0ull);
                packed[i] = out;
                count_digits(out, -1);
            }
            return;
        }
        uint32_t id = kNoSlot;
        bool defer = false;
        if (c.tag) {
            if (hres && c.hidx >= 0) {
                id = s_hslot[c.hidx];
            } else if (c.tag == 1) {
                // the slot's head READY with this key, or its mirror entry (d = 0 / 1)
                const uint64_t want0 = kMir ? mir_entry(c.k0, idt.seed, idt.mir_shift, 0u)
                                            : id_head(idt.gen, kIdReady, 1u, c.k0);
                const uint64_t want1 = kMir ? want0 | 1u << 14 : want0;
#ifdef FSX_MEASURE_NO_PROBE
                id = c.h;
                c.hint0 = want0;
                c.m.x = (unsigned short)want0;
#endif
                const uint64_t got0 = kMir ? (uint64_t)c.m.x : c.hint0;
                const uint64_t got1 = kMir ? (uint64_t)c.m.y : c.hint1;
                if (got0 == want0) id = c.h;
                else if (got1 == want1) id = (uint32_t)((c.h + 1) & idt.mask);
                else defer = true;
            } else {
                defer = true;
            }
        }
        // kHf: the light packets' positions in the chunk, in arrival order (deferred or not)
        uint32_t lpos = 0;
        if constexpr (kHr) {   // (parse_step counted this step's light packets into crun)
            const uint64_t lm = __ballot(c.tag != 0 && c.hidx < 0);
            lpos = ((t >> 4) << 10) + crun - (uint32_t)__popcll(lm) + (uint32_t)__popcll(lm & lt_mask);
        } else if constexpr (kHf) {
            const uint64_t lm = __ballot(c.tag != 0 && c.hidx < 0);
            if (lane == 0 && t < ntiles) lmask[t] = lm;
            lpos = ((t >> 4) << 10) + crun + (uint32_t)__popcll(lm & lt_mask);
            crun += (uint32_t)__popcll(lm);
        }
        const uint64_t dm = __ballot(defer);
        if (dm) {
            if (ndef + 64 > kDefCap) flush();
            if (defer) {
                uint32_t *q = dq + (ndef + (uint32_t)__popcll(dm & lt_mask)) * kDefW;
                q[0] = i; q[1] = c.tag | (uint32_t)(c.hidx + 1) << 8; q[2] = c.k0;
                if constexpr (kDefW >= 5) { q[3] = (uint32_t)c.hint0; q[4] = (uint32_t)(c.hint0 >> 32); }
                if constexpr (kHf) q[kDefPos] = lpos;
            }
            ndef += (uint32_t)__popcll(dm);
        }
        if (c.tag && !defer) {
            const uint64_t out = word_of(id, c.tag, i, c.hidx);
            if constexpr (kHf) {
                if (c.hidx < 0) packed[lpos] = out;
            } else {
                packed[i] = out;
            }
            count_digits(out, c.hidx);
        }
    };
    // The wave's steps in order: s -> (tile blockIdx.x + (s / kSteps) * gridDim.x, step
    // s % kSteps). Three register sets, the loop unrolled by three, so no register holding
    // an in-flight load is ever moved (a move would wait for the load): iteration s
    // resolves step s, parses step s + 1 from set (s + 1) % 3 and loads step s + 3 into
    // set s % 3.
    const uint32_t my_tiles = nsort > blockIdx.x ? (nsort - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
    const uint32_t S = my_tiles * kSteps;
    auto tile_of = [&](uint32_t q) { return blockIdx.x + (q / kSteps) * gridDim.x; };
    auto step_at = [&](uint32_t q) { return q < S ? step_of(tile_of(q), q % kSteps) : ntiles; };
    uint4 h0[kHv], h1[kHv], h2[kHv];
    uint32_t L0, L1, L2;
    uint64_t T0, T1, T2, P0, P1, P2;
    load(step_at(0), h0, L0, T0, P0);
    load(step_at(1), h1, L1, T1, P1);
    load(step_at(2), h2, L2, T2, P2);
    ProbeSet c;
    if (S) parse_step(c, step_at(0), h0, L0, T0, P0);
    auto tile_end = [&](uint32_t q) {
        if (q % kSteps == kSteps - 1) {   // sort tile done: its deferred packets, then its digit-0 counts
            flush();
            if constexpr (kHf) {   // the wave's chunk: its light word count
                if (lane == 0) chunk_cnt[step_at(q) >> 4] = crun;
                crun = 0;
            }
            if constexpr (kHr) {   // the chunk's first / last timestamp
                if (lane == 0) { s_cb[w] = c_base; s_cz[w] = c_prev; }
            }
            if (ghist) {
                __syncthreads();
                const uint32_t c0 = s_t0[threadIdx.x];
                s_hist[0][threadIdx.x] += c0;
                if (thist && threadIdx.x <= dp.mask[0]) thist[(size_t)threadIdx.x * tcap + tile_of(q)] = c0;
                s_t0[threadIdx.x] = 0;
                if constexpr (kHr) {
                    // a tile spanning 2^32 ns or more: no unsorted path (k_hmode; with a clock
                    // that goes back it is refused anyway, so first / last bound the span)
                    const uint32_t tt = tile_of(q);
                    if (threadIdx.x == 0) {
                        uint64_t last = s_cz[0];
                        bool back = false;   // (a chunk starting before the one before it ended)
                        for (uint32_t k = 1; k < 4; ++k)
                            if (tt * kSortTile + k * 1024u < n) {
                                back |= s_cb[k] < s_cz[k - 1];
                                last = s_cz[k];
                            }
                        if (last >= s_cb[0] && last - s_cb[0] >= (1ull << 32)) atomicOr(&bs->span_big, 1u);
                        if (back) atomicOr(&bs->nonmono, 1u);
                    }
                }
                __syncthreads();
            }
        }
    };
    auto iter = [&](uint32_t q, const uint4 (&hp)[kHv], uint32_t Lp, uint64_t Tp, uint64_t Pp,
                    uint4 (&hl)[kHv], uint32_t &Ll, uint64_t &Tl, uint64_t &Pl) {
        // C: resolve step q with the probes issued one iteration ago
        resolve_step(c, step_at(q));
        wave_lds_order();
        tile_end(q);
        // A: parse step q + 1 (its records were loaded two iterations ago), probes issued
        c = ProbeSet{};
        if (q + 1 < S) parse_step(c, step_at(q + 1), hp, Lp, Tp, Pp);
        // B: the record loads of step q + 3 into the set step q used
        load(step_at(q + 3), hl, Ll, Tl, Pl);
    };
    for (uint32_t q = 0; q < S; q += 3) {
        iter(q, h1, L1, T1, P1, h0, L0, T0, P0);
        if (q + 1 < S) iter(q + 1, h2, L2, T2, P2, h1, L1, T1, P1);
        if (q + 2 < S) iter(q + 2, h0, L0, T0, P0, h2, L2, T2, P2);
    }
    if (ghist) {
        __syncthreads();
#pragma unroll
        for (int dg = 0; dg < 4; ++dg) {
            const uint32_t c = s_hist[dg][threadIdx.x];
            if (c) atomicAdd(&ghist[dg * 256 + threadIdx.x], c);
        }
    }
    // one add per wave: a per-step add to one counter serializes at the memory side
    if (lane == 0 && nfresh && idt.slots) atomicAdd(&bs->n_new, nfresh);
    if constexpr (kRules) {
        nrule = wave_incl_sum(nrule);
        if (lane == 63 && nrule) atomicAdd(&bs->n_rule, nrule);
    }
    any6 = __ballot(any6 != 0) ? 1u : 0u;
    nonmono = __ballot(nonmono != 0) ? 1u : 0u;
    maxlen = wave_max(maxlen);
    maxts = wave_max(maxts);
    inv_mints = wave_max(inv_mints);
    if (lane == 0) {
        s_red[w][0] = any6; s_red[w][1] = nonmono; s_red[w][2] = maxlen;
        s_ts[w] = maxts; s_its[w] = inv_mints;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, m = 0, l = 0;
        uint64_t mt = 0, imt = 0;
        for (int k = 0; k < 4; ++k) {
            a |= s_red[k][0]; m |= s_red[k][1];
            l = s_red[k][2] > l ? s_red[k][2] : l;
            mt = s_ts[k] > mt ? s_ts[k] : mt;
            imt = s_its[k] > imt ? s_its[k] : imt;
        }
        if (a) atomicOr(&bs->any_v6, 1u);
        if (m) atomicOr(&bs->nonmono, 1u);
        atomicMax(&bs->max_len, l);
        atomicMax(reinterpret_cast<unsigned long long *>(&bs->max_ts), (unsigned long long)mt);
        atomicMax(reinterpret_cast<unsigned long long *>(&bs->inv_min_ts), (unsigned long long)imt);
    }
}

// ------------------------------------------------------------------ radix sort
// LSD radix sort of the sort words on their 32-bit key: 4 passes of 8 bits, the
// payload words (kPayLenBits) following the same permutation. Per pass the keys are
// cut into 4096-key tiles:
//   k_tile_hist     per-tile digit counts, digit-major [256][tiles]
//   k_tile_scan     per digit: exclusive scan over the tiles plus the digit's global
//                   base (exclusive scan of the k_parse histogram of that digit)
//   k_tile_scatter  stable in-tile ranking (wave-ballot matching), LDS-sorted tile,
//                   runs written to the digit buckets: keys, then payload words
// Pass 0 reads the parse output in arrival order: it drops the non-IP sentinels and
// builds the payload words from (ts, len).
//
// The single-pass "onesweep" variant (decoupled look-back instead of k_tile_hist /
// k_tile_scan) is kept for A/B runs behind FSX_FLAG_ONESWEEP_SORT: on MI355X its
// look-back polls must bypass the per-XCD L2s, and a tile waited ~11 us in it
// (scripts/micro/sort_micro.hip), more than the extra key read of k_tile_hist costs.

// n_valid and the per-pass digit bases (exclusive scans of the k_parse histograms).
// light_b: pass-0 buckets below it hold the light entries (256: all entries).
__global__ __launch_bounds__(256) void k_hist_prep(const uint32_t *__restrict__ ghist,
                                                   uint32_t *__restrict__ gbase, BatchState *bs,
                                                   uint32_t light_b) {
    __shared__ uint32_t s_tmp[4];
#pragma unroll
    for (int dg = 0; dg < 4; ++dg) {
        uint32_t tot;
        const uint32_t b = block256_excl(ghist[dg * 256 + threadIdx.x], s_tmp, &tot);
        gbase[dg * 256 + threadIdx.x] = b;
        if (dg == 0 && threadIdx.x == 0) bs->n_valid = tot;
        if (dg == 0 && light_b == 256 && threadIdx.x == 0) bs->n_light = tot;
        if (dg == 0 && light_b < 256 && threadIdx.x == light_b) bs->n_light = b;
        if (dg == 0 && threadIdx.x == 0) bs->light_b = light_b;
    }
    if (threadIdx.x == 0)
        bs->pay_ok = bs->max_len < (1u << kPayLenBits) && bs->max_ts - ~bs->inv_min_ts < kPayTsRange;
}

__device__ __forceinline__ bool sort_item(uint32_t i, uint32_t end, int first, uint64_t v) {
    return i < end && !(first && v == kSentinel);
}

// Per-tile digit counts (one block per tile; per-wave LDS counters).
// din (passes >= 1): the digits the previous pass's scatter wrote, one byte per position —
// 4 KiB per tile read instead of 32 KiB of keys (kDig = 512, the 9-bit light passes: one
// 16-bit word per position, 8 KiB per tile).
template <int kDig>
__global__ __launch_bounds__(256) void k_tile_hist(const uint64_t *__restrict__ in, uint32_t L_host,
                                                   const uint32_t *L_dev, uint32_t shift, uint32_t dmask,
                                                   int first, uint32_t *__restrict__ thist, uint32_t tcap,
                                                   const void *__restrict__ din) {
    static_assert(kDig == 256 || kDig == 512, "8- or 9-bit digits");
    constexpr int kPer = kDig / 256;   // digits per thread
    __shared__ uint32_t sh[4][kDig];
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    const uint32_t L = L_dev ? *L_dev : L_host;
    const uint32_t nact = (L + kSortTile - 1) / kSortTile;   // tiles of this pass
    if (blockIdx.x >= nact) return;
    // (XCD-aware order: neighbouring tiles' counts share the lines of each digit row)
    const uint32_t t = xcd_swizzle(blockIdx.x, nact);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < kPer; ++q) sh[k][tid + 256 * q] = 0;
    __syncthreads();
    const uint32_t t0 = t * kSortTile, end = min(L, t0 + kSortTile);
    const uint32_t lane = lane_id();
    auto store_rows = [&]() {   // digit-major rows (only the dmask + 1 live digits)
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const uint32_t d = tid + 256u * (uint32_t)q;
            if (d <= dmask) thist[(size_t)d * tcap + t] = sh[0][d] + sh[1][d] + sh[2][d] + sh[3][d];
        }
    };
    if (din) {   // thread x: positions t0 + 16x .. t0 + 16x + 15
        static_assert(kSortTile == 16 * 256, "16 digits per thread");
        const uint32_t p0 = t0 + 16u * tid;
        constexpr uint32_t kW = kDig == 256 ? 4 : 8;   // 32-bit words of the thread's 16 digits
        constexpr uint32_t kB = kDig == 256 ? 8 : 16;  // bits per digit slot
        uint32_t wd[kW];
#pragma unroll
        for (uint32_t k = 0; k < kW; ++k) wd[k] = 0;
        if (p0 + 16u <= end) {
            const uint4 *src = reinterpret_cast<const uint4 *>(static_cast<const uint8_t *>(din) + (size_t)p0 * (kB / 8));
#pragma unroll
            for (uint32_t k = 0; k < kW / 4; ++k) {
                const uint4 x = src[k];
                wd[4 * k] = x.x; wd[4 * k + 1] = x.y; wd[4 * k + 2] = x.z; wd[4 * k + 3] = x.w;
            }
        } else {
            for (uint32_t k = 0; k < 16; ++k)
                if (p0 + k < end) {
                    const uint32_t x = kDig == 256 ? (uint32_t)static_cast<const uint8_t *>(din)[p0 + k]
                                                   : (uint32_t)static_cast<const uint16_t *>(din)[p0 + k];
                    wd[k * kB / 32] |= x << ((k * kB) & 31);
                }
        }
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const bool ok = p0 + k < end;
            const uint32_t d = (wd[k * kB / 32] >> ((k * kB) & 31)) & dmask;
            const uint64_t act = __ballot(ok);
            if (!act) continue;
            const int lead = __ffsll((unsigned long long)act) - 1;
            const uint32_t dl = __shfl(d, lead);
            if (__ballot(ok && d == dl) == act) {
                if ((int)lane == lead) atomicAdd(&sh[w][dl], (uint32_t)__popcll(act));
            } else if (ok) {
                atomicAdd(&sh[w][d], 1u);
            }
        }
        __syncthreads();
        store_rows();
        return;
    }
    // 16-byte loads: thread x holds keys 2(256 r + x) and 2(256 r + x) + 1 (the order of
    // a histogram's inputs is irrelevant)
    uint64_t v[kSortItems];
    auto item = [&](int r) { return t0 + 2u * ((uint32_t)(r >> 1) * 256u + tid) + (uint32_t)(r & 1); };
    if (t0 + kSortTile <= end) {
#pragma unroll
        for (int r = 0; r < kSortItems; r += 2) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(in + item(r));
            v[r] = x.x; v[r + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < kSortItems; ++r) v[r] = item(r) < end ? in[item(r)] : kSentinel;
    }
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        const uint32_t i = item(r);
        const bool ok = sort_item(i, end, first, v[r]);
        const uint32_t d = (uint32_t)(v[r] >> shift) & dmask;
        const uint64_t act = __ballot(ok);
        if (!act) continue;
        // runs of one heavy source make whole waves share a digit: one add for them
        const int lead = __ffsll((unsigned long long)act) - 1;
        const uint32_t dl = __shfl(d, lead);
        if (__ballot(ok && d == dl) == act) {
            if ((int)lane == lead) atomicAdd(&sh[w][dl], (uint32_t)__popcll(act));
        } else if (ok) {
            atomicAdd(&sh[w][d], 1u);
        }
    }
    __syncthreads();
    store_rows();   // (one partial line per count)
}

// Block d: offs[d][t] = base[d] + sum of thist[d][t'] over t' < t (in place), in chunks of
// 4096 tiles with a running carry: a chunk's counts are loaded and stored coalesced (16 per
// thread, strided by 256) and staged through LDS (padded: conflict-free), where thread x
// scans the 16 consecutive tiles 16x..16x+15. A light pass of a 64M-packet batch (~8K tiles)
// is two chunks: the scan is a chain of block scans on the front's critical path.
#ifndef FSX_TILE_SCAN_WIDE
#define FSX_TILE_SCAN_WIDE 1   // 0: round 4's chunks of 1024 tiles, 4 per thread (A/B)
#endif
// gbase == nullptr (the 9-bit light passes, whose digit totals k_parse does not count): the
// rows are scanned from 0 and each digit's total goes to tot[d] (k_digit_base turns those
// into the bases the scatter adds).
__global__ __launch_bounds__(256) void k_tile_scan(uint32_t *__restrict__ thist, uint32_t tcap,
                                                   uint32_t L_host, const uint32_t *L_dev,
                                                   const uint32_t *__restrict__ gbase,
                                                   uint32_t *__restrict__ tot_out = nullptr) {
    __shared__ uint32_t s_tmp[4];
    const uint32_t L = L_dev ? *L_dev : L_host;
    const uint32_t ntiles = (L + kSortTile - 1) / kSortTile;
    uint32_t *row = thist + (size_t)blockIdx.x * tcap;
    uint32_t carry = gbase ? gbase[blockIdx.x] : 0u;
    const uint32_t tid = threadIdx.x;
#if FSX_TILE_SCAN_WIDE
    __shared__ uint32_t s_x[4096 + 256];   // tile e of the chunk at e + e / 16
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 4096u) {
        uint32_t x[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t e = k * 256u + tid;
            x[k] = c0 + e < ntiles ? row[c0 + e] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t e = k * 256u + tid;
            s_x[e + (e >> 4)] = x[k];
        }
        __syncthreads();
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) { x[j] = s_x[tid * 17u + j]; sum += x[j]; }
        uint32_t tot;
        uint32_t off = carry + block256_excl(sum, s_tmp, &tot);
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) { s_x[tid * 17u + j] = off; off += x[j]; }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t e = k * 256u + tid;
            if (c0 + e < ntiles) row[c0 + e] = s_x[e + (e >> 4)];
        }
        carry += tot;
        __syncthreads();
    }
#else
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint32_t i = c0 + tid * 4u;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = i + k < ntiles ? row[i + k] : 0u;
        uint32_t tot;
        uint32_t off = carry + block256_excl(x[0] + x[1] + x[2] + x[3], s_tmp, &tot);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < ntiles) { row[i + k] = off; off += x[k]; }
        carry += tot;
    }
#endif
    if (tot_out && tid == 0) tot_out[blockIdx.x] = carry;
}

// The 9-bit light passes' digit bases: exclusive scan of the 512 digit totals k_tile_scan
// left in tot (in place; thread x: digits 2x, 2x + 1).
__global__ __launch_bounds__(256) void k_digit_base(uint32_t *__restrict__ tot) {
    __shared__ uint32_t s_tmp[4];
    const uint32_t a = tot[2 * threadIdx.x], b = tot[2 * threadIdx.x + 1];
    const uint32_t x = block256_excl(a + b, s_tmp, nullptr);
    tot[2 * threadIdx.x] = x;
    tot[2 * threadIdx.x + 1] = x + a;
}

// One tile: stable rank, global bases from offs(d, tile count of d), LDS-sorted
// tile, runs to the buckets; payload words through the same LDS slots. kDig: 256 (8-bit
// digits) or 512 (the 9-bit light passes of 24- / 25-bit ids); dwide: the next pass's
// digit goes to dout as a 16-bit word (a 9-bit next digit), else a byte.
template <bool kLatePay, class Offs, int kDig = 256>
__device__ __forceinline__ void sort_tile(uint32_t t, const uint64_t *__restrict__ in,
                                          uint64_t *__restrict__ out, uint32_t L, uint32_t shift,
                                          uint32_t dmask, int first, const BatchState *bs,
                                          const uint64_t *__restrict__ pin, uint64_t *__restrict__ pout,
                                          const uint64_t *__restrict__ ts,
                                          const uint32_t *__restrict__ len, Offs offs,
                                          void *__restrict__ dout = nullptr, uint32_t nshift = 0,
                                          uint32_t nmask = 0, bool dwide = false) {
    static_assert(kDig == 256 || kDig == 512, "8- or 9-bit digits");
    constexpr int kPer = kDig / 256;   // digits per thread
    __shared__ unsigned long long s_el[kSortTile];
    __shared__ uint32_t s_wc[4][kDig];
    __shared__ uint32_t s_dst[kDig], s_tbase[kDig], s_tcnt[kDig];
    __shared__ uint32_t s_tmp[4];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
#pragma unroll
    for (int k = 0; k < 4 * kPer; ++k) s_wc[w][lane * 4 * kPer + k] = 0;
    __syncthreads();
    FSX_STAMP(t, 0);
    const uint32_t t0 = t * kSortTile;
    const uint32_t end = min(L, t0 + kSortTile);
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    uint64_t v[kSortItems];
    uint32_t lr[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        const uint32_t i = t0 + w * (kSortItems * 64u) + (uint32_t)r * 64u + lane;
        v[r] = i < end ? in[i] : kSentinel;
    }
    // payload words: built from (ts, len) in pass 0 (positions are arrival indices
    // there), carried afterwards
    const bool pay = bs->pay_ok != 0;
    uint64_t pv[kSortItems];
    auto load_pay = [&]() {
        const uint64_t tbase = ~bs->inv_min_ts;
#pragma unroll
        for (int r = 0; r < kSortItems; ++r) {
            const uint32_t i = t0 + w * (kSortItems * 64u) + (uint32_t)r * 64u + lane;
            if (first) pv[r] = i < end ? ((ts[i] - tbase) << kPayLenBits) | len[i] : 0ull;
            else pv[r] = i < end ? pin[i] : 0ull;
        }
    };
    // kLatePay: load the payload words only after the keys are out (fewer live
    // registers through the ranking, one more memory latency per tile)
    if (!kLatePay && pay) load_pay();
    // Stable ranking inside the wave: lanes with equal digits are matched by ballots
    // (one compare for a wave that shares a digit), the group leader reserves the
    // group's slots with one returning LDS add, and the group reads the old count from
    // its leader. A wave's LDS operations execute in order, so consecutive items'
    // reservations need no round trip in between.
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        const uint32_t i = t0 + w * (kSortItems * 64u) + (uint32_t)r * 64u + lane;
        const bool valid = sort_item(i, end, first, v[r]);
        const uint64_t act = __ballot(valid);
        const uint32_t d = (uint32_t)(v[r] >> shift) & dmask;
        const int lead0 = act ? __ffsll((unsigned long long)act) - 1 : 0;
        const uint32_t dl = __shfl(d, lead0);
        const uint64_t peers = __ballot(valid && d == dl) == act ? act : match_digit<kDig == 256 ? 8 : 9>(d, act);
        const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
        uint32_t base = 0;
        if (valid && below == 0) base = atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
        base = __shfl(base, __ffsll((unsigned long long)peers) - 1);
        lr[r] = valid ? base + below : 0xFFFFFFFFu;
    }
    __syncthreads();
    FSX_STAMP(t, 1);
    // thread x owns digits kPer * x .. kPer * x + kPer - 1 (consecutive: one block scan)
    uint32_t c[kPer][4], tc[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const uint32_t d = kPer * tid + q;
#pragma unroll
        for (int k = 0; k < 4; ++k) c[q][k] = s_wc[k][d];
        tc[q] = c[q][0] + c[q][1] + c[q][2] + c[q][3];
        s_dst[d] = d <= dmask ? offs(d, tc[q]) : 0u;   // rows of dead digits are never written
    }
    __syncthreads();
    FSX_STAMP(t, 2);
    uint32_t tsum = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const uint32_t d = kPer * tid + q;
        s_wc[0][d] = 0; s_wc[1][d] = c[q][0]; s_wc[2][d] = c[q][0] + c[q][1]; s_wc[3][d] = c[q][0] + c[q][1] + c[q][2];
        s_tcnt[d] = tc[q];
        tsum += tc[q];
    }
    uint32_t tb = block256_excl(tsum, s_tmp, nullptr);
#pragma unroll
    for (int q = 0; q < kPer; ++q) { s_tbase[kPer * tid + q] = tb; tb += tc[q]; }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        if (lr[r] != 0xFFFFFFFFu) {
            const uint32_t dd = (uint32_t)(v[r] >> shift) & dmask;
            lr[r] += s_tbase[dd] + s_wc[w][dd];  // tile-sorted slot
            s_el[lr[r]] = v[r];
        }
    }
    __syncthreads();
    FSX_STAMP(t, 3);
    const uint32_t T = s_tbase[kDig - 1] + s_tcnt[kDig - 1];
    uint32_t dst[kSortItems];
#pragma unroll
    for (int m = 0; m < kSortItems; ++m) {
        const uint32_t j = tid + 256u * (uint32_t)m;
        if (j < T) {
            const uint64_t x = s_el[j];
            const uint32_t dd = (uint32_t)(x >> shift) & dmask;
            dst[m] = s_dst[dd] + (j - s_tbase[dd]);
            out[dst[m]] = x;
            if (dout) {   // (the next pass's digit)
                const uint32_t nd = (uint32_t)(x >> nshift) & nmask;
                if (dwide) static_cast<uint16_t *>(dout)[dst[m]] = (uint16_t)nd;
                else static_cast<uint8_t *>(dout)[dst[m]] = (uint8_t)nd;
            }
        }
    }
    FSX_STAMP(t, 4);
    if (!pay) return;
    if (kLatePay) load_pay();
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; ++r)
        if (lr[r] != 0xFFFFFFFFu) s_el[lr[r]] = pv[r];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kSortItems; ++m) {
        const uint32_t j = tid + 256u * (uint32_t)m;
        if (j < T) pout[dst[m]] = s_el[j];
    }
    FSX_STAMP(t, 5);
}

constexpr bool kLatePayDefault = true;
#ifndef FSX_SCATTER_MINB
#define FSX_SCATTER_MINB 3   // waves/SIMD bound of k_tile_scatter (A/B: scripts/build_variant.sh; 4: profiles/r04/ab_r04z.txt)
#endif

struct TileOffs {
    const uint32_t *offs;
    uint32_t tcap, t;
    __device__ __forceinline__ uint32_t operator()(uint32_t d, uint32_t) const {
        return offs[(size_t)d * tcap + t];
    }
};
// (the 9-bit plan's light passes: rows scanned from 0, the digit bases from k_digit_base)
struct TileOffsB {
    const uint32_t *offs, *base;
    uint32_t tcap, t;
    __device__ __forceinline__ uint32_t operator()(uint32_t d, uint32_t) const {
        return base[d] + offs[(size_t)d * tcap + t];
    }
};

template <bool kLatePay, int kDig = 256, bool kBase = false>
__global__ __launch_bounds__(256, kLatePay ? FSX_SCATTER_MINB : 1) void k_tile_scatter(const uint64_t *__restrict__ in,
                                                      uint64_t *__restrict__ out, uint32_t L_host,
                                                      const uint32_t *L_dev, uint32_t shift, uint32_t dmask,
                                                      int first, const uint32_t *__restrict__ offs,
                                                      uint32_t tcap,
                                                      const BatchState *bs,
                                                      const uint64_t *__restrict__ pin,
                                                      uint64_t *__restrict__ pout,
                                                      const uint64_t *__restrict__ ts,
                                                      const uint32_t *__restrict__ len,
                                                      void *__restrict__ dout, uint32_t nshift,
                                                      uint32_t nmask, const uint32_t *__restrict__ dbase,
                                                      int dwide) {
    const uint32_t L = L_dev ? *L_dev : L_host;
    const uint32_t nact = (L + kSortTile - 1) / kSortTile;   // tiles of this pass
    if (blockIdx.x >= nact) return;
    const uint32_t t = xcd_swizzle(blockIdx.x, nact);
    if constexpr (kBase)
        sort_tile<kLatePay, TileOffsB, kDig>(t, in, out, L, shift, dmask, first, bs, pin, pout, ts, len,
                                             TileOffsB{offs, dbase, tcap, t}, dout, nshift, nmask, dwide != 0);
    else
        sort_tile<kLatePay, TileOffs, kDig>(t, in, out, L, shift, dmask, first, bs, pin, pout, ts, len,
                                            TileOffs{offs, tcap, t}, dout, nshift, nmask, dwide != 0);
}

// ---- pass 0 with the heavy sources outside the sort (k_parse<..., kHf>; fsx_heavy.hip).
// One block per sort tile t, wave w = the tile's parse chunk w (1024 arrival positions).
// kRecs = false (FSX_PARSE_PAY, the default): k_parse computed the clock facts and wrote each
// light word's payload word beside it, and k_heavy_recs builds the tile records in the tail,
// so this is step 2 alone — the chunk's light words and payload words read from their
// compacted runs, ranked and scattered (16 B read + 16 B written per light entry).
// kRecs = true (round 4):
//   1. every packet's timestamp, length and verdict byte (coalesced): the batch's clock facts
//      (non-decreasing?, min / max, tile span), and for every heavy source h (byte 0x80 | h)
//      its sums over the tile (HeavyTileRec): lengths, squared lengths, first / last
//      timestamp and the gaps between its consecutive packets — a packet's predecessor is
//      the last lane below it with the same h (eight ballots), else the wave's last packet
//      of h in an earlier row; the waves' chunks are joined at the tile end;
//   2. pass 0 of the light sort words, which k_parse compacted per chunk (chunk_cnt): the
//      stable in-tile ranking of sort_tile. The payload words come from step 1's registers:
//      the chunk's light words mark their packets in an LDS bitmap, every lane compacts the
//      payload words of its light packets into the wave's LDS row, and light word j of the
//      chunk takes entry j (k_parse compacted them in arrival order). (Gathering them from
//      ts / len by arrival index missed L2 beside the tail kernels: 0.8 GB per batch.)
#ifndef FSX_PASS0H_GATHER
#define FSX_PASS0H_GATHER 0   // 1: the payload words gathered from ts / len (A/B)
#endif
// (k_pass0h and k_parse<..., kHf> cut a sort tile into four 1024-packet chunks of 16 rows)
static_assert(kSortTile == 4096 && kSortItems == 16, "k_pass0h / kHf parse: 4 x 1024-packet chunks per tile");
#ifndef FSX_PASS0H_MINB
#define FSX_PASS0H_MINB FSX_SCATTER_MINB
#endif
template <bool kRecs>
__global__ __launch_bounds__(256, FSX_PASS0H_MINB) void k_pass0h(const uint64_t *__restrict__ in,
                                                                  uint64_t *__restrict__ out, uint32_t n,
                                                                  uint32_t shift, uint32_t dmask,
                                                                  const uint32_t *__restrict__ offs, uint32_t tcap,
                                                                  BatchState *bs, uint64_t *__restrict__ pout,
                                                                  const uint64_t *__restrict__ ts,
                                                                  const uint32_t *__restrict__ len,
                                                                  const uint8_t *__restrict__ tags,
                                                                  const uint32_t *__restrict__ chunk_cnt,
                                                                  const uint64_t *__restrict__ lmask,
                                                                  HeavyTileRec *__restrict__ rec,
                                                                  const HeavySet *__restrict__ hs,
                                                                  const uint64_t *__restrict__ pin,
                                                                  void *__restrict__ dout, uint32_t nshift,
                                                                  uint32_t nmask, int dwide) {
    __shared__ unsigned long long s_el[kSortTile];
    __shared__ uint32_t s_wc[4][256];
    __shared__ uint32_t s_dst[256], s_tbase[256], s_tcnt[256];
    __shared__ uint32_t s_tmp[4];
    __shared__ unsigned long long s_red[4][3];
    __shared__ uint32_t s_flag[4];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    if (blockIdx.x >= ntiles) return;
    const uint32_t t = xcd_swizzle(blockIdx.x, ntiles);
    const uint32_t t0 = t * kSortTile;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint32_t c0 = t0 + w * 1024u;
    unsigned long long *row = s_el + w * 1024u;
    if constexpr (!kRecs) {   // (k_parse checked the clock inside each tile; here across tiles)
        if (tid == 0 && t > 0 && t0 < n && ts[t0] < ts[t0 - 1]) atomicOr(&bs->nonmono, 1u);
    }
    if constexpr (kRecs) {
    const uint32_t nh = hs->n;
    const uint64_t tb = ts[0];
    // ---- 1. heavy sums and clock facts (LDS: the scratch region of s_el)
    uint32_t *h_s1 = reinterpret_cast<uint32_t *>(s_el);            // [128]
    uint32_t *h_dmax = h_s1 + kHeavyMax;                            // [128]
    uint32_t *h_fo = h_dmax + kHeavyMax;                            // [128]
    unsigned long long *h_s2 = s_el + 256;                          // [128] (bytes 2048..)
    unsigned long long *h_d2 = h_s2 + kHeavyMax;                    // [128]
    unsigned long long *h_first = h_d2 + kHeavyMax;                 // [4][128]
    unsigned long long *h_last = h_first + 4 * kHeavyMax;           // [4][128]
    constexpr unsigned long long kNone = ~0ull;
    if (tid < kHeavyMax) {
        h_s1[tid] = 0; h_dmax[tid] = 0; h_fo[tid] = 0xFFFFFFFFu;
        h_s2[tid] = 0; h_d2[tid] = 0;
    }
    for (uint32_t j = tid; j < 4 * kHeavyMax; j += 256) { h_first[j] = kNone; h_last[j] = kNone; }
    __syncthreads();
    uint64_t prev_t = lane == 0 && c0 > 0 && c0 < n ? ts[c0 - 1] : 0ull;   // (lane 0: before the chunk)
    uint32_t nonmono = 0;
    uint64_t mx = 0, imn = 0;   // max, ~min
    // the chunk's 16 rows loaded up front (the LDS ordering below is a compiler barrier: loads
    // issued inside the row loop would each wait a full memory latency)
    uint64_t Tr[16];
    uint32_t Lr[16], Gr[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t i = c0 + r * 64u + lane;
        const bool live = i < n;
        Tr[r] = ts[live ? i : 0u];
        Lr[r] = len[live ? i : 0u];
        Gr[r] = live ? tags[i] : 0u;
    }
    uint64_t Pr[16];   // the payload words of the lane's packets (step 2)
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        const uint32_t i = c0 + r * 64u + lane;
        const bool live = i < n;
        const uint64_t T = live ? Tr[r] : 0ull;
        const uint32_t L = live ? Lr[r] : 0u;
        const uint32_t g = Gr[r];
        uint64_t pv = __shfl_up(T, 1);
        if (lane == 0) pv = (c0 + r * 64u > 0) ? prev_t : T;
        if (live) {
            nonmono |= T < pv ? 1u : 0u;
            mx = T > mx ? T : mx;
            imn = ~T > imn ? ~T : imn;
        }
        prev_t = __shfl(T, 63);
        const bool hv = g >= 0x80u && (g & 0x7Fu) < nh;
        const uint64_t act = __ballot(hv);
        if (act) {
            const uint32_t h = g & 0x7Fu;
            const uint64_t peers = match_digit(h, act);   // (every lane: ballots)
            const uint64_t below = peers & lt_mask;
            const uint32_t pl = below ? 63u - (uint32_t)__clzll((long long)below) : lane;
            const uint64_t tpl = __shfl(T, (int)pl);
            if (hv) {
                uint64_t tp = tpl;
                bool gap = below != 0;
                if (!gap) {   // first of h in this row: the wave's last packet of h so far
                    tp = h_last[w * kHeavyMax + h];
                    gap = tp != kNone;
                    if (!gap) {
                        h_first[w * kHeavyMax + h] = T;
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
                if ((peers >> lane) == 1ull) h_last[w * kHeavyMax + h] = T;   // the row's last of h
            }
            wave_lds_order();
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) Pr[r] = ((Tr[r] - tb) << kPayLenBits) | Lr[r];
    // the chunk's light-packet masks (k_parse; wave-uniform: scalar loads)
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(c0 >> 6);
    uint64_t Mr[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) Mr[r] = !FSX_PASS0H_GATHER && (s0 + r) * 64u < n ? lmask[s0 + r] : 0ull;
    nonmono = __ballot(nonmono != 0) ? 1u : 0u;
    mx = wave_max(mx);
    imn = wave_max(imn);
    if (lane == 0) { s_red[w][0] = mx; s_red[w][1] = imn; s_flag[w] = nonmono; }
    __syncthreads();
    if (tid < kHeavyMax) {   // join the waves' chunks: the gaps across chunk boundaries
        const uint32_t h = tid;
        uint64_t d2 = h_d2[h], first = kNone, last = kNone;
        uint32_t dm = h_dmax[h];
        for (uint32_t ww = 0; ww < 4; ++ww) {
            const uint64_t f = h_first[ww * kHeavyMax + h];
            if (f == kNone) continue;
            if (last != kNone) {
                const uint64_t d = f - last;
                d2 += d * d;
                const uint32_t d32 = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
                dm = d32 > dm ? d32 : dm;
            } else {
                first = f;
            }
            last = h_last[ww * kHeavyMax + h];
        }
        HeavyTileRec &R = rec[t];
        R.s1[h] = h_s1[h]; R.dmax[h] = dm; R.fo[h] = h_fo[h];
        R.s2[h] = h_s2[h]; R.t0[h] = first; R.t1[h] = last; R.d2[h] = d2;
    }
    if (tid == 0) {
        uint64_t m = 0, im = 0;
        uint32_t nm = 0;
        for (int k = 0; k < 4; ++k) {
            m = s_red[k][0] > m ? s_red[k][0] : m;
            im = s_red[k][1] > im ? s_red[k][1] : im;
            nm |= s_flag[k];
        }
        if (nm) atomicOr(&bs->nonmono, 1u);
        if (m - ~im >= (1ull << 32) && m >= ~im) atomicOr(&bs->span_big, 1u);
        atomicMax(reinterpret_cast<unsigned long long *>(&bs->max_ts), (unsigned long long)m);
        atomicMax(reinterpret_cast<unsigned long long *>(&bs->inv_min_ts), (unsigned long long)im);
    }
    __syncthreads();
    // the payload words of the chunk's light packets in arrival order: row w * 1024 + j of s_el
    // (light word j of the chunk is its j-th light packet)
    if constexpr (!FSX_PASS0H_GATHER) {
        uint32_t run = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint64_t m = Mr[r];
            if ((m >> lane) & 1ull) row[run + (uint32_t)__popcll(m & lt_mask)] = Pr[r];
            run += (uint32_t)__popcll(m);
        }
    }
    }   // kRecs
    // ---- 2. pass 0 of the tile's light words (sort_tile, keys from the chunk runs)
#pragma unroll
    for (int k = 0; k < 4; ++k) s_wc[w][lane * 4 + k] = 0;
    __syncthreads();
    const uint32_t ccnt = chunk_cnt[t * 4u + w];
    uint64_t v[kSortItems];
    uint32_t lr[kSortItems];
    uint64_t pv[kSortItems];   // payload words (ts - ts[0]) << kPayLenBits | len (k_hmode: pay_ok)
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        const uint32_t j = (uint32_t)r * 64u + lane;
        v[r] = j < ccnt ? in[c0 + j] : kSentinel;
        if constexpr (!kRecs) pv[r] = j < ccnt ? pin[c0 + j] : 0ull;   // (k_parse's, compacted like the words)
    }
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        const bool valid = v[r] != kSentinel;
        const uint64_t act = __ballot(valid);
        const uint32_t d = (uint32_t)((v[r] & ~kFreshBit) >> shift) & dmask;
        const int lead0 = act ? __ffsll((unsigned long long)act) - 1 : 0;
        const uint32_t dl = __shfl(d, lead0);
        const uint64_t peers = __ballot(valid && d == dl) == act ? act : match_digit(d, act);
        const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
        uint32_t base = 0;
        if (valid && below == 0) base = atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
        base = __shfl(base, __ffsll((unsigned long long)peers) - 1);
        lr[r] = valid ? base + below : 0xFFFFFFFFu;
    }
    if constexpr (kRecs && !FSX_PASS0H_GATHER) {
#pragma unroll
        for (int r = 0; r < kSortItems; ++r)
            pv[r] = lr[r] != 0xFFFFFFFFu ? row[(uint32_t)r * 64u + lane] : 0ull;
    }
    __syncthreads();
    const uint32_t d = tid;
    const uint32_t q0 = s_wc[0][d], q1 = s_wc[1][d], q2 = s_wc[2][d], q3 = s_wc[3][d];
    const uint32_t tc = q0 + q1 + q2 + q3;
    s_dst[d] = d <= dmask && tc ? offs[(size_t)d * tcap + t] : 0u;
    __syncthreads();
    s_wc[0][d] = 0; s_wc[1][d] = q0; s_wc[2][d] = q0 + q1; s_wc[3][d] = q0 + q1 + q2;
    s_tcnt[d] = tc;
    s_tbase[d] = block256_excl(tc, s_tmp, nullptr);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; ++r) {
        if (lr[r] != 0xFFFFFFFFu) {
            const uint32_t dd = (uint32_t)((v[r] & ~kFreshBit) >> shift) & dmask;
            lr[r] += s_tbase[dd] + s_wc[w][dd];
            s_el[lr[r]] = v[r];
        }
    }
    __syncthreads();
    const uint32_t T = s_tbase[255] + s_tcnt[255];
    uint32_t dst[kSortItems];
#pragma unroll
    for (int m = 0; m < kSortItems; ++m) {
        const uint32_t j = tid + 256u * (uint32_t)m;
        if (j < T) {
            const uint64_t x = s_el[j];
            const uint32_t dd = (uint32_t)((x & ~kFreshBit) >> shift) & dmask;
            dst[m] = s_dst[dd] + (j - s_tbase[dd]);
            out[dst[m]] = x;
            if (dout) {   // (pass 1's digit: a byte, or a 16-bit word for a 9-bit digit)
                const uint32_t nd = (uint32_t)((x & ~kFreshBit) >> nshift) & nmask;
                if (dwide) static_cast<uint16_t *>(dout)[dst[m]] = (uint16_t)nd;
                else static_cast<uint8_t *>(dout)[dst[m]] = (uint8_t)nd;
            }
        }
    }
    if constexpr (kRecs && FSX_PASS0H_GATHER) {   // (A/B: gathered by arrival index)
        const uint64_t tb = ts[0];
#pragma unroll
        for (int r = 0; r < kSortItems; ++r) {
            if (lr[r] != 0xFFFFFFFFu) {
                const uint32_t i = pk_idx(v[r]);
                pv[r] = ((ts[i] - tb) << kPayLenBits) | len[i];
            } else {
                pv[r] = 0;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; ++r)
        if (lr[r] != 0xFFFFFFFFu) s_el[lr[r]] = pv[r];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kSortItems; ++m) {
        const uint32_t j = tid + 256u * (uint32_t)m;
        if (j < T) pout[dst[m]] = s_el[j];
    }
}

hipError_t launch_pass0h(const uint64_t *in, uint64_t *out, uint32_t n, uint32_t shift, uint32_t dmask,
                         const uint32_t *offs, uint32_t tcap, BatchState *bs, uint64_t *pout, const uint64_t *ts,
                         const uint32_t *len, const uint8_t *tags, const uint32_t *chunk_cnt,
                         const uint64_t *lmask, void *rec, const HeavySet *hs, const uint64_t *pin, hipStream_t st,
                         void *dout, uint32_t nshift, uint32_t nmask, int dwide) {
    const uint32_t ntiles = std::max<uint32_t>(1, (n + kSortTile - 1) / kSortTile);
    if (pin)   // (FSX_PARSE_PAY: the clock facts and payload words came from k_parse)
        k_pass0h<false><<<ntiles, 256, 0, st>>>(in, out, n, shift, dmask, offs, tcap, bs, pout, ts, len, tags,
                                                chunk_cnt, lmask, static_cast<HeavyTileRec *>(rec), hs, pin,
                                                dout, nshift, nmask, dwide);
    else
        k_pass0h<true><<<ntiles, 256, 0, st>>>(in, out, n, shift, dmask, offs, tcap, bs, pout, ts, len, tags,
                                               chunk_cnt, lmask, static_cast<HeavyTileRec *>(rec), hs, nullptr,
                                               dout, nshift, nmask, dwide);
    return hipGetLastError();
}

// ---- onesweep variant (FSX_FLAG_ONESWEEP_SORT): per-digit decoupled look-back.
// Status words are 8-byte {generation, inclusive?, count} granules written with one
// agent-scope store and polled with agent-scope loads; tiles take ids from an atomic
// counter, so a tile only waits on tiles whose blocks already started; every pass of
// every batch has its own generation, so stale words never match.
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr int kLookW = 8;  // predecessor statuses per look-back round trip

__device__ __forceinline__ unsigned long long os_word(uint32_t gen, bool inclusive, uint32_t cnt) {
    return ((unsigned long long)gen << 33) | ((unsigned long long)(inclusive ? 1u : 0u) << 32) | cnt;
}

template <int kLW>
struct LookbackOffs {
    unsigned long long *status;
    const uint32_t *gbase;
    BatchState *bs;
    uint32_t t, gen;
    __device__ __forceinline__ uint32_t operator()(uint32_t d, uint32_t tc) const {
        unsigned long long *my = status + (size_t)t * 256u + d;
        __hip_atomic_store(my, os_word(gen, t == 0, tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t excl = 0;
        if (t == 0) return gbase[d];
        int32_t tt = (int32_t)t - 1;
        uint32_t spins = 0;
        for (;;) {
            unsigned long long wv[kLW];
#pragma unroll
            for (int j = 0; j < kLW; ++j)
                wv[j] = tt - j >= 0 ? __hip_atomic_load(status + (size_t)(tt - j) * 256u + d,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : os_word(gen, true, 0);
            int used = 0;
            bool done = false;
#pragma unroll
            for (int j = 0; j < kLW; ++j) {
                if (done || used < j) break;
                if ((uint32_t)(wv[j] >> 33) != gen) break;  // not published yet
                excl += (uint32_t)wv[j];
                used = j + 1;
                done = ((wv[j] >> 32) & 1ull) != 0;
            }
            if (done) break;
            tt -= used;
            if (used == 0) {
                if (++spins > kSpinLimit) { atomicOr(&bs->err, ERR_SORT_HANG); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __hip_atomic_store(my, os_word(gen, true, excl + tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return gbase[d] + excl;
    }
};

template <int kLW>
__global__ __launch_bounds__(256) void k_onesweep(const uint64_t *__restrict__ in,
                                                  uint64_t *__restrict__ out, uint32_t L_host,
                                                  const uint32_t *L_dev, uint32_t shift, uint32_t dmask,
                                                  const uint32_t *__restrict__ gbase,
                                                  unsigned long long *status, uint32_t *tile_ctr,
                                                  uint32_t gen, int first, BatchState *bs,
                                                  const uint64_t *__restrict__ pin,
                                                  uint64_t *__restrict__ pout,
                                                  const uint64_t *__restrict__ ts,
                                                  const uint32_t *__restrict__ len) {
    __shared__ uint32_t s_tile;
    const uint32_t L = L_dev ? *L_dev : L_host;
    const uint32_t ntiles = (L + kSortTile - 1) / kSortTile;
    if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t t = s_tile;
    if (t >= ntiles) return;
    sort_tile<false>(t, in, out, L, shift, dmask, first, bs, pin, pout, ts, len,
                     LookbackOffs<kLW>{status, gbase, bs, t, gen});
}

// ------------------------------------------------------------------ segment heads
// A source starts wherever the id changes (ids are exact: one per (family, address)).
// Tile = kTile sorted positions; 256 threads x 16 consecutive positions. light_only
// (heavy verdict lists): the heads of [0, n_light) only; each heavy source is one run of
// pass 0 and k_heads_heavy appends those segments from pass 0's bucket counts.
__global__ __launch_bounds__(256) void k_heads_count(const uint64_t *__restrict__ S,
                                                     BatchState *bs,
                                                     const uint8_t *__restrict__ hdr,
                                                     uint8_t *__restrict__ headf,
                                                     uint32_t *__restrict__ tile_cnt,
                                                     uint32_t *__restrict__ sub_cnt, uint32_t light_only,
                                                     uint32_t ord = 0) {
    __shared__ uint32_t s_tmp[4];
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const uint32_t lane = lane_id();
    // (ord: k_ord_fix marked the starts of the sources it separated inside a key-hash run)
    const bool ofix = ord != 0;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // coalesced: round k covers positions [t*kTile + 256k, +256), one per thread
        uint64_t cur[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t p = t * kTile + (uint32_t)k * 256u + threadIdx.x;
            cur[k] = p < M ? S[p] : kSentinel;
        }
        uint32_t cnt = 0;
        uint32_t sub[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t p = t * kTile + (uint32_t)k * 256u + threadIdx.x;
            uint64_t prev = __shfl_up(cur[k], 1);
            if (lane == 0 && p > 0 && p < M) prev = S[p - 1];
            if (p < M) {
                const bool h = p == 0 || ((prev ^ cur[k]) & ~kFreshBit) >> kIdShift != 0 || (ofix && headf[p]);
                headf[p] = h ? 1u : 0u;
                cnt += h;
                sub[k >> 2] += h;
            }
        }
        // per-1024-position sub-tile head counts (flow tiles, fsx_flows.hip)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t st;
            block256_excl(sub[j], s_tmp, &st);
            if (threadIdx.x == 0 && sub_cnt) sub_cnt[t * 4 + j] = st;
            sub[j] = 0;
        }
        uint32_t tot;
        block256_excl(cnt, s_tmp, &tot);
        if (threadIdx.x == 0) tile_cnt[t] = tot;
    }
}

// Single block: exclusive scan of per-tile counts (in place), nseg, seg_start[nseg]=M.
// (256 threads, four tiles each per round: a single block of this size still finds a CU
// while the side streams' grids occupy the chip)
__global__ __launch_bounds__(256) void k_scan_tiles_u32(uint32_t *__restrict__ cnt, BatchState *bs,
                                                        uint32_t *seg_start, uint32_t light_only) {
    __shared__ uint32_t s_tmp[4];
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint32_t i = c0 + threadIdx.x * 4u;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = i + k < ntiles ? cnt[i + k] : 0u;
        uint32_t tot;
        uint32_t off = carry + block256_excl(x[0] + x[1] + x[2] + x[3], s_tmp, &tot);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < ntiles) { cnt[i + k] = off; off += x[k]; }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        bs->nseg = carry;
        seg_start[carry] = M;
    }
}

__global__ __launch_bounds__(256) void k_heads_write(BatchState *bs, const uint8_t *__restrict__ headf,
                                                     const uint32_t *__restrict__ tile_off,
                                                     uint32_t *__restrict__ seg_start,
                                                     const uint64_t *__restrict__ S,
                                                     uint32_t *__restrict__ seg_slot, uint64_t id_mask,
                                                     uint32_t light_only, uint32_t *__restrict__ seg_lo) {
    __shared__ uint32_t s_tmp[4];
    __shared__ uint32_t s_pos[kTile];   // the tile's head positions, compacted
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    for (uint32_t b = blockIdx.x; b < ntiles; b += gridDim.x) {
        // XCD-aware order: the compacted runs of neighbouring tiles share cache lines
        const uint32_t t = xcd_swizzle(b, ntiles);
        const uint32_t p0 = t * kTile + threadIdx.x * 16u;
        uint32_t f[4] = {0, 0, 0, 0};
        if (p0 + 16 <= M) {
            const uint4 v = *reinterpret_cast<const uint4 *>(headf + p0);
            f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
        } else {
            for (uint32_t k = 0; p0 + k < M && k < 16; ++k) f[k >> 2] |= (uint32_t)headf[p0 + k] << (8 * (k & 3));
        }
        uint32_t cnt = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) cnt += __popc(f[k] & 0x01010101u);
        uint32_t tot;
        uint32_t off = block256_excl(cnt, s_tmp, &tot);
        // positions through LDS, then written out by consecutive threads (a tile full of
        // one-packet sources, config 5's carpet, has 4096 heads: 16 per thread would be
        // 16 strided 4-byte stores per array)
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((f[k >> 2] >> (8 * (k & 3))) & 1u) s_pos[off++] = p0 + k;
        __syncthreads();
        const uint32_t base = tile_off[t];
        for (uint32_t j = threadIdx.x; j < tot; j += 256u) {
            const uint32_t p = s_pos[j];
            seg_start[base + j] = p;
            const uint64_t v = S[p];
            if (seg_slot) seg_slot[base + j] = pk_id(v, id_mask);   // id = table slot
            if (seg_lo) seg_lo[base + j] = (uint32_t)v;
        }
        __syncthreads();
    }
}

// The heavy sources' segments after the light ones (light_only heads): non-empty heavy
// bucket h of pass 0 is segment nseg_light + (its rank among the non-empty buckets), its
// run [gbase, gbase + count) as positions; nseg and the end sentinel follow.
__global__ __launch_bounds__(256) void k_heads_heavy(BatchState *bs, const uint32_t *__restrict__ cnt0,
                                                     const uint32_t *__restrict__ base0,
                                                     uint32_t *__restrict__ seg_start,
                                                     uint32_t *__restrict__ seg_slot,
                                                     const uint64_t *__restrict__ S, uint64_t id_mask,
                                                     uint32_t *__restrict__ seg_lo, const HeavySet *hs) {
    __shared__ uint32_t s_tmp[4];
    const uint32_t h = threadIdx.x;
    const uint32_t L = bs->nseg;   // light segments (k_scan_tiles_u32); read before the barrier
    const uint32_t lb = bs->light_b;
    const bool live = h < kHeavyMax && cnt0[lb + h] > 0;
    uint32_t H;
    const uint32_t r = block256_excl(live ? 1u : 0u, s_tmp, &H);
    if (live) {
        const uint32_t a = base0[lb + h];
        seg_start[L + r] = a;
        // (hfast: no runs in S; the heavy sources' slots are resolved in k_heavy_pick)
        const bool runs = !bs->hfast;
        if (seg_slot) seg_slot[L + r] = runs ? pk_id(S[a], id_mask) : hs->slot[h];
        if (seg_lo) seg_lo[L + r] = runs ? (uint32_t)S[a] : 0u;
    }
    if (h == 0) {
        bs->nseg_light = L;
        bs->nseg = L + H;
        seg_start[L + H] = bs->n_valid;
    }
}

// ------------------------------------------------------------------ home-ordered inserts
// (DESIGN.md §3 "Home-ordered inserts") A flood of new sources inserted as k_parse meets them
// claims index heads at random: one 128-byte line read and written back per 8-byte head
// (config 5: 25.8 of 52.6 ms per step). Instead k_parse writes the home-ordered key hash
// (ord_hkey: the first probe slot in the top bits), the sort brings each source's packets
// together in home order, and k_ord_resolve finds / inserts one slot per segment in that order:
// consecutive heads claim neighbouring slots (the lines stay in L2). IPv4 keys are exact (a
// bijection of the address); sources sharing an IPv6 (or mixed-family) key hash are separated
// here: a run of equal hashes holding an IPv6 packet is regrouped stably by (family, address)
// and every source after the first gets a head mark (k_heads_count ORs them in).
constexpr uint32_t kOrdSmall = 8;     // runs up to this length: one thread
constexpr uint32_t kOrdLong = 512;    // longer mixed runs: one wave with the keys in LDS

__device__ __forceinline__ uint32_t ord_key_of(uint64_t w) { return (uint32_t)(w >> kIdShift); }

// The source of a home-ordered sort word (bit 63: IPv6): IPv4 from the key hash itself (no
// memory access), IPv6 from its record's address bytes.
__device__ __forceinline__ uint32_t ord_src(uint64_t w, const uint8_t *hdr, uint64_t seed, uint32_t s,
                                            uint32_t k[4]) {
    if (w >> 63) {
        load_key6(hdr, pk_idx(w), k);
        return 2u;
    }
    k[0] = ord_v4_key(ord_key_of(w), seed, s);
    k[1] = k[2] = k[3] = 0;
    return 1u;
}

// Block-chunked list append: block b owns positions [b * chunk, (b + 1) * chunk); it counts
// its flags, takes its range of the list with ONE atomic (a single counter hit once per wave
// serialized at the L2: 26 ms for config 5), then writes the flagged positions in order.
template <class F>
__device__ __forceinline__ void chunk_append(uint32_t M, uint32_t *counter, uint32_t *out, uint32_t *s_tmp,
                                             const F &flag) {
    const uint32_t chunk = ((M + gridDim.x - 1) / gridDim.x + 255u) & ~255u;
    const uint32_t c0 = blockIdx.x * chunk, c1 = min(M, c0 + chunk);
    if (c0 >= c1) return;
    uint32_t cnt = 0;
    for (uint32_t p = c0 + threadIdx.x; p < c1; p += 256u) cnt += flag(p) ? 1u : 0u;
    uint32_t tot;
    block256_excl(cnt, s_tmp, &tot);
    __shared__ uint32_t s_base;
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(counter, tot) : 0u;
    __syncthreads();
    uint32_t base = s_base;
    for (uint32_t p0 = c0; p0 < c1; p0 += 256u) {
        const uint32_t p = p0 + threadIdx.x;
        const bool f = p < c1 && flag(p);
        uint32_t stot;
        const uint32_t off = block256_excl(f ? 1u : 0u, s_tmp, &stot);
        if (f) out[base + off] = p;
        base += stot;
    }
}

// The starts of the runs of two or more equal key hashes, listed (bs->n_orun).
__global__ __launch_bounds__(256) void k_ord_scan(const uint64_t *__restrict__ S, BatchState *bs,
                                                  uint32_t *__restrict__ runs) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t M = bs->n_valid;
    chunk_append(M, &bs->n_orun, runs, s_tmp, [&](uint32_t p) {
        const uint32_t hk = ord_key_of(S[p]);
        return (p == 0 || ord_key_of(S[p - 1]) != hk) && p + 1 < M && ord_key_of(S[p + 1]) == hk;
    });
}

// One thread per listed run; runs of 2 .. kOrdSmall regrouped in registers, longer ones listed
// (bs->n_ofix, positions in `list`) for k_ord_long.
__global__ __launch_bounds__(256) void k_ord_fix(uint64_t *__restrict__ S, uint64_t *__restrict__ pay,
                                                 BatchState *bs, PacketIn in, const uint32_t *__restrict__ len,
                                                 uint8_t *__restrict__ headf, const uint32_t *__restrict__ runs,
                                                 uint32_t *__restrict__ list, uint64_t seed, uint32_t s) {
    if (bs->err) return;
    const uint32_t M = bs->n_valid, nr = bs->n_orun;
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < nr; r += gridDim.x * 256u) {
        const uint32_t p = runs[r];
        const uint64_t w0 = S[p];
        const uint32_t hk = ord_key_of(w0);
        uint64_t W[kOrdSmall], Pw[kOrdSmall];
        uint32_t L = 0;
        bool any6 = false, more = false;
#pragma unroll
        for (uint32_t j = 0; j < kOrdSmall; ++j) {
            const uint64_t x = p + j < M ? S[p + j] : 0ull;
            const bool in_run = p + j < M && ord_key_of(x) == hk && L == j;
            W[j] = x;
            L += in_run ? 1u : 0u;
            any6 |= in_run && (x >> 63);
        }
        if (L == kOrdSmall && p + kOrdSmall < M && ord_key_of(S[p + kOrdSmall]) == hk) more = true;
        if (more) {   // a long run: k_ord_long
            list[atomicAdd(&bs->n_ofix, 1u)] = p;
            continue;
        }
        if (!any6) continue;   // IPv4 only: equal hashes are equal addresses
        uint32_t T[kOrdSmall], K[kOrdSmall][4];
#pragma unroll
        for (uint32_t j = 0; j < kOrdSmall; ++j) {
            K[j][0] = K[j][1] = K[j][2] = K[j][3] = 0;
            T[j] = j < L ? ord_src(W[j], in.hdr, seed, s, K[j]) : 0u;
            Pw[j] = j < L ? pay[p + j] : 0ull;
        }
        // group leader of j: the first entry of its source; rank: stable order by leader
        uint32_t G[kOrdSmall];
#pragma unroll
        for (uint32_t j = 0; j < kOrdSmall; ++j) {
            G[j] = j;
#pragma unroll
            for (uint32_t m = 0; m < kOrdSmall; ++m)
                if (m < j && G[j] == j && T[m] == T[j] && K[m][0] == K[j][0] && K[m][1] == K[j][1] &&
                    K[m][2] == K[j][2] && K[m][3] == K[j][3])
                    G[j] = m;
        }
        bool moved = false;
        uint32_t R[kOrdSmall];
#pragma unroll
        for (uint32_t j = 0; j < kOrdSmall; ++j) {
            uint32_t r = 0;
#pragma unroll
            for (uint32_t m = 0; m < kOrdSmall; ++m)
                r += (m < L && (G[m] < G[j] || (G[m] == G[j] && m < j))) ? 1u : 0u;
            R[j] = r;
            moved |= j < L && r != j;
        }
#pragma unroll
        for (uint32_t j = 0; j < kOrdSmall; ++j) {
            if (j >= L) continue;
            if (moved) {
                S[p + R[j]] = W[j];
                pay[p + R[j]] = Pw[j];
            }
            if (G[j] == j && j > 0) headf[p + R[j]] = 1;   // a further source of the run
        }
    }
}

// A mixed run longer than kOrdLong (a heavy IPv6 source whose 32-bit key hash a flood source
// shares: rare, but not impossible under a flood of ~10^6 IPv6 sources): its sources are taken
// out one at a time, stably — the run's first remaining packet names the next source, one pass
// moves that source's packets to tmp / ptmp (after the sources taken before) and compacts the
// others in place (a write never passes the chunk being read) — then the run is copied back.
// O(L · sources); more than kOrdMaxSrc sources in one run (not reachable by chance): false.
constexpr uint32_t kOrdMaxSrc = 1024;

__device__ bool ord_extract(uint64_t *S, uint64_t *pay, uint8_t *headf, uint64_t *tmp, uint64_t *ptmp,
                            uint32_t p, uint32_t L, const uint8_t *hdr, uint64_t seed, uint32_t s) {
    const uint32_t lane = lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t rem = L, out = 0;
    for (uint32_t round = 0; rem; ++round) {
        if (round == kOrdMaxSrc) return false;
        uint32_t kl[4];
        const uint32_t tl = ord_src(S[p], hdr, seed, s, kl);
        const uint32_t out0 = out;
        uint32_t nm = 0;
        for (uint32_t j0 = 0; j0 < rem; j0 += 64) {
            const uint32_t j = j0 + lane;
            const bool in = j < rem;
            uint64_t x = 0, pw = 0;
            bool match = false;
            if (in) {
                x = S[p + j];
                pw = pay[p + j];
                uint32_t k[4];
                const uint32_t t = ord_src(x, hdr, seed, s, k);
                match = t == tl && k[0] == kl[0] && k[1] == kl[1] && k[2] == kl[2] && k[3] == kl[3];
            }
            const uint64_t mm = __ballot(in && match), mn = __ballot(in && !match);
            if (in && match) {
                const uint32_t o = out + (uint32_t)__popcll(mm & below);
                tmp[p + o] = x;
                ptmp[p + o] = pw;
            } else if (in) {   // (o <= j: only positions this wave has read already)
                const uint32_t o = nm + (uint32_t)__popcll(mn & below);
                S[p + o] = x;
                pay[p + o] = pw;
            }
            out += (uint32_t)__popcll(mm);
            nm += (uint32_t)__popcll(mn);
        }
        if (out0 && lane == 0) headf[p + out0] = 1;   // a further source of the run
        rem = nm;
        __threadfence_block();   // (this wave's compacted words: read back next round)
    }
    __threadfence_block();
    for (uint32_t j = lane; j < L; j += 64) {
        S[p + j] = tmp[p + j];
        pay[p + j] = ptmp[p + j];
    }
    __threadfence_block();
    return true;
}

// One wave per listed run (longer than kOrdSmall): its length, then — if it holds an IPv6
// packet — every packet's (family, address) in LDS, leaders, stable ranks; the words move through
// the idle sort buffer (tmp / ptmp) at the same positions. Longer mixed runs: ord_extract.
__global__ __launch_bounds__(64) void k_ord_long(uint64_t *__restrict__ S, uint64_t *__restrict__ pay,
                                                 BatchState *bs, PacketIn in, const uint32_t *__restrict__ len,
                                                 uint8_t *__restrict__ headf, const uint32_t *__restrict__ list,
                                                 uint64_t *__restrict__ tmp, uint64_t *__restrict__ ptmp, uint64_t seed,
                                                 uint32_t s) {
    __shared__ uint32_t s_t[kOrdLong], s_k[kOrdLong][4], s_g[kOrdLong];
    if (bs->err) return;
    const uint32_t M = bs->n_valid, nl = bs->n_ofix, lane = lane_id();
    for (uint32_t r = blockIdx.x; r < nl; r += gridDim.x) {
        const uint32_t p = list[r];
        const uint32_t hk = ord_key_of(S[p]);
        uint32_t e = p;
        bool any6 = false;
        for (;;) {   // the run's end and whether it holds an IPv6 packet
            const uint32_t q = e + lane;
            const uint64_t x = q < M ? S[q] : 0ull;
            const bool in_run = q < M && ord_key_of(x) == hk;
            const uint64_t m = __ballot(in_run);
            any6 |= __ballot(in_run && (x >> 63)) != 0;
            if (~m) { e += (uint32_t)__ffsll((unsigned long long)~m) - 1u; break; }
            e += 64;
        }
        if (!any6) continue;
        const uint32_t L = e - p;
        // the run's first source against every packet (a repeated source: nothing to move)
        uint32_t k0[4];
        const uint32_t t0 = ord_src(S[p], in.hdr, seed, s, k0);
        bool same = true;
        for (uint32_t j = lane; j < L; j += 64) {
            uint32_t k[4];
            const uint32_t t = ord_src(S[p + j], in.hdr, seed, s, k);
            same &= t == t0 && k[0] == k0[0] && k[1] == k0[1] && k[2] == k0[2] && k[3] == k0[3];
        }
        if (__ballot(!same) == 0) continue;
        if (L > kOrdLong) {   // (an IPv6 flood source sharing a heavy source's hash)
            if (!ord_extract(S, pay, headf, tmp, ptmp, p, L, in.hdr, seed, s)) {
                if (lane == 0) atomicOr(&bs->err, ERR_FIXUP);
                return;
            }
            continue;
        }
        for (uint32_t j = lane; j < L; j += 64) s_t[j] = ord_src(S[p + j], in.hdr, seed, s, s_k[j]);
        __syncthreads();
        for (uint32_t j = lane; j < L; j += 64) {
            uint32_t g = j;
            for (uint32_t m = 0; m < j; ++m)
                if (s_t[m] == s_t[j] && s_k[m][0] == s_k[j][0] && s_k[m][1] == s_k[j][1] &&
                    s_k[m][2] == s_k[j][2] && s_k[m][3] == s_k[j][3]) { g = m; break; }
            s_g[j] = g;
        }
        __syncthreads();
        for (uint32_t j = lane; j < L; j += 64) {
            const uint32_t gj = s_g[j];
            uint32_t rk = 0;
            for (uint32_t m = 0; m < L; ++m) rk += (s_g[m] < gj || (s_g[m] == gj && m < j)) ? 1u : 0u;
            tmp[p + rk] = S[p + j];
            ptmp[p + rk] = pay[p + j];
            if (gj == j && j > 0) headf[p + rk] = 1;
        }
        __syncthreads();   // (global writes of this wave: ordered for its own later reads)
        __threadfence_block();
        for (uint32_t j = lane; j < L; j += 64) {
            S[p + j] = tmp[p + j];
            pay[p + j] = ptmp[p + j];
        }
        __syncthreads();
    }
}

// One thread per segment, in home order: the source from its first word, its slot found or
// inserted from its home (id_resolve, lazy: the head only), the slot into seg_slot and
// "inserted here" into the first word's bit 63 (kFreshBit, the walkers' flood path; bit 63
// marked IPv6 until now). New sources counted. Block b owns a contiguous chunk of segments;
// k_ord_resolve4 takes the IPv4 ones (the key from the hash: no memory access before the
// claim) and leaves the chunk's IPv6 ones in order at the chunk's own positions of `list6`
// (their count in cnt6[b]), so that k_ord_resolve6 — the same blocks — runs them densely,
// without IPv4 lanes waiting on their record reads and key publication.
__device__ __forceinline__ void ord_chunk(uint32_t nseg, uint32_t &c0, uint32_t &c1) {
    const uint32_t chunk = ((nseg + gridDim.x - 1) / gridDim.x + 255u) & ~255u;
    c0 = min(nseg, blockIdx.x * chunk);
    c1 = min(nseg, c0 + chunk);
}

__device__ __forceinline__ bool ord_claim(const IdTable &idt, uint32_t s, uint32_t g, uint64_t *S,
                                          const uint32_t *seg_start, uint32_t *seg_slot, const uint8_t *hdr,
                                          BatchState *bs) {
    const uint32_t a = seg_start[g];
    const uint64_t w = S[a];
    uint32_t k[4];
    const uint32_t tag = ord_src(w, hdr, idt.seed, s, k);
    const uint64_t home = ord_key_of(w) >> (32 - s);
    bool fresh = false;
    const uint32_t id = id_resolve<true>(idt, tag, k, home, idt.head[home], &fresh);
    if (id == kNoSlot) atomicOr(&bs->err, ERR_TABLE_FULL);
    seg_slot[g] = id;
    S[a] = (w & ~kFreshBit) | (fresh ? kFreshBit : 0ull);
    return fresh;
}

// kOrdU segments per thread and step, their loads and first-probe claims in flight together:
// a head whose first probe slot is empty in this epoch is claimed by one CAS issued beside the
// others; a READY head with the source's key is found; anything else (a lost race, a longer
// probe chain, an IPv6 key to compare) takes id_resolve's full protocol from there.
constexpr uint32_t kOrdU = 4;

__device__ __forceinline__ void ord_finish(const IdTable &idt, uint32_t g, uint32_t a, uint64_t w, uint32_t id,
                                           bool fresh, uint64_t *S, uint32_t *seg_slot, BatchState *bs) {
    if (id == kNoSlot) atomicOr(&bs->err, ERR_TABLE_FULL);
    seg_slot[g] = id;
    S[a] = (w & ~kFreshBit) | (fresh ? kFreshBit : 0ull);
}

__global__ __launch_bounds__(256) void k_ord_resolve4(BatchState *bs, const uint32_t *__restrict__ seg_start,
                                                      uint64_t *__restrict__ S, PacketIn in, IdTable idt,
                                                      uint32_t *__restrict__ seg_slot, uint32_t *__restrict__ list6,
                                                      uint32_t *__restrict__ cnt6) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t s = (uint32_t)__popcll(idt.mask), lane = lane_id();
    if (blockIdx.x == 0 && threadIdx.x == 0) bs->ord = 1;
    uint32_t c0, c1;
    ord_chunk(bs->nseg, c0, c1);
    uint32_t nfresh = 0, n6 = 0;
    for (uint32_t g0 = c0; g0 < c1; g0 += 256u * kOrdU) {   // (block-uniform trips)
        uint32_t a[kOrdU], k0[kOrdU];
        uint64_t w[kOrdU], home[kOrdU], hint[kOrdU], prev[kOrdU];
        bool v4[kOrdU], six[kOrdU];
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            const uint32_t g = g0 + u * 256u + threadIdx.x;
            a[u] = g < c1 ? seg_start[g] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            const uint32_t g = g0 + u * 256u + threadIdx.x;
            w[u] = g < c1 ? S[a[u]] : 0ull;
            six[u] = g < c1 && (w[u] >> 63);
            v4[u] = g < c1 && !six[u];
            k0[u] = ord_v4_key(ord_key_of(w[u]), idt.seed, s);
            home[u] = ord_key_of(w[u]) >> (32 - s);
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) hint[u] = v4[u] ? idt.head[home[u]] : 0ull;
        const uint64_t want_hi = id_head(idt.gen, kIdReady, 1u, 0u);
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {   // first-slot claims, all in flight
            const bool empty = v4[u] && (uint32_t)(hint[u] >> 48) != idt.gen;
            prev[u] = empty ? atomicCAS(idt.head + home[u], (unsigned long long)hint[u],
                                        (unsigned long long)(want_hi | k0[u]))
                            : hint[u];
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            bool fresh = false;
            if (v4[u]) {
                const uint32_t g = g0 + u * 256u + threadIdx.x;
                const uint64_t want = want_hi | k0[u];
                const bool empty = (uint32_t)(hint[u] >> 48) != idt.gen;
                uint32_t id;
                if (empty && prev[u] == hint[u]) {   // claimed here
                    fresh = true;
                    id = (uint32_t)home[u];
                    mir_publish(idt.mir, idt.mir_shift, idt.mask, idt.seed, home[u], k0[u]);
                } else if (prev[u] == want) {          // found (or another lane claimed it for us: never —
                    id = (uint32_t)home[u];            // one segment per source)
                } else {
                    const uint32_t kk[4] = {k0[u], 0u, 0u, 0u};
                    id = id_resolve<true>(idt, 1u, kk, home[u], prev[u], &fresh);
                }
                ord_finish(idt, g, a[u], w[u], id, fresh, S, seg_slot, bs);
            }
            nfresh += (uint32_t)__popcll(__ballot(fresh));
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {   // the IPv6 segments, listed in order
            uint32_t t6;
            const uint32_t off = block256_excl(six[u] ? 1u : 0u, s_tmp, &t6);
            if (six[u]) list6[c0 + n6 + off] = g0 + u * 256u + threadIdx.x;
            n6 += t6;
        }
    }
    if (threadIdx.x == 0) cnt6[blockIdx.x] = n6;
    if (lane == 0 && nfresh) atomicAdd(&bs->n_new, nfresh);
}

// The chunk's IPv6 segments, kOrdU per thread: records and first-slot heads loaded together,
// an empty first slot claimed BUSY (CAS), the three key words published by returning
// exchanges for all claims at once, then READY (id_resolve's protocol); the rest by id_resolve.
__global__ __launch_bounds__(256) void k_ord_resolve6(BatchState *bs, const uint32_t *__restrict__ seg_start,
                                                      uint64_t *__restrict__ S, PacketIn in, IdTable idt,
                                                      uint32_t *__restrict__ seg_slot,
                                                      const uint32_t *__restrict__ list6,
                                                      const uint32_t *__restrict__ cnt6) {
    if (bs->err) return;
    const uint32_t s = (uint32_t)__popcll(idt.mask), lane = lane_id();
    uint32_t c0, c1;
    ord_chunk(bs->nseg, c0, c1);
    const uint32_t m = c0 < c1 ? cnt6[blockIdx.x] : 0u;
    uint32_t nfresh = 0;
    const uint64_t busy_hi = id_head(idt.gen, kIdBusy, 2u, 0u), ready_hi = id_head(idt.gen, kIdReady, 2u, 0u);
    for (uint32_t j0 = 0; j0 < m; j0 += 256u * kOrdU) {   // (block-uniform trips)
        uint32_t g[kOrdU], a[kOrdU], k[kOrdU][4];
        uint64_t w[kOrdU], home[kOrdU], hint[kOrdU], prev[kOrdU];
        bool live[kOrdU], claimed[kOrdU];
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            const uint32_t j = j0 + u * 256u + threadIdx.x;
            live[u] = j < m;
            g[u] = live[u] ? list6[c0 + j] : c0;
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) a[u] = live[u] ? seg_start[g[u]] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            w[u] = live[u] ? S[a[u]] : 0ull;
            home[u] = ord_key_of(w[u]) >> (32 - s);
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            if (live[u]) load_key6(in.hdr, pk_idx(w[u]), k[u]);
            else k[u][0] = k[u][1] = k[u][2] = k[u][3] = 0;
            hint[u] = live[u] ? idt.head[home[u]] : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            const bool empty = live[u] && (uint32_t)(hint[u] >> 48) != idt.gen;
            prev[u] = empty ? atomicCAS(idt.head + home[u], (unsigned long long)hint[u],
                                        (unsigned long long)(busy_hi | k[u][0]))
                            : hint[u];
            claimed[u] = empty && prev[u] == hint[u];
        }
        uint32_t r[kOrdU][3];
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {   // the claimed heads' key words, all in flight
            if (claimed[u]) {
                uint32_t *kw = idt.k6 + home[u] * 4;
                r[u][0] = __hip_atomic_exchange(kw + 0, k[u][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                r[u][1] = __hip_atomic_exchange(kw + 1, k[u][2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                r[u][2] = __hip_atomic_exchange(kw + 2, k[u][3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                r[u][0] = r[u][1] = r[u][2] = 0;
            }
        }
        // every claim of this wave READY (after its key words returned) before any lane of it
        // may wait on a BUSY head in id_resolve
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            if (claimed[u]) {
                asm volatile("" ::"v"(r[u][0]), "v"(r[u][1]), "v"(r[u][2]) : "memory");
                __hip_atomic_store(idt.head + home[u], (unsigned long long)(ready_hi | k[u][0]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                ord_finish(idt, g[u], a[u], w[u], (uint32_t)home[u], true, S, seg_slot, bs);
            }
            nfresh += (uint32_t)__popcll(__ballot(claimed[u]));
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrdU; ++u) {
            bool fresh = false;
            if (live[u] && !claimed[u]) {
                const uint32_t id = id_resolve<true>(idt, 2u, k[u], home[u], prev[u], &fresh);
                ord_finish(idt, g[u], a[u], w[u], id, fresh, S, seg_slot, bs);
            }
            nfresh += (uint32_t)__popcll(__ballot(fresh));
        }
    }
    if (lane == 0 && nfresh) atomicAdd(&bs->n_new, nfresh);
}

// Region claims (the ordered path's default): block b takes kRegSeg consecutive segments
// and, exclusively, the heads from its first segment's home to the next block's first home
// (at most kRegMax of them): they are loaded into LDS, every segment probes / claims there
// (LDS CAS; a slot claimed in this block is another source — one segment per source — so no
// key comparison against it), and the block's claims go back to HBM as plain stores (heads,
// IPv6 key words, IPv4 mirror entries): no global atomic for a flood's inserts, which the
// device processes at ~30 G/s (k_ord_resolve4 / 6: 18 ms for config 5's 2^28). A probe that
// leaves the region is spilled to k_ord_spill (the global protocol, after this kernel).
constexpr uint32_t kRegSeg = 512, kRegMax = 2048;
constexpr uint64_t kIdLocal = 3;   // head state in LDS: claimed by this block

__global__ __launch_bounds__(256) void k_ord_claim(BatchState *bs, const uint32_t *__restrict__ seg_start,
                                                   uint64_t *__restrict__ S, PacketIn in, IdTable idt,
                                                   uint32_t *__restrict__ seg_slot, uint32_t *__restrict__ spill,
                                                   uint32_t *__restrict__ nspill, uint32_t *__restrict__ nfresh_b,
                                                   const uint64_t *__restrict__ pay, const uint64_t *__restrict__ ts,
                                                   const uint32_t *__restrict__ len, uint8_t *__restrict__ marks,
                                                   Slot *table, Limits lim) {
    __shared__ unsigned long long H[kRegMax];
    __shared__ uint32_t s_nsp, s_fresh, s_fused;
    __shared__ uint64_t s_r[2];
    if (bs->err) return;
    const uint32_t nseg = bs->nseg, b = blockIdx.x, tid = threadIdx.x;
    const uint32_t c0 = b * kRegSeg;
    if (c0 >= nseg) {
        if (tid == 0) { nspill[b] = 0; nfresh_b[b] = 0; nfresh_b[gridDim.x + b] = 0; }
        return;
    }
    const uint32_t c1 = min(nseg, c0 + kRegSeg);
    const uint32_t s = (uint32_t)__popcll(idt.mask), gen = idt.gen;
    if (tid == 0) {
        s_r[0] = ord_key_of(S[seg_start[c0]]) >> (32 - s);
        s_r[1] = c1 < nseg ? ord_key_of(S[seg_start[c1]]) >> (32 - s) : idt.mask + 1;
        s_nsp = 0;
        s_fresh = 0;
        s_fused = 0;
    }
    __syncthreads();
    const uint64_t R0 = s_r[0];
    const uint32_t Rn = (uint32_t)min<uint64_t>(s_r[1] - R0, kRegMax);
    const bool pay_ok = bs->pay_ok != 0;
    const uint64_t tbase = ~bs->inv_min_ts;
    for (uint32_t r = tid; r < Rn; r += 256u) H[r] = idt.head[R0 + r];
    __syncthreads();
    uint32_t nfr = 0, nfu = 0;
    for (uint32_t j = tid; j < c1 - c0; j += 256u) {
        const uint32_t g = c0 + j, a = seg_start[g];
        const uint64_t w = S[a];
        uint32_t k[4];
        const uint32_t tag = ord_src(w, in.hdr, idt.seed, s, k);
        uint32_t r = (uint32_t)((ord_key_of(w) >> (32 - s)) - R0);
        const uint64_t mine = id_head(gen, kIdLocal, tag, tag == 1 ? k[0] : j);
        int res = 0;   // 1 claimed, 2 found, 3 spilled
        while (!res) {
            if (r >= Rn) { res = 3; break; }
            const unsigned long long cur = H[r];
            if ((uint32_t)(cur >> 48) != gen) {   // empty in this epoch: claim it in LDS
                if (atomicCAS(&H[r], cur, (unsigned long long)mine) == cur) res = 1;
                continue;
            }
            const uint32_t st = (uint32_t)(cur >> 40) & 0xFFu, ct = (uint32_t)(cur >> 32) & 0xFFu;
            if (st == kIdReady && ct == tag && (uint32_t)cur == k[0]) {   // a source of the index
                if (tag == 1) { res = 2; break; }
                const uint32_t *kw = idt.k6 + (R0 + r) * 4;
                if (kw[0] == k[1] && kw[1] == k[2] && kw[2] == k[3]) { res = 2; break; }
            } else if (st != kIdReady && st != kIdLocal) {   // (no BUSY head outside a claim)
                res = 3;
                break;
            }
            ++r;
        }
        if (res == 3) {
            spill[c0 + atomicAdd(&s_nsp, 1u)] = g;
            continue;
        }
        const uint64_t pos = R0 + r;
        if (res == 1) {   // the claim to HBM right away (no other block reads this region):
            ++nfr;        // head READY, IPv6 key words, IPv4 mirror entry
            if (tag == 2) {
                uint32_t *kw = idt.k6 + pos * 4;
                kw[0] = k[1]; kw[1] = k[2]; kw[2] = k[3];
            } else {
                mir_publish(idt.mir, idt.mir_shift, idt.mask, idt.seed, pos, k[0]);
            }
            idt.head[pos] = id_head(gen, kIdReady, tag, k[0]);
            if (seg_start[g + 1] - a == 1) {
                // a new source's only packet (a flood): its walk here — fw_step from no state
                // (src/fsx_kern.c:265-284, :312-326), the mark at its position, its whole line
                // stamped with the batch generation (a failed batch's lines are rolled back; the
                // stamps of a passed one are cleared at the generation wrap) — and no walker
                // visit (seg_slot = kNoSlot)
                uint64_t T;
                uint32_t L;
                if (pay_ok) {
                    const uint64_t pw = pay[a];
                    T = tbase + (pw >> kPayLenBits);
                    L = (uint32_t)pw & ((1u << kPayLenBits) - 1u);
                } else {
                    T = ts[pk_idx(w)];
                    L = len[pk_idx(w)];
                }
                FwState st{false, false, 0, 0, 0, 0};
                MarkWriter<false> mw{marks, 0};
                fw_step(st, T, L, a, lim, mw);
                const uint32_t fl = (st.has_st ? SLOT_HAS_ST : 0u) | (st.has_bl ? SLOT_HAS_BL : 0u) |
                                    (idt.born << kBornShift);
                uint4 *p = reinterpret_cast<uint4 *>(table + pos);
                p[0] = make_uint4(slot_tag(tag, lim.tgen), fl, k[0], tag == 2 ? k[1] : 0u);
                p[1] = make_uint4(tag == 2 ? k[2] : 0u, tag == 2 ? k[3] : 0u, (uint32_t)st.pps, (uint32_t)(st.pps >> 32));
                p[2] = make_uint4((uint32_t)st.bps, (uint32_t)(st.bps >> 32), (uint32_t)st.tt, (uint32_t)(st.tt >> 32));
                p[3] = make_uint4((uint32_t)st.till, (uint32_t)(st.till >> 32), 0u, 0u);
                seg_slot[g] = kNoSlot;
                S[a] = w & ~kFreshBit;
                ++nfu;
                continue;
            }
        }
        seg_slot[g] = (uint32_t)pos;
        S[a] = (w & ~kFreshBit) | (res == 1 ? kFreshBit : 0ull);
    }
    if (nfr) atomicAdd(&s_fresh, nfr);
    if (nfu) atomicAdd(&s_fused, nfu);
    __syncthreads();
    if (tid == 0) { nspill[b] = s_nsp; nfresh_b[b] = s_fresh; nfresh_b[gridDim.x + b] = s_fused; }
}

// The segments k_ord_claim spilled (their probe left the block's region): the global protocol.
__global__ __launch_bounds__(256) void k_ord_spill(BatchState *bs, const uint32_t *__restrict__ seg_start,
                                                   uint64_t *__restrict__ S, PacketIn in, IdTable idt,
                                                   uint32_t *__restrict__ seg_slot, const uint32_t *__restrict__ spill,
                                                   const uint32_t *__restrict__ nspill, uint32_t *__restrict__ nfresh_b) {
    if (bs->err) return;
    const uint32_t b = blockIdx.x, c0 = b * kRegSeg;
    if (c0 >= bs->nseg) return;
    const uint32_t m = nspill[b], s = (uint32_t)__popcll(idt.mask);
    uint32_t nfr = 0;
    for (uint32_t j = threadIdx.x; j < m; j += 256u)
        nfr += ord_claim(idt, s, spill[c0 + j], S, seg_start, seg_slot, in.hdr, bs) ? 1u : 0u;
    if (nfr) atomicAdd(nfresh_b + b, nfr);
}

__global__ void k_bs_flag(BatchState *bs) { bs->ord = 1; }

// Every slot's generation stamp cleared (at the 16-bit batch-generation wrap: k_ord_claim leaves
// the stamps of the lines it writes, which a failed batch of the same generation 65536 batches
// later would otherwise roll back).
__global__ __launch_bounds__(256) void k_born_clear(Slot *table, uint64_t nslots) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256u)
        if (table[i].flags >> kBornShift) table[i].flags &= kFlagBits;
}
hipError_t launch_born_clear(Slot *table, uint64_t nslots, hipStream_t st) {
    k_born_clear<<<4096, 256, 0, st>>>(table, nslots);
    return hipGetLastError();
}

// n_new += the blocks' fresh counts (one block); every segment walked by k_ord_claim: the
// walkers have nothing to do.
__global__ __launch_bounds__(256) void k_ord_count(BatchState *bs, const uint32_t *__restrict__ nfresh_b, uint32_t nb) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    uint64_t t = 0, f = 0;
    for (uint32_t i = threadIdx.x; i < nb; i += 256u) { t += nfresh_b[i]; f += nfresh_b[nb + i]; }
    uint32_t tot, fu;
    block256_excl((uint32_t)t, s_tmp, &tot);
    block256_excl((uint32_t)f, s_tmp, &fu);
    if (threadIdx.x == 0) {
        bs->n_new += tot;
        bs->ord_walked = fu == bs->nseg ? 1u : 0u;
    }
}

hipError_t launch_ord_heads(uint64_t *S, uint64_t *pay, BatchState *bs, const PacketIn &in, const uint32_t *len,
                            uint8_t *headf, uint32_t *list, uint64_t *tmp, uint64_t *ptmp, uint32_t n,
                            uint64_t seed, uint64_t mask, hipStream_t st) {
    const uint32_t s = (uint32_t)__builtin_popcountll(mask);
    hipError_t e;
    if ((e = hipMemsetAsync(headf, 0, n, st)) != hipSuccess) return e;
    const uint32_t grid = std::min<uint32_t>(4096, std::max<uint32_t>(1, (n + 255) / 256));
    // (list: the run starts in [0, n / 2) — a run holds two packets or more —, the long ones after)
    uint32_t *runs = list, *longs = list + n / 2;
    k_ord_scan<<<grid, 256, 0, st>>>(S, bs, runs);
    k_ord_fix<<<grid, 256, 0, st>>>(S, pay, bs, in, len, headf, runs, longs, seed, s);
    k_ord_long<<<1024, 64, 0, st>>>(S, pay, bs, in, len, headf, longs, tmp, ptmp, seed, s);
    return hipGetLastError();
}

// ------------------------------------------------------------------ table lookup / insert

// Publish slot i of (tag, key) in the persistent index (single writer, between batches).
__device__ __forceinline__ void index_publish(const TableIndex &X, const Limits &lim, uint64_t i,
                                              uint32_t tag, const uint32_t k[4]) {
    if (tag == 2) {
        X.k6[i * 4 + 0] = k[1]; X.k6[i * 4 + 1] = k[2]; X.k6[i * 4 + 2] = k[3];
    }
    __threadfence();
    X.heads[i] = id_head(X.epoch, kIdReady, tag, k[0]);
    if (tag == 1) mir_publish(X.mir, X.mir_shift, lim.table_mask, lim.seed, i, k[0]);
}

// Claim an empty slot for a key known to be absent (map ops: one thread, no batch in
// flight) and publish it in the index.
__device__ __forceinline__ uint32_t table_claim(Slot *table, const Limits &lim, const TableIndex &X,
                                                uint32_t tag, const uint32_t k[4]) {
    uint64_t i = probe_start(tag, k, lim.seed, lim.table_mask, lim.test_flags);
    for (uint64_t probes = 0; probes <= lim.table_mask; ++probes) {
        if (slot_fam(table[i].tag, lim.tgen) == 0) {
            Slot &s = table[i];
            s.tag = slot_tag(tag, lim.tgen);
            s.flags = 0;
            s.key[0] = k[0]; s.key[1] = k[1]; s.key[2] = k[2]; s.key[3] = k[3];
            s.pps = s.bps = s.tt = s.till = s.aux = 0;
            index_publish(X, lim, i, tag, k);
            return (uint32_t)i;
        }
        i = (i + 1) & lim.table_mask;
    }
    return kNoSlot;
}

// After k_parse (one thread): the batch's new sources must fit max_entries, and with the
// sliding window its carried logs plus packets the history buffer — checked before any
// limiter state changes; a failing batch is rolled back by the host (fsx_api.hip).
// Pipelined batches: a batch whose predecessor failed is cancelled (the host rolls both back).
// (hist_in_tail: a split sliding-window batch checks its history room in its tail, after the
// previous tail has set hist_total: k_sw_tail_check)
// The source count moves atomically: a split tail (k_sw_tail_check) may undo its batch's
// count on another stream meanwhile.
__global__ void k_batch_check(BatchState *bs, TableState *tstate, Limits lim, const BatchState *prev,
                              uint32_t hist_in_tail = 0) {
    if (bs->err) return;
    if (prev && prev->err) { bs->err |= ERR_CANCELED; return; }
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(&tstate->count);
    const uint64_t count = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (count + bs->n_new > lim.max_entries) { bs->err |= ERR_TABLE_FULL; return; }
    if (lim.limiter == 1 && !hist_in_tail && tstate->hist_total + bs->n_valid > lim.hist_cap) {
        bs->err |= ERR_HIST_FULL;
        return;
    }
    if (bs->n_new) atomicAdd(cnt, (unsigned long long)bs->n_new);
    if (bs->n_rule) {   // prefix-rule drops count in stats_map like blacklist drops
        // (atomic: a pipelined batch's tail may be adding its counters meanwhile)
        atomicAdd(reinterpret_cast<unsigned long long *>(&tstate->stats[1]), (unsigned long long)bs->n_rule);
        bs->dropped += bs->n_rule;
    }
}

// The first kernel of a split sliding-window batch's tail (the previous tail has finished
// and set hist_total): the batch fails with ERR_HIST_FULL when its packets do not fit the
// history buffer, and is cancelled when an earlier split batch failed in its own tail
// (TableState::tail_fail; its k_batch_check may have run before that failure was known,
// and its predecessor's BatchState may already belong to a later front) — in both cases
// before any state changes, undoing what k_batch_check counted (the rollback rebuilds the
// index).
__global__ void k_sw_tail_check(BatchState *bs, TableState *tstate, Limits lim) {
    if (bs->err) return;
    uint32_t err = 0;
    if (tstate->tail_fail) err = ERR_CANCELED;
    else if (tstate->hist_total + bs->n_valid > lim.hist_cap) err = ERR_HIST_FULL;
    if (!err) return;
    bs->err |= err;
    tstate->tail_fail = 1;
    if (bs->n_new)
        atomicAdd(reinterpret_cast<unsigned long long *>(&tstate->count), (unsigned long long)(0ull - bs->n_new));
    if (bs->n_rule) {
        atomicAdd(reinterpret_cast<unsigned long long *>(&tstate->stats[1]), (unsigned long long)(0ull - bs->n_rule));
        bs->dropped -= bs->n_rule;
    }
}

// ------------------------------------------------------------------ overflow admission
// FSX_FLAG_OVERFLOW_ADMIT (include/fsx_hip.h): the batch's sources carry
// per-batch ids; after the segment heads, every source is found in the persistent index
// (read only) or flagged at its first packet's arrival index; the flags' exclusive scan in
// arrival order is each new source's admission rank; ranks below the free room are inserted
// into the index (their fresh table slot), the others get a slot of the transient region
// after the table (slots + segment id), fresh for this batch and never dumped or looked up.

// Slot of (tag, key) in the persistent index, kNoSlot when absent (no inserts race it).
__device__ __forceinline__ uint32_t index_find(const TableIndex &X, const Limits &lim, uint32_t tag,
                                               const uint32_t k[4]) {
    // (the probe start computed from scalars: through the array, the compiler kept two of
    // the key words in scratch)
    const uint32_t k0 = k[0], k1 = k[1], k2 = k[2], k3 = k[3];
    const uint64_t hv6 = mix64(mix64(lim.seed ^ (2ull << 56) ^ ((uint64_t)k0 | ((uint64_t)k1 << 32))) ^
                               ((uint64_t)k2 | ((uint64_t)k3 << 32)));
    uint64_t h = tag == 1 ? (uint64_t)v4_hash(k0, lim.seed)
                          : (lim.test_flags & 1u) ? (uint64_t)v4_hash(0x0100000Au, lim.seed) : hv6;
    h &= lim.table_mask;
    for (uint64_t probes = 0; probes <= lim.table_mask; ++probes, h = (h + 1) & lim.table_mask) {
        const uint64_t cur = __hip_atomic_load(X.heads + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(cur >> 48) != X.epoch) return kNoSlot;   // empty in this epoch
        if (((cur >> 32) & 0xFFu) != tag || (uint32_t)cur != k0) continue;
        if (tag == 1) return (uint32_t)h;
        const uint32_t *kw = X.k6 + h * 4;
        if (__hip_atomic_load(kw + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k1 &&
            __hip_atomic_load(kw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k2 &&
            __hip_atomic_load(kw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k3)
            return (uint32_t)h;
    }
    return kNoSlot;
}

// The source of segment g (its first packet's record), and that packet's arrival index.
__device__ __forceinline__ uint32_t seg_source(const uint64_t *S, const uint32_t *seg_start, uint32_t g,
                                               const PacketIn &in, uint32_t salt, uint32_t k[4], uint32_t &idx) {
    (void)salt;
    const uint64_t v = S[seg_start[g]];
    idx = pk_idx(v);
    // (the key words as scalars, written once: branches that filled the array differently
    // made the compiler select them through scratch)
    uint32_t k0, k1 = 0, k2 = 0, k3 = 0, tag;
    if (in.rec) {   // ShardRecord16 {key, len | dport << 16, ts} / ShardRecord {key[4], ts, len, ...}
        if (in.rec_bytes == 16) {
            k0 = reinterpret_cast<const uint4 *>(in.rec)[idx].x;
            tag = 1;
        } else {
            const uint4 *p = reinterpret_cast<const uint4 *>(in.rec) + 2 * (size_t)idx;
            const uint4 a = p[0], b = p[1];
            k0 = a.x; k1 = a.y; k2 = a.z; k3 = a.w;
            tag = ((b.w >> 16) & 0xFFu) == 6 ? 2u : 1u;
        }
    } else {        // key_of, both families' words computed and selected
        const uint32_t *d = reinterpret_cast<const uint32_t *>(in.hdr + (size_t)idx * 64);
        const uint32_t d3 = d[3], d5 = d[5], d6 = d[6], d7 = d[7], d8 = d[8], d9 = d[9];
        const bool v6 = (d3 & 0xFFFFu) == 0xDD86u;
        k0 = v6 ? (d5 >> 16) | (d6 << 16) : (d6 >> 16) | (d7 << 16);
        k1 = v6 ? (d6 >> 16) | (d7 << 16) : 0u;
        k2 = v6 ? (d7 >> 16) | (d8 << 16) : 0u;
        k3 = v6 ? (d8 >> 16) | (d9 << 16) : 0u;
        tag = v6 ? 2u : 1u;
    }
    k[0] = k0; k[1] = k1; k[2] = k2; k[3] = k3;
    return tag;
}

__global__ __launch_bounds__(256) void k_admit_find(const BatchState *bs, const uint64_t *__restrict__ S,
                                                    const uint32_t *__restrict__ seg_start,
                                                    uint32_t *__restrict__ seg_slot, PacketIn in, TableIndex X,
                                                    Limits lim, uint32_t *__restrict__ flag) {
    if (bs->err) return;
    const uint32_t nseg = bs->nseg;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nseg; g += gridDim.x * 256u) {
        uint32_t k[4], idx;
        const uint32_t tag = seg_source(S, seg_start, g, in, lim.salt32, k, idx);
        const uint32_t s = index_find(X, lim, tag, k);
        seg_slot[g] = s;
        if (s == kNoSlot) flag[idx] = 1u;
    }
}

// per 4096 arrival positions: the flagged ones (tile_cnt), then (mode 1, after the scan of
// tile_cnt) each flagged position's rank in place
template <int kMode>
__global__ __launch_bounds__(256) void k_admit_rank(const BatchState *bs, uint32_t *__restrict__ flag, uint32_t n,
                                                    uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t p0 = t * kTile + threadIdx.x * 16u;
        uint32_t f[16], c = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            f[j] = p0 + j < n ? flag[p0 + j] : 0u;
            c += f[j];
        }
        uint32_t tot;
        uint32_t off = block256_excl(c, s_tmp, &tot);
        if constexpr (kMode == 0) {
            if (threadIdx.x == 0) tile_cnt[t] = tot;
        } else {
            off += tile_cnt[t];
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (f[j]) flag[p0 + j] = off++;
        }
    }
}

// one block: exclusive scan of the per-tile counts in place
__global__ __launch_bounds__(256) void k_admit_scan(const BatchState *bs, uint32_t *__restrict__ cnt, uint32_t n) {
    __shared__ uint32_t s_tmp[4];
    if (bs->err) return;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 256) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t x = i < ntiles ? cnt[i] : 0u;
        uint32_t tot;
        const uint32_t e = block256_excl(x, s_tmp, &tot);
        if (i < ntiles) cnt[i] = carry + e;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void k_admit_insert(BatchState *bs, const TableState *tstate,
                                                      const uint64_t *__restrict__ S,
                                                      const uint32_t *__restrict__ seg_start,
                                                      uint32_t *__restrict__ seg_slot, PacketIn in, IdTable idt,
                                                      Limits lim, const uint32_t *__restrict__ rank, Slot *table,
                                                      uint64_t tbase) {
    if (bs->err) return;
    const uint64_t cnt = tstate->count;
    const uint64_t room = cnt < lim.max_entries ? lim.max_entries - cnt : 0ull;
    const uint32_t nseg = bs->nseg;
    uint32_t na = 0, nt = 0;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nseg; g += gridDim.x * 256u) {
        if (seg_slot[g] != kNoSlot) continue;
        uint32_t k[4], idx;
        const uint32_t tag = seg_source(S, seg_start, g, in, lim.salt32, k, idx);
        if (rank[idx] < room) {   // admitted: its slot in the persistent index
            const uint64_t h = id_start(idt, tag, k);
            const uint64_t hint = __hip_atomic_load(idt.head + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool fresh = false;
            const uint32_t s = id_resolve(idt, tag, k, h, hint, &fresh);
            if (s == kNoSlot) atomicOr(&bs->err, ERR_TABLE_FULL);
            seg_slot[g] = s;
            ++na;
        } else {                  // transient: a fresh slot of its own for this batch
            Slot &sl = table[tbase + g];
            sl.tag = slot_tag(tag, lim.tgen);
            sl.flags = 0;
            sl.key[0] = k[0]; sl.key[1] = k[1]; sl.key[2] = k[2]; sl.key[3] = k[3];
            sl.pps = sl.bps = sl.tt = sl.till = sl.aux = 0;
            seg_slot[g] = (uint32_t)(tbase + g);
            ++nt;
        }
    }
    na = wave_sum(na);
    nt = wave_sum(nt);
    if (lane_id() == 0) {
        if (na) atomicAdd(&bs->n_admit, na);
        if (nt) atomicAdd(&bs->n_trans, nt);
    }
}

__global__ void k_admit_commit(BatchState *bs, TableState *tstate) {
    if (bs->err) return;
    tstate->count += bs->n_admit;
}

// Rollback / epoch change: re-publish every live slot under the new epoch; slots born in
// the failed batch `born` (nonzero) are emptied instead.
__global__ __launch_bounds__(256) void k_index_rebuild(Slot *table, Limits lim, TableIndex X, uint32_t born) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= lim.table_mask;
         i += (uint64_t)gridDim.x * 256u) {
        Slot &s = table[i];
        const uint32_t fam = slot_fam(s.tag, lim.tgen);
        if (fam == 0) continue;
        if (born && (s.flags >> kBornShift) == born) {
            s.tag = 0;
            s.flags = 0;
            continue;
        }
        if (fam == 2) {
            X.k6[i * 4 + 0] = s.key[1]; X.k6[i * 4 + 1] = s.key[2]; X.k6[i * 4 + 2] = s.key[3];
        }
        X.heads[i] = id_head(X.epoch, kIdReady, fam, s.key[0]);
        if (fam == 1) mir_publish(X.mir, X.mir_shift, lim.table_mask, lim.seed, i, s.key[0]);
    }
}

hipError_t launch_index_rebuild(Slot *table, const Limits &lim, const TableIndex &X, uint32_t born,
                                hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, (lim.table_mask + 256) / 256);
    k_index_rebuild<<<grid, 256, 0, st>>>(table, lim, X, born);
    return hipGetLastError();
}

// ------------------------------------------------------------------ fixed-window walker
// Segments of at most short_seg packets: one thread, exact per-packet replay with 16
// packets' loads in flight. Longer segments (the heavy sources): one wave each,
// epoch jumps with 64-wide cooperative searches (few dependent round trips per
// search instead of one per binary-search step). The boundary is per limiter: the
// fixed-window wave walker runs beside the thread walker on its own stream, so a
// lower boundary balances the two (measured on config 2: 256 fixed, 512 sliding).
#ifndef FSX_SHORT_SEG_FIXED
#define FSX_SHORT_SEG_FIXED 256   // (A/B: scripts/build_variant.sh)
#endif
constexpr uint32_t kShortSegFixed = FSX_SHORT_SEG_FIXED;
#ifndef FSX_WALK_LONG_BLOCKS
#define FSX_WALK_LONG_BLOCKS 2048   // blocks of the wave walker (one source per wave)
#endif
#ifndef FSX_WALK_SHORT_BLOCKS
#define FSX_WALK_SHORT_BLOCKS 2048  // blocks of the thread walker
#endif
constexpr uint32_t kShortSegSliding = 512;


// Segments are walked in order of length class (ceil log2 of the packet count), so
// the lanes of a wave replay segments of similar length; the last class (longer
// than short_seg) goes to the wave walkers, one wave per segment.
__device__ __forceinline__ uint32_t seg_class(uint32_t L, uint32_t short_seg) {
    if (L > short_seg) return kSegClasses - 1;
    return L <= 1 ? 0u : 32u - (uint32_t)__clz((int)(L - 1));
}

// Counting sort of the segment ids by class: per-block counts over contiguous
// chunks, one scan, then per-block LDS cursors (no contended global atomics; order
// inside a class is irrelevant to the result).
constexpr uint32_t kSegBlocks = 1024;
static_assert(kSegClasses * kSegBlocks == kSegClassWords, "Scratch::seg_cls size");

__device__ __forceinline__ void seg_chunk(uint32_t nseg, uint32_t b, uint32_t &lo, uint32_t &hi) {
    const uint32_t chunk = (nseg + kSegBlocks - 1) / kSegBlocks;
    lo = min(nseg, b * chunk);
    hi = min(nseg, lo + chunk);
}

template <bool kWrite>
__device__ __forceinline__ void seg_classes_pass(const uint32_t *seg_start, uint32_t lo, uint32_t hi,
                                                 uint32_t short_seg, uint32_t *sh, uint32_t *order) {
    const uint32_t lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t b = lo; b < hi; b += 256u) {
        const uint32_t g = b + threadIdx.x;
        const bool ok = g < hi;
        const uint32_t c = ok ? seg_class(seg_start[g + 1] - seg_start[g], short_seg) : kSegClasses;
#pragma unroll
        for (uint32_t k = 0; k < kSegClasses; ++k) {
            const uint64_t m = __ballot(c == k);
            if (!m) continue;
            uint32_t off = 0;
            if (lane == 0) off = atomicAdd(&sh[k], (uint32_t)__popcll(m));
            if constexpr (kWrite) {
                off = __shfl(off, 0);
                if (c == k) order[off + (uint32_t)__popcll(m & lt)] = g;
            }
        }
    }
}

// Every segment one packet (a carpet of new sources, config 5): class 0 throughout, the
// order the identity (no seg_start reads).
__device__ __forceinline__ bool seg_all_single(const BatchState *bs) {
    return bs->nseg == bs->n_valid && bs->n_light == bs->n_valid;
}

__global__ __launch_bounds__(256) void k_seg_count(const BatchState *bs,
                                                   const uint32_t *__restrict__ seg_start,
                                                   uint32_t *__restrict__ blk, uint32_t short_seg) {
    __shared__ uint32_t sh[kSegClasses];
    uint32_t lo, hi;
    seg_chunk(bs->nseg, blockIdx.x, lo, hi);
    if (seg_all_single(bs)) {
        if (threadIdx.x < kSegClasses) blk[threadIdx.x * kSegBlocks + blockIdx.x] = threadIdx.x == 0 ? hi - lo : 0u;
        return;
    }
    if (threadIdx.x < kSegClasses) sh[threadIdx.x] = 0;
    __syncthreads();
    seg_classes_pass<false>(seg_start, lo, hi, short_seg, sh, nullptr);
    __syncthreads();
    if (threadIdx.x < kSegClasses) blk[threadIdx.x * kSegBlocks + blockIdx.x] = sh[threadIdx.x];
}

// Exclusive scan of the class-major [class][block] counts; class totals to cls (256
// threads, 64 consecutive counts each: a run never crosses a class).
__global__ __launch_bounds__(256) void k_seg_scan(uint32_t *__restrict__ blk, uint32_t *cls) {
    static_assert(kSegClasses * kSegBlocks == 64 * 256 && kSegBlocks % 64 == 0, "one 64-count run per thread");
    __shared__ uint32_t s_tmp[4];
    __shared__ uint32_t s_cls[kSegClasses];
    const uint32_t t = threadIdx.x;
    if (t < kSegClasses) s_cls[t] = 0;
    uint32_t v[64], sum = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) { v[k] = blk[t * 64 + k]; sum += v[k]; }
    uint32_t off = block256_excl(sum, s_tmp, nullptr);   // (its barriers order the s_cls reset)
#pragma unroll
    for (int k = 0; k < 64; ++k) { blk[t * 64 + k] = off; off += v[k]; }
    if (sum) atomicAdd(&s_cls[(t * 64) / kSegBlocks], sum);
    __syncthreads();
    if (t < kSegClasses) cls[t] = s_cls[t];
}

__global__ __launch_bounds__(256) void k_seg_order(const BatchState *bs,
                                                   const uint32_t *__restrict__ seg_start,
                                                   const uint32_t *__restrict__ blk,
                                                   uint32_t *__restrict__ order, uint32_t short_seg) {
    __shared__ uint32_t cur[kSegClasses];
    uint32_t lo, hi;
    seg_chunk(bs->nseg, blockIdx.x, lo, hi);
    if (seg_all_single(bs)) {   // (block b's class-0 cursor is lo)
        for (uint32_t g = lo + threadIdx.x; g < hi; g += 256u) order[g] = g;
        return;
    }
    if (threadIdx.x < kSegClasses) cur[threadIdx.x] = blk[threadIdx.x * kSegBlocks + blockIdx.x];
    __syncthreads();
    seg_classes_pass<true>(seg_start, lo, hi, short_seg, cur, order);
}

template <class SV>
__device__ __forceinline__ void walk_short(const SV &sv, const BatchState *bs,
                                           const uint32_t *seg_start, const uint32_t *seg_slot,
                                           const uint32_t *order, const uint32_t *cls,
                                           uint8_t *marks, Slot *table, const Limits &lim,
                                           const HeavyLists &H, const SlotKeys &K) {
    const uint32_t nshort = bs->nseg - cls[kSegClasses - 1];
    // (a batch without new sources loads no heads: warm streams keep their walker as it was)
    const bool knew = K.heads && bs->n_new != 0;
    // mostly new sources (a flood, config 5): a segment whose first word carries kFreshBit
    // has a slot this batch claimed, written whole without reading it
    const bool flood = knew && K.fresh_bit && 2ull * bs->n_new > bs->nseg;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nshort; i += gridDim.x * 256u) {
        const uint32_t g = order[i];
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        if (H.list && a >= bs->n_light) continue;   // a heavy source: k_walk_heavy
        const uint32_t si = seg_slot[g];
        if (si == kNoSlot) continue;   // (home-ordered inserts walked it: k_ord_claim)
        Slot &sl = table[si];
        if (flood && (sv.S[a] & kFreshBit)) {
            const unsigned long long hd = K.heads[si];
            FwState st{false, false, 0, 0, 0, 0};
            MarkWriter<false> mw{marks, 0};
            walk_fixed_exact_thread(sv, a, b, lim, mw, st);
            store_new_line(sl, st, K, si, hd);
            continue;
        }
        const SlotLine L0 = load_line(sl);
        const uint32_t flags0 = L0.q[0].y;
        const bool fresh = knew && slot_fam(tag_of(L0), lim.tgen) == 0;
        // (a fresh slot's line may hold an older table generation's source: no state)
        FwState st = fresh ? FwState{false, false, 0, 0, 0, 0} : state_of(L0);
        const unsigned long long hd = knew ? K.heads[si] : 0ull;
        MarkWriter<false> mw{marks, 0};
        walk_fixed_exact_thread(sv, a, b, lim, mw, st);
        if (fresh) store_new_line(sl, st, K, si, hd);
        else store_state_f(sl, st, flags0);
    }
}

__global__ __launch_bounds__(256) void k_walk_fixed(const uint64_t *__restrict__ S, BatchState *bs,
                                                    const uint32_t *__restrict__ seg_start,
                                                    const uint32_t *__restrict__ seg_slot,
                                                    const uint64_t *__restrict__ ts,
                                                    const uint32_t *__restrict__ len,
                                                    const uint64_t *__restrict__ pay,
                                                    const uint32_t *__restrict__ order,
                                                    const uint32_t *__restrict__ cls,
                                                    uint8_t *__restrict__ marks, Slot *table,
                                                    Limits lim, HeavyLists H, SlotKeys K) {
    if (bs->err || bs->ord_walked) return;
    if (bs->pay_ok) {
        const SegView<true> sv{S, ts, len, pay, ~bs->inv_min_ts};
        walk_short(sv, bs, seg_start, seg_slot, order, cls, marks, table, lim, H, K);
    } else {
        const SegView<false> sv{S, ts, len, pay, 0};
        walk_short(sv, bs, seg_start, seg_slot, order, cls, marks, table, lim, H, K);
    }
}

template <class SV>
__device__ __forceinline__ void walk_long(const SV &sv, const BatchState *bs,
                                          const uint32_t *seg_start, const uint32_t *seg_slot,
                                          const uint32_t *order, const uint32_t *cls,
                                          uint8_t *marks, Slot *table, const Limits &lim,
                                          const HeavyLists &H, const SlotKeys &K) {
    const uint32_t nl = cls[kSegClasses - 1], first = bs->nseg - nl;
    const bool glob_fast = fast_ok(bs, lim);
    const uint32_t maxL = bs->max_len;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const bool knew = K.heads && bs->n_new != 0;
    for (uint32_t i = wave; i < nl; i += gridDim.x * 4u) {
        const uint32_t g = order[first + i];
        const uint32_t a = seg_start[g], b = seg_start[g + 1];
        if (H.list && a >= bs->n_light) continue;   // a heavy source: k_walk_heavy
        const uint32_t si = seg_slot[g];
        if (si == kNoSlot) continue;   // (k_ord_claim walked it)
        Slot &sl = table[si];
        const SlotLine L0 = load_line(sl);
        const uint32_t flags0 = L0.q[0].y;
        const bool fresh = knew && slot_fam(tag_of(L0), lim.tgen) == 0;
        FwState st = fresh ? FwState{false, false, 0, 0, 0, 0} : state_of(L0);
        const unsigned long long hd = knew ? K.heads[si] : 0ull;
        const bool fast = glob_fast && (!st.has_st || (st.tt <= ~0ull - lim.window &&
                                                       st.pps < kBig && st.bps < kBig));
        MarkWriter<true> mw{marks, 0};
        if (fast) walk_fixed_fast<true>(sv, a, b, lim, maxL, mw, st);
        else walk_fixed_exact_wave(sv, a, b, lim, mw, st);
        if (lane_id() == 0) {
            if (fresh) store_new_line(sl, st, K, si, hd);
            else store_state_f(sl, st, flags0);
        }
    }
}

__global__ __launch_bounds__(256) void k_walk_fixed_long(const uint64_t *__restrict__ S,
                                                         BatchState *bs,
                                                         const uint32_t *__restrict__ seg_start,
                                                         const uint32_t *__restrict__ seg_slot,
                                                         const uint64_t *__restrict__ ts,
                                                         const uint32_t *__restrict__ len,
                                                         const uint64_t *__restrict__ pay,
                                                         const uint32_t *__restrict__ order,
                                                         const uint32_t *__restrict__ cls,
                                                         uint8_t *__restrict__ marks, Slot *table,
                                                         Limits lim, HeavyLists H, SlotKeys K) {
    if (bs->err || bs->ord_walked) return;
    if (bs->pay_ok) {
        const SegView<true> sv{S, ts, len, pay, ~bs->inv_min_ts};
        walk_long(sv, bs, seg_start, seg_slot, order, cls, marks, table, lim, H, K);
    } else {
        const SegView<false> sv{S, ts, len, pay, 0};
        walk_long(sv, bs, seg_start, seg_slot, order, cls, marks, table, lim, H, K);
    }
}

// The heavy sources' segments (heavy verdict lists): one wave per heavy bucket of pass 0,
// whose run [gbase, gbase + count) of sorted positions is the source's segment.
template <class SV>
__device__ __forceinline__ void walk_heavy(const SV &sv, const BatchState *bs, const uint32_t *cnt0,
                                           const uint32_t *base0, Slot *table, const Limits &lim,
                                           const HeavyLists &H, const SlotKeys &K) {
    const bool glob_fast = fast_ok(bs, lim);
    const uint32_t maxL = bs->max_len;
    const uint32_t h = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (h >= H.hs->n) return;
    const uint32_t c = cnt0[bs->light_b + h];
    if (c == 0) return;
    const uint32_t a = base0[bs->light_b + h], b = a + c;
    const uint32_t si = pk_id(sv.S[a], lim.table_mask);
    Slot &sl = table[si];
    // (unresolved heavy sources, under prefix rules, are inserted by k_parse: lazily — a line
    // of another table generation is a new source's, with no state)
    const bool adopt = K.heads && slot_fam(sl.tag, lim.tgen) == 0;
    FwState st = adopt ? FwState{false, false, 0, 0, 0, 0} : load_state(sl);
    const unsigned long long hd = K.heads ? K.heads[si] : 0ull;
    const bool fast = glob_fast && (!st.has_st || (st.tt <= ~0ull - lim.window &&
                                                   st.pps < kBig && st.bps < kBig));
    MarkWriter<true, true> mw{nullptr, 0};
    heavy_list_open(H, sv.S, a, mw);   // (h: this wave's heavy bucket)
    if (fast) walk_fixed_fast<true>(sv, a, b, lim, maxL, mw, st);
    else walk_fixed_exact_wave(sv, a, b, lim, mw, st);
    heavy_list_close(H, (int)h, a, b, mw);
    if (lane_id() == 0) {
        store_state(sl, st);
        if (adopt) slot_adopt(sl, K, si, hd, lim.tgen);
    }
}

__global__ __launch_bounds__(256) void k_walk_heavy(const uint64_t *__restrict__ S, BatchState *bs,
                                                    const uint32_t *__restrict__ cnt0,
                                                    const uint32_t *__restrict__ base0,
                                                    const uint64_t *__restrict__ ts,
                                                    const uint32_t *__restrict__ len,
                                                    const uint64_t *__restrict__ pay, Slot *table,
                                                    Limits lim, HeavyLists H, SlotKeys K) {
    if (bs->err || bs->hfast) return;   // (hfast: k_walk_heavy_sel)
    if (bs->pay_ok) {
        const SegView<true> sv{S, ts, len, pay, ~bs->inv_min_ts};
        walk_heavy(sv, bs, cnt0, base0, table, lim, H, K);
    } else {
        const SegView<false> sv{S, ts, len, pay, 0};
        walk_heavy(sv, bs, cnt0, base0, table, lim, H, K);
    }
}

// ------------------------------------------------------------------ fill + scatter
// Tile of kTile sorted positions; thread j owns marks [16j, 16j+16).
__device__ __forceinline__ void load_marks16(const uint8_t *marks, uint32_t p0, uint32_t M, uint32_t f[4]) {
    if (p0 + 16 <= M) {
        const uint4 v = *reinterpret_cast<const uint4 *>(marks + p0);
        f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
    } else {
        f[0] = f[1] = f[2] = f[3] = 0;
        for (uint32_t k = 0; k < 16 && p0 + k < M; ++k) f[k >> 2] |= (uint32_t)marks[p0 + k] << (8 * (k & 3));
    }
}

// (light_only: the heavy sources' positions [n_light, n_valid) have verdict lists instead;
// 2: the token bucket's heavy sources, decided outside the sort only on the unsorted path)
__global__ __launch_bounds__(256) void k_fill_last(const uint8_t *__restrict__ marks, BatchState *bs,
                                                   uint8_t *__restrict__ tile_last, uint32_t light_only) {
    __shared__ uint32_t s_w[4];
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t p0 = t * kTile + threadIdx.x * 16u;
        uint32_t f[4];
        load_marks16(marks, p0, M, f);
        uint32_t enc = 0;  // (local index + 1) << 8 | mark of the last non-zero mark
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t m = (f[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            if (m) enc = ((threadIdx.x * 16u + k + 1u) << 8) | m;
        }
        enc = wave_max(enc);
        if (lane_id() == 0) s_w[threadIdx.x >> 6] = enc;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t e = s_w[0];
            for (int k = 1; k < 4; ++k) e = s_w[k] > e ? s_w[k] : e;
            tile_last[t] = (uint8_t)(e & 0xFFu);
        }
        __syncthreads();
    }
}

// Single block: carry[t] = last non-zero of tile_last[0..t-1] (in place, exclusive).
__global__ __launch_bounds__(1024) void k_fill_carry(uint8_t *__restrict__ tile_last, BatchState *bs,
                                                     uint32_t light_only) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t m = i < ntiles ? tile_last[i] : 0u;
        const uint32_t enc = m ? (((i + 1u) << 8) | m) : 0u;
        const uint32_t incl = wave_incl_max(enc);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t pre = s_carry;
        uint32_t tot = s_carry;
        for (uint32_t k = 0; k < 16; ++k) {
            if (k < w) pre = s_w[k] > pre ? s_w[k] : pre;
            tot = s_w[k] > tot ? s_w[k] : tot;
        }
        uint32_t excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0;
        excl = excl > pre ? excl : pre;
        __syncthreads();
        if (i < ntiles) tile_last[i] = (uint8_t)(excl & 0xFFu);
        if (threadIdx.x == 0) s_carry = tot;
        __syncthreads();
    }
}

// Fill + DROP collection: the verdict of every sorted position (last mark at or before
// it), counted into stats_map; DROP positions append their arrival index to the list of
// their arrival chunk (one cursor add per chunk and wave: a heavy source's run of drops
// lands in few chunks), so k_verdict_apply writes the verdict bytes chunk by chunk
// instead of one scattered byte store per drop.
__global__ __launch_bounds__(256) void k_fill_scatter(const uint8_t *__restrict__ marks,
                                                      const uint64_t *__restrict__ S, BatchState *bs,
                                                      const uint8_t *__restrict__ carry,
                                                      uint32_t *__restrict__ drop_list,
                                                      uint32_t *__restrict__ drop_cur,
                                                      TableState *tstate, uint32_t nchunks,
                                                      uint32_t light_only, uint8_t *__restrict__ verdict) {
    __shared__ uint8_t s_v[kTile];
    __shared__ uint32_t s_w[4];
    __shared__ unsigned long long s_cnt[4][2];
    __shared__ uint32_t s_cc[kMaxTileChunks];   // per arrival chunk: tile count, then base
    __shared__ uint16_t s_rk[kTile];            // per DROP position: rank in its chunk
    if (bs->err) return;
    const uint32_t M = cover_n(bs, light_only);
    const uint32_t ntiles = (M + kTile - 1) / kTile;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    // batches of <= kMaxTileChunks chunks: a tile reserves its DROPs' list slots with one
    // cursor add per chunk it touches, all in parallel (otherwise one per chunk and wave)
    const bool agg = nchunks <= kMaxTileChunks;
    if (agg)
        for (uint32_t c = threadIdx.x; c < nchunks; c += 256) s_cc[c] = 0;
    uint64_t n_pass = 0, n_drop = 0;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t p0 = t * kTile + threadIdx.x * 16u;
        uint32_t f[4];
        load_marks16(marks, p0, M, f);
        uint32_t enc = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t m = (f[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            if (m) enc = ((threadIdx.x * 16u + k + 1u) << 8) | m;
        }
        // exclusive "last non-zero" over the threads before me, then the tile carry
        const uint32_t incl = wave_incl_max(enc);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t k = 0; k < w; ++k) pre = s_w[k] > pre ? s_w[k] : pre;
        uint32_t excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0;
        excl = excl > pre ? excl : pre;
        uint8_t cur = excl ? (uint8_t)(excl & 0xFFu) : carry[t];
        bool mine = false;   // a DROP among this thread's valid positions
        uint32_t nvalid = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t m = (f[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            if (m) cur = (uint8_t)m;
            s_v[threadIdx.x * 16u + k] = cur;
            if (p0 + (uint32_t)k < M) {
                ++nvalid;
                mine |= cur == XDP_DROP;
            }
        }
        // most light tiles hold no DROP at all (the floods are the heavy sources, whose
        // verdicts travel as lists): count them PASS and move on
        if (!__syncthreads_or(mine ? 1 : 0)) {
            n_pass += nvalid;
            continue;
        }
        const uint32_t tile0 = t * kTile;
        const uint64_t lt = (1ull << lane) - 1ull;
        if (verdict) {   // every DROP straight to its arrival index (one byte store each)
            for (uint32_t j0 = 0; j0 < kTile && tile0 + j0 < M; j0 += 256) {
                const uint32_t j = j0 + threadIdx.x;
                const uint8_t v = tile0 + j < M ? s_v[j] : 0;
                n_pass += v == XDP_PASS;
                n_drop += v == XDP_DROP;
                if (v == XDP_DROP) verdict[pk_idx(S[tile0 + j])] = XDP_DROP;
            }
            __syncthreads();
            continue;
        }
        if (agg) {
            for (uint32_t j0 = 0; j0 < kTile; j0 += 256) {
                const uint32_t j = j0 + threadIdx.x;
                const bool ok = tile0 + j < M;
                const uint8_t v = ok ? s_v[j] : 0;
                n_pass += v == XDP_PASS;
                n_drop += v == XDP_DROP;
                // its slot among the tile's drops of its arrival chunk (a list's order is
                // irrelevant to k_verdict_apply): one returning LDS add per DROP
                if (v == XDP_DROP) s_rk[j] = (uint16_t)atomicAdd(&s_cc[pk_idx(S[tile0 + j]) >> kVChunkBits], 1u);
            }
            __syncthreads();
            for (uint32_t c = threadIdx.x; c < nchunks; c += 256) {
                const uint32_t cnt = s_cc[c];
                if (cnt) s_cc[c] = atomicAdd(&drop_cur[c], cnt);
            }
            __syncthreads();
            for (uint32_t j = threadIdx.x; j < kTile && tile0 + j < M; j += 256) {
                if (s_v[j] != XDP_DROP) continue;
                const uint32_t idx = pk_idx(S[tile0 + j]);   // (an L2 hit: read above)
                const uint32_t ch = idx >> kVChunkBits;
                drop_list[(size_t)ch * kVChunk + s_cc[ch] + s_rk[j]] = idx;
            }
            __syncthreads();
            for (uint32_t c = threadIdx.x; c < nchunks; c += 256) s_cc[c] = 0;
            __syncthreads();
            continue;
        }
        for (uint32_t j0 = 0; j0 < kTile && tile0 + j0 < M; j0 += 256) {   // block-uniform trips
            const uint32_t j = j0 + threadIdx.x;
            const bool ok = tile0 + j < M;
            const uint8_t v = ok ? s_v[j] : 0;
            n_pass += v == XDP_PASS;
            n_drop += v == XDP_DROP;
            const bool drop = v == XDP_DROP;
            const uint32_t idx = drop ? pk_idx(S[tile0 + j]) : 0u;
            const uint32_t ch = idx >> kVChunkBits;
            uint64_t pending = __ballot(drop);
            while (pending) {
                const int lead = __ffsll((unsigned long long)pending) - 1;
                const uint32_t lc = __shfl(ch, lead);
                const uint64_t same = __ballot(drop && ch == lc) & pending;
                uint32_t base = 0;
                if ((int)lane == lead) base = atomicAdd(&drop_cur[lc], (uint32_t)__popcll(same));
                base = __shfl(base, lead);
                if ((same >> lane) & 1ull)
                    drop_list[(size_t)lc * kVChunk + base + (uint32_t)__popcll(same & lt)] = idx;
                pending &= ~same;
            }
        }
        __syncthreads();
    }
    n_pass = wave_incl_sum(n_pass);
    n_drop = wave_incl_sum(n_drop);
    if (lane == 63) { s_cnt[w][0] = n_pass; s_cnt[w][1] = n_drop; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, d = 0;
        for (int k = 0; k < 4; ++k) { a += s_cnt[k][0]; d += s_cnt[k][1]; }
        if (a) {
            atomicAdd(reinterpret_cast<unsigned long long *>(&tstate->stats[0]), a);
            atomicAdd(reinterpret_cast<unsigned long long *>(&bs->allowed), a);
        }
        if (d) {
            atomicAdd(reinterpret_cast<unsigned long long *>(&tstate->stats[1]), d);
            atomicAdd(reinterpret_cast<unsigned long long *>(&bs->dropped), d);
        }
    }
}

// One block per arrival chunk of kVChunk verdict bytes: the chunk through LDS, its DROP
// list applied, written back with 16-byte stores (IP packets were written PASS by
// k_parse). Resets the chunk's cursor for the next batch.
// With heavy verdict lists (hl != nullptr) every chunk is rewritten: the bytes k_parse
// tagged 0x80 | h take heavy source h's verdict at their arrival index (the last list entry
// at or before it; each block first narrows every list to the entries around its chunk).
__global__ __launch_bounds__(256) void k_verdict_apply(uint8_t *__restrict__ verdict, uint32_t n,
                                                       const uint32_t *__restrict__ drop_list,
                                                       uint32_t *__restrict__ drop_cur,
                                                       const BatchState *bs, const HeavySet *hs,
                                                       const uint32_t *__restrict__ hl) {
    __shared__ uint4 s_v4[kVChunk / 16];
    __shared__ uint32_t s_lo[kHeavyMax], s_hi[kHeavyMax], s_tmp4[4];
    uint8_t *s_v = reinterpret_cast<uint8_t *>(s_v4);
    const uint32_t c = blockIdx.x;
    const uint32_t cnt = drop_cur[c];
    __syncthreads();
    if (threadIdx.x == 0) drop_cur[c] = 0;
    if ((cnt == 0 && !hl) || bs->err) return;
    const uint32_t b0 = c * kVChunk, nb = min(kVChunk, n - b0);
    const bool vec = ((reinterpret_cast<uintptr_t>(verdict) & 15u) == 0) && nb == kVChunk;
    if (vec) {
        const uint4 *src = reinterpret_cast<const uint4 *>(verdict + b0);
        for (uint32_t q = threadIdx.x; q < kVChunk / 16; q += 256) s_v4[q] = src[q];
    } else {
        for (uint32_t q = threadIdx.x; q < nb; q += 256) s_v[q] = verdict[b0 + q];
    }
    __syncthreads();
    const uint32_t *lst = drop_list + (size_t)c * kVChunk;
    for (uint32_t q = threadIdx.x; q < cnt; q += 256) s_v[lst[q] - b0] = XDP_DROP;
    if (hl) {
        // entries [lo, hi) of list h decide this chunk's packets of h; they are copied to
        // LDS (s_ent from s_off[h]) when all lists' chunk entries fit, else read in place
        constexpr uint32_t kEnt = 2048;
        __shared__ uint32_t s_off[kHeavyMax + 1], s_ent[kEnt];
        const uint32_t nh = hs->n;
        uint32_t lo = 0, hi = 0;
        if (threadIdx.x < nh) {
            const uint32_t *L = hl + hs->lbase[threadIdx.x];
            const uint32_t m = hs->lcnt[threadIdx.x];
            uint32_t l = 0, r = m;   // first entry with index > b0
            while (l < r) { const uint32_t md = (l + r) >> 1; if ((L[md] >> 1) <= b0) l = md + 1; else r = md; }
            lo = l ? l - 1 : 0;
            r = m;                   // first entry with index >= b0 + nb
            while (l < r) { const uint32_t md = (l + r) >> 1; if ((L[md] >> 1) < b0 + nb) l = md + 1; else r = md; }
            hi = m == 0 ? 0 : l > lo ? l : lo + 1;   // (a source without packets: no entries)
            s_lo[threadIdx.x] = lo;
            s_hi[threadIdx.x] = hi;
        }
        uint32_t tot;
        const uint32_t off = block256_excl(threadIdx.x < nh ? hi - lo : 0u, s_tmp4, &tot);
        const bool staged = tot <= kEnt;
        if (threadIdx.x < nh) {
            s_off[threadIdx.x] = off;
            if (staged) {
                const uint32_t *L = hl + hs->lbase[threadIdx.x];
                for (uint32_t e = lo; e < hi; ++e) s_ent[off + e - lo] = L[e];
            }
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb; q += 256) {
            const uint32_t v = s_v[q];
            if (v < 0x80u) continue;
            const uint32_t h = v & 0x7Fu, i = b0 + q;
            uint32_t l = 0, r = s_hi[h] - s_lo[h];   // last entry with index <= i
            const uint32_t *L = staged ? s_ent + s_off[h] : hl + hs->lbase[h] + s_lo[h];
            while (r - l > 1) { const uint32_t md = (l + r) >> 1; if ((L[md] >> 1) <= i) l = md; else r = md; }
            s_v[q] = (L[l] & 1u) ? XDP_DROP : XDP_PASS;
        }
    }
    __syncthreads();
    if (vec) {
        uint4 *dst = reinterpret_cast<uint4 *>(verdict + b0);
        for (uint32_t q = threadIdx.x; q < kVChunk / 16; q += 256) dst[q] = s_v4[q];
    } else {
        for (uint32_t q = threadIdx.x; q < nb; q += 256) verdict[b0 + q] = s_v[q];
    }
}

// ------------------------------------------------------------------ pipeline
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Look-back generations: every onesweep pass of every batch gets a fresh value, so
// stale status words of earlier passes never match (no per-pass memset).
static std::atomic<uint32_t> g_generation{0};
static uint32_t next_generation() {
    uint32_t g = g_generation.fetch_add(4) & 0x3FFFFFFFu;
    if (g == 0) g = g_generation.fetch_add(4) & 0x3FFFFFFFu;
    return g;
}

// The tail of a batch (after its sort): heavy walker and flow sums, segment heads, flows,
// the limiter's walkers, verdict fill and apply. Enqueued right after the front, or — for
// pipelined batches — later, after the next batch's parse (fsx_api.hip run_pipelined).
hipError_t launch_tail(const TailArgs &a) {
    const PacketIn &in = a.in;
    const uint32_t *len = a.len;
    const uint64_t *ts = a.ts;
    const uint32_t n = a.n;
    uint8_t *verdict = a.verdict;
    Slot *table = a.table;
    TableState *tstate = a.tstate;
    BatchState *bs = a.bs;
    Scratch sc = a.sc;
    const Limits &lim = a.lim;
    const bool do_limit = a.do_limit;
    const FlowRequest *flows = a.has_flows ? &a.fq : nullptr;
    const HistBufs &hist = a.hist;
    hipStream_t st = a.st, st2 = a.st2, st3 = a.st3;
    hipEvent_t fork_ev = a.fork_ev, join_ev = a.join_ev, walk_fork_ev = a.walk_fork_ev,
               walk_join_ev = a.walk_join_ev, heavy_fork_ev = a.heavy_fork_ev, heavy_flow_ev = a.heavy_flow_ev;
    PipeTiming *tm = a.tm;
    const PipeSplit *split = a.split ? &a.sp : nullptr;
    const int npass = a.npass;
    const uint32_t tcap = (uint32_t)(a.sc.cap / kSortTile + 2);
    const bool tagh = a.tagh;
    const uint32_t gridTiles = a.gridTiles;
    int last[3] = {a.last[0], a.last[1], a.last[2]};
    auto mark_on = [&](const char *name, int s_id) {
        if (!tm || tm->used >= tm->cap) return;
        const int i = tm->used++;
        tm->names[i] = name;
        tm->prev[i] = last[s_id];
        (void)hipEventRecord(tm->ev[i], s_id == 2 ? st3 : s_id == 1 ? st2 : st);
        last[s_id] = i;
    };
    auto mark = [&](const char *name) { mark_on(name, 0); };
    const Marker mk{[](void *p, const char *name) { (*static_cast<decltype(mark) *>(p))(name); }, &mark};
    hipError_t e;
    hipStream_t hs = (st3 && heavy_fork_ev && heavy_flow_ev) ? st3 : st;
    int hs_id = hs == st ? 0 : 2;
    // the heavy flow sums: on the flow stream ahead of the light flow tiles (a fourth stream
    // would share a hardware queue with the limiter chain: GPU_MAX_HW_QUEUES is 4)
    const bool fork = a.fork;   // flows beside the limiter
    hipStream_t hf = (hs != st && fork) ? st2 : hs;
    int hf_id = hf == st2 && hf != st ? 1 : hs_id;
    // the heavy runs: pass 0's output (packed[1]), which the light passes never write in
    // [n_light, n) (with 3 passes also the light entries' final buffer)
    uint64_t *S_fin = sc.packed[1], *pay_fin = sc.pay[1];
    // heavy verdict lists live in the parse buffer over the heavy positions (which no pass
    // writes after pass 0 read it)
    // (the token bucket's heavy packets get their verdict bytes directly: launch_tb_heavy, or on
    // the run path the fill's DROP stores and k_tb_untag)
    const bool tb_tag = tagh && do_limit && lim.limiter == 2;
    const HeavyLists hlists{tagh && !tb_tag ? reinterpret_cast<uint32_t *>(sc.packed[0]) : nullptr, sc.heavy,
                            tstate, bs};
    // (lazy slots: the fixed window's walkers write a new source's family and key)
    const SlotKeys skeys{a.lazy ? a.X.heads : nullptr, a.X.k6, a.lazy && a.fresh_bit ? 1u : 0u, lim.tgen};
    // the heavy runs' walker and flow sums, forked right after the sort (A/B, config 2: right
    // after pass 0 they slowed passes 1-2, after the heads they delayed the walkers; a fourth
    // stream shared a hardware queue with the limiter chain)
    bool heavy_join = false;
    // FSX_PARSE_PAY: the heavy tile records (k_heavy_recs) before the heavy walker and the
    // heavy flow sums read them — on their stream when both run there, else before the fork
    const bool recs = a.hfm && FSX_PARSE_PAY;
    const bool recs_on_hs = recs && hs != st && (!flows || hf == hs);
    auto launch_recs = [&](hipStream_t rs, int rs_id) -> hipError_t {
        hipError_t e = launch_heavy_recs(bs, ts, len, verdict, n, sc.heavy, sc.hrec, rs);
        mark_on("k_heavy_recs", rs_id);
        return e;
    };
    auto launch_heavy = [&]() -> hipError_t {
        hipError_t e;
        if (recs && !recs_on_hs && (e = launch_recs(st, 0)) != hipSuccess) return e;
        if (hs != st) {
            if ((e = hipEventRecord(heavy_fork_ev, st)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(hs, heavy_fork_ev, 0)) != hipSuccess) return e;
            mark_on(nullptr, hs_id);
            if (flows && hf != hs) {
                if ((e = hipStreamWaitEvent(hf, heavy_fork_ev, 0)) != hipSuccess) return e;
                mark_on(nullptr, hf_id);
            }
        }
        if (recs_on_hs && (e = launch_recs(hs, hs_id)) != hipSuccess) return e;
        if (lim.limiter == 0) {   // (the sliding window's heavy walker: launch_sliding_window)
            k_walk_heavy<<<kHeavyMax / 4, 256, 0, hs>>>(S_fin, bs, sc.sort_ctl, sc.gbase, ts, len, pay_fin,
                                                          table, lim, hlists, skeys);
            mark_on("k_walk_heavy", hs_id);
        }
        if (a.hfm && lim.limiter == 0) {   // (the path k_hmode picked runs; the other returns at once)
            if ((e = launch_walk_heavy_sel(bs, sc.sort_ctl, sc.gbase, sc.hist, tcap, verdict, ts, len, n, sc.hrec,
                                           table, lim, sc.heavy, hlists.list, tstate, hs)) != hipSuccess)
                return e;
            mark_on("k_walk_heavy_sel", hs_id);
        }
        if (a.hfm && tb_tag) {   // token bucket: the heavy packets' verdicts in arrival order (unsorted path)
            if ((e = launch_tb_heavy(bs, sc.sort_ctl, sc.gbase, sc.hist, tcap, verdict, ts, n, sc.hrec, sc.tbh, table,
                                     lim, sc.heavy, tstate, hs)) != hipSuccess)
                return e;
            mark_on("k_tb_heavy", hs_id);
        }
        // (pipelined: the heavy walker beside the tail's chain; k_verdict_apply joins it)
        if (heavy_join && (e = hipEventRecord(walk_join_ev, hs)) != hipSuccess) return e;
        if (flows) {
            if ((e = launch_flows_heavy(S_fin, pay_fin, ts, len, bs, sc.sort_ctl, sc.gbase, sc.heavy_flow,
                                        sc.cap, hf)) != hipSuccess)
                return e;
            if (a.hfm && (e = launch_hflow_combine(bs, sc.sort_ctl, sc.gbase, sc.hist, tcap, n, sc.hrec, sc.hflow,
                                                   hf)) != hipSuccess)
                return e;
            mark_on("k_flow_heavy", hf_id);
            if (hf != st && (e = hipEventRecord(heavy_flow_ev, hf)) != hipSuccess) return e;
        }
        return hipSuccess;
    };
    if (split && split->tail) {
        // pipelined: the tail on its own stream (the caller made it and st2 wait for the
        // front); walkers serial on it, the heavy flow sums and the flows on st2
        st = split->tail;
        if ((e = hipMemsetAsync(sc.marks, 0, n, st)) != hipSuccess) return e;
        st3 = nullptr;
        hs = st;
        hs_id = 0;
        hf = fork ? st2 : st;
        hf_id = fork ? 1 : 0;
        // unsorted heavy sources: their walker (select / rank searches, latency-bound on 32
        // blocks) on the flow stream ahead of the heavy flow rows, not ahead of the heads
        if (a.hfm && (lim.limiter == 0 || tb_tag) && st2 && walk_join_ev) {
            hs = st2;
            hs_id = 1;
            heavy_join = true;
        }
    }
    // (unsplit: the token bucket's heavy kernels on the walker stream are joined before the
    // verdicts are final — no fork of walkers follows them there)
    if (!(split && split->tail) && a.hfm && tb_tag && hs != st && walk_join_ev) heavy_join = true;
    if (split && split->tail && do_limit && lim.limiter == 1) k_sw_tail_check<<<1, 1, 0, st>>>(bs, tstate, lim);
    // unsorted heavy sources: their carried state decides the path now that the previous
    // batch's walkers have stored it; those sent back to the run path get their runs first
    if (a.hfm && (e = launch_hmode_state(sc.sort_ctl, n, bs, sc.heavy, table, lim, tstate, st)) != hipSuccess)
        return e;
    if (a.hfm && (e = launch_heavy_gather(bs, verdict, ts, len, n, sc.hist, tcap, sc.heavy, a.shift0, lim.table_mask,
                                          S_fin, pay_fin, st)) != hipSuccess)
        return e;
    if (a.hfm) mark("k_heavy_gather");
    if (tagh && (e = launch_heavy()) != hipSuccess) return e;
    if (npass & 1) {
        std::swap(sc.packed[0], sc.packed[1]);
        std::swap(sc.pay[0], sc.pay[1]);
    }
    uint64_t *S = sc.packed[0];
    const uint32_t lo = tagh ? 1u : 0u;   // light-only heads
    if (a.ord) {   // home-ordered inserts: sources sharing a key hash separated (the idle sort buffer as scratch)
        if ((e = launch_ord_heads(S, sc.pay[0], bs, in, len, sc.headf, sc.seg_order, sc.packed[1], sc.pay[1], n,
                                  lim.seed, lim.table_mask, st)) != hipSuccess)
            return e;
        mark("k_ord_fix");
    }
    k_heads_count<<<gridTiles, 256, 0, st>>>(S, bs, in.hdr, sc.headf, sc.tile_aux, sc.sub_cnt, lo, a.ord ? 1u : 0u);
    mark("k_heads_count");
    k_scan_tiles_u32<<<1, 256, 0, st>>>(sc.tile_aux, bs, sc.seg_start, lo);
    // (the first sort word's low half per segment only for the flow rows)
    uint32_t *seg_lo = flows && !in.rec ? sc.seg_lo : nullptr;
    k_heads_write<<<gridTiles, 256, 0, st>>>(bs, sc.headf, sc.tile_aux, sc.seg_start, S,
                                             do_limit ? sc.seg_slot : nullptr,
                                             a.admit ? lim.admit_mask : lim.table_mask, lo, seg_lo);
    if (tagh)
        k_heads_heavy<<<1, 256, 0, st>>>(bs, sc.sort_ctl, sc.gbase, sc.seg_start, do_limit ? sc.seg_slot : nullptr,
                                         S_fin, lim.table_mask, seg_lo, sc.heavy);
    mark("k_heads_write");
    if (a.ord) {   // every segment's slot found / inserted in home order, then the table check
        static const uint32_t coh = getenv("FSX_ID_COHERENT") ? 1u : 0u;
        IdTable idt{a.X.heads, a.X.k6, lim.table_mask, lim.seed, a.X.epoch, lim.test_flags, table, a.id_gen, coh,
                    a.X.mir, a.X.mir_shift};
        idt.init = 0;   // (lazy slots: the walkers write a new source's line)
        idt.tgen = lim.tgen;
        // (the segment-order buffer holds the IPv6 lists, pass 0's tile rows — unused without
        // the heavy sort — their per-block counts)
        static const bool no_region = getenv("FSX_ORD_NO_REGION") != nullptr;   // A/B: global claims only
        if (!no_region) {
            // (pass 0's tile rows, unused without the heavy sort, hold the per-block counts)
            const uint32_t nb = std::max<uint32_t>(1, cdiv(n, kRegSeg));
            k_bs_flag<<<1, 1, 0, st>>>(bs);
            k_ord_claim<<<nb, 256, 0, st>>>(bs, sc.seg_start, S, in, idt, sc.seg_slot, sc.seg_order, sc.hist,
                                            sc.hist + nb, sc.pay[0], ts, len, sc.marks, table, lim);
            k_ord_spill<<<nb, 256, 0, st>>>(bs, sc.seg_start, S, in, idt, sc.seg_slot, sc.seg_order, sc.hist,
                                            sc.hist + nb);
            k_ord_count<<<1, 256, 0, st>>>(bs, sc.hist + nb, nb);
        } else {
            const uint32_t gr = std::min<uint32_t>(4096, std::max<uint32_t>(1, cdiv(n, 256)));
            k_ord_resolve4<<<gr, 256, 0, st>>>(bs, sc.seg_start, S, in, idt, sc.seg_slot, sc.seg_order, sc.hist);
            k_ord_resolve6<<<gr, 256, 0, st>>>(bs, sc.seg_start, S, in, idt, sc.seg_slot, sc.seg_order, sc.hist);
        }
        k_batch_check<<<1, 1, 0, st>>>(bs, tstate, lim, nullptr, 0u);
        mark("k_ord_resolve");
    }
    if (a.admit) {   // FSX_FLAG_OVERFLOW_ADMIT: every segment's table slot (admitted / transient)
        const uint32_t ga = std::min<uint32_t>(2048, std::max<uint32_t>(1, cdiv(n, 256)));
        const uint32_t gt = std::min<uint32_t>(4096, std::max<uint32_t>(1, cdiv(n, kTile)));
        k_admit_find<<<ga, 256, 0, st>>>(bs, S, sc.seg_start, sc.seg_slot, in, a.X, lim, sc.admit_rank);
        k_admit_rank<0><<<gt, 256, 0, st>>>(bs, sc.admit_rank, n, sc.admit_cnt);
        k_admit_scan<<<1, 256, 0, st>>>(bs, sc.admit_cnt, n);
        k_admit_rank<1><<<gt, 256, 0, st>>>(bs, sc.admit_rank, n, sc.admit_cnt);
        static const uint32_t coherent = getenv("FSX_ID_COHERENT") ? 1u : 0u;
        IdTable pidt{a.X.heads, a.X.k6, lim.table_mask, lim.seed, a.X.epoch, lim.test_flags, table, a.id_gen,
                     coherent, a.X.mir, a.X.mir_shift};
        pidt.tgen = lim.tgen;
        k_admit_insert<<<ga, 256, 0, st>>>(bs, tstate, S, sc.seg_start, sc.seg_slot, in, pidt, lim, sc.admit_rank,
                                           table, lim.table_mask + 1);
        k_admit_commit<<<1, 1, 0, st>>>(bs, tstate);
        mark("k_admit");
    }
    // pipelined sliding window with heavy lists: the heavy walkers (latency-bound, 32 blocks)
    // on the flow stream ahead of the flows, beside the light walkers; k_sw_hist joins them
    hipEvent_t sw_heavy_done = nullptr;
    if (do_limit && lim.limiter == 1 && tagh && split && split->tail && st2 && walk_fork_ev && walk_join_ev) {
        if ((e = hipEventRecord(walk_fork_ev, st)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(st2, walk_fork_ev, 0)) != hipSuccess) return e;
        mark_on(nullptr, 1);
        if ((e = launch_sw_heavy(S, ts, len, bs, sc, table, tstate, hist, lim, n, hlists,
                                 a.hfm ? verdict : nullptr, st2)) != hipSuccess)
            return e;
        mark_on("k_walk_sw_heavy", 1);
        if ((e = hipEventRecord(walk_join_ev, st2)) != hipSuccess) return e;
        sw_heavy_done = walk_join_ev;
    }
    if (flows) {
        hipStream_t fs = st;
        if (fork) {   // the features run beside the limiter
            if ((e = hipEventRecord(fork_ev, st)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(st2, fork_ev, 0)) != hipSuccess) return e;
            fs = st2;
            mark_on(nullptr, 1);
        }
        if ((e = launch_flows(S, sc.pay[0], bs, sc.headf, len, ts, in, sc.tile_aux, sc.sub_cnt, sc.seg_start,
                              sc.flow_first, sc.flow_last, sc.span_list, flows->acc, flows->keys16,
                              flows->fam, flows->feat, flows->prob, flows->dec, flows->cap, flows->score,
                              lim.salt32, n, do_limit ? flows->sacc : nullptr, flows->epoch, sc.seg_slot,
                              tagh, seg_lo, seg_lo ? sc.seg_len : nullptr, flows->part, fs)) != hipSuccess)
            return e;
        if (tagh) {   // the heavy sources' rows, from their sums (k_flow_heavy)
            if (hf != fs && (e = hipStreamWaitEvent(fs, heavy_flow_ev, 0)) != hipSuccess) return e;
            if ((e = launch_flows_heavy_finish(S_fin, bs, sc.sort_ctl, sc.seg_start, in, len, ts, sc.heavy_flow, sc.cap,
                                               flows->keys16, flows->fam, flows->feat, flows->prob, flows->dec,
                                               flows->cap, flows->score, lim.salt32,
                                               do_limit ? flows->sacc : nullptr, flows->epoch, sc.seg_slot, fs)) !=
                hipSuccess)
                return e;
            if (a.hfm && (e = launch_hflow_finish(bs, sc.sort_ctl, sc.heavy, sc.hflow, n, in, len, ts, flows->keys16,
                                                  flows->fam, flows->feat, flows->prob, flows->dec, flows->cap,
                                                  flows->score, do_limit ? flows->sacc : nullptr, flows->epoch,
                                                  PartialOut{}, fs)) != hipSuccess)
                return e;
        }
        mark_on("k_flow_features", fork ? 1 : 0);
        if (fork && (e = hipEventRecord(join_ev, st2)) != hipSuccess) return e;
    }
    if (!do_limit) return hipGetLastError();
    if (lim.limiter == 2) {   // FSX_LIMIT_TOKEN_BUCKET
        // (tagged heavy packets on the run path: their runs' heads and the tiles' segment offsets)
        if (tb_tag && (e = launch_tb_run_heads(bs, sc.seg_start, sc.headf, sc.tile_aux, n, st)) != hipSuccess)
            return e;
        if ((e = launch_token_bucket(S, ts, len, bs, sc, table, lim, n, st, mk, tb_tag ? 2u : 0u)) != hipSuccess)
            return e;
    } else {
        uint32_t *cls = sc.sort_ctl + 1028;
        const uint32_t short_seg = lim.limiter == 1 ? kShortSegSliding : kShortSegFixed;
        k_seg_count<<<kSegBlocks, 256, 0, st>>>(bs, sc.seg_start, sc.seg_cls, short_seg);
        k_seg_scan<<<1, 256, 0, st>>>(sc.seg_cls, cls);
        k_seg_order<<<kSegBlocks, 256, 0, st>>>(bs, sc.seg_start, sc.seg_cls, sc.seg_order, short_seg);
        mark("k_seg_order");
        if (lim.limiter == 1) {   // FSX_LIMIT_SLIDING_WINDOW
            if ((e = launch_sliding_window(S, ts, len, bs, sc, table, tstate, hist, lim, n, st, mk, st3,
                                           walk_fork_ev, walk_join_ev, &hlists, a.hfm ? verdict : nullptr,
                                           sw_heavy_done)) != hipSuccess)
                return e;
        } else {
            // short and long segments are disjoint: the wave walker runs on its own
            // stream beside the thread walker when a third stream is available
            const bool fork3 = st3 && walk_fork_ev && walk_join_ev;
            if (fork3) {
                if ((e = hipEventRecord(walk_fork_ev, st)) != hipSuccess) return e;
                if ((e = hipStreamWaitEvent(st3, walk_fork_ev, 0)) != hipSuccess) return e;
                mark_on(nullptr, 2);
            }
            k_walk_fixed_long<<<FSX_WALK_LONG_BLOCKS, 256, 0, fork3 ? st3 : st>>>(S, bs, sc.seg_start, sc.seg_slot, ts, len,
                                                                  sc.pay[0], sc.seg_order, cls, sc.marks,
                                                                  table, lim, hlists, skeys);
            mark_on("k_walk_fixed_long", fork3 ? 2 : 0);
            if (fork3 && (e = hipEventRecord(walk_join_ev, st3)) != hipSuccess) return e;
            // Unused dynamic LDS caps the thread walker's blocks per CU (53000 B: three) beside the
            // next batch's front when the host saw an all-light stream (Limits::light_dom): config 3
            // from a stream 5.96 / 6.04 -> 5.75 / 5.76 ms, while the headline (+5 %) and config 4
            // (+1.5 %) want it uncapped (profiles/r06/ab_r06wk*). FSX_WALK_LDS=B: B bytes always (A/B)
            static const int walk_env = getenv("FSX_WALK_LDS") ? atoi(getenv("FSX_WALK_LDS")) : -1;
            const uint32_t walk_lds = walk_env >= 0 ? (uint32_t)walk_env : lim.light_dom ? 53000u : 0u;
            k_walk_fixed<<<std::min<uint32_t>(FSX_WALK_SHORT_BLOCKS, cdiv(n, 256)), 256, walk_lds, st>>>(S, bs, sc.seg_start, sc.seg_slot, ts, len, sc.pay[0],
                                                     sc.seg_order, cls, sc.marks, table, lim, hlists, skeys);
            mark("k_walk_fixed");
            if (fork3 && (e = hipStreamWaitEvent(st, walk_join_ev, 0)) != hipSuccess) return e;
        }
    }
    const uint32_t fill_lo = tb_tag ? 2u : tagh ? 1u : 0u;   // (cover_n)
    k_fill_last<<<gridTiles, 256, 0, st>>>(sc.marks, bs, sc.tile_last, fill_lo);
    k_fill_carry<<<1, 1024, 0, st>>>(sc.tile_last, bs, fill_lo);
    mark("k_fill_last");
    // Light DROPs (heavy verdict lists on: the rest are lists) stored straight into the
    // verdicts: config 4's 12.8M light DROPs 1.11 -> 0.32 ms. Without heavy lists (the token
    // bucket: about every other packet a DROP) per-chunk lists that k_verdict_apply merges:
    // 33M scattered byte stores took 0.44 ms and 1.15 GB. (FSX_DROP_LISTS=1: lists always.)
    static const bool drop_lists = getenv("FSX_DROP_LISTS") != nullptr;
    k_fill_scatter<<<gridTiles, 256, 0, st>>>(sc.marks, S, bs, sc.tile_last, sc.drop_list, sc.drop_cur,
                                              tstate, cdiv(n, kVChunk), fill_lo,
                                              drop_lists || !tagh ? nullptr : verdict);
    mark("k_fill_scatter");
    if (tb_tag && (e = launch_tb_untag(bs, verdict, n, st)) != hipSuccess) return e;   // (run path only)
    if (heavy_join && (e = hipStreamWaitEvent(st, walk_join_ev, 0)) != hipSuccess) return e;
    k_verdict_apply<<<cdiv(n, kVChunk), 256, 0, st>>>(verdict, n, sc.drop_list, sc.drop_cur, bs, sc.heavy,
                                                      hlists.list);
    mark("k_verdict_apply");
    if (fork) {
        static const bool end_aux = getenv("FSX_TAIL_END_AUX") != nullptr;   // A/B (slower: 2.99 vs 2.96 ms)
        if (split && split->tail && end_aux) {   // pipelined: the tail ends on the flow stream (flush_tail)
            if ((e = hipEventRecord(walk_join_ev, st)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(st2, walk_join_ev, 0)) != hipSuccess) return e;
        } else if ((e = hipStreamWaitEvent(st, join_ev, 0)) != hipSuccess) {
            return e;
        }
    }
    return hipGetLastError();
}

hipError_t launch_verdict_pipeline(const PacketIn &in, const uint32_t *len, const uint64_t *ts,
                                   uint32_t n, uint8_t *verdict, Slot *table, TableState *tstate,
                                   BatchState *bs, const Scratch &sc_in, uint32_t id_gen,
                                   const TableIndex &X, const Limits &lim, const RuleSet &rules,
                                   bool do_limit, const FlowRequest *flows,
                                   const HistBufs &hist, hipStream_t st, hipStream_t st2,
                                   hipEvent_t fork_ev, hipEvent_t join_ev, hipStream_t st3,
                                   hipEvent_t walk_fork_ev, hipEvent_t walk_join_ev, hipEvent_t heavy_fork_ev,
                                   hipEvent_t heavy_flow_ev, PipeTiming *tm, const PipeSplit *split) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    Scratch sc = sc_in;        // packed[0] / pay[0] become the sorted output below
    int last[3] = {-1, -1, -1};   // last event index per stream (timing)
    // mark(name) closes the interval of the kernel just enqueued on stream s (0: st, 1: st2,
    // 2: st3)
    auto mark_on = [&](const char *name, int s_id) {
        if (!tm || tm->used >= tm->cap) return;
        const int i = tm->used++;
        tm->names[i] = name;
        tm->prev[i] = last[s_id];
        (void)hipEventRecord(tm->ev[i], s_id == 2 ? st3 : s_id == 1 ? st2 : st);
        last[s_id] = i;
    };
    auto mark = [&](const char *name) { mark_on(name, 0); };
    const Marker mk{[](void *p, const char *name) { (*static_cast<decltype(mark) *>(p))(name); }, &mark};
    if (tm) tm->used = 0;
    hipError_t e;
    // the prologue's stream: a pipelined batch resets its own scratch and picks its heavy
    // sources on `split->pro` while the previous batch's sort runs on st (it needs only the
    // previous batch's parse: the index); the parse waits for it below
    const bool early = split && split->pro && split->pro_wait && split->pro_done && !tm && n > 0;
    hipStream_t sp0 = early ? split->pro : st;
    if (early && (e = hipStreamWaitEvent(sp0, split->pro_wait, 0)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(bs, 0, sizeof(BatchState), sp0)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;

    const uint32_t gridStream = std::min<uint32_t>(2048, std::max<uint32_t>(1, cdiv(n, 256)));
    const uint32_t gridTiles = std::min<uint32_t>(4096, std::max<uint32_t>(1, cdiv(n, kTile)));

    // mark(name) closes the interval of the kernel just enqueued (per-kernel timing)
    const bool onesweep = (lim.test_flags & 2u) != 0;
    // with the limiter, sources are found / inserted in the persistent index (sort id =
    // table slot); flow features alone use a per-batch id table and touch no map state
    static const uint32_t coherent = getenv("FSX_ID_COHERENT") ? 1u : 0u;
    // FSX_FLAG_OVERFLOW_ADMIT: per-batch ids for every source; table slots from the admission
    // kernels after the heads (launch_tail)
    const bool admit = do_limit && (lim.test_flags & kFlagAdmit) != 0;
    const uint64_t bmask = admit ? lim.admit_mask : lim.table_mask;   // the per-batch id table's
    IdTable idt = do_limit && !admit
        ? IdTable{X.heads, X.k6, lim.table_mask, lim.seed, X.epoch, lim.test_flags, table, id_gen, coherent,
                  X.mir, X.mir_shift}
        : IdTable{reinterpret_cast<unsigned long long *>(sc.id_tab), sc.id_tab + 2 * (bmask + 1),
                  bmask, lim.seed, id_gen, lim.test_flags, nullptr, 0, coherent};
    idt.tgen = lim.tgen;
    if ((e = hipMemsetAsync(sc.sort_ctl, 0, kSortCtlWords * 4, sp0)) != hipSuccess) return e;
    if (admit && (e = hipMemsetAsync(sc.admit_rank, 0, (size_t)n * 4, sp0)) != hipSuccess) return e;
    mark("start");
    const uint32_t ntiles = std::max<uint32_t>(1, cdiv(n, kSortTile));
    const uint32_t tcap = (uint32_t)(sc.cap / kSortTile + 2);
    // source ids have log2(slots) bits: ceil(bits / 8) LSD passes of equal digits of at
    // most 8 bits (21 bits: 3 x 7 — fewer buckets, longer runs per tile than 8 + 8 + 5)
    uint32_t idbits = 0;
    while ((1ull << idbits) <= idt.mask) ++idbits;
    // home-ordered inserts (the host asks per batch: a flood of new sources; fixed window with
    // lazy slots, header records, no flows): 32-bit key hashes sort in four 8-bit passes
    static const bool eager_slots = getenv("FSX_EAGER_SLOTS") != nullptr;
    const bool ord = lim.ord && do_limit && lim.limiter == 0 && !(lim.test_flags & kFlagAdmit) && !eager_slots &&
                     !flows && !in.rec && idbits >= 1 && idbits <= 31;
    if (ord) idbits = 32;
    static const bool full_digits = getenv("FSX_SORT_FULL_DIGITS") != nullptr;   // A/B: 8,8,..,rest
    static const bool no_heavy = getenv("FSX_NO_HEAVY_SORT") != nullptr;          // A/B: plain LSD
    // Heavy-source sort (tables of <= 2^25 slots): pass 0 buckets the light entries by a
    // low id digit and every heavy source into a bucket of its own (the bucket in bits
    // [bshift, 64) above the id: 8 bits, light digit 7 bits and 128 heavy sources for every
    // id width it takes, up to 25 bits: bshift = 56); the later passes sort
    // the light entries only, by the remaining id bits in equal digits. Pass 0 writes the
    // other sort buffer, which then holds the heavy runs for good (the later passes cover
    // [0, n_light)); with an even pass count the light entries end in the parse buffer, so
    // the heavy runs are read from pass 0's buffer (S_heavy in the tail): only the fixed
    // window's heavy verdict lists consume them apart from the light entries, so an even
    // count is taken with those lists only. The sliding window's heavy lists (its history
    // rebuild reads every segment from the final buffer) need an odd count.
    static const bool no_hlists = getenv("FSX_NO_HEAVY_LISTS") != nullptr;
    const bool lists_any = do_limit && verdict && !no_hlists && !admit;
    const bool lists_ok = lists_any && lim.limiter == 0;
    // heavy verdict lists (fixed / sliding window with the heavy-source sort; FSX_NO_HEAVY_LISTS=1: A/B)
    const bool lists_sw0 = lists_any && lim.limiter == 1;
    // The digit plan (fsx_plan.h). 24- / 25-bit ids (17 / 18 light bits after pass 0's 7): two
    // light passes of 9-bit digits (512-digit tiles, bases from the tile scan: k_digit_base)
    // instead of three of 6 bits, for every limiter batch with verdicts — the fixed window (heavy
    // lists), the sliding window (heavy lists: the odd count they need) and the token bucket
    // (sorted heavy runs); FSX_SORT_LIGHT6=1: the three 6-bit passes (A/B; the sliding window
    // and the token bucket then take the plain sort). Plain sorts of 25- / 26-bit ids (flow-only
    // batches, admission off): three passes of 8 + 8 + 9 / 8 + 9 + 9 bits instead of four of 7
    // (FSX_SORT_PLAIN4=1: the four passes, A/B).
    static const bool light6 = getenv("FSX_SORT_LIGHT6") != nullptr;
    static const bool plain4 = getenv("FSX_SORT_PLAIN4") != nullptr;
    static_assert(kPlanIdShift == kIdShift, "fsx_plan.h's id position");
    SortPlanIn pq;
    pq.idbits = idbits; pq.onesweep = onesweep; pq.full_digits = full_digits; pq.no_heavy = no_heavy;
    pq.admit = admit; pq.lists_any = lists_any; pq.lists_ok = lists_ok; pq.light6 = light6; pq.plain4 = plain4;
    const SortPlan plan = make_sort_plan(pq);
    const int npass = plan.npass;
    const bool heavy_sort = plan.heavy_sort;
    const uint32_t bshift = plan.bshift;
    const bool lists_sw = lists_sw0 && (npass & 1);
    // heavy slots resolved once in k_heavy_pick (FSX_NO_HEAVY_SLOTS=1: A/B). Under prefix rules
    // the pick leaves every source whose /24 a rule touches light (rule_maybe), so a heavy
    // source is never rule-dropped and may be inserted there (round 5; FSX_RULES_LAZY_HEAVY=1:
    // round 4's unresolved heavy sources under rules, inserted by the parse, on the run path)
    static const bool no_hslots = getenv("FSX_NO_HEAVY_SLOTS") != nullptr;
    static const bool rules_lazy = getenv("FSX_RULES_LAZY_HEAVY") != nullptr;
    const bool rl_batch = do_limit && rules.slot;
    const uint32_t resolve = !no_hslots && !(rl_batch && (rules_lazy || in.rec)) ? 1u : 0u;
    // token bucket: the heavy sources outside the sort (launch_tb_heavy; round 6, VERDICT r05
    // item 4) — tagged heavy packets with resolved slots, the heavy runs in the light entries'
    // final buffer (an odd pass count) for the run path. Bit-exact and measured slower than the
    // heavy-source sort (4.70 / 4.74 vs 3.96 / 3.94 ms per 64M packets), so
    // opt-in: FSX_TB_UNSORTED=1 (read per batch: tests switch it)
    const bool tb_unsorted = getenv("FSX_TB_UNSORTED") != nullptr;
    const bool lists_tb = lists_any && lim.limiter == 2 && (npass & 1) && resolve && tb_unsorted;
    const bool tagh = heavy_sort && (lists_ok || lists_sw || lists_tb);
    // heavy sources outside the sort (fsx_heavy.hip): header records with resolved heavy
    // slots; k_hmode picks the batch's path on the device (FSX_NO_HFAST=1: the runs, A/B)
    static const bool no_hfast = getenv("FSX_NO_HFAST") != nullptr;
    // (record mode too: the records' len / ts go to in.rec_len / rec_ts, which k_pass0h reads)
    // (sliding window: FSX_FLAG_SW_UNSORTED only — measured slower than the sort)
    const bool hfm = tagh && (lim.limiter == 0 || lim.limiter == 2 ||
                              (lim.limiter == 1 && (lim.test_flags & kFlagSwUnsorted))) &&
                     resolve && !no_hfast;
    if (!(split && split->tail) && (e = hipMemsetAsync(sc.marks, 0, n, st)) != hipSuccess) return e;
    DigitPlan dp{};
    dp.npass = (uint32_t)npass;
    dp.nhist = plan.nhist;
    dp.light_b = plan.light_b;
    for (int p = 0; p < 4; ++p) { dp.shift[p] = plan.shift[p]; dp.mask[p] = plan.mask[p]; }
    const bool wide_plan = plan.tile_bases;   // (passes >= 1: bases from the tile scan)
    uint32_t nheavy = kHeavyMax;
    if (heavy_sort) {
        nheavy = std::min<uint32_t>(kHeavyMax, (1u << (64 - bshift)) - dp.light_b);
        static const uint32_t heavy_n = getenv("FSX_HEAVY_N") ? (uint32_t)atoi(getenv("FSX_HEAVY_N")) : 0u;
        if (heavy_n) nheavy = std::min(nheavy, heavy_n);   // (A/B: fewer heavy sources)
    }
    if (heavy_sort) {
        k_heavy_sample<<<64, 256, 0, sp0>>>(in, len, n, sc.sketch, lim.seed, lim.table_mask, lim.test_flags);
        // (sliding window on the unsorted path: only sources with >= 1/96 of the sample — the
        // rank walker's dense ones, k_hmode_state sends any under 1/128 of the batch to the
        // run path — the rest sort with the light sources)
        const uint32_t S = std::min<uint32_t>(n, kHeavySample);
        // (FSX_SW_FLOOR=D: 1/D of the sample instead, 0 the fixed window's floor — A/B)
        static const uint32_t sw_div = getenv("FSX_SW_FLOOR") ? (uint32_t)atoi(getenv("FSX_SW_FLOOR")) : 96u;
        const bool sw_dense = hfm && lim.limiter == 1 && !(lim.test_flags & kFlagSwSparse) && sw_div;
        const uint32_t floor_cnt = sw_dense ? std::max<uint32_t>(16, S / sw_div) : 16u;
        k_heavy_pick<<<1, 1024, 0, sp0>>>(in, len, sc.sketch, sc.heavy, nheavy, floor_cnt, lim.seed,
                                          lim.table_mask, lim.test_flags, idt, resolve, bs,
                                          rl_batch ? rules : RuleSet{});
        mark("k_heavy_pick");
    }
    if (early) {   // the parse after the prologue
        if ((e = hipEventRecord(split->pro_done, sp0)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(st, split->pro_done, 0)) != hipSuccess) return e;
    }
    // Lazy slots (fixed window): k_parse claims a new source's index head only; the walker
    // that first stores its state writes the rest (one random line per insert instead of
    // two: the head's and the slot's; FSX_EAGER_SLOTS=1: A/B). The heavy pick, the other
    // limiters and the admission path initialise slots as they insert.
    static const bool eager = getenv("FSX_EAGER_SLOTS") != nullptr;
    const bool lazy = do_limit && !admit && lim.limiter == 0 && !eager;
    // pipelined: the previous batch's tail goes in right before this batch's parse, so it
    // overlaps the parse and the sort (the parse touches the index heads and new sources'
    // slots only, the previous batch's walkers its own sources' slots; the heavy sources'
    // carried state is read at the tail's start, k_hmode_state). A/B, FSX_TAIL_AT: -1 before
    // the parse (default; 2.914 / 2.918 vs 2.937 / 2.939 ms, profiles/r04/ab_r04ab.txt), 0
    // after it (round 3's default), 1 after the first pass's offsets scan, 2 after the first
    // scatter (3.46 / 3.77 vs 3.46 ms in round 3).
    const bool pw = split && split->pro_wait;
    static const int tail_at = getenv("FSX_TAIL_AT") ? atoi(getenv("FSX_TAIL_AT")) : -1;
    bool hooked = false;   // (exactly once per pipelined batch: a tail left unhooked would be lost)
    auto tail_hook = [&](int at) -> hipError_t {
        if (hooked || !split || !split->on_parse || (at != tail_at && at != 3)) return hipSuccess;
        hooked = true;
        // (right after the parse the tail waits on the prologue's event: one marker, not two)
        return split->on_parse(split->cb, at == 0 && pw ? split->pro_wait : nullptr);
    };
    if ((e = tail_hook(-1)) != hipSuccess) return e;
    IdTable pidt = idt;
    if (lazy) pidt.init = 0;
    {
        const uint32_t g = std::min<uint32_t>(FSX_PARSE_GRID, ntiles);   // one resident block per slot
        const HeavySet *hs = heavy_sort ? sc.heavy : nullptr;
        uint32_t *th = onesweep ? nullptr : sc.hist;
        // (FSX_PARSE_PAY: the light payload words, compacted like the words, into pay[0], which
        // pass 0 reads before pass 1 writes it; else the light-packet masks)
        uint64_t *lmask = hfm && FSX_PARSE_PAY ? sc.pay[0] : light_masks(sc.chunk_cnt, sc.cap);
        // the prefix rules apply to limiter batches (an instantiation of its own, so the
        // rule-free parse keeps its registers)
        const bool rl = do_limit && rules.slot;
        // (kMir: light IPv4 sources probe the persistent index's mirror, not its heads)
#define FSX_PARSE(R, Q, H) (idt.mir ? k_parse<R, Q, true, H><<<g, 256, 0, st>>>(in, len, ts, n, sc.packed[0], verdict, bs, pidt, \
                                                        sc.sort_ctl, th, tcap, dp, hs, rules, tagh ? 1u : 0u, sc.chunk_cnt, lmask) \
                                 : k_parse<R, Q, false, H><<<g, 256, 0, st>>>(in, len, ts, n, sc.packed[0], verdict, bs, pidt, \
                                                        sc.sort_ctl, th, tcap, dp, hs, rules, tagh ? 1u : 0u, sc.chunk_cnt, lmask))
        if (ord)
            rl ? k_parse<0, true, false, false, true><<<g, 256, 0, st>>>(in, len, ts, n, sc.packed[0], verdict, bs, pidt,
                                                                        sc.sort_ctl, th, tcap, dp, hs, rules, 0u,
                                                                        sc.chunk_cnt, lmask)
               : k_parse<0, false, false, false, true><<<g, 256, 0, st>>>(in, len, ts, n, sc.packed[0], verdict, bs,
                                                                         pidt, sc.sort_ctl, th, tcap, dp, hs, rules,
                                                                         0u, sc.chunk_cnt, lmask);
        else if (hfm)   // (with prefix rules: header records only, resolve above)
            !in.rec ? (rl ? FSX_PARSE(0, true, true) : FSX_PARSE(0, false, true))
                    : in.rec_bytes == 16 ? FSX_PARSE(16, false, true) : FSX_PARSE(32, false, true);
        else if (!in.rec)
            rl ? FSX_PARSE(0, true, false) : FSX_PARSE(0, false, false);
        else if (in.rec_bytes == 16)
            rl ? FSX_PARSE(16, true, false) : FSX_PARSE(16, false, false);
        else
            rl ? FSX_PARSE(32, true, false) : FSX_PARSE(32, false, false);
#undef FSX_PARSE
    }
    mark("k_parse");
    // (the next batch's prologue may start once this parse has updated the index; recorded
    // after every split batch's parse, also one whose own prologue ran on st)
    if (pw && (e = hipEventRecord(split->pro_wait, st)) != hipSuccess) return e;
    // Heavy verdict lists: every heavy source is one run of pass 0's output (the later passes
    // write [0, n_light) only) whose segment needs no head search, so its walker and its flow
    // sums run on the third stream beside the heads, the classes and the light walkers, which
    // like the light flow tiles cover [0, n_light) only (k_heads_heavy appends the heavy
    // segments).
    static const bool no_fork = getenv("FSX_NO_FLOW_FORK") != nullptr;   // A/B: flows serialized
    if ((e = tail_hook(0)) != hipSuccess) return e;
    k_hist_prep<<<1, 256, 0, st>>>(sc.sort_ctl, sc.gbase, bs, heavy_sort ? dp.light_b : 256u);
    if (do_limit && !ord)   // (home-ordered: after the slots are found, launch_tail)
        k_batch_check<<<1, 1, 0, st>>>(bs, tstate, lim, split ? split->prev : nullptr,
                                       split && split->tail && lim.limiter == 1 ? 1u : 0u);
    const uint32_t gen0 = onesweep ? next_generation() : 0u;
    for (int pass = 0; pass < npass; ++pass) {
        const uint64_t *in = sc.packed[pass & 1];
        uint64_t *out = sc.packed[(pass + 1) & 1];
        const uint64_t *pin = pass == 0 ? nullptr : sc.pay[pass & 1];
        uint64_t *pout = sc.pay[(pass + 1) & 1];
        const uint32_t shift = dp.shift[pass], pmask = dp.mask[pass];
        // the light passes' tile rows in a region of their own: pass 0's rows of the heavy
        // buckets (light_b + h) are read in the tail (k_walk_heavy_sel, k_hflow_combine,
        // k_heavy_gather) — an 8-bit light digit (tables of 2^22 / 2^23 slots) would overwrite them
        uint32_t *hst = pass > 0 && heavy_sort ? sc.hist + 256ull * tcap : sc.hist;
        // the next pass's digit byte per output position (its tile histogram reads those
        // instead of the keys; FSX_SORT_KEY_HIST=1: the keys, A/B)
        static const bool key_hist = getenv("FSX_SORT_KEY_HIST") != nullptr;
        const bool dig_on = !key_hist && sc.dig;
        uint8_t *dout = dig_on && pass + 1 < npass ? sc.dig : nullptr;
        const uint32_t nshift = pass + 1 < npass ? dp.shift[pass + 1] : 0u;
        const uint32_t nmask = pass + 1 < npass ? dp.mask[pass + 1] : 0u;
        // the 9-bit plan's light passes: 512-digit tiles, 16-bit digit words, bases from the
        // tile scan's row totals (k_parse counted pass 0's digits only)
        const bool kwide = pmask > 255u, nwide = nmask > 255u;
        const bool tbase = wide_plan && pass > 0;
        uint32_t *dbase = sc.gbase + 1024;
        if (onesweep) {
            const uint32_t *Ld = pass == 0 ? nullptr : &bs->n_valid;
            k_onesweep<kLookW><<<ntiles, 256, 0, st>>>(in, out, n, Ld, shift, pmask, sc.gbase + 256 * pass,
                                                       sc.status, sc.sort_ctl + 1024 + pass,
                                                       gen0 + (uint32_t)pass, pass == 0, bs, pin, pout,
                                                       ts, len);
            mark("k_onesweep");
        } else {
            // passes >= 1 cover [0, n_light): the heavy entries (pass 0's top buckets) are
            // final in pass 0's output (packed[1]; the light entries end there too when npass
            // is odd, in packed[0] when it is even)
            const uint32_t *Ld = pass == 0 ? nullptr : &bs->n_light;
            if (pass > 0) {   // pass 0's per-tile counts come from k_parse
                if (kwide)
                    k_tile_hist<512><<<ntiles, 256, 0, st>>>(in, n, Ld, shift, pmask, pass == 0, hst, tcap,
                                                             dig_on ? sc.dig : nullptr);
                else
                    k_tile_hist<256><<<ntiles, 256, 0, st>>>(in, n, Ld, shift, pmask, pass == 0, hst, tcap,
                                                             dig_on ? sc.dig : nullptr);
                mark("k_tile_hist");
            }
            if (tbase) {
                k_tile_scan<<<pmask + 1, 256, 0, st>>>(hst, tcap, n, Ld, nullptr, dbase);
                k_digit_base<<<1, 256, 0, st>>>(dbase);
            } else {
                k_tile_scan<<<pmask + 1, 256, 0, st>>>(hst, tcap, n, Ld, sc.gbase + 256 * pass);
            }
            mark("k_tile_scan");
            if (pass == 0 && (e = tail_hook(1)) != hipSuccess) return e;
            if (pass == 0 && hfm) {   // light words from the parse chunks; heavy tile sums; the path
                if ((e = launch_pass0h(in, out, n, shift, pmask, sc.hist, tcap, bs, pout, ts, len, verdict,
                                       sc.chunk_cnt, light_masks(sc.chunk_cnt, sc.cap), sc.hrec, sc.heavy,
                                       FSX_PARSE_PAY ? sc.pay[0] : nullptr, st, dout, nshift, nmask,
                                       nwide ? 1 : 0)) != hipSuccess)
                    return e;
                mark("k_pass0h");
                if ((e = launch_hmode(bs, ts, n, lim, st)) != hipSuccess) return e;
                mark("k_hmode");
            } else {
#define FSX_SCATTER(D, B) k_tile_scatter<kLatePayDefault, D, B><<<ntiles, 256, 0, st>>>( \
                    in, out, n, Ld, shift, pmask, pass == 0, hst, tcap, bs, pin, pout, ts, len, dout, nshift, nmask, \
                    dbase, nwide ? 1 : 0)
                if (!tbase) FSX_SCATTER(256, false);
                else if (!kwide) FSX_SCATTER(256, true);
                else FSX_SCATTER(512, true);
#undef FSX_SCATTER
                mark("k_tile_scatter");
            }
            if (pass == 0 && (e = tail_hook(2)) != hipSuccess) return e;
        }
    }
    if ((e = tail_hook(3)) != hipSuccess) return e;   // (any position not reached: onesweep)
    if (split && split->front_done) {   // pipelined: the front is done; the tail is handed back
        if ((e = hipEventRecord(split->front_done, st)) != hipSuccess) return e;
    }
    TailArgs ta{};
    ta.in = in; ta.len = len; ta.ts = ts; ta.n = n; ta.verdict = verdict; ta.table = table; ta.tstate = tstate;
    ta.bs = bs; ta.sc = sc; ta.lim = lim; ta.do_limit = do_limit;
    ta.has_flows = flows != nullptr;
    if (flows) ta.fq = *flows;
    ta.hist = hist; ta.st = st; ta.st2 = st2; ta.st3 = st3; ta.fork_ev = fork_ev; ta.join_ev = join_ev;
    ta.walk_fork_ev = walk_fork_ev; ta.walk_join_ev = walk_join_ev; ta.heavy_fork_ev = heavy_fork_ev;
    ta.heavy_flow_ev = heavy_flow_ev; ta.tm = tm; ta.split = split != nullptr;
    if (split) ta.sp = *split;
    ta.npass = npass; ta.tagh = tagh; ta.gridTiles = gridTiles;
    ta.hfm = hfm; ta.shift0 = dp.shift[0];
    ta.admit = admit; ta.X = X; ta.id_gen = id_gen; ta.lazy = lazy; ta.fresh_bit = lazy && (!heavy_sort || hfm);
    ta.ord = ord;
    ta.fork = flows && do_limit && st2 && fork_ev && join_ev && !no_fork;
    for (int k = 0; k < 3; ++k) ta.last[k] = last[k];
    if (split && split->tail_out) {
        *split->tail_out = ta;
        return hipGetLastError();
    }
    return launch_tail(ta);
}

// ------------------------------------------------------------------ table clear
// fsx_reset / the eviction rebuild: the slot table zeroed with 16-byte stores, each wave
// writing 1 KiB runs (whole lines), four stores in flight per lane, XCD-contiguous chunks
// (FSX_CLEAR_MEMSET=1: hipMemsetAsync, A/B; config 5's 32 GiB table).
__global__ __launch_bounds__(256) void k_clear16(uint4 *__restrict__ p, uint64_t n16) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u *q = reinterpret_cast<v4u *>(p);
    const uint64_t nb = gridDim.x;
    const uint64_t b = xcd_swizzle(blockIdx.x, gridDim.x);
    // block b owns the contiguous share [lo, hi) of the 16-byte words
    const uint64_t lo = n16 * b / nb, hi = n16 * (b + 1) / nb;
    const v4u z = {0u, 0u, 0u, 0u};
    uint64_t i = lo + threadIdx.x;
    for (; i + 768 < hi; i += 1024) {
        __builtin_nontemporal_store(z, q + i);
        __builtin_nontemporal_store(z, q + i + 256);
        __builtin_nontemporal_store(z, q + i + 512);
        __builtin_nontemporal_store(z, q + i + 768);
    }
    for (; i < hi; i += 256) __builtin_nontemporal_store(z, q + i);
}

hipError_t launch_clear(void *p, uint64_t bytes, hipStream_t st) {
    static const bool memset = getenv("FSX_CLEAR_MEMSET") != nullptr;
    if (memset || (bytes & 15) || (reinterpret_cast<uintptr_t>(p) & 15)) return hipMemsetAsync(p, 0, bytes, st);
    const uint64_t n16 = bytes / 16;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, n16 / 4096));
    k_clear16<<<grid, 256, 0, st>>>(static_cast<uint4 *>(p), n16);
    return hipGetLastError();
}

// ------------------------------------------------------------------ map syscalls
// op: 0 lookup, 1 update, 2 delete. Result: 0 / -ENOENT(-2) / -EEXIST(-17) / -ENOSPC(-28).
// Map id -> table tag (1 IPv4, 2 IPv6) and slot flag bit (include/fsx_hip.h map ids).
__host__ __device__ inline uint32_t map_tag(int map_id) { return (map_id == 2 || map_id == 4 || map_id == 6) ? 2u : 1u; }
__host__ __device__ inline uint32_t map_bit(int map_id) {
    return (map_id == 1 || map_id == 2) ? SLOT_HAS_ST : (map_id == 5 || map_id == 6) ? SLOT_HAS_TB : SLOT_HAS_BL;
}

__global__ void k_map_op(Slot *table, TableState *tstate, Limits lim, TableIndex X, int op, int map_id,
                         uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint64_t v0,
                         uint64_t v1, uint64_t v2, uint64_t flags, int32_t *res, uint64_t *outv) {
    if (threadIdx.x || blockIdx.x) return;
    const uint32_t k[4] = {k0, k1, k2, k3};
    const uint32_t tag = map_tag(map_id);
    const uint32_t bit = map_bit(map_id);
    uint32_t s = table_find(table, lim, tag, k);
    const bool present = s != kNoSlot && (table[s].flags & bit);
    if (op == 0) {
        if (!present) { *res = -2; return; }
        if (bit == SLOT_HAS_ST) { outv[0] = table[s].pps; outv[1] = table[s].bps; outv[2] = table[s].tt; }
        else if (bit == SLOT_HAS_TB) { outv[0] = table[s].aux; outv[1] = table[s].tt; }
        else outv[0] = table[s].till;
        *res = 0;
        return;
    }
    if (op == 2) {
        if (!present) { *res = -2; return; }
        table[s].flags &= ~bit;
        *res = 0;
        return;
    }
    if (flags == 1 && present) { *res = -17; return; }
    if (flags == 2 && !present) { *res = -2; return; }
    if (s == kNoSlot) {
        if (tstate->count >= lim.max_entries) { *res = -28; return; }
        s = table_claim(table, lim, X, tag, k);
        if (s == kNoSlot) { *res = -28; return; }
        tstate->count += 1;
    }
    if (bit == SLOT_HAS_ST) { table[s].pps = v0; table[s].bps = v1; table[s].tt = v2; }
    else if (bit == SLOT_HAS_TB) { table[s].aux = v0; table[s].tt = v1; }
    else table[s].till = v0;
    table[s].flags |= bit;
    *res = 0;
}

// Batched update (BPF_MAP_UPDATE_BATCH with BPF_ANY; distinct keys): one thread per
// entry finds or inserts its source in the index exactly as k_parse does (CAS claims,
// slots stamped with generation `born` so a failing import rolls back like a batch),
// then writes the value; new sources are counted in bs->n_new and checked against
// max_entries by k_batch_check.
__global__ __launch_bounds__(256) void k_map_import(Slot *table, Limits lim, TableIndex X, uint32_t born,
                                                    int map_id, const uint32_t *__restrict__ keys,
                                                    const uint64_t *__restrict__ vals, uint32_t n,
                                                    BatchState *bs) {
    const uint32_t tag = map_tag(map_id), bit = map_bit(map_id);
    const uint32_t kw = tag == 2 ? 4u : 1u;
    const uint32_t vw = bit == SLOT_HAS_ST ? 3u : bit == SLOT_HAS_TB ? 2u : 1u;
    IdTable idt{X.heads, X.k6, lim.table_mask, lim.seed, X.epoch, lim.test_flags, table, born, 0u,
                X.mir, X.mir_shift};
    idt.tgen = lim.tgen;
    uint32_t fresh_n = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        uint32_t k[4] = {0, 0, 0, 0};
        for (uint32_t q = 0; q < kw; ++q) k[q] = keys[(size_t)i * kw + q];
        const uint64_t h = probe_start(tag, k, lim.seed, lim.table_mask, lim.test_flags);
        bool fresh = false;
        const uint32_t s = id_resolve(idt, tag, k, h, X.heads[h], &fresh);
        if (s == kNoSlot) { atomicOr(&bs->err, ERR_TABLE_FULL); continue; }
        fresh_n += fresh;
        Slot &sl = table[s];
        const uint64_t *v = vals + (size_t)i * vw;
        if (bit == SLOT_HAS_ST) { sl.pps = v[0]; sl.bps = v[1]; sl.tt = v[2]; }
        else if (bit == SLOT_HAS_TB) { sl.aux = v[0]; sl.tt = v[1]; }
        else sl.till = v[0];
        atomicOr(&sl.flags, bit);
    }
    if (fresh_n) atomicAdd(&bs->n_new, fresh_n);
}

hipError_t launch_map_import(Slot *table, TableState *tstate, BatchState *bs, const Limits &lim,
                             const TableIndex &X, uint32_t born, int map_id, const uint32_t *d_keys,
                             const uint64_t *d_vals, uint32_t n, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    hipError_t e = hipMemsetAsync(bs, 0, sizeof(BatchState), st);
    if (e != hipSuccess || n == 0) return e;
    const uint32_t grid = std::min<uint32_t>(4096, (n + 255) / 256);
    k_map_import<<<grid, 256, 0, st>>>(table, lim, X, born, map_id, d_keys, d_vals, n, bs);
    k_batch_check<<<1, 1, 0, st>>>(bs, tstate, lim, nullptr);
    return hipGetLastError();
}

// ------------------------------------------------------------------ idle eviction
// FSX_FLAG_EVICT_IDLE (oracle/fsx_oracle.c evict_idle). Open addressing
// cannot drop an entry in place (a later key's probe chain may run through it), so the
// survivors are copied out and re-inserted under a new index epoch.
__device__ __forceinline__ uint64_t batch_ts(const PacketIn &in, const uint64_t *ts, uint32_t i) {
    if (!in.rec) return ts[i];
    const uint4 *r = reinterpret_cast<const uint4 *>(in.rec);
    if (in.rec_bytes == 16) {   // ShardRecord16 {key, len | dport << 16, ts}
        const uint4 w = r[i];
        return (uint64_t)w.z | ((uint64_t)w.w << 32);
    }
    const uint4 w = r[(size_t)i * 2 + 1];   // ShardRecord: ts after the 16 key bytes
    return (uint64_t)w.x | ((uint64_t)w.y << 32);
}

__global__ __launch_bounds__(256) void k_evict_min_ts(PacketIn in, const uint64_t *__restrict__ ts, uint32_t n,
                                                      unsigned long long *scal) {
    uint64_t m = ~0ull;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint64_t t = batch_ts(in, ts, i);
        m = t < m ? t : m;
    }
    m = ~wave_max(~m);
    if (lane_id() == 0 && m != ~0ull) atomicMin(&scal[0], (unsigned long long)m);
}

// Live at now0: a window still open (the reset test of src/fsx_kern.c:245 fails), a live
// blacklist entry (src/fsx_kern.c:189-204), or token-bucket state.
__device__ __forceinline__ bool slot_live(const Slot &s, const Limits &lim, uint64_t now0) {
    return ((s.flags & SLOT_HAS_ST) && !(now0 - s.tt > lim.window)) ||
           ((s.flags & SLOT_HAS_BL) && s.till > 0 && !(now0 > s.till)) || (s.flags & SLOT_HAS_TB);
}

__global__ __launch_bounds__(256) void k_evict_compact(const Slot *__restrict__ table, Limits lim, Slot *buf,
                                                       uint64_t cap, unsigned long long *scal) {
    const uint64_t now0 = scal[0];
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= lim.table_mask;
         i += (uint64_t)gridDim.x * 256u) {
        const Slot s = table[i];
        if (slot_fam(s.tag, lim.tgen) == 0 || !slot_live(s, lim, now0)) continue;
        const unsigned long long o = atomicAdd(&scal[1], 1ull);
        if (o < cap) buf[o] = s;
    }
}

__global__ __launch_bounds__(256) void k_evict_reinsert(Slot *table, TableState *tstate, Limits lim, TableIndex X,
                                                        const Slot *__restrict__ buf, uint64_t m) {
    IdTable idt{X.heads, X.k6, lim.table_mask, lim.seed, X.epoch, lim.test_flags, table, 0u, 0u,
                X.mir, X.mir_shift};
    idt.tgen = lim.tgen;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256u) {
        Slot s = buf[i];
        const uint32_t fam = slot_fam(s.tag, lim.tgen);
        const uint64_t h = id_start(idt, fam, s.key);
        bool fresh = false;
        const uint32_t id = id_resolve(idt, fam, s.key, h, X.heads[h], &fresh);
        if (id != kNoSlot) table[id] = s;   // (2x the entries in slots: never full)
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) tstate->count = m;
}

hipError_t launch_evict_scan(const Slot *table, const Limits &lim, const PacketIn &in, const uint64_t *ts,
                             uint32_t n, Slot *buf, uint64_t cap, unsigned long long *scal, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t g0 = std::max<uint32_t>(1, std::min<uint32_t>(2048, (n + 255) / 256));
    k_evict_min_ts<<<g0, 256, 0, st>>>(in, ts, n, scal);
    const uint32_t g1 = (uint32_t)std::min<uint64_t>(4096, (lim.table_mask + 256) / 256);
    k_evict_compact<<<g1, 256, 0, st>>>(table, lim, buf, cap, scal);
    return hipGetLastError();
}

hipError_t launch_evict_reinsert(Slot *table, TableState *tstate, const Limits &lim, const TableIndex &X,
                                 const Slot *buf, uint64_t m, hipStream_t st) {
    (void)hipGetLastError();
    const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, (m + 255) / 256));
    k_evict_reinsert<<<g, 256, 0, st>>>(table, tstate, lim, X, buf, m);
    return hipGetLastError();
}

hipError_t launch_map_op(Slot *table, TableState *tstate, const Limits &lim, const TableIndex &X, int op,
                         int map_id, const uint32_t key[4], const uint64_t val[3], uint64_t flags,
                         int32_t *d_result, uint64_t *d_val, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    k_map_op<<<1, 64, 0, st>>>(table, tstate, lim, X, op, map_id, key[0], key[1], key[2], key[3],
                               val[0], val[1], val[2], flags, d_result, d_val);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_map_dump(const Slot *table, Limits lim, int map_id,
                                                  uint8_t *keys, uint64_t *vals, uint64_t cap,
                                                  unsigned long long *count) {
    const uint32_t tag = map_tag(map_id);
    const uint32_t bit = map_bit(map_id);
    const uint32_t klen = tag == 2 ? 16u : 4u;
    const uint32_t vw = bit == SLOT_HAS_ST ? 3u : bit == SLOT_HAS_TB ? 2u : 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= lim.table_mask;
         i += (uint64_t)gridDim.x * 256u) {
        const Slot &s = table[i];
        if (slot_fam(s.tag, lim.tgen) != tag || !(s.flags & bit)) continue;
        const unsigned long long o = atomicAdd(count, 1ull);
        if (o >= cap) continue;
        const uint8_t *kb = reinterpret_cast<const uint8_t *>(s.key);
        for (uint32_t b = 0; b < klen; ++b) keys[o * klen + b] = kb[b];
        if (vw == 3) { vals[o * 3] = s.pps; vals[o * 3 + 1] = s.bps; vals[o * 3 + 2] = s.tt; }
        else if (vw == 2) { vals[o * 2] = s.aux; vals[o * 2 + 1] = s.tt; }
        else vals[o] = s.till;
    }
}

hipError_t launch_map_dump(const Slot *table, const Limits &lim, int map_id, uint8_t *d_keys,
                           uint64_t *d_vals, uint64_t cap, unsigned long long *d_count,
                           hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint64_t slots = lim.table_mask + 1;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, (slots + 255) / 256);
    k_map_dump<<<grid, 256, 0, st>>>(table, lim, map_id, d_keys, d_vals, cap, d_count);
    return hipGetLastError();
}

}  // namespace fsx
