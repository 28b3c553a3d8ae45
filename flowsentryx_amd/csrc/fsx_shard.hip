// fsx_shard.hip — hash(src IP) sharding of the verdict path over G GPUs (SURVEY.md §8 e).
//
// Every rank holds a contiguous slice of the arrival stream. All limiter state is per
// source IP, so a source's packets are routed to one owner rank, owner = H(family, key)
// (fsx_shard_owner), which runs the unchanged batch pipeline on them:
//   k_shard_parse     parse (src/parsing_helper.h:49-136 rules) + owner of every IP
//                     packet from coalesced, LDS-staged header loads; per-tile per-owner
//                     counts, local verdicts, and the 16-byte records in arrival order
//   k_shard_scan      per owner (one block each): exclusive scan over its tiles, its total
//   k_shard_pack16 /  stable partition by owner (16-byte records from k_shard_parse's
//   k_shard_pack      arrival-order copy / re-parsed into 32-byte records {src key, ts, len,
//                     L4 dst port, family} (16-byte {IPv4 key, len, dport, ts} when the
//                     caller allows it and the slice has no IPv6 source and no frame of
//                     64 KiB or more); local verdicts for the packets that never
//                     reach a limiter (short frames DROP, non-IP PASS: src/fsx_kern.c:
//                     123-131); for each send slot the local packet index
//   (RCCL all-to-all of the records, host side: flowsentryx_amd/shard.py)
//   k_shard_unpack    owner side: records -> 64-byte header records + len + ts whose parse
//                     and flow features equal the originals'
//   (owner: fsx_verdict_batch_device / fsx_process_batch_device; all-to-all back)
//   k_shard_scatter   verdicts back to local arrival positions
// Slices are contiguous and concatenated by rank on the owner, so every source's
// packets reach its owner in global arrival order and the result equals the 1-GPU run.
#include <hip/hip_runtime.h>

#include "fsx_dev_common.h"
#include "fsx_internal.h"
#include "fsx_shard.h"

namespace fsx {

constexpr uint32_t kShardTile = 4096;  // 256 threads x 16 packets
constexpr uint32_t kMaxShards = 64;

// Parse one 64-byte record (same rules as k_parse / the oracle): 0 DROP, 1 PASS
// (non-IP), 4 / 6 IP family with its key words and L4 destination port.
__device__ __forceinline__ uint32_t shard_parse(const uint8_t *rec, uint32_t L, uint32_t k[4],
                                                uint32_t &dport) {
    const uint32_t *d = reinterpret_cast<const uint32_t *>(rec);
    const uint32_t d3 = d[3];
    const uint32_t proto = ((d3 & 0xFFu) << 8) | ((d3 >> 8) & 0xFFu);
    k[0] = k[1] = k[2] = k[3] = 0;
    dport = 0;
    if (L < 14u) return 0;
    uint32_t off, l4;
    if (proto == 0x86DDu) {
        if (L < 54u) return 0;
        const uint32_t d5 = d[5], d6 = d[6], d7 = d[7], d8 = d[8], d9 = d[9];
        k[0] = (d5 >> 16) | (d6 << 16);
        k[1] = (d6 >> 16) | (d7 << 16);
        k[2] = (d7 >> 16) | (d8 << 16);
        k[3] = (d8 >> 16) | (d9 << 16);
        off = 54;
        l4 = (d5 & 0xFFu);   // byte 20: next header
    } else if (proto == 0x0800u) {
        if (L < 34u) return 0;
        k[0] = (d[6] >> 16) | (d[7] << 16);
        off = 14u + 4u * (((d3 >> 16) & 0xFFu) & 0x0Fu);   // byte 14: version/IHL
        l4 = (d[5] >> 24) & 0xFFu;                           // byte 23: protocol
    } else {
        return 1;
    }
    if ((l4 == 6 || l4 == 17) && off + 4 <= L && off + 4 <= 64)
        dport = ((uint32_t)rec[off + 2] << 8) | rec[off + 3];
    return proto == 0x86DDu ? 6u : 4u;
}

__device__ __forceinline__ uint32_t owner_dev(uint32_t fam, const uint32_t k[4], uint32_t G) {
    return shard_owner_of(fam == 6 ? 2u : 1u, k, G);
}

constexpr uint64_t kReplicaSeed = kShardSeed ^ 0xB10C;

// Blacklist entry of (tag, key) in the replica, or null.
__device__ __forceinline__ const ShardBlock *replica_find(const Replica &r, uint32_t tag, const uint32_t k[4]) {
    uint64_t i = slot_hash(tag, k, kReplicaSeed) & r.mask;
    for (uint64_t probes = 0; probes <= r.mask; ++probes) {
        const ShardBlock &b = r.slots[i];
        if (b.tag == 0) return nullptr;
        if (b.tag == tag && b.key[0] == k[0] && b.key[1] == k[1] && b.key[2] == k[2] && b.key[3] == k[3])
            return &b;
        i = (i + 1) & r.mask;
    }
    return nullptr;
}

// Parse + replica check: 0 DROP (parse), 1 PASS (non-IP), 2 DROP (blacklisted in the
// replica: till > 0 and now <= till, src/fsx_kern.c:189-215 — exact when the clock is
// monotone over the batches so far, which the host checks before asking for it),
// 4 / 6 an IP packet for its owner.
// (fam: the family 4 / 6 of an IP packet, also of a replica-dropped one; the replica by
// reference plus a flag: selecting between its address and null put the kernel argument
// in scratch)
__device__ __forceinline__ uint32_t shard_classify(const uint8_t *rec, uint32_t L, uint64_t now,
                                                   const Replica &rep, bool use_rep, uint32_t k[4],
                                                   uint32_t &dport, uint32_t &fam) {
    const uint32_t f = shard_parse(rec, L, k, dport);
    fam = f;
    if (f >= 4 && use_rep) {
        const ShardBlock *b = replica_find(rep, f == 6 ? 2u : 1u, k);
        if (b && b->till > 0 && !(now > b->till)) return 2;
    }
    return f;
}

// Per tile: per-owner IP-packet counts, owner-major [G][tiles].
__global__ void k_shard_fmt_init(unsigned long long *wide) { *wide = 0; }

// One pass over the headers (the k_count counts of k_shard_count, plus everything the
// compact pack needs): a tile of 4096 packets per block, wave w owns [w*1024, +1024) in
// 64-packet steps whose records are loaded with four coalesced 1 KiB wave loads and
// staged through LDS (17-dword pitch, as k_parse). Per packet: its verdict when it never
// reaches a limiter (and a PASS placeholder otherwise), its owner (0xFF: not sent) and,
// for an IPv4 packet, its 16-byte record in arrival order (compact requests).
__global__ __launch_bounds__(256) void k_shard_parse(const uint8_t *__restrict__ hdr,
                                                     const uint32_t *__restrict__ len,
                                                     const uint64_t *__restrict__ ts, uint32_t n,
                                                     uint32_t G, uint32_t *__restrict__ cnt,
                                                     uint32_t ntiles, Replica rep, int use_rep0,
                                                     const uint32_t *__restrict__ use_dev,
                                                     unsigned long long *wide,
                                                     uint8_t *__restrict__ verdict,
                                                     uint8_t *__restrict__ own8,
                                                     ShardRecord16 *__restrict__ crec,
                                                     uint64_t *__restrict__ owner_total, uint32_t drop_rec) {
    __shared__ uint32_t s_rec[4][64 * 17];
    __shared__ uint32_t sh[kMaxShards + 1];
    // (use_dev: the sub-batch's filter decision, made on the device: fsx_shard_filter_plan_device)
    const int use_rep = use_rep0 && (!use_dev || *use_dev);
    const uint32_t t = blockIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x <= kMaxShards) sh[threadIdx.x] = 0;
    __syncthreads();
    uint32_t *rec = s_rec[w];
    bool need_wide = false;
    uint32_t filtered = 0;
    for (uint32_t j = 0; j < kShardTile / 256u; ++j) {
        const uint32_t base = t * kShardTile + w * 1024u + j * 64u;
        const uint8_t *src = hdr + (size_t)base * 64;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t g = (uint32_t)k * 1024u + lane * 16u;
            uint4 x = make_uint4(0, 0, 0, 0);
            if (base + (g >> 6) < n) x = *reinterpret_cast<const uint4 *>(src + g);
            uint32_t *d = rec + (g >> 6) * 17u + ((g & 63u) >> 2);
            d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
        }
        wave_lds_order();
        const uint32_t i = base + lane;
        if (i < n) {
            // the staged record: 64 contiguous LDS bytes (shard_parse reads dwords and the
            // L4 port bytes)
            const uint32_t L = len[i];
            const uint64_t now = ts[i];
            uint32_t k[4], dp, fam;
            const uint32_t f = shard_classify(reinterpret_cast<const uint8_t *>(rec + lane * 17u), L, now,
                                              rep, use_rep != 0, k, dp, fam);
            uint8_t o = 0xFFu;
            // an IP packet for its owner, or (drop_rec) a replica-dropped one for group G
            if (f >= 4 || (f == 2 && drop_rec)) {
                o = (uint8_t)(f >= 4 ? owner_dev(f, k, G) : G);
                atomicAdd(&sh[o], 1u);
                need_wide |= fam == 6 || L > 0xFFFFu;
                if (crec && fam == 4) {
                    ShardRecord16 x;
                    x.key = k[0];
                    x.len = (uint16_t)L;
                    x.dport = (uint16_t)dp;
                    x.ts = now;
                    crec[i] = x;
                }
            }
            // parse DROP / non-IP PASS are never counted; a replica DROP is counted in
            // stats_map.dropped (src/fsx_kern.c:208-214) by the host
            verdict[i] = f == 1 || f >= 4 ? 2u : 1u;
            filtered += f == 2;
            own8[i] = o;
        }
        wave_lds_order();
    }
    if (wide && __ballot(need_wide) && lane == 0) atomicOr(wide, 1ull);
    filtered = wave_sum(filtered);
    if (lane == 0 && filtered)
        atomicAdd(reinterpret_cast<unsigned long long *>(&owner_total[G]), (unsigned long long)filtered);
    __syncthreads();
    if (threadIdx.x < G + drop_rec) cnt[(size_t)threadIdx.x * ntiles + t] = sh[threadIdx.x];
}

// Regions (FSX_SHARD_REGIONS) with compact requests: k_shard_parse's work, and every record
// placed at once — owner o's run starts at record o * n (group G, the replica drops, at G * n),
// in arrival order — so no arrival-order copy is written and read back (k_shard_pack16).
// A tile's offsets inside each region come from a decoupled look-back over the tiles before
// it: tiles are taken in ticket order, each publishes its per-owner count (flag 1) and then
// its inclusive prefix (flag 2) in one 64-bit word per (tile, owner) — the data is the flag.
// Each lane keeps its 16 packets' records in registers between the parse and the placement.
// The per-tile counts still go to `cnt`, for k_shard_scan and the 32-byte fallback
// (k_shard_pack re-places a wide slice).
constexpr uint32_t kPlaceSpin = 1u << 22;

__device__ __forceinline__ uint32_t place_lookback(unsigned long long *status, uint32_t t, uint32_t o,
                                                   uint32_t Gx, uint32_t tot, unsigned long long *wide) {
    unsigned long long *my = status + (size_t)t * Gx + o;
    if (t == 0) {
        __hip_atomic_store(my, (2ull << 62) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    __hip_atomic_store(my, (1ull << 62) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t excl = 0, spins = 0;
    for (int64_t tt = (int64_t)t - 1; tt >= 0;) {
        const unsigned long long w = __hip_atomic_load(status + (size_t)tt * Gx + o, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t flag = (uint32_t)(w >> 62);
        if (flag == 0) {   // not published yet (its block holds a lower ticket: it is running)
            if (++spins > kPlaceSpin) {   // (never expected; a bounded wait, not a hang)
                atomicOr(wide, 2ull);   // -> the pack's record size reads kShardPackErr
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += (uint32_t)w;
        if (flag == 2) break;
        --tt;
    }
    __hip_atomic_store(my, (2ull << 62) | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

__global__ __launch_bounds__(256) void k_shard_place16(const uint8_t *__restrict__ hdr,
                                                       const uint32_t *__restrict__ len,
                                                       const uint64_t *__restrict__ ts, uint32_t n,
                                                       uint32_t G, uint32_t *__restrict__ cnt,
                                                       uint32_t ntiles, Replica rep, int use_rep0,
                                                       const uint32_t *__restrict__ use_dev,
                                                       unsigned long long *wide,
                                                       uint8_t *__restrict__ verdict,
                                                       uint4 *__restrict__ out, uint32_t *__restrict__ send_idx,
                                                       uint64_t *__restrict__ owner_total, uint32_t drop_rec,
                                                       unsigned long long *status, uint32_t *ticket) {
    __shared__ uint32_t s_rec[4][64 * 17];
    __shared__ uint32_t s_wc[4][kMaxShards + 1];
    __shared__ uint32_t s_tile;
    const int use_rep = use_rep0 && (!use_dev || *use_dev);
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t Gx = G + drop_rec;
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    for (uint32_t o = threadIdx.x; o < 4 * (kMaxShards + 1); o += 256) (&s_wc[0][0])[o] = 0;
    __syncthreads();
    const uint32_t t = s_tile;
    uint32_t *rec = s_rec[w];
    bool need_wide = false;
    uint32_t filtered = 0;
    uint4 r[16];
    uint32_t ob[4] = {~0u, ~0u, ~0u, ~0u};   // owners, a byte per packet (0xFF: not sent)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t base = t * kShardTile + w * 1024u + (uint32_t)j * 64u;
        const uint8_t *src = hdr + (size_t)base * 64;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t g = (uint32_t)k * 1024u + lane * 16u;
            uint4 x = make_uint4(0, 0, 0, 0);
            if (base + (g >> 6) < n) x = *reinterpret_cast<const uint4 *>(src + g);
            uint32_t *d = rec + (g >> 6) * 17u + ((g & 63u) >> 2);
            d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
        }
        wave_lds_order();
        const uint32_t i = base + lane;
        r[j] = make_uint4(0, 0, 0, 0);
        if (i < n) {
            const uint32_t L = len[i];
            const uint64_t now = ts[i];
            uint32_t k[4], dp, fam;
            const uint32_t f = shard_classify(reinterpret_cast<const uint8_t *>(rec + lane * 17u), L, now,
                                              rep, use_rep != 0, k, dp, fam);
            if (f >= 4 || (f == 2 && drop_rec)) {
                const uint32_t o = f >= 4 ? owner_dev(f, k, G) : G;
                atomicAdd(&s_wc[w][o], 1u);
                need_wide |= fam == 6 || L > 0xFFFFu;
                ob[j >> 2] = (ob[j >> 2] & ~(0xFFu << (8 * (j & 3)))) | (o << (8 * (j & 3)));
                // (ShardRecord16 {key, len | dport << 16, ts}; a wide slice is re-placed)
                r[j] = make_uint4(k[0], (L & 0xFFFFu) | (dp << 16), (uint32_t)now, (uint32_t)(now >> 32));
            }
            verdict[i] = f == 1 || f >= 4 ? 2u : 1u;
            filtered += f == 2;
        }
        wave_lds_order();
    }
    if (wide && __ballot(need_wide) && lane == 0) atomicOr(wide, 1ull);
    filtered = wave_sum(filtered);
    if (lane == 0 && filtered)
        atomicAdd(reinterpret_cast<unsigned long long *>(&owner_total[G]), (unsigned long long)filtered);
    __syncthreads();
    if (threadIdx.x < Gx) {   // per owner: the tile's count, its offset in the region, per wave
        const uint32_t o = threadIdx.x;
        const uint32_t c0 = s_wc[0][o], c1 = s_wc[1][o], c2 = s_wc[2][o], c3 = s_wc[3][o];
        const uint32_t tot = c0 + c1 + c2 + c3;
        cnt[(size_t)o * ntiles + t] = tot;
        const uint32_t b = place_lookback(status, t, o, Gx, tot, wide);
        s_wc[0][o] = b;
        s_wc[1][o] = b + c0;
        s_wc[2][o] = b + c0 + c1;
        s_wc[3][o] = b + c0 + c1 + c2;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t i = t * kShardTile + w * 1024u + (uint32_t)j * 64u + lane;
        const uint32_t own = (ob[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        const bool ip = own != 0xFFu;
        uint64_t peers = __ballot(ip);
        for (uint32_t b = 0; (1u << b) < Gx; ++b) {
            const bool bit = (own >> b) & 1u;
            const uint64_t bal = __ballot(ip && bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        uint32_t base = 0;
        if (ip && below == 0) base = atomicAdd(&s_wc[w][own], (uint32_t)__popcll(peers));
        base = __shfl(base, ip ? __ffsll((unsigned long long)peers) - 1 : 0);
        if (ip) {
            const size_t slot = (size_t)own * n + base + below;
            out[slot] = r[j];
            send_idx[slot] = i;
        }
    }
}

// The first record slot of owner o: the totals of the owners before it.
__device__ __forceinline__ uint32_t owner_base(const uint64_t *owner_total, uint32_t o) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < o; ++k) b += (uint32_t)owner_total[k];
    return b;
}

// Compact pack (16-byte records, no header re-read): per tile, the owners and records
// k_shard_parse left in arrival order are placed stably at their owners' offsets.
__global__ __launch_bounds__(256) void k_shard_pack16(const uint8_t *__restrict__ own8,
                                                      const ShardRecord16 *__restrict__ crec,
                                                      uint32_t n, uint32_t G,
                                                      const uint32_t *__restrict__ offs, uint32_t ntiles,
                                                      ShardRecord16 *__restrict__ rec,
                                                      uint32_t *__restrict__ send_idx,
                                                      const uint64_t *__restrict__ owner_total, uint32_t Gx) {
    __shared__ uint32_t s_wc[4][kMaxShards + 1];
    if (owner_total[G + 1] != 16u) return;   // wide slice: k_shard_pack places 32-byte records
    const uint32_t t = blockIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
    for (uint32_t o = threadIdx.x; o < 4 * (kMaxShards + 1); o += 256) (&s_wc[0][0])[o] = 0;
    __syncthreads();
    uint8_t ob[16];
    // (loading the records here too, 16 per lane, made the kernel slower: 0.70 -> 0.96 ms)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t i = t * kShardTile + w * 1024u + (uint32_t)r * 64u + lane;
        ob[r] = i < n ? own8[i] : 0xFFu;
        if (ob[r] != 0xFFu) atomicAdd(&s_wc[w][ob[r]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < Gx) {   // exclusive over the waves, from the tile's owner base
        const uint32_t o = threadIdx.x;
        uint32_t b = offs[(size_t)o * ntiles + t] + owner_base(owner_total, o);
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = s_wc[k][o];
            s_wc[k][o] = b;
            b += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t i = t * kShardTile + w * 1024u + (uint32_t)r * 64u + lane;
        const uint32_t own = ob[r];
        const bool ip = own != 0xFFu;
        uint64_t peers = __ballot(ip);
        for (uint32_t b = 0; (1u << b) < Gx; ++b) {
            const bool bit = (own >> b) & 1u;
            const uint64_t bal = __ballot(ip && bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        uint32_t base = 0;
        if (ip && below == 0) base = atomicAdd(&s_wc[w][own], (uint32_t)__popcll(peers));
        base = __shfl(base, ip ? __ffsll((unsigned long long)peers) - 1 : 0);
        if (ip) {
            const uint32_t slot = base + below;
            rec[slot] = crec[i];
            send_idx[slot] = i;
        }
    }
}

// One block per owner: exclusive scan of its row of per-tile counts (in place, from 0) and
// its total; the packs add the owner's base (the totals of the owners before it,
// owner_base). Rows of 4096 tiles per round (4 per thread).
__global__ __launch_bounds__(1024) void k_shard_scan(uint32_t *__restrict__ cnt, uint64_t *__restrict__ owner_total,
                                                     uint32_t G, uint32_t ntiles, int compact) {
    __shared__ uint32_t s_w[16];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6, o = blockIdx.x;
    uint32_t *row = cnt + (size_t)o * ntiles;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 4096) {
        const uint32_t i = c0 + threadIdx.x * 4u;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = i + k < ntiles ? row[i + k] : 0u;
        const uint32_t sum = x[0] + x[1] + x[2] + x[3];
        const uint32_t incl = wave_incl_sum(sum);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t off = carry, tot = 0;
        for (uint32_t k = 0; k < 16; ++k) {
            off += k < w ? s_w[k] : 0u;
            tot += s_w[k];
        }
        off += incl - sum;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < ntiles) { row[i + k] = off; off += x[k]; }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        owner_total[o] = carry;
        // compact requests: the wide flag of k_shard_parse becomes the record size
        // (bit 1: a look-back of k_shard_place16 timed out — the host raises on kShardPackErr)
        if (o == 0 && compact) {
            const uint64_t wf = owner_total[G + 1];
            owner_total[G + 1] = (wf & 2u) ? kShardPackErr : wf ? 32u : 16u;
        }
    }
}

// Per tile: stable (arrival order) placement of every IP packet at its owner's offset.
__global__ __launch_bounds__(256) void k_shard_pack(const uint8_t *__restrict__ hdr,
                                                    const uint32_t *__restrict__ len,
                                                    const uint64_t *__restrict__ ts, uint32_t n,
                                                    uint32_t G, const uint32_t *__restrict__ offs,
                                                    uint32_t ntiles, void *__restrict__ rec,
                                                    uint32_t *__restrict__ send_idx,
                                                    uint8_t *__restrict__ verdict, Replica rep,
                                                    int use_rep0, const uint32_t *__restrict__ use_dev,
                                                    uint64_t *__restrict__ owner_total,
                                                    int compact, uint32_t drop_rec, int regions) {
    const int use_rep = use_rep0 && (!use_dev || *use_dev);
    // (k_shard_pack16 / k_shard_place16 placed them; or a failed placement: nothing more)
    if (compact && (owner_total[G + 1] == 16u || owner_total[G + 1] == kShardPackErr)) return;
    __shared__ uint32_t s_base[kMaxShards + 1];
    __shared__ uint32_t s_wc[4][kMaxShards + 1];
    const uint32_t t = blockIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t Gx = G + drop_rec;   // (group G: the replica-dropped packets)
    // (regions: owner o's run starts at record o * n; else after the owners before it)
    if (threadIdx.x < Gx)
        s_base[threadIdx.x] = offs[(size_t)threadIdx.x * ntiles + t] + (regions ? 0u : owner_base(owner_total, threadIdx.x));
    // wave w owns packets [t*4096 + w*1024, +1024) in arrival order: count per owner
    // first (so a wave places after the waves before it), then place in order
    uint32_t of[16];   // owner << 4 | class (0 DROP, 1 PASS, 4/6 IP, 8 | 4/6 replica-dropped IP, 15 none)
    for (uint32_t o = threadIdx.x; o < 4 * (kMaxShards + 1); o += 256) (&s_wc[0][0])[o] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t i = t * kShardTile + w * 1024u + (uint32_t)r * 64u + lane;
        of[r] = 15u;
        if (i < n) {
            uint32_t k[4], dp, fam;
            const uint32_t f = shard_classify(hdr + (size_t)i * 64, len[i], ts[i], rep, use_rep != 0, k, dp,
                                              fam);
            if (f >= 4 || (f == 2 && drop_rec)) {
                const uint32_t o = f >= 4 ? owner_dev(f, k, G) : G;
                of[r] = (o << 4) | (f >= 4 ? f : 8u | fam);
                atomicAdd(&s_wc[w][o], 1u);
                if (f == 2) verdict[i] = 1u;
            } else {
                of[r] = f;
                // parse DROP / non-IP PASS are never counted; a replica DROP is counted
                // in stats_map.dropped (src/fsx_kern.c:208-214) by the host
                verdict[i] = f == 1 ? 2u : 1u;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < Gx) {   // exclusive over the waves, from the tile's owner base
        const uint32_t o = threadIdx.x;
        uint32_t b = s_base[o];
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = s_wc[k][o];
            s_wc[k][o] = b;
            b += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t i = t * kShardTile + w * 1024u + (uint32_t)r * 64u + lane;
        const uint32_t f = of[r] & 7u, own = of[r] >> 4;
        const bool ip = (of[r] & 15u) != 15u && (f == 4u || f == 6u);
        const bool dropped = (of[r] & 8u) != 0 && ip;
        // rank among this step's lanes with the same owner (ballots over the owner bits)
        uint64_t peers = __ballot(ip);
        for (uint32_t b = 0; (1u << b) < Gx; ++b) {
            const bool bit = (own >> b) & 1u;
            const uint64_t bal = __ballot(ip && bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        uint32_t base = 0;
        if (ip && below == 0) base = atomicAdd(&s_wc[w][own], (uint32_t)__popcll(peers));
        base = __shfl(base, ip ? __ffsll((unsigned long long)peers) - 1 : 0);
        if (ip) {
            uint32_t k[4], dp;
            shard_parse(hdr + (size_t)i * 64, len[i], k, dp);
            const size_t slot = (regions ? (size_t)own * n : 0) + base + below;
            ShardRecord x;
            x.key[0] = k[0]; x.key[1] = k[1]; x.key[2] = k[2]; x.key[3] = k[3];
            x.ts = ts[i];
            x.len = len[i];
            x.dport = (uint16_t)dp;
            x.family = (uint8_t)f;
            x.pad = 0;
            reinterpret_cast<ShardRecord *>(rec)[slot] = x;
            send_idx[slot] = i;
            if (!dropped) verdict[i] = 2u;   // placeholder until the owner's verdict returns
        }
    }
}

// Owner side: 32-byte records -> header records that parse to the same key, family and
// dst port, frame length and timestamp.
__device__ __forceinline__ ShardRecord widen(const ShardRecord &x) { return x; }
__device__ __forceinline__ ShardRecord widen(const ShardRecord16 &c) {
    ShardRecord x;
    x.key[0] = c.key; x.key[1] = x.key[2] = x.key[3] = 0;
    x.ts = c.ts;
    x.len = c.len;
    x.dport = c.dport;
    x.family = 4;
    x.pad = 0;
    return x;
}

template <class R>
__global__ __launch_bounds__(256) void k_shard_unpack(const R *__restrict__ rec, uint32_t m,
                                                      uint8_t *__restrict__ hdr,
                                                      uint32_t *__restrict__ len,
                                                      uint64_t *__restrict__ ts) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < m; i += gridDim.x * 256u) {
        const ShardRecord x = widen(rec[i]);
        uint32_t d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = 0;
        const uint32_t dp = ((x.dport & 0xFFu) << 8) | (x.dport >> 8);   // network order
        if (x.family == 6) {
            d[3] = 0xDD86u;                                   // bytes 12-13: 0x86DD
            d[5] = 17u | (x.key[0] << 16);                    // byte 20 next header = UDP
            d[6] = (x.key[0] >> 16) | (x.key[1] << 16);
            d[7] = (x.key[1] >> 16) | (x.key[2] << 16);
            d[8] = (x.key[2] >> 16) | (x.key[3] << 16);
            d[9] = x.key[3] >> 16;
            d[14] = dp;                                       // bytes 56-57 (54 + 2)
        } else {
            d[3] = 0x0008u | (0x45u << 16);                   // 0x0800, version 4 / IHL 5
            d[5] = 17u << 24;                                 // byte 23 protocol = UDP
            d[6] = x.key[0] << 16;                            // bytes 26-27
            d[7] = x.key[0] >> 16;                            // bytes 28-29
            d[9] = dp;                                        // bytes 36-37 (34 + 2)
        }
        uint4 *o = reinterpret_cast<uint4 *>(hdr + (size_t)i * 64);
        o[0] = make_uint4(d[0], d[1], d[2], d[3]);
        o[1] = make_uint4(d[4], d[5], d[6], d[7]);
        o[2] = make_uint4(d[8], d[9], d[10], d[11]);
        o[3] = make_uint4(d[12], d[13], d[14], d[15]);
        len[i] = x.len;
        ts[i] = x.ts;
    }
}

__global__ __launch_bounds__(256) void k_shard_scatter(const uint8_t *__restrict__ ret,
                                                       const uint32_t *__restrict__ send_idx, uint32_t m,
                                                       uint8_t *__restrict__ verdict) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < m; i += gridDim.x * 256u)
        verdict[send_idx[i]] = ret[i];
}

// Regions: returned verdict i (owner by owner, counts[o] each) -> its owner's region entry.
__global__ __launch_bounds__(256) void k_shard_scatter_regions(const uint8_t *__restrict__ ret,
                                                               const uint32_t *__restrict__ send_idx, uint32_t m,
                                                               uint64_t region, const uint64_t *__restrict__ counts,
                                                               uint32_t G, uint8_t *__restrict__ verdict) {
    __shared__ uint32_t s_pre[kMaxShards + 1];
    if (threadIdx.x == 0) {
        uint32_t a = 0;
        for (uint32_t o = 0; o < G; ++o) { s_pre[o] = a; a += (uint32_t)counts[o]; }
        s_pre[G] = a;
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < m && i < s_pre[G]; i += gridDim.x * 256u) {
        uint32_t lo = 0, hi = G;   // the owner o with s_pre[o] <= i < s_pre[o + 1]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] <= i) lo = mid; else hi = mid;
        }
        verdict[send_idx[(size_t)lo * region + (i - s_pre[lo])]] = ret[i];
    }
}

__global__ void k_shard_empty(uint64_t *owner_total, uint32_t G, int compact) {
    for (uint32_t o = 0; o <= G; ++o) owner_total[o] = 0;
    if (compact) owner_total[G + 1] = 16u;
}

hipError_t launch_shard_pack(const uint8_t *hdr, const uint32_t *len, const uint64_t *ts, uint32_t n,
                             uint32_t G, uint8_t *verdict, void *rec, uint32_t *send_idx,
                             uint64_t *owner_total, uint32_t *scratch, uint8_t *own8, void *crec,
                             const Replica *rep, bool compact, bool drop_rec, const uint32_t *use_dev,
                             bool regions, unsigned long long *status, uint32_t *ticket, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    k_shard_empty<<<1, 1, 0, st>>>(owner_total, G, compact);   // also the wide flag / filtered
    if (n == 0) return hipGetLastError();
    const uint32_t ntiles = (n + kShardTile - 1) / kShardTile;
    const Replica r = rep ? *rep : Replica{nullptr, 0};
    const int use = rep != nullptr && rep->slots != nullptr;
    unsigned long long *wide = compact ? reinterpret_cast<unsigned long long *>(owner_total + G + 1) : nullptr;
    if (wide) k_shard_fmt_init<<<1, 1, 0, st>>>(wide);
    ShardRecord16 *cr = compact ? reinterpret_cast<ShardRecord16 *>(crec) : nullptr;
    const uint32_t dr = drop_rec && use ? 1u : 0u;   // (records of the replica drops: group G)
    const bool place = compact && regions;   // (k_shard_place16: no arrival-order copy)
    if (place) {
        hipError_t e = hipMemsetAsync(status, 0, (size_t)ntiles * (G + dr) * 8, st);
        if (e == hipSuccess) e = hipMemsetAsync(ticket, 0, 4, st);
        if (e != hipSuccess) return e;
        k_shard_place16<<<ntiles, 256, 0, st>>>(hdr, len, ts, n, G, scratch, ntiles, r, use, use_dev, wide, verdict,
                                                reinterpret_cast<uint4 *>(rec), send_idx, owner_total, dr, status,
                                                ticket);
    } else {
        k_shard_parse<<<ntiles, 256, 0, st>>>(hdr, len, ts, n, G, scratch, ntiles, r, use, use_dev, wide, verdict,
                                              own8, cr, owner_total, dr);
    }
    k_shard_scan<<<G + dr, 1024, 0, st>>>(scratch, owner_total, G, ntiles, compact);
    if (compact && !place)
        k_shard_pack16<<<ntiles, 256, 0, st>>>(own8, cr, n, G, scratch, ntiles,
                                               reinterpret_cast<ShardRecord16 *>(rec), send_idx, owner_total,
                                               G + dr);
    k_shard_pack<<<ntiles, 256, 0, st>>>(hdr, len, ts, n, G, scratch, ntiles, rec, send_idx, verdict, r,
                                         use, use_dev, owner_total, compact, dr, regions ? 1 : 0);
    return hipGetLastError();
}

// Clock facts of a local batch: {min ts, max ts, any decrease in arrival order}.
__global__ __launch_bounds__(256) void k_shard_clock(const uint64_t *__restrict__ ts, uint32_t n,
                                                     unsigned long long *out3) {
    uint64_t mn = ~0ull, mx = 0;
    uint32_t dec = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint64_t t = ts[i];
        mn = t < mn ? t : mn;
        mx = t > mx ? t : mx;
        if (i > 0 && ts[i - 1] > t) dec = 1;
    }
    mx = wave_max(mx);
    mn = ~wave_max(~mn);
    dec = __ballot(dec != 0) ? 1u : 0u;
    if (lane_id() == 0) {
        atomicMin(&out3[0], (unsigned long long)mn);
        atomicMax(&out3[1], (unsigned long long)mx);
        if (dec) atomicOr(&out3[2], 1ull);
    }
}

hipError_t launch_shard_clock(const uint64_t *ts, uint32_t n, uint64_t *out3, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint64_t init[3] = {~0ull, 0ull, 0ull};
    hipError_t e = hipMemcpyAsync(out3, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e != hipSuccess || n == 0) return e;
    const uint32_t grid = std::min<uint32_t>(2048, (n + 255) / 256);
    k_shard_clock<<<grid, 256, 0, st>>>(ts, n, reinterpret_cast<unsigned long long *>(out3));
    return hipGetLastError();
}

// Every live blacklist entry (till > 0) of this rank's table.
__global__ __launch_bounds__(256) void k_blocklist_export(const Slot *table, uint64_t mask, uint32_t tgen,
                                                          ShardBlock *out, uint64_t cap, unsigned long long *count) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= mask; i += (uint64_t)gridDim.x * 256u) {
        const Slot &s = table[i];
        const uint32_t fam = slot_fam(s.tag, tgen);
        if (fam == 0 || !(s.flags & SLOT_HAS_BL) || s.till == 0) continue;
        const unsigned long long o = atomicAdd(count, 1ull);
        if (o >= cap) continue;
        ShardBlock b;
        b.key[0] = s.key[0]; b.key[1] = s.key[1]; b.key[2] = s.key[2]; b.key[3] = s.key[3];
        b.till = s.till;
        b.tag = fam;
        b.pad = 0;
        out[o] = b;
    }
}

hipError_t launch_blocklist_export(const Slot *table, uint64_t table_mask, uint32_t tgen, ShardBlock *out,
                                   uint64_t cap, unsigned long long *count, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    hipError_t e = hipMemsetAsync(count, 0, 8, st);
    if (e != hipSuccess) return e;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, (table_mask + 256) / 256);
    k_blocklist_export<<<grid, 256, 0, st>>>(table, table_mask, tgen, out, cap, count);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_replica_clear(ShardBlock *slots, uint64_t mask) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= mask; i += (uint64_t)gridDim.x * 256u)
        slots[i].tag = 0;
}

// Insert m distinct entries (every source has one owner) into cleared replica slots.
__global__ __launch_bounds__(256) void k_replica_build(const ShardBlock *__restrict__ in, uint64_t m,
                                                       ShardBlock *slots, uint64_t mask) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256u) {
        const ShardBlock b = in[j];
        uint64_t i = slot_hash(b.tag, b.key, kReplicaSeed) & mask;
        for (uint64_t probes = 0; probes <= mask; ++probes) {
            if (atomicCAS(&slots[i].tag, 0u, b.tag) == 0u) {
                slots[i].key[0] = b.key[0]; slots[i].key[1] = b.key[1];
                slots[i].key[2] = b.key[2]; slots[i].key[3] = b.key[3];
                slots[i].till = b.till;
                break;
            }
            i = (i + 1) & mask;
        }
    }
}

hipError_t launch_replica_build(const ShardBlock *in, uint64_t m, ShardBlock *slots, uint64_t mask,
                                hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t cgrid = (uint32_t)std::min<uint64_t>(1024, (mask + 256) / 256);
    k_replica_clear<<<cgrid, 256, 0, st>>>(slots, mask);
    if (m == 0) return hipGetLastError();
    const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (m + 255) / 256);
    k_replica_build<<<grid, 256, 0, st>>>(in, m, slots, mask);
    return hipGetLastError();
}

// The replica from n_blocks all-gathered fixed-capacity blocks (fsx_blocklist_replica_blocks_device):
// block b = a 32-byte header (its entry count, int64) then cap entries; min(count, cap) used.
__global__ __launch_bounds__(256) void k_replica_build_blocks(const uint8_t *__restrict__ blocks, uint32_t nb,
                                                              uint64_t cap, ShardBlock *slots, uint64_t mask) {
    const uint64_t per = (cap + 1) * sizeof(ShardBlock);
    for (uint32_t b = 0; b < nb; ++b) {
        const uint8_t *blk = blocks + (size_t)b * per;
        const uint64_t cnt = *reinterpret_cast<const unsigned long long *>(blk);
        const uint64_t m = cnt < cap ? cnt : cap;
        const ShardBlock *in = reinterpret_cast<const ShardBlock *>(blk + sizeof(ShardBlock));
        for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256u) {
            const ShardBlock e = in[j];
            uint64_t i = slot_hash(e.tag, e.key, kReplicaSeed) & mask;
            for (uint64_t probes = 0; probes <= mask; ++probes) {
                if (atomicCAS(&slots[i].tag, 0u, e.tag) == 0u) {
                    slots[i].key[0] = e.key[0]; slots[i].key[1] = e.key[1];
                    slots[i].key[2] = e.key[2]; slots[i].key[3] = e.key[3];
                    slots[i].till = e.till;
                    break;
                }
                i = (i + 1) & mask;
            }
        }
    }
}

hipError_t launch_replica_build_blocks(const void *blocks, uint32_t nb, uint64_t cap, ShardBlock *slots,
                                       uint64_t mask, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    const uint32_t cgrid = (uint32_t)std::min<uint64_t>(1024, (mask + 256) / 256);
    k_replica_clear<<<cgrid, 256, 0, st>>>(slots, mask);
    if (nb == 0 || cap == 0) return hipGetLastError();
    const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (cap + 255) / 256);
    k_replica_build_blocks<<<grid, 256, 0, st>>>(static_cast<const uint8_t *>(blocks), nb, cap, slots, mask);
    return hipGetLastError();
}

// The replica filter's per-sub-batch decision from every rank's piece clocks
// {min, max, decreases} ([G][k][3], all-gathered; an empty piece is {~0, 0, 0}): sub-batch j
// filters iff no piece of it goes back, its pieces follow each other in rank order, and no
// earlier sub-batch holds a packet later than its first — the global clock does not go back
// up to it, so no earlier packet can have deleted a replica entry at a later time.
__global__ void k_filter_plan(const unsigned long long *__restrict__ clk, uint32_t G, uint32_t k,
                              uint32_t *__restrict__ out) {
    if (threadIdx.x || blockIdx.x) return;
    bool any_prev = false;
    uint64_t prev_hi = 0;
    for (uint32_t j = 0; j < k; ++j) {
        bool ok = true, seen = false, have = false;
        uint64_t last = 0, lo = 0, hi = 0;
        for (uint32_t r = 0; r < G; ++r) {
            const unsigned long long *c = clk + 3ull * ((uint64_t)r * k + j);
            const uint64_t mn = c[0], mx = c[1];
            if (c[2]) ok = false;
            if (mx == 0 && mn == ~0ull) continue;   // empty piece
            if (seen && mn < last) ok = false;
            seen = true;
            last = mx;
            lo = have ? (mn < lo ? mn : lo) : mn;
            hi = have ? (mx > hi ? mx : hi) : mx;
            have = true;
        }
        if (ok && any_prev && have && lo < prev_hi) ok = false;
        out[j] = ok ? 1u : 0u;
        if (have) {
            prev_hi = any_prev ? (hi > prev_hi ? hi : prev_hi) : hi;
            any_prev = true;
        }
    }
}

hipError_t launch_filter_plan(const uint64_t *clk, uint32_t G, uint32_t k, uint32_t *out, hipStream_t st) {
    (void)hipGetLastError();
    k_filter_plan<<<1, 1, 0, st>>>(reinterpret_cast<const unsigned long long *>(clk), G, k, out);
    return hipGetLastError();
}

hipError_t launch_shard_unpack(const void *rec, uint32_t rec_bytes, uint32_t m, uint8_t *hdr, uint32_t *len,
                               uint64_t *ts, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    if (m == 0) return hipSuccess;
    const uint32_t grid = std::min<uint32_t>(4096, (m + 255) / 256);
    if (rec_bytes == 16)
        k_shard_unpack<<<grid, 256, 0, st>>>(reinterpret_cast<const ShardRecord16 *>(rec), m, hdr, len, ts);
    else
        k_shard_unpack<<<grid, 256, 0, st>>>(reinterpret_cast<const ShardRecord *>(rec), m, hdr, len, ts);
    return hipGetLastError();
}

hipError_t launch_shard_scatter_regions(const uint8_t *ret, const uint32_t *send_idx, uint32_t m, uint64_t region,
                                        const uint64_t *counts, uint32_t G, uint8_t *verdict, hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    if (m == 0) return hipSuccess;
    const uint32_t grid = std::min<uint32_t>(4096, (m + 255) / 256);
    k_shard_scatter_regions<<<grid, 256, 0, st>>>(ret, send_idx, m, region, counts, G, verdict);
    return hipGetLastError();
}

hipError_t launch_shard_scatter(const uint8_t *ret, const uint32_t *send_idx, uint32_t m, uint8_t *verdict,
                                hipStream_t st) {
    (void)hipGetLastError();   // a stale error of another caller is not ours
    if (m == 0) return hipSuccess;
    const uint32_t grid = std::min<uint32_t>(4096, (m + 255) / 256);
    k_shard_scatter<<<grid, 256, 0, st>>>(ret, send_idx, m, verdict);
    return hipGetLastError();
}

}  // namespace fsx
