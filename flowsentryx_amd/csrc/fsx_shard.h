// fsx_shard.h — record layout and owner function of the hash(src IP) sharded path
// (SURVEY.md §8 e; fsx_shard.hip). Shared by host (C ABI) and device code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fsx_internal.h"

namespace fsx {

// One IP packet on the wire between ranks (32 bytes).
struct alignas(16) ShardRecord {
    uint32_t key[4];      // raw source address words (IPv4: key[0] only)
    uint64_t ts;          // arrival time (ns)
    uint32_t len;         // frame length
    uint16_t dport;       // L4 destination port (host order; 0 when absent)
    uint8_t family;       // 4 or 6
    uint8_t pad;
};
static_assert(sizeof(ShardRecord) == 32, "32-byte exchange records");

// Compact record of an IPv4 packet: a sender whose slice has no IPv6 source and no frame
// of 64 KiB or more ships these instead (half the all-to-all volume of the common case).
struct alignas(16) ShardRecord16 {
    uint32_t key;         // raw IPv4 source address
    uint16_t len;         // frame length
    uint16_t dport;       // L4 destination port (host order; 0 when absent)
    uint64_t ts;          // arrival time (ns)
};
static_assert(sizeof(ShardRecord16) == 16, "16-byte compact records");

// Exchange record i of a record-mode batch (every record an IP packet): family tag 1 / 2,
// source key, frame length, timestamp and L4 destination port.
__device__ __forceinline__ uint32_t rec_read(const void *rec, uint32_t rec_bytes, uint32_t i, uint32_t k[4],
                                             uint32_t &L, uint64_t &T, uint32_t &dport) {
    if (rec_bytes == sizeof(ShardRecord16)) {
        const uint4 a = reinterpret_cast<const uint4 *>(rec)[i];
        k[0] = a.x; k[1] = k[2] = k[3] = 0;
        L = a.y & 0xFFFFu;
        dport = a.y >> 16;
        T = (uint64_t)a.z | ((uint64_t)a.w << 32);
        return 1;
    }
    const uint4 *p = reinterpret_cast<const uint4 *>(rec) + 2 * (size_t)i;
    const uint4 a = p[0], b = p[1];
    k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
    T = (uint64_t)b.x | ((uint64_t)b.y << 32);
    L = b.z;
    dport = b.w & 0xFFFFu;
    return ((b.w >> 16) & 0xFFu) == 6 ? 2u : 1u;
}

constexpr uint64_t kShardSeed = 0x5A4D0F5EED5ull;   // fixed: every rank must agree

// One blacklist entry of the replicated blocklist (all-gathered between ranks).
struct alignas(16) ShardBlock {
    uint32_t key[4];
    uint64_t till;        // ipv{4,6}_blacklist_map value
    uint32_t tag;         // 1 IPv4, 2 IPv6
    uint32_t pad;
};
static_assert(sizeof(ShardBlock) == 32, "32-byte blocklist entries");

// The replica: open addressing over next_pow2(2 m) ShardBlock slots (tag 0 = empty).
struct Replica {
    const ShardBlock *slots;
    uint64_t mask;
};

constexpr uint32_t kShardFilter = 1u;   // fsx_shard_pack_device flag (FSX_SHARD_FILTER_BLOCKLIST)
constexpr uint32_t kShardCompact = 2u;  // fsx_shard_pack_device flag (FSX_SHARD_COMPACT)
constexpr uint32_t kShardDropRecords = 4u;   // fsx_shard_pack_device flag (FSX_SHARD_DROP_RECORDS)
constexpr uint32_t kShardRegions = 8u;       // fsx_shard_pack_device flag (FSX_SHARD_REGIONS)
// counts[G + 1] of a pack whose placement look-back timed out (never expected): the host raises
constexpr uint32_t kShardPackErr = 1u;

// owner = floor(h * G / 2^32) of a 32-bit mix of (family tag, address).
__host__ __device__ inline uint32_t shard_owner_of(uint32_t tag, const uint32_t k[4], uint32_t G) {
    const uint64_t h = slot_hash(tag, k, kShardSeed);
    return (uint32_t)(((h >> 32) * (uint64_t)G) >> 32);
}

// owner_total: [G] per-owner records, [G] replica drops, [G + 1] (compact only) record bytes.
// own8 [n] and crec [n] (16-byte records in arrival order) are scratch.
hipError_t launch_shard_pack(const uint8_t *hdr, const uint32_t *len, const uint64_t *ts, uint32_t n,
                             uint32_t G, uint8_t *verdict, void *rec, uint32_t *send_idx,
                             uint64_t *owner_total, uint32_t *scratch, uint8_t *own8, void *crec,
                             const Replica *rep, bool compact, bool drop_rec, const uint32_t *use_dev,
                             bool regions, unsigned long long *status, uint32_t *ticket, hipStream_t st);
hipError_t launch_shard_clock(const uint64_t *ts, uint32_t n, uint64_t *out3, hipStream_t st);
hipError_t launch_blocklist_export(const Slot *table, uint64_t table_mask, uint32_t tgen, ShardBlock *out,
                                   uint64_t cap, unsigned long long *count, hipStream_t st);
hipError_t launch_replica_build(const ShardBlock *in, uint64_t m, ShardBlock *slots, uint64_t mask,
                                hipStream_t st);
hipError_t launch_replica_build_blocks(const void *blocks, uint32_t nb, uint64_t cap, ShardBlock *slots,
                                       uint64_t mask, hipStream_t st);
hipError_t launch_filter_plan(const uint64_t *clk, uint32_t G, uint32_t k, uint32_t *out, hipStream_t st);
hipError_t launch_shard_unpack(const void *rec, uint32_t rec_bytes, uint32_t m, uint8_t *hdr, uint32_t *len,
                               uint64_t *ts, hipStream_t st);
hipError_t launch_shard_scatter(const uint8_t *ret, const uint32_t *send_idx, uint32_t m, uint8_t *verdict,
                                hipStream_t st);
hipError_t launch_shard_scatter_regions(const uint8_t *ret, const uint32_t *send_idx, uint32_t m, uint64_t region,
                                        const uint64_t *counts, uint32_t G, uint8_t *verdict, hipStream_t st);

}  // namespace fsx
