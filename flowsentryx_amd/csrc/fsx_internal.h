// fsx_internal.h — device data layout and kernel launchers of libfsx_hip.so.
//
// HBM layout:
//   * the five reference maps live in ONE device-resident open-addressing table of
//     64-byte slots (one cache line per source IP: tag, key, ip_stats, blacklist),
//     capacity = next_pow2(2 * max_entries) — src/fsx_kern.c:56-94;
//   * per-batch scratch sized for cfg.max_batch packets: the packed sort words
//     (two ping-pong arrays of u64), a u8 mark per sorted position, the ordered
//     segment starts and their table slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "fsx_q8.h"

namespace fsx {

constexpr uint64_t kSentinel = ~0ull;     // "not an IP packet" in the packed array
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// Radix sort geometry: 8-bit digits, 256-thread blocks, 16 items/thread tiles.
constexpr int kSortThreads = 256;
#ifndef FSX_SORT_ITEMS
#define FSX_SORT_ITEMS 16   // keys per thread of a sort tile (A/B: scripts/build_variant.sh)
#endif
constexpr int kSortItems = FSX_SORT_ITEMS;
constexpr int kSortTile = kSortThreads * kSortItems;  // 4096
constexpr int kSortMaxBlocks = 2048;
constexpr int kTile = 4096;                            // fill / compaction tile
constexpr uint32_t kVChunkBits = 14;
constexpr uint32_t kVChunk = 1u << kVChunkBits;         // verdict bytes per k_verdict_apply block
constexpr uint32_t kMaxTileChunks = 4096;               // k_fill_scatter's per-tile chunk counters

enum : uint32_t {
    ERR_TABLE_FULL = 1u,
    ERR_PROBE = 2u,
    ERR_FIXUP = 4u,
    ERR_SORT_HANG = 8u,
    ERR_HIST_FULL = 16u,
    ERR_CANCELED = 32u,   // pipelined batches: the batch before this one failed
    ERR_HEAVY_VIEW = 64u, // a heavy source's tile-count row / tags inconsistent (fsx_heavy_view.h)
};

enum : uint32_t { SLOT_HAS_ST = 1u, SLOT_HAS_BL = 2u, SLOT_HAS_TB = 4u };
// Slot.flags bits 16..31: the batch generation that inserted the slot (0 once a batch
// has walked it, or for map-op inserts); a failed batch's inserts are rolled back.
constexpr uint32_t kBornShift = 16;
constexpr uint32_t kFlagBits = (1u << kBornShift) - 1u;

// Persistent source index: one 8-byte head per table slot {epoch 16 | state 8 | tag 8 |
// key word 0} plus IPv6 key words 1..3, mirroring Slot.tag/key. k_parse probes the
// dense heads (not the 64-byte slots) and inserts new sources, so a source's sort id IS
// its table slot. The epoch changes on fsx_reset and after a rolled-back batch, which
// empties every head at once (no clearing; stale cached lines read as empty).
struct TableIndex {
    unsigned long long *heads;
    uint32_t *k6;          // [slots][4]: IPv6 key words 1..3
    uint32_t epoch;
    void *mir = nullptr;   // IPv4 mirror of the heads (mir_entry; null: off), cleared every epoch
    uint32_t mir_shift = 0;   // log2(slots)
};

// One source IP (either family). tag: 0 empty, 1 IPv4, 2 IPv6.
struct alignas(64) Slot {
    uint32_t tag;
    uint32_t flags;       // SLOT_HAS_*
    uint32_t key[4];      // raw saddr bytes (IPv4: key[0] only)
    uint64_t pps;         // struct ip_stats, src/fsx_struct.h:17-22
    uint64_t bps;
    uint64_t tt;          // track_time
    uint64_t till;        // ipv{4,6}_blacklist_map value
    uint64_t aux;         // token bucket: nano-tokens (tt = last refill time, SLOT_HAS_TB)
};
static_assert(sizeof(Slot) == 64, "slot is one cache line");

// Device-side per-batch scalars (zeroed before each batch).
struct BatchState {
    uint32_t n_valid;     // IP packets (entries that go through the sort)
    uint32_t any_v6;
    uint32_t nonmono;     // a timestamp decreased in arrival order
    uint32_t nseg;        // distinct source IPs in the batch
    uint32_t n_new;
    uint32_t err;
    uint32_t max_len;
    uint32_t n_rule;      // IP packets dropped by a prefix rule (not in n_valid)
    uint32_t n_long;      // segments longer than the short-segment bound (wave walker)
    uint32_t n_span;      // sources crossing flow tiles (k_flow_combine)
    uint64_t max_ts;
    uint64_t allowed;     // this batch
    uint64_t dropped;
    uint64_t inv_min_ts;  // ~(smallest timestamp): max-reduced from 0
    uint32_t pay_ok;      // sorted payload words valid (see kPayLenBits)
    uint32_t n_light;     // entries of non-heavy sources: sort passes >= 1 cover [0, n_light)
    uint32_t nseg_light;  // heavy verdict lists: segments ids [0, nseg_light) are light, the
                          // heavy sources' segments follow (k_heads_heavy)
    uint32_t light_b;     // heavy-source sort: heavy source h is pass-0 bucket light_b + h
                          // (k_hist_prep; 256 without the heavy sort)
    // unsorted heavy sources (DESIGN.md §3 "Heavy sources outside the sort"): k_pass0h's
    // clock facts and k_hmode's verdict — 1: the heavy walker and flow rows work on the
    // arrival order (select / rank over the tagged verdict bytes); 0: k_heavy_gather
    // builds the heavy runs and the run-based kernels take over
    uint32_t hfast;
    uint32_t span_big;    // some sort tile spans >= 2^32 ns (u64 gap-square sums could wrap)
    uint32_t n_admit;     // FSX_FLAG_OVERFLOW_ADMIT: sources admitted / transient this batch
    uint32_t n_trans;
    uint32_t n_ofix;      // home-ordered batches: key-hash runs longer than 8 (k_ord_long)
    uint32_t n_orun;      // ... key-hash runs of two or more packets (k_ord_scan)
    uint32_t ord;         // home-ordered inserts (Limits::ord) ran for this batch
    uint32_t ord_walked;  // ... and walked every segment (k_ord_claim): the walkers return at once
};

// Sorted payload word carried through the onesweep passes next to each sort word:
// (ts - min_ts) << 24 | len. Valid when every ts is within 2^40 ns (~18 min) of the
// batch minimum and every len < 2^24; otherwise consumers gather ts/len by index.
constexpr uint32_t kPayLenBits = 24;
constexpr uint32_t kSegClasses = 16;  // walker length classes (last: wave-walked segments)
constexpr uint32_t kSortCtlWords = 1028 + 2 * kSegClasses;
constexpr uint32_t kSegClassWords = kSegClasses * 1024;   // Scratch::seg_cls (kSegBlocks per class)
constexpr uint64_t kPayTsRange = 1ull << (64 - kPayLenBits);

// Persistent device scalars.
struct TableState {
    uint64_t count;       // occupied slots
    uint64_t stats[2];    // stats_map {allowed, dropped}, src/fsx_struct.h:11-15
    // sliding window: carried logs and the clock facts pruning needs
    uint64_t hist_total;  // entries in the current history buffer
    uint64_t last_max_ts; // largest timestamp of all batches so far
    uint32_t ever_nonmono;  // some batch (or batch boundary) went back in time
    uint32_t hist_cur;    // which of the two history buffers is current
    uint32_t max_len_seen;  // largest frame length of all batches so far
    // a split sliding-window batch failed in its tail (k_sw_tail_check): every later split
    // batch cancels itself there too, until the host has rolled them back and cleared it
    uint32_t tail_fail;
    // (kept by fsx_reset: diagnostics since fsx_open) fixed-window batches whose heavy
    // sources took the unsorted path / the run path (k_hmode_state)
    uint32_t n_hfast, n_hrun;
};
constexpr size_t kTableStateResetBytes = offsetof(TableState, n_hfast);

// Sliding-window logs carried between batches: per source, the log of counted packets
// still inside the window (<= pps_threshold entries, oldest first), packed by source in
// one of two ping-pong buffers. Slot.aux = offset << kHistCntBits | count.
constexpr uint32_t kHistCntBits = 24;
// The sliding window's heavy sources by rank (k_walk_sw_heavy_sel) stage every heavy source's
// final log (<= pps_threshold entries) past the history's capacity: pps_threshold <= this,
// else the run path.
constexpr uint32_t kSwHeavyMaxP = 4096;
constexpr uint64_t kAuxWalked = 1ull << 63;   // Slot.aux during a batch: walked segment id

struct HistBufs {
    uint64_t *t[2];
    uint32_t *l[2];
    uint64_t cap;
    uint32_t *tile_cnt;   // per 4096 table slots: surviving log entries
    uint64_t *tile_off;   // their exclusive scan
    uint64_t *total;      // entries after the rebuild
};

// Per walked source: the final log as a virtual range [lo, hi) over its old history
// (hoff, m) followed by its sorted positions j0, j0+1, ...
struct SwSeg {
    uint64_t hoff;
    uint32_t m, j0, lo, hi;
    uint32_t pad_[2];
};

struct Limits {           // the rate-limiter constants, src/fsx_kern.c:245,308-310
    uint64_t pps, bps, window, block;
    uint64_t tb_rate, tb_cap;  // token bucket, nano-tokens
    uint64_t max_entries;
    uint64_t hist_cap;    // sliding window: history entries per buffer
    uint64_t table_mask;
    uint64_t seed;
    uint32_t salt32;
    int32_t limiter;
    uint32_t test_flags;  // fsx_config.flags (FSX_FLAG_TEST_* test hooks, policies)
    // FSX_FLAG_OVERFLOW_ADMIT: the batch's sources get ids in the per-batch id table (this
    // mask), their table slots come from the admission kernels
    uint64_t admit_mask;
    // home-ordered inserts for this batch (DESIGN.md §3 "Home-ordered inserts"; set by the
    // host per batch: a flood of new sources): k_parse writes a key-hash sort word, the
    // segment heads find / insert their slots in home-slot order after the sort
    uint32_t ord;
    // table generation (16 bits): a slot's tag word is its family | tgen << 16, and a line of
    // another generation reads as empty — fsx_reset moves to the next generation instead of
    // clearing the table (DESIGN.md §3 "Clear-free reset")
    uint32_t tgen;
    // host hint (set per batch): the last batch the host checked had >= 90 % of its IP packets
    // in light sources (an all-light stream, config 3's shape) — the thread walker then runs
    // with its blocks per CU capped beside the next batch's front
    uint32_t light_dom;
};
constexpr uint32_t kFlagAdmit = 8u;   // include/fsx_hip.h FSX_FLAG_OVERFLOW_ADMIT
constexpr uint32_t kFlagSwUnsorted = 16u;   // include/fsx_hip.h FSX_FLAG_SW_UNSORTED
constexpr uint32_t kFlagSwSparse = 32u;     // include/fsx_hip.h FSX_FLAG_TEST_SW_SPARSE
constexpr uint32_t kFlagOrdered = 64u;      // include/fsx_hip.h FSX_FLAG_ORDERED_INSERTS

// ------------------------------------------------------------ hashing
__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t fmix32_inv(uint32_t h) {
    h ^= h >> 16; h *= 0x7ed1b41du; h ^= (h >> 13) ^ (h >> 26); h *= 0xa5cb9243u; h ^= h >> 16;
    return h;
}
// IPv4 sort key: a bijection of the address, so equal sort keys <=> equal address.
__host__ __device__ inline uint32_t skey_v4(uint32_t ip, uint32_t salt) { return fmix32(ip ^ salt); }
__host__ __device__ inline uint32_t ip_of_skey(uint32_t sk, uint32_t salt) { return fmix32_inv(sk) ^ salt; }
// IPv6 sort key: salted 32-bit hash (collisions resolved exactly by the fixup pass).
__host__ __device__ inline uint32_t skey_v6(const uint32_t k[4], uint64_t seed) {
    uint64_t a = (uint64_t)k[0] | ((uint64_t)k[1] << 32);
    uint64_t b = (uint64_t)k[2] | ((uint64_t)k[3] << 32);
    return (uint32_t)(mix64(mix64(seed ^ a) ^ b) >> 32);
}
__host__ __device__ inline uint64_t slot_hash(uint32_t tag, const uint32_t k[4], uint64_t seed) {
    uint64_t h = mix64(seed ^ ((uint64_t)tag << 56) ^ ((uint64_t)k[0] | ((uint64_t)k[1] << 32)));
    if (tag == 2) h = mix64(h ^ ((uint64_t)k[2] | ((uint64_t)k[3] << 32)));
    return h;
}

// ------------------------------------------------------------ prefix rules
// Prefix blocklist (FSX_MAP_IPV4_PREFIX / _IPV6_PREFIX): one open-addressing
// table of both families' rules keyed by (family, prefix length, masked address), built by
// the host when the rules change; the lookup probes the family's distinct lengths longest
// first, so the first hit is the longest match.
struct RuleSlot {
    uint32_t tag;        // family << 8 | prefix length (family 1 / 2: never 0); 0 = empty
    uint32_t fp;         // rule_fp(a): the IPv4 address itself, an IPv6 fingerprint
    uint64_t till;       // blocked while 0 < now <= till
    uint32_t a[4];       // the address words (key byte order), bits past the length zero
};
static_assert(sizeof(RuleSlot) == 32, "one 32-byte probe per slot");
constexpr uint32_t kRuleLens6 = 64;  // RuleSet::lens: [0, 33) IPv4, [64, 193) IPv6
constexpr uint32_t kRuleFilterBits = 24;   // filter: one bit per /24 (per family)
struct RuleSet {
    const RuleSlot *slot = nullptr;   // nullptr: no rules
    const uint8_t *lens = nullptr;    // distinct prefix lengths per family, descending
    // per family 2^24 bits: bit p set when some rule covers part of the /24 p (the
    // first 24 address bits), so most packets are cleared by one load (2 MiB per family)
    const uint32_t *filter = nullptr;
    uint32_t mask = 0;                // slots - 1
    uint32_t nlen4 = 0, nlen6 = 0;
};
// The first len bits (network order) of the key words k (raw address bytes, little-endian
// words) kept, the rest zeroed.
__host__ __device__ inline void rule_mask(const uint32_t k[4], uint32_t len, uint32_t a[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int bits = (int)len - 32 * w;
        const uint32_t be = bits <= 0 ? 0u : bits >= 32 ? 0xFFFFFFFFu : ~0u << (32 - bits);
        // byte-swap the big-endian mask into the key word's byte order
        const uint32_t le = (be >> 24) | ((be >> 8) & 0xFF00u) | ((be << 8) & 0xFF0000u) | (be << 24);
        a[w] = k[w] & le;
    }
}
__host__ __device__ inline uint32_t rule_fp(const uint32_t a[4]) {
    return a[0] ^ (a[1] * 0x9E3779B1u) ^ (a[2] * 0x85EBCA77u) ^ (a[3] * 0xC2B2AE3Du);
}
__host__ __device__ inline uint32_t rule_hash(uint32_t tag, const uint32_t a[4]) {
    uint64_t h = mix64(((uint64_t)tag << 32) ^ a[0]);
    if ((tag >> 8) == 2) h = mix64(h ^ ((uint64_t)a[1] | ((uint64_t)a[2] << 32)) ^ ((uint64_t)a[3] << 17));
    return (uint32_t)(h >> 32);
}

// IPv4 table hash: a bijection of the 32-bit address (salted fmix32), so a source's home
// slot (the low log2(slots) bits) plus the remaining high bits name its address exactly.
__host__ __device__ inline uint32_t v4_hash(uint32_t k0, uint64_t seed) {
    return fmix32(k0 ^ (uint32_t)seed ^ (uint32_t)(seed >> 32));
}

// First probe slot of a source in the table (shared by k_parse, the map ops and the
// index rebuild). Test hook FSX_FLAG_TEST_V6_COLLIDE: every IPv6 source starts at IPv4
// 10.0.0.1's slot.
__host__ __device__ inline uint64_t probe_start(uint32_t tag, const uint32_t k[4], uint64_t seed,
                                                uint64_t mask, uint32_t test_flags) {
    if (tag == 2 && (test_flags & 1u)) return v4_hash(0x0100000Au, seed) & mask;
    if (tag == 1) return v4_hash(k[0], seed) & mask;
    return slot_hash(tag, k, seed) & mask;
}

// Home-ordered sort key (DESIGN.md §3 "Home-ordered inserts"): the source's first probe slot
// `home` (probe_start, s = log2(slots) bits, 1 <= s <= 31) in the top s bits, hash bits below.
// IPv4: rotr(v4_hash, s) — a bijection of the address (ord_v4_key inverts it); IPv6: 32 bits
// of its table hash (equal keys of different sources are separated by k_ord_fix).
__host__ __device__ inline uint32_t ord_hkey(uint32_t tag, const uint32_t k[4], uint64_t home, uint64_t seed,
                                             uint32_t s) {
    const uint32_t h = tag == 1 ? v4_hash(k[0], seed) : (uint32_t)slot_hash(tag, k, seed);
    return (uint32_t)(home << (32 - s)) | (h >> s);
}
__host__ __device__ inline uint32_t ord_v4_key(uint32_t hk, uint64_t seed, uint32_t s) {
    const uint32_t h = (hk << s) | (hk >> (32 - s));   // v4_hash
    return fmix32_inv(h) ^ (uint32_t)seed ^ (uint32_t)(seed >> 32);
}

// IPv4 mirror of the source index: one 2-byte entry per table slot, written
// when an IPv4 source is published at its home slot (d = 0) or the slot after it (d = 1):
// a valid bit, d and the 32 - log2(slots) hash bits above the home slot. v4_hash is a
// bijection, so an entry equal to the one computed for an address IS that address: k_parse
// matches light sources on 2-byte entries instead of the 8-byte heads (a quarter of the
// bytes to keep in the XCD's L2). Tables of 2^18 .. 2^26 slots (<= 14 high bits); smaller
// ones (<= 2 MiB of heads) have none, and neither do larger ones: beyond 128 MiB the mirror
// no longer stays in the caches, and a flood's every insert pays one more random line
// (config 5's 2^29 slots: 78.9 vs 76.6 ms per step with it, profiles/r03/ab_mirror/).
#ifndef FSX_MIR_MAX_SHIFT
#define FSX_MIR_MAX_SHIFT 26   // (A/B: scripts/build_variant.sh)
#endif
constexpr uint32_t kMirShift = 18, kMirMaxShift = FSX_MIR_MAX_SHIFT;
__host__ __device__ inline size_t mir_bytes(uint32_t shift) {
    return shift < kMirShift || shift > kMirMaxShift ? 0 : ((size_t)1 << shift) * 2;
}
__host__ __device__ inline uint32_t mir_entry(uint32_t k0, uint64_t seed, uint32_t shift, uint32_t d) {
    return 0x8000u | d << 14 | (shift >= 32 ? 0u : v4_hash(k0, seed) >> shift);
}
// IPv4 source k0 published at slot pos: its mirror entry when pos is its first or second
// probe slot.
__device__ __forceinline__ void mir_publish(void *mir, uint32_t shift, uint64_t mask, uint64_t seed,
                                            uint64_t pos, uint32_t k0) {
    if (!mir) return;
    const uint64_t d = (pos - (v4_hash(k0, seed) & mask)) & mask;
    if (d <= 1) static_cast<uint16_t *>(mir)[pos] = (uint16_t)mir_entry(k0, seed, shift, (uint32_t)d);
}

// Slot tag words: family (1 IPv4, 2 IPv6) | table generation << 16 (Limits::tgen); the
// family of a line, 0 when it is empty or of another generation.
__host__ __device__ inline uint32_t slot_tag(uint32_t fam, uint32_t tgen) { return fam | tgen << 16; }
__host__ __device__ inline uint32_t slot_fam(uint32_t tagw, uint32_t tgen) {
    return (tagw >> 16) == tgen ? (tagw & 0xFFFFu) : 0u;
}

// Slot of (tag, key) in the table (linear probing from its probe start), or kNoSlot.
__device__ inline bool slot_key_eq(const Slot &s, uint32_t tag, const uint32_t k[4]) {
    return s.key[0] == k[0] && s.key[1] == k[1] && s.key[2] == k[2] && s.key[3] == k[3];
}

__device__ inline uint32_t table_find(const Slot *table, const Limits &lim, uint32_t tag,
                                               const uint32_t k[4]) {
    uint64_t i = probe_start(tag, k, lim.seed, lim.table_mask, lim.test_flags);
    for (uint64_t probes = 0; probes <= lim.table_mask; ++probes) {
        const uint32_t t = slot_fam(table[i].tag, lim.tgen);
        if (t == 0) return kNoSlot;
        if (t == tag && slot_key_eq(table[i], tag, k)) return (uint32_t)i;
        i = (i + 1) & lim.table_mask;
    }
    return kNoSlot;
}

// packed sort word: bucket << bshift | source id << 31 | arrival index (n <= 2^31 - 1; ids
// < 2^32, max_entries <= 2^31). The source id is the source's slot in the id table
// (k_parse), so equal ids <=> equal (family, address) and the sort needs only log2(slots)
// key bits; the family is read from the packet's own record where it is needed (key_of).
// The bucket (heavy-source sort only, ids of <= 25 bits: bits 56..63) is the first sort
// pass's digit: the source's heavy index above the light digits, or a low id digit
// (HeavySet).
constexpr uint32_t kIdShift = 31;
// id_mask = table_mask: with the heavy-source sort the top byte holds the first-pass bucket;
// without it the id may use bits 31..62 (tables of up to 2^32 slots).
__host__ __device__ inline uint32_t pk_id(uint64_t v, uint64_t id_mask) { return (uint32_t)((v >> kIdShift) & id_mask); }
__host__ __device__ inline uint32_t pk_idx(uint64_t v) { return (uint32_t)v & 0x7FFFFFFFu; }
// Without the heavy-source sort no digit reaches bit 63, and with the heavy sources outside
// the sort a light word's pass-0 bucket is below 128 (k_pass0h ranks it without the bit):
// there bit 63 marks the packet that inserted its source in this batch (lazy slots; the
// walker writes that slot's line without reading it). Segment heads compare the words
// without it.
constexpr uint64_t kFreshBit = 1ull << 63;

// ------------------------------------------------------------ launchers (fsx_device.hip)
// Heavy sources of a batch: up to kHeavyMax source keys picked from a
// strided sample of the batch by k_heavy_sample / k_heavy_pick. Their packets get a
// first-pass sort bucket of their own, so after that pass each of them is one run in
// arrival order and the later passes sort only the other sources' entries. A wrong pick
// costs time only: the grouping is exact for any set of keys.
constexpr uint32_t kHeavyMax = 128;
constexpr uint32_t kSketchBits = 12;
constexpr uint32_t kSketch = 1u << kSketchBits;   // count sketch buckets
constexpr uint32_t kHeavySample = 65536;           // sampled packets per batch
constexpr uint32_t kHeavyMapBits = 10;
struct HeavySet {
    uint32_t n;
    uint32_t resolved;   // slot[] holds each heavy source's table slot (k_heavy_pick inserted
                         // new ones), so k_parse takes it from LDS instead of probing
    uint32_t tag[kHeavyMax];
    uint32_t key[kHeavyMax][4];
    uint32_t slot[kHeavyMax];
    // heavy verdict lists (fixed window): heavy source h's verdict changes
    // are lcnt[h] entries {arrival index << 1 | DROP} at list + lbase[h] (written by the
    // walker of its segment; read by k_verdict_apply for the packets k_parse tagged 0x80 | h)
    uint32_t lbase[kHeavyMax];
    uint32_t lcnt[kHeavyMax];
    // sliding window on the unsorted path (k_hmode_state): bit h set = heavy source h is too
    // sparse for the rank walker (select / rank cost a verdict-tile scan each) and takes the
    // run path (k_heavy_gather, k_walk_sw_heavy); nrun = their count
    uint64_t srun[2];
    uint32_t nrun, pad_;
    // open addressing on the source's probe start (its table hash) modulo the map size:
    // heavy index + 1, 0 empty
    alignas(16) uint8_t map[1u << kHeavyMapBits];
};

struct Scratch {
    uint64_t *packed[2];
    uint64_t *pay[2];      // payload words in sort order (kPayLenBits)
    uint8_t *marks;        // per sorted position: 0 none, else verdict starting there
    uint8_t *headf;        // per sorted position: segment-head flag
    uint32_t *seg_start;   // nseg + 1
    uint32_t *seg_slot;
    uint32_t *seg_lo;      // per segment: low word of its first sort word (family, arrival index)
    uint32_t *seg_len;     // per light segment: frame length of its first packet (flow tiles)
    uint32_t *hist;        // sort: per-tile digit counts [256][cap/kSortTile+2]; walker classes
    uint32_t *tile_aux;    // per kTile tile
    uint8_t *tile_last;
    uint32_t *seg_order;   // segment ids grouped by length class (walker load balance)
    // per-block length-class counts of k_seg_count / scan / order (their own buffer: the
    // tail's heavy kernels read pass 0's scanned rows in hist beside them on another stream)
    uint32_t *seg_cls;
    uint32_t *sub_cnt;     // heads per 1024-position flow tile
    void *flow_first;      // FlowAcc per flow tile (fsx_flows.hip)
    void *flow_last;
    uint32_t *span_list;
    uint32_t *sort_ctl;    // [0,1024) digit histograms of the 4 passes, [1024,1028) tile
                           // counters, [1028,1028+2*kSegClasses) segment class counts, cursors
    uint32_t *gbase;       // 4 x 256 digit bases
    unsigned long long *status;  // onesweep look-back words, 256 per tile
    uint64_t *lim_tiles;   // limiter scans: 4 u64 per kTile tile (token bucket: map + carry)
    uint64_t lim_tiles_n;  // tiles lim_tiles is sized for
    SwSeg *sw_seg;         // sliding window: per source (null for other limiters)
    uint32_t *id_tab;      // per-batch source ids: u64 heads [slots] then u32 IPv6 key
                           // words [slots][4] (generation-tagged, never cleared)
    uint32_t *drop_list;   // DROP verdicts by arrival chunk: chunk c owns [c, c + 1) * kVChunk
    uint32_t *drop_cur;    // entries per chunk (zeroed by k_verdict_apply after use)
    uint32_t *sketch;      // heavy-source sample, two sketches: counts [kSketch], candidate
                           // packets [kSketch] each (counts zeroed by k_heavy_pick after use)
    HeavySet *heavy;
    void *heavy_flow;      // heavy sources' flow chunk sums (heavy_flow_bytes)
    // unsorted heavy sources (front buffers, one per pipelined set): light sort-word count
    // of every 1024-packet parse chunk (k_parse writes the light words compacted per chunk)
    // and one HeavyTileRec per sort tile (k_pass0h)
    uint32_t *chunk_cnt;
    void *hrec;
    void *hflow;           // tail: per (group of kHGroupTiles tiles, heavy source) flow sums
    uint8_t *dig;          // the next sort pass's digit of every output position (cap bytes):
                           // written by pass p's scatter, read by pass p + 1's tile histogram
    void *tbh;             // token bucket, heavy sources unsorted: per (sort tile, heavy source)
                           // map + state (tb_heavy_bytes; null for the other limiters)
    // FSX_FLAG_OVERFLOW_ADMIT: per arrival index, 1 at a new source's first packet, then its
    // admission rank; per 4096 positions, their count / exclusive scan
    uint32_t *admit_rank;
    uint32_t *admit_cnt;
    uint64_t cap;          // packets the scratch is sized for
};

// Unsorted heavy sources: per sort tile (4096 arrival positions) and heavy source h, the
// sums the flow features need over h's packets of the tile (SoA, so a block writes one
// contiguous record per tile and a thread per h reads it coalesced). Exact while the batch
// clock is non-decreasing, every frame < 2^16 B and every tile spans < 2^32 ns (k_hmode
// checks; otherwise the runs are built and the records ignored).
struct HeavyTileRec {
    uint32_t s1[kHeavyMax];     // sum of frame lengths
    uint32_t dmax[kHeavyMax];   // largest gap between consecutive packets of h inside the tile
    uint32_t fo[kHeavyMax];     // arrival offset (in the tile) of h's first packet
    uint32_t pad_[kHeavyMax];
    uint64_t s2[kHeavyMax];     // sum of squared lengths
    uint64_t t0[kHeavyMax];     // first and last timestamp
    uint64_t t1[kHeavyMax];
    uint64_t d2[kHeavyMax];     // sum of squared gaps inside the tile
};
constexpr uint32_t kHGroupTiles = 64;    // tiles per k_hflow_combine group
inline size_t heavy_rec_bytes(uint64_t cap) { return (cap / kSortTile + 2) * sizeof(HeavyTileRec); }
// ... followed (16-byte aligned) by the light-packet mask of every 64-packet parse step
// (k_parse's ballot; k_pass0h compacts the light packets' payload words by it)
inline size_t chunk_cnt_head(uint64_t cap) { return ((cap / 1024 + 8) * 4 + 15) / 16 * 16; }
inline size_t chunk_cnt_bytes(uint64_t cap) { return chunk_cnt_head(cap) + (cap / 64 + 8) * 8; }
inline uint64_t *light_masks(uint32_t *chunk_cnt, uint64_t cap) {
    return reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(chunk_cnt) + chunk_cnt_head(cap));
}

// Flow partials (fsx_flow_partials_records_device): every source's raw sums go to the run of
// its owner rank (G runs of cap partials, cnt[o] per run) instead of a row.
struct PartialOut {
    void *buf;
    uint32_t cap, G;
    unsigned long long *cnt;
};

// Optional per-source outputs of a batch (flow features + q8 scores), device pointers.
struct FlowRequest {
    uint8_t *keys16;
    uint8_t *fam;
    float *feat;      // n_sources x 8, may be null
    float *prob;      // may be null (then no scoring)
    uint8_t *dec;
    uint32_t cap;
    ScoreParams score;
    void *acc;        // cap x FlowAcc scratch (owned by the context)
    // accumulate mode (fsx_flows_begin .. fsx_flows_end): every source's sums merge into
    // its table slot's SlotAcc of this epoch instead of becoming an output row
    void *sacc;
    uint32_t epoch;
    PartialOut part;  // (buf null: rows / accumulate as above)
};

// do_limit: run the rate limiter (verdicts + maps); flows: also per-source features.
// Per-kernel timing of one batch: events recorded after each kernel; interval i runs
// from event prev[i] to event i (on the same stream; prev < 0: a start marker).
struct PipeTiming {
    hipEvent_t *ev;
    const char **names;
    int *prev;
    int cap;
    int used;
};

// The packets of a batch: 64-byte header records (hdr, with the caller's len / ts), or
// the exchange records of the sharded path (record mode: rec, rec_bytes 16 / 32, every
// record an IP packet; k_parse writes their len / ts into rec_len / rec_ts for the rest
// of the pipeline).
struct PacketIn {
    const uint8_t *hdr;
    const void *rec;
    uint32_t rec_bytes;
    uint32_t *rec_len;
    uint64_t *rec_ts;
};

// Batch pipelining (fsx_set_pipeline, DESIGN.md §3 "Pipelined batches"): the front of a
// batch (heavy pick, parse, sort) stays on st; the rest (heads, walkers, fill, verdicts;
// flows on st2) runs on tail, after `front_done`, so the next batch's front overlaps this
// batch's tail. Its front buffers (Scratch sort arrays, BatchState) alternate between two
// sets; prev (the batch before, or null) cancels this one when it failed.
struct TailArgs;
struct PipeSplit {
    hipStream_t tail;
    hipEvent_t front_done;     // recorded on st after the sort
    const BatchState *prev;
    // called right after this batch's parse (enqueues the previous batch's deferred tail, so
    // it overlaps this batch's sort rather than its parse)
    // (recorded: an event already recorded on st at this point, or null)
    hipError_t (*on_parse)(void *cb, hipEvent_t recorded);
    void *cb;
    TailArgs *tail_out;        // this batch's tail is returned here, not enqueued
    // early prologue (null: on st): this batch's scratch resets and heavy-source pick run on
    // `pro` after `pro_wait` (the previous batch's parse), beside the previous batch's sort;
    // st waits for `pro_done` before the parse; `pro_wait` is recorded after this parse
    hipStream_t pro = nullptr;
    hipEvent_t pro_wait = nullptr, pro_done = nullptr;
};

// Everything the tail of a batch needs (launch_tail): by value, so a pipelined batch's tail can
// be enqueued after the call that built it has returned.
struct TailArgs {
    PacketIn in;
    const uint32_t *len;
    const uint64_t *ts;
    uint32_t n;
    uint8_t *verdict;
    Slot *table;
    TableState *tstate;
    BatchState *bs;
    Scratch sc;
    Limits lim;
    bool do_limit, has_flows, split, tagh, fork;
    bool hfm;             // heavy sources outside the sort (k_pass0h ran; k_hmode picks the path)
    bool admit;           // FSX_FLAG_OVERFLOW_ADMIT (admission kernels after the heads)
    TableIndex X;         // (admission: the persistent index)
    uint32_t id_gen;      // (admission: the batch generation stamped on admitted slots)
    bool lazy;            // k_parse left new sources' slots to the fixed window's walkers
    bool fresh_bit;       // ... and marked the inserting packets' sort words (kFreshBit)
    bool ord;             // home-ordered inserts: key-hash words, slots found after the heads
    uint32_t shift0;      // pass 0's bucket shift (k_heavy_gather's sort words)
    FlowRequest fq;
    HistBufs hist;
    hipStream_t st, st2, st3;
    hipEvent_t fork_ev, join_ev, walk_fork_ev, walk_join_ev, heavy_fork_ev, heavy_flow_ev;
    PipeTiming *tm;
    PipeSplit sp;
    int npass;
    uint32_t gridTiles;
    int last[3];
};
hipError_t launch_tail(const TailArgs &a);
hipError_t launch_born_clear(Slot *table, uint64_t nslots, hipStream_t st);

// st: the batch stream. st2 (optional, with fork/join events): the flow features run
// on it concurrently with the rate limiter (they share only read-only inputs). st3
// (optional): the fixed-window wave walker beside the thread walker.
hipError_t launch_verdict_pipeline(const PacketIn &in, const uint32_t *len, const uint64_t *ts,
                                   uint32_t n, uint8_t *verdict, Slot *table, TableState *tstate,
                                   BatchState *bs, const Scratch &sc, uint32_t id_gen,
                                   const TableIndex &X, const Limits &lim, const RuleSet &rules,
                                   bool do_limit, const FlowRequest *flows, const HistBufs &hist,
                                   hipStream_t st, hipStream_t st2, hipEvent_t fork_ev,
                                   hipEvent_t join_ev, hipStream_t st3, hipEvent_t walk_fork_ev,
                                   hipEvent_t walk_join_ev, hipEvent_t heavy_fork_ev,
                                   hipEvent_t heavy_flow_ev, PipeTiming *tm,
                                   const PipeSplit *split = nullptr);

// Build-defined limiters (fsx_limiters.hip), after the table lookup/insert of a batch:
// one verdict mark per sorted position, final per-source state in the table.
// mark(name) closes the timing interval of the kernels just enqueued (may be empty).
typedef void (*MarkFn)(void *ctx, const char *name);
struct Marker {
    MarkFn fn;
    void *ctx;
    void operator()(const char *name) const { if (fn) fn(ctx, name); }
};

struct HeavyLists;
// light_only 2: the heavy sources' packets are decided outside the sort when the batch takes
// the unsorted path (launch_tb_heavy), so the scan covers the light entries only then
hipError_t launch_token_bucket(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                               const Scratch &sc, Slot *table, const Limits &lim, uint32_t n,
                               hipStream_t st, const Marker &mark, uint32_t light_only = 0);
// token bucket, heavy sources outside the sort (fsx_limiters.hip): per-tile maps, a scan per
// heavy source over its tiles, the replay writing its verdict bytes; the run path's heavy heads
// and the untagging of its passed heavy packets
size_t tb_heavy_bytes(uint64_t cap);
hipError_t launch_tb_heavy(BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, const uint32_t *offs,
                           uint32_t tcap, uint8_t *verdict, const uint64_t *ts, uint32_t n, const void *rec,
                           void *tbh, Slot *table, const Limits &lim, const HeavySet *hs, TableState *tstate,
                           hipStream_t st);
hipError_t launch_tb_run_heads(const BatchState *bs, const uint32_t *seg_start, uint8_t *headf, uint32_t *tile_off,
                               uint32_t n, hipStream_t st);
hipError_t launch_tb_untag(const BatchState *bs, uint8_t *verdict, uint32_t n, hipStream_t st);

// st3 (optional, with fork/join events): the long-segment walker beside the short one.
hipError_t launch_sliding_window(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                                 const Scratch &sc, Slot *table, TableState *tstate, const HistBufs &hb,
                                 const Limits &lim, uint32_t n, hipStream_t st, const Marker &mark,
                                 hipStream_t st3, hipEvent_t fork_ev, hipEvent_t join_ev,
                                 const HeavyLists *H,    // (H->list: heavy verdict lists)
                                 const uint8_t *tags,    // (heavy sources outside the sort: verdict tags)
                                 hipEvent_t heavy_done); // (launch_sw_heavy ran on another stream)
hipError_t launch_sw_heavy(const uint64_t *S, const uint64_t *ts, const uint32_t *len, BatchState *bs,
                           const Scratch &sc, Slot *table, TableState *tstate, const HistBufs &hb,
                           const Limits &lim, uint32_t n, const HeavyLists &H, const uint8_t *tags,
                           hipStream_t st);

hipError_t launch_pcap_records(const uint8_t *buf, const uint64_t *off, const uint32_t *caplen, uint32_t n,
                               uint8_t *hdr, hipStream_t st);

hipError_t launch_flows(const uint64_t *S, const uint64_t *pay, BatchState *bs, const uint8_t *headf, const uint32_t *len,
                        const uint64_t *ts, const PacketIn &in, const uint32_t *tile_off,
                        const uint32_t *sub_cnt, const uint32_t *seg_start, void *firstp, void *lastp,
                        uint32_t *span_list, void *acc, uint8_t *keys16, uint8_t *fam, float *feat,
                        float *prob, uint8_t *dec, uint32_t cap, const ScoreParams &P, uint32_t salt,
                        uint32_t n, void *sacc, uint32_t epoch, const uint32_t *seg_slot, bool light_only,
                        const uint32_t *seg_lo, uint32_t *seg_len, const PartialOut &part, hipStream_t st);
// Heavy verdict lists: the heavy sources' flow sums right after sort pass 0, their rows
// after the heads (fsx_flows.hip "heavy sources"); scratch of heavy_flow_bytes(cap).
size_t heavy_flow_bytes(uint64_t cap);
hipError_t launch_flows_heavy(const uint64_t *S, const uint64_t *pay, const uint64_t *ts, const uint32_t *len,
                              const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, void *scratch,
                              uint64_t cap, hipStream_t st);
hipError_t launch_flows_heavy_finish(const uint64_t *S, const BatchState *bs, const uint32_t *cnt0,
                                     const uint32_t *seg_start, const PacketIn &in, const uint32_t *len,
                                     const uint64_t *ts, void *scratch, uint64_t cap, uint8_t *keys16, uint8_t *fam,
                                     float *feat, float *prob, uint8_t *dec, uint32_t rows_cap,
                                     const ScoreParams &P, uint32_t salt, void *sacc, uint32_t epoch,
                                     const uint32_t *seg_slot, hipStream_t st);

// Heavy sources outside the sort (fsx_heavy.hip; k_pass0h in fsx_device.hip), DESIGN.md §3.
hipError_t launch_pass0h(const uint64_t *in, uint64_t *out, uint32_t n, uint32_t shift, uint32_t dmask,
                         const uint32_t *offs, uint32_t tcap, BatchState *bs, uint64_t *pout, const uint64_t *ts,
                         const uint32_t *len, const uint8_t *tags, const uint32_t *chunk_cnt,
                         const uint64_t *lmask, void *rec,
                         const HeavySet *hs, const uint64_t *pin, hipStream_t st,
                         void *dout = nullptr, uint32_t nshift = 0, uint32_t nmask = 0, int dwide = 0);
hipError_t launch_hmode(BatchState *bs, const uint64_t *ts, uint32_t n, const Limits &lim, hipStream_t st);
// (FSX_PARSE_PAY: every sort tile's HeavyTileRec, at the start of the tail)
hipError_t launch_heavy_recs(const BatchState *bs, const uint64_t *ts, const uint32_t *len, const uint8_t *tags,
                             uint32_t n, const HeavySet *hs, void *rec, hipStream_t st);
// (the tail's first kernel: the heavy sources' carried state, after the previous tail stored it)
hipError_t launch_hmode_state(const uint32_t *cnt0, uint32_t n, BatchState *bs, HeavySet *hs, const Slot *table,
                              const Limits &lim, TableState *tstate, hipStream_t st);
hipError_t launch_heavy_gather(const BatchState *bs, const uint8_t *tags, const uint64_t *ts, const uint32_t *len,
                               uint32_t n, const uint32_t *offs, uint32_t tcap, const HeavySet *hs, uint32_t shift0,
                               uint64_t id_mask, uint64_t *out, uint64_t *pout, hipStream_t st);
hipError_t launch_walk_heavy_sel(BatchState *bs, const uint32_t *cnt0, const uint32_t *base0, const uint32_t *offs,
                                 uint32_t tcap, const uint8_t *tags, const uint64_t *ts, const uint32_t *len,
                                 uint32_t n, const void *rec, Slot *table, const Limits &lim, HeavySet *hs,
                                 uint32_t *list, TableState *tstate, hipStream_t st);
size_t hflow_bytes(uint64_t cap);
hipError_t launch_hflow_combine(const BatchState *bs, const uint32_t *cnt0, const uint32_t *base0,
                                const uint32_t *offs, uint32_t tcap, uint32_t n, const void *rec, void *part,
                                hipStream_t st);
hipError_t launch_hflow_finish(const BatchState *bs, const uint32_t *cnt0, const HeavySet *hs, const void *part,
                               uint32_t n, const PacketIn &in, const uint32_t *len, const uint64_t *ts,
                               uint8_t *keys16, uint8_t *fam, float *feat, float *prob, uint8_t *dec,
                               uint32_t rows_cap, const ScoreParams &P, void *sacc, uint32_t epoch,
                               const PartialOut &partial, hipStream_t st);

size_t flow_acc_bytes();
size_t slot_acc_bytes();
// Accumulate mode: merge m flow partials (fsx_flow_partial) into the epoch's per-slot sums.
// (d_m non-null: the count is min(*d_m, m), read on the device)
hipError_t launch_flows_merge(const void *partials, uint32_t m, const Slot *table, const Limits &lim, void *sacc,
                              uint32_t epoch, hipStream_t st, const uint64_t *d_m = nullptr);
// Rows of every source accumulated in epoch `epoch` (slots of the table), *d_count = rows.
hipError_t launch_flows_end(const void *sacc, uint32_t epoch, const Slot *table, uint64_t slots, uint32_t tgen,
                            uint8_t *keys16, uint8_t *fam, float *feat, float *prob, uint8_t *dec,
                            uint32_t cap, const ScoreParams &P, unsigned long long *d_count,
                            hipStream_t st);
ScoreParams make_score_params(const int8_t w[8], float inv_in, int32_t zp_in, float bias_over_ats,
                              float mult, int32_t zp_out, const uint8_t lut[256]);

hipError_t launch_map_op(Slot *table, TableState *tstate, const Limits &lim, const TableIndex &X, int op,
                         int map_id, const uint32_t key[4], const uint64_t val[3], uint64_t flags,
                         int32_t *d_result, uint64_t *d_val, hipStream_t st);
// Batched BPF_ANY update of distinct keys (key words: 1 per IPv4 / 4 per IPv6 key; value
// words: 3 stats / 2 token state / 1 blacklist); new sources counted and checked like a
// batch's (bs->err, rollback by generation `born`).
hipError_t launch_map_import(Slot *table, TableState *tstate, BatchState *bs, const Limits &lim,
                             const TableIndex &X, uint32_t born, int map_id, const uint32_t *d_keys,
                             const uint64_t *d_vals, uint32_t n, hipStream_t st);
// Re-publish the live slots under X.epoch; slots born in batch `born` (nonzero) are
// emptied (rollback of a failed batch).
hipError_t launch_index_rebuild(Slot *table, const Limits &lim, const TableIndex &X, uint32_t born,
                                hipStream_t st);

// FSX_FLAG_EVICT_IDLE, with the device idle before a limiter batch:
// scan: the batch's smallest timestamp into scal[0] (preset ~0), then every source that
// is not idle at it is copied into buf (scal[1] counts them, preset 0; at most cap);
// reinsert (after the host started a new index epoch and cleared the table): the m
// survivors go back into the table under X.epoch with their state, count = m.
hipError_t launch_evict_scan(const Slot *table, const Limits &lim, const PacketIn &in, const uint64_t *ts,
                             uint32_t n, Slot *buf, uint64_t cap, unsigned long long *scal, hipStream_t st);
hipError_t launch_evict_reinsert(Slot *table, TableState *tstate, const Limits &lim, const TableIndex &X,
                                 const Slot *buf, uint64_t m, hipStream_t st);

hipError_t launch_map_dump(const Slot *table, const Limits &lim, int map_id, uint8_t *d_keys,
                           uint64_t *d_vals, uint64_t cap, unsigned long long *d_count,
                           hipStream_t st);

// Zero `bytes` of device memory on st (the slot table: fsx_reset, eviction).
hipError_t launch_clear(void *p, uint64_t bytes, hipStream_t st);

hipError_t launch_score(const float *feat, size_t n, float *prob, uint8_t *dec,
                        const int8_t w[8], float inv_in, int32_t zp_in, float bias_over_ats,
                        float mult, int32_t zp_out, const uint8_t lut[256], hipStream_t st);

}  // namespace fsx
