/*
 * fsx_hip.h — C ABI of libfsx_hip.so, the MI355X (gfx950) batch data plane that
 * replaces FlowSentryX's packet-verdict hot path.
 *
 * Reference boundary being replaced (paths relative to the FlowSentryX tree):
 *   - the XDP program ABI  `SEC("xdp") int fsx(struct xdp_md *ctx)`
 *       src/fsx_kern.c:96-97  -> fsx_verdict_batch / fsx_verdict_batch_device
 *     returning XDP_DROP (1) / XDP_PASS (2) per packet, in arrival order;
 *   - the five BPF maps that are its state/control ABI, src/fsx_kern.c:56-94
 *       stats_map           ARRAY[1]  key u32 0 -> struct stats {allowed,dropped}
 *       ipv4_stats_map      LRU_HASH  key 4 B   -> struct ip_stats {pps,bps,track_time}
 *       ipv6_stats_map      LRU_HASH  key 16 B  -> struct ip_stats
 *       ipv4_blacklist_map  LRU_HASH  key 4 B   -> u64 blocked_till_ns
 *       ipv6_blacklist_map  LRU_HASH  key 16 B  -> u64 blocked_till_ns
 *     -> fsx_map_lookup / fsx_map_update / fsx_map_delete / fsx_map_dump with the
 *        exact key/value byte layouts of src/fsx_struct.h:11-22;
 *   - the host weight loader role of src/fsx_load.py:1-18 (push the quantized
 *     model_weights.pth into the data plane) -> fsx_load_q8_model;
 *   - the model forward of model/model.py:132-137 and its decision y > 0.5
 *     (model/model.py:206) -> fsx_score / fsx_score_device.
 *
 * Conventions
 *   - Every entry point returns 0 or a negative errno (-EINVAL, -ENOMEM, -EIO for
 *     HIP runtime errors, -ENOENT, -EEXIST, -ENOSPC, -E2BIG). Nothing throws or
 *     longjmps across this boundary. fsx_last_error() returns a message.
 *   - Host pointers are owned by the caller and are not retained after return.
 *   - One context per host thread; calls on one context are serialized by the
 *     caller. Results are deterministic and equal to the reference program's
 *     single-CPU, arrival-order semantics.
 *   - A packet is a 64-byte header record (the first min(len,64) frame bytes,
 *     zero padded), its frame length `len` (data_end - data, FCS excluded) and
 *     its arrival time `ts_ns` (the value bpf_ktime_get_ns() returns at
 *     src/fsx_kern.c:150).
 */
#ifndef FSX_HIP_H
#define FSX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSX_ABI_VERSION 1

/* Verdict codes: the XDP return values of src/fsx_kern.c (enum xdp_action). */
#define FSX_XDP_DROP 1
#define FSX_XDP_PASS 2

#define FSX_HDR_BYTES 64

/* fsx_config.flags — FSX_FLAG_TEST_V6_COLLIDE and FSX_FLAG_ONESWEEP_SORT are test / A-B
 * hooks. FSX_FLAG_TEST_V6_COLLIDE makes every IPv6
 * source start its probe of the per-batch source-id table at IPv4 10.0.0.1's slot
 * (one long probe chain shared by all of them; results must not change). */
#define FSX_FLAG_TEST_V6_COLLIDE 1u
/* Sort with the single-pass onesweep variant (decoupled look-back) instead of the
 * per-pass tile histograms (A/B measurements only). */
#define FSX_FLAG_ONESWEEP_SORT 2u
/* Opt-in overflow policy (fixed window only; DESIGN.md §2.1, parity unpinned like the
 * reference's LRU_HASH eviction). Default (flag clear): a batch whose new sources would
 * exceed max_entries fails with -ENOSPC. With the flag: before a limiter batch of n
 * packets, when the tracked sources plus n exceed max_entries, every source that is idle
 * at the batch's smallest timestamp now0 leaves the maps first: its window has expired
 * (no ip_stats, or now0 - track_time > window_ns: the reset test of src/fsx_kern.c:245),
 * it holds no live blacklist entry (none, till 0 or now0 > till) and no token-bucket
 * state. The batch then runs as usual (-ENOSPC if it still overflows). The check reads the
 * tracked count (a context sync: previous batches finish first) only when a host-side bound
 * (the last count read plus the packets of every batch since) plus n could exceed
 * max_entries, so pipelined batches far below capacity do not wait; an eviction is not
 * undone if the batch then fails;
 * the number evicted is fsx_last_batch_info()[12]. Not with fsx_flows_begin. */
#define FSX_FLAG_EVICT_IDLE 4u
/* Opt-in overflow policy for floods beyond max_entries (any limiter; DESIGN.md §2.2,
 * build-defined, parity unpinned like the reference's LRU_HASH maps of
 * MAX_TRACK_IPS = 100000 entries, src/fsx_struct.h:7, src/fsx_kern.c:64-94). A source is
 * tracked once it has map state (as for FSX_FLAG_EVICT_IDLE). Within a limiter batch, in
 * arrival order, a source that is not tracked when its first packet reaches the per-source
 * maps (after the prefix rules) is ADMITTED — tracked from then on, with the maps as usual —
 * while fewer than max_entries sources are tracked; otherwise it is TRANSIENT for this
 * batch: its packets are evaluated exactly like a new source's (fixed window: ip_stats
 * {1, len, now} on its first packet, then src/fsx_kern.c:150-346; sliding window / token
 * bucket: their specs), with state that lives for this batch only and is never visible in
 * the maps. So every packet gets a verdict (stats_map counts them all) and a batch never
 * fails with -ENOSPC for lack of table room. With FSX_FLAG_EVICT_IDLE the idle eviction
 * runs first. Batches run unpipelined (mode 2) and the heavy-source sort is off; not with
 * fsx_flows_begin. fsx_last_batch_info()[14] / [15]: sources admitted / transient. */
#define FSX_FLAG_OVERFLOW_ADMIT 8u
/* A/B hook: the sliding window's heaviest sources outside the sort (walked by rank over the
 * arrival order, as the fixed window's always are). Off by default: on
 * config 2 it measured slower than the heavy-source sort (3.74 vs 3.44 ms per step). */
#define FSX_FLAG_SW_UNSORTED 16u
/* Test hook (with FSX_FLAG_SW_UNSORTED): the heavy-source pick keeps the fixed window's
 * floor, so heavy sources too sparse for the rank walker reach its per-source run path. */
#define FSX_FLAG_TEST_SW_SPARSE 32u
/* Home-ordered inserts on every fixed-window batch (header records, no flows):
 * k_parse writes each IP packet's home-ordered source hash instead of probing the index, and
 * the segment heads find / insert their slots in home-slot order after the sort. Without the
 * flag a batch takes them when the previous checked batch was a flood (new sources > half of
 * its IP packets). Results are the same either way. */
#define FSX_FLAG_ORDERED_INSERTS 64u

/* Map ids: the five maps of src/fsx_kern.c:56-94, then the token-bucket state maps of
 * the build-defined token bucket (value fsx_tb_state), then the
 * build-defined prefix blocklists: BPF_MAP_TYPE_LPM_TRIE-style maps
 * whose key is struct bpf_lpm_trie_key {u32 prefixlen; u8 addr[4 | 16]} (8 / 20 bytes)
 * and whose value is a u64 "blocked till" in ns like the blacklists'. */
enum fsx_map_id {
    FSX_MAP_STATS = 0,          /* stats_map          src/fsx_kern.c:56-62 */
    FSX_MAP_IPV4_STATS = 1,     /* ipv4_stats_map     src/fsx_kern.c:64-70 */
    FSX_MAP_IPV6_STATS = 2,     /* ipv6_stats_map     src/fsx_kern.c:72-78 */
    FSX_MAP_IPV4_BLACKLIST = 3, /* ipv4_blacklist_map src/fsx_kern.c:80-86 */
    FSX_MAP_IPV6_BLACKLIST = 4, /* ipv6_blacklist_map src/fsx_kern.c:88-94 */
    FSX_MAP_IPV4_TOKENS = 5,    /* build-defined: key 4 B  -> fsx_tb_state */
    FSX_MAP_IPV6_TOKENS = 6,    /* build-defined: key 16 B -> fsx_tb_state */
    FSX_MAP_IPV4_PREFIX = 7,    /* build-defined: fsx_prefix_key4 -> u64 till */
    FSX_MAP_IPV6_PREFIX = 8,    /* build-defined: fsx_prefix_key6 -> u64 till */
    FSX_MAP_COUNT = 9
};

/* Prefix-blocklist keys (struct bpf_lpm_trie_key layout; prefixlen in host order).
 * Update and delete are exact on (prefixlen, the first prefixlen bits of addr); the
 * address bits past prefixlen are ignored. Lookup is a longest-prefix match of addr
 * over the rules of length <= prefixlen (BPF LPM-trie lookup semantics). Every IP packet
 * of a limiter batch is first matched against its family's rules: when the longest
 * matching rule has 0 < now <= till the packet is dropped (stats_map dropped + 1) and
 * never reaches the per-source maps; a longest match with till == 0 or expired lets it
 * through (an exception inside a shorter blocked prefix). */
typedef struct fsx_prefix_key4 { uint32_t prefixlen; uint8_t addr[4]; } fsx_prefix_key4;
typedef struct fsx_prefix_key6 { uint32_t prefixlen; uint8_t addr[16]; } fsx_prefix_key6;
#define FSX_PREFIX_MAX_ENTRIES 65536   /* rules per prefix map */

/* bpf_map_update_elem flags (linux/bpf.h). */
#define FSX_BPF_ANY 0
#define FSX_BPF_NOEXIST 1
#define FSX_BPF_EXIST 2

/* Limiter algorithms. FIXED is the reference program (src/fsx_kern.c:225-336).
 * SLIDING and TOKEN_BUCKET are build-defined (README.md:155-162 only names them);
 * their semantics are specified in DESIGN.md §4. */
enum fsx_limiter {
    FSX_LIMIT_FIXED_WINDOW = 0,
    FSX_LIMIT_SLIDING_WINDOW = 1,
    FSX_LIMIT_TOKEN_BUCKET = 2
};

/* struct stats, src/fsx_struct.h:11-15 */
typedef struct fsx_stats {
    uint64_t allowed;
    uint64_t dropped;
} fsx_stats;

/* struct ip_stats, src/fsx_struct.h:17-22 */
typedef struct fsx_ip_stats {
    uint64_t pps;
    uint64_t bps;
    uint64_t track_time;
} fsx_ip_stats;

/* Token-bucket state of one source (build-defined). */
typedef struct fsx_tb_state {
    uint64_t tokens;          /* nano-tokens (1e9 = one packet) */
    uint64_t last;            /* ns of the last counted packet */
} fsx_tb_state;

/* Largest tb_burst (tokens) a token-bucket context accepts: capacity <= 2^61 nano-tokens. */
#define FSX_TB_MAX_BURST 2305843009ull
/* Largest pps_threshold a sliding-window context accepts (a carried log holds at most
 * pps_threshold entries per source). */
#define FSX_SW_MAX_PPS 16777214ull

typedef struct fsx_config {
    uint64_t pps_threshold;   /* 1000       src/fsx_kern.c:309 */
    uint64_t bps_threshold;   /* 125000000  src/fsx_kern.c:310 */
    uint64_t window_ns;       /* 1000000000 src/fsx_kern.c:245 */
    uint64_t block_ns;        /* 10 s       src/fsx_kern.c:308,317 */
    uint64_t max_entries;     /* per map; MAX_TRACK_IPS=100000 src/fsx_struct.h:7.
                                 No LRU eviction: a full table makes a batch fail
                                 with -ENOSPC, unless
                                 FSX_FLAG_EVICT_IDLE. 1 .. 2^31. */
    uint64_t max_batch;       /* largest n per call (device scratch is sized for it) */
    uint64_t tb_rate;         /* token bucket: refill in nano-tokens per ns (1000 = 1000 tok/s) */
    uint64_t tb_burst;        /* token bucket: capacity in tokens (<= FSX_TB_MAX_BURST) */
    uint64_t hash_seed;       /* salt of the table/IPv6 sort hashes */
    int32_t limiter;          /* enum fsx_limiter */
    int32_t device;           /* HIP device ordinal */
    uint32_t flags;           /* FSX_FLAG_*: 0 or FSX_FLAG_EVICT_IDLE in production */
    uint32_t reserved[7];
} fsx_config;

/* Quantized scorer: QuantStub -> Linear(8,1) -> sigmoid -> DeQuantStub,
 * model/model.py:124-137, eager-mode int8 after torch.ao convert(). */
typedef struct fsx_q8_model {
    int8_t weight[8];         /* linear._packed_params weight int_repr (per-tensor, zp 0) */
    float weight_scale;       /* 0.002657087752595544 */
    float bias;               /* 0.02776797 (fp32) */
    float in_scale;           /* quant.scale       944881.875 */
    int32_t in_zero_point;    /* quant.zero_point  0 */
    float out_scale;          /* linear.scale      398330.96875 */
    int32_t out_zero_point;   /* linear.zero_point 84 */
} fsx_q8_model;

typedef struct fsx_ctx fsx_ctx;

/* Fill *cfg with the reference constants. */
void fsx_config_default(fsx_config *cfg);
int fsx_abi_version(void);

int fsx_open(fsx_ctx **out, const fsx_config *cfg);
void fsx_close(fsx_ctx *ctx);
const char *fsx_last_error(const fsx_ctx *ctx);

/* Attach a caller-owned hipStream_t (NULL restores the context's own stream). */
int fsx_set_stream(fsx_ctx *ctx, void *hip_stream);
/* Wait for enqueued device work and report deferred device-side errors. */
int fsx_sync(fsx_ctx *ctx);
/* Batch pipelining (default off; DESIGN.md §3 "Pipelined batches"). When on, a fixed- or
 * sliding-window fsx_verdict_batch_device / fsx_process_batch_device call enqueues the batch's front
 * (parse, sort) on the context stream and its tail (walkers, verdicts, flows) on the
 * context's own side streams, so the next batch's front overlaps this batch's tail; results
 * and map state are exactly those of the same calls without pipelining. Record batches
 * (fsx_verdict_records_device / fsx_process_records_device) split the same way. Up to three batches
 * are in flight: a call first waits (on the host) for the batch three calls back. The caller
 * keeps a batch's input and output buffers untouched until that batch completes: read the
 * outputs after fsx_sync (or any other entry point, which orders the context stream after
 * the last tail). A failed batch cancels the batch after it; the error (e.g. -ENOSPC) is
 * returned by fsx_sync or by the call that found it, which enqueues nothing, and neither
 * failed batch changes any map (a sliding-window batch whose history does not fit fails
 * with -ENOSPC when its tail starts). The overflow
 * admission flag runs each batch whole on the context stream (no overlap, but still no host
 * synchronization per call); so does every
 * batch with on = 2 (a caller that reuses input buffers in stream order); timed batches
 * (fsx_enable_timing) run unpipelined. on = 0 turns it off. on = 1 also allocates a second
 * table set (fixed window / token bucket, tables of <= 2^25 slots) so that fsx_reset between
 * pipelined batches does not wait for them. */
int fsx_set_pipeline(fsx_ctx *ctx, int on);
/* Order a caller's hipStream_t after the batches enqueued so far, without a host
 * synchronization: `hip_stream` waits for the context stream's work and for every split
 * tail already enqueued. A pipelined batch's tail is enqueued by the next batch call (beside
 * its parse) or by any other entry point, so with all = 0 the last split batch is NOT
 * covered — the caller keeps overlapping it with the next batch and waits for batch j after
 * enqueueing batch j + 1 (the sharded plane's owners, flowsentryx_amd/shard.py); all = 1
 * enqueues that tail first and covers every batch. */
int fsx_stream_wait_batches(fsx_ctx *ctx, void *hip_stream, int all);

/* Replaces fsx() (src/fsx_kern.c:96-347) over a batch of n packets in arrival
 * order. Host pointers; hdr is n*64 bytes; verdict receives n bytes (1/2).
 * Map state and stats carry over between calls exactly as the BPF maps do. */
int fsx_verdict_batch(fsx_ctx *ctx, const uint8_t *hdr, const uint32_t *len,
                      const uint64_t *ts_ns, size_t n, uint8_t *verdict);
/* Same with device (HBM-resident) pointers, enqueued on the context stream.
 * Returns after enqueue; errors detected on the device surface at fsx_sync. */
int fsx_verdict_batch_device(fsx_ctx *ctx, const uint8_t *d_hdr, const uint32_t *d_len,
                             const uint64_t *d_ts, size_t n, uint8_t *d_verdict);

/* The full hot path on one device batch: verdicts and map state exactly as
 * fsx_verdict_batch_device, plus, for every distinct source IP of the batch, its
 * key (16 bytes, IPv4 in the first 4), family (4 or 6), the eight flow features of
 * model/model.py:117 (d_features may be NULL) and, when a model is
 * loaded, its q8 probability and decision (model/model.py:132-137, :206). Source
 * outputs are indexed 0..sources-1 (sources = fsx_last_batch_info()[1] after
 * fsx_sync); flow_cap bounds the rows written. */
int fsx_process_batch_device(fsx_ctx *ctx, const uint8_t *d_hdr, const uint32_t *d_len,
                             const uint64_t *d_ts, size_t n, uint8_t *d_verdict,
                             uint8_t *d_keys16, uint8_t *d_family, float *d_features,
                             float *d_prob, uint8_t *d_malicious, size_t flow_cap);

/* BPF map syscalls on the five reference maps (bpf_map_*_elem semantics). */
int fsx_map_lookup(fsx_ctx *ctx, int map_id, const void *key, void *value);
int fsx_map_update(fsx_ctx *ctx, int map_id, const void *key, const void *value,
                   uint64_t flags);
int fsx_map_delete(fsx_ctx *ctx, int map_id, const void *key);
/* BPF_MAP_UPDATE_BATCH analogue (flags = FSX_BPF_ANY): n entries of map 1..6, keys and
 * values in the map's byte layouts, keys distinct. All or nothing: when the new sources
 * would exceed max_entries the call fails with -ENOSPC and no map changes (restore of a
 * map_dump after a restart, bulk rule-table loads). */
int fsx_map_update_batch(fsx_ctx *ctx, int map_id, const void *keys, const void *values, size_t n,
                         uint64_t flags);
/* Copy up to cap entries (unordered) into keys/values; *n_out = entries present. */
int fsx_map_dump(fsx_ctx *ctx, int map_id, void *keys, void *values, size_t cap,
                 size_t *n_out);
int fsx_get_stats(fsx_ctx *ctx, fsx_stats *out);
/* Empty every per-source map and zero the stats (a fresh program load). The prefix
 * blocklists are operator configuration, like the loaded model, and stay. With pipelined
 * batches in flight (fsx_set_pipeline 1; fixed window / token bucket) it does not wait for
 * them: a second set of tables is swapped in and cleared on the device, and the next batch
 * overlaps their tails; an in-flight batch's error is then returned by the next fsx_sync
 * (it changed nothing the reset keeps) and does not cancel the batches after the reset. */
int fsx_reset(fsx_ctx *ctx);

/* Scoring (model/model.py:132-137, decision model/model.py:206). */
int fsx_load_q8_model(fsx_ctx *ctx, const fsx_q8_model *model);
int fsx_score(fsx_ctx *ctx, const float *features, size_t n, float *prob,
              uint8_t *malicious);
int fsx_score_device(fsx_ctx *ctx, const float *d_features, size_t n, float *d_prob,
                     uint8_t *d_malicious);

/* One global batch's flow features delivered over several calls (the owner side of the
 * sharded path, where a source's packets arrive in sub-batches, in global arrival order):
 * after fsx_flows_begin, every fsx_process_batch_device / fsx_process_records_device call
 * merges its per-source sums into the source's running sums (table slot) instead of writing
 * rows (its keys/family/feature/score pointers may be NULL); fsx_flows_end writes one row
 * per source merged since fsx_flows_begin — exactly the row one call over the whole batch
 * would give — and the row count to *d_rows (device pointer; NULL: none). Asynchronous.
 * Rows are in no particular order; with cap < rows, which rows are written is unspecified
 * (*d_rows still counts all of them). The calls' own flow_cap does not limit the merge. */
int fsx_flows_begin(fsx_ctx *ctx);
int fsx_flows_end(fsx_ctx *ctx, uint8_t *d_keys16, uint8_t *d_family, float *d_features,
                  float *d_prob, uint8_t *d_malicious, size_t cap, uint64_t *d_rows);

/* Per-source-IP flow features (build-defined) for the packets of
 * one batch (host pointers; the maps are not touched). n_flows_out = distinct
 * source IPs; up to cap rows of keys (16 B), family (4/6) and features (8 x fp32,
 * model/model.py:117 order) are written, in no particular order. */
int fsx_flow_features(fsx_ctx *ctx, const uint8_t *hdr, const uint32_t *len,
                      const uint64_t *ts_ns, size_t n, size_t cap, uint8_t *keys16,
                      uint8_t *family, float *features, size_t *n_flows_out);

/* ---- hash(src IP) sharding over G GPUs (SURVEY.md §8 e; host protocol in
 * flowsentryx_amd/shard.py). Every rank holds a contiguous slice of the arrival stream;
 * every source IP has one owner rank that runs the limiter on all of its packets, so
 * a sharded run equals the 1-GPU run. No reference counterpart: the reference is one
 * XDP program per host (src/fsx_kern.c:96-97). */
#define FSX_MAX_SHARDS 64
#define FSX_SHARD_RECORD_BYTES 32   /* {u32 key[4]; u64 ts; u32 len; u16 dport; u8 family; u8 pad} */

/* Owner rank of a source: key16 = raw address (IPv4 in the first 4 bytes), family 4/6.
 * Host-only (no device work). */
uint32_t fsx_shard_owner(const uint8_t *key16, int family, uint32_t n_shards);
#define FSX_SHARD_RECORD16_BYTES 16 /* {u32 ipv4 key; u16 len; u16 dport; u64 ts} */
#define FSX_SHARD_PACK_ERR 1        /* d_counts[n_shards + 1] of a failed placement */
#define FSX_SHARD_BLOCK_BYTES 32    /* {u32 key[4]; u64 till; u32 tag (1 v4, 2 v6); u32 pad} */
#define FSX_SHARD_FILTER_BLOCKLIST 1u
#define FSX_SHARD_COMPACT 2u
#define FSX_SHARD_DROP_RECORDS 4u
#define FSX_SHARD_REGIONS 8u

/* Parse a device batch and partition its IP packets by owner, stable in arrival order:
 * d_records (n * 32 bytes capacity) receives the records owner by owner, d_send_idx the
 * local packet index of every record, d_counts[n_shards] the records per owner.
 * Packets that never reach a limiter get their verdict in d_verdict here (frames too
 * short for their header: DROP; non-IP: PASS; src/fsx_kern.c:123-148). With
 * FSX_SHARD_FILTER_BLOCKLIST, IP packets whose source is in the context's blocklist
 * replica with till > 0 and now <= till are dropped here (src/fsx_kern.c:189-215) and
 * counted in d_counts[n_shards] (the caller adds them to stats_map.dropped); exact only
 * when timestamps are non-decreasing over all batches so far (fsx_shard_clock_device).
 * With FSX_SHARD_COMPACT, d_counts has n_shards + 2 entries and d_counts[n_shards + 1]
 * receives the record size written: FSX_SHARD_RECORD16_BYTES when no IP packet of the
 * slice is IPv6 or 64 KiB or longer, else FSX_SHARD_RECORD_BYTES — or FSX_SHARD_PACK_ERR
 * when the placement failed on the device (a bounded look-back timed out; the caller must
 * treat the pack as failed). With
 * FSX_SHARD_DROP_RECORDS (and the filter), the replica-dropped packets are written as
 * records too, after every owner's run, in arrival order (d_counts[n_shards] of them; the
 * first sum(d_counts[0..n_shards)) records are the ones to send), so the arrival rank can
 * take their flow sums (fsx_flow_partials_records_device). With FSX_SHARD_REGIONS every
 * owner has a region of n records instead: owner o's records (and d_send_idx entries) start at
 * record o * n, the replica-dropped ones at n_shards * n — d_records holds (n_shards + 1) * n
 * records of 32 bytes, d_send_idx as many entries; with FSX_SHARD_COMPACT too, the records
 * are placed as the headers are parsed (one pass: DESIGN.md §7). */
int fsx_shard_pack_device(fsx_ctx *ctx, const uint8_t *d_hdr, const uint32_t *d_len,
                          const uint64_t *d_ts, size_t n, uint32_t n_shards, uint32_t flags,
                          uint8_t *d_verdict, void *d_records, uint32_t *d_send_idx,
                          uint64_t *d_counts);
/* The same with the replica filter decided on the device: the blocklist filter applies iff
 * *d_filter != 0 (fsx_shard_filter_plan_device), so no host read is needed to decide it. */
int fsx_shard_pack_filtered_device(fsx_ctx *ctx, const uint8_t *d_hdr, const uint32_t *d_len,
                                   const uint64_t *d_ts, size_t n, uint32_t n_shards, uint32_t flags,
                                   const uint32_t *d_filter, uint8_t *d_verdict, void *d_records,
                                   uint32_t *d_send_idx, uint64_t *d_counts);
/* The replica filter's decision for each of k sub-batches, on the device: d_clocks holds the
 * all-gathered {min, max, decreases} (fsx_shard_clock_device) of every rank's piece of every
 * sub-batch ([n_shards][k][3] u64; an empty piece is {~0, 0, 0}); d_filter[j] = 1 when the
 * global clock (rank 0's piece, then rank 1's, ...) does not go back up to the end of
 * sub-batch j, which makes the filter exact. */
int fsx_shard_filter_plan_device(fsx_ctx *ctx, const uint64_t *d_clocks, uint32_t n_shards, uint32_t k,
                                 uint32_t *d_filter);
/* Flow partial: the exact flow sums of one source over a run of its packets
 * in arrival order, with the run's first / last timestamp and its first packet's L4
 * destination port; u128 sums as {low, high} u64 words. */
#define FSX_FLOW_PARTIAL_BYTES 112
typedef struct fsx_flow_partial {
    uint32_t key[4];       /* raw source address words (IPv4: key[0]) */
    uint32_t tag;          /* 1 IPv4, 2 IPv6 */
    uint32_t dport;
    uint64_t n, s1, dmax;  /* packets, sum of frame lengths, largest inter-arrival time */
    uint64_t first_ts, last_ts;
    uint64_t s2[2], d1[2], d2[2];   /* sum L^2, sum d, sum d^2 (d: inter-arrival ns) */
} fsx_flow_partial;
/* Arrival side of the blocklist filter with flow features: the flow partial of every
 * source of n exchange records (rec_bytes FSX_SHARD_RECORD_BYTES or
 * FSX_SHARD_RECORD16_BYTES, in arrival order) into the run of its owner: d_partials holds
 * n_shards runs of cap_per_shard partials (run o from o * cap_per_shard), d_counts[o] =
 * sources of owner o (beyond cap_per_shard: counted, not written). Touches no map state. */
int fsx_flow_partials_records_device(fsx_ctx *ctx, const void *d_records, size_t n, uint32_t rec_bytes,
                                     uint32_t n_shards, void *d_partials, size_t cap_per_shard,
                                     uint64_t *d_counts);
/* Owner side, between fsx_flows_begin and fsx_flows_end: merge m partials of distinct
 * sources into their running sums, as if the partial's packets were processed right after
 * everything merged so far (a source absent from the maps is skipped: the protocol sends
 * partials only for sources of this owner's blocklist). */
int fsx_flows_merge_device(fsx_ctx *ctx, const void *d_partials, size_t m);
/* The same for min(*d_count, cap) partials: a fixed-capacity exchange block whose count is
 * on the device (no host read). */
int fsx_flows_merge_counted_device(fsx_ctx *ctx, const void *d_partials, size_t cap, const uint64_t *d_count);
/* d_out3 = {min ts, max ts, 1 if some ts decreases in arrival order}. */
int fsx_shard_clock_device(fsx_ctx *ctx, const uint64_t *d_ts, size_t n, uint64_t *d_out3);
/* Every live blacklist entry (till > 0) of this context's maps as FSX_SHARD_BLOCK_BYTES
 * records; *d_count = entries present (records beyond cap are not written). */
int fsx_blocklist_export_device(fsx_ctx *ctx, void *d_entries, size_t cap, uint64_t *d_count);
/* Replace the context's blocklist replica with m all-gathered entries (distinct keys). */
int fsx_blocklist_replica_device(fsx_ctx *ctx, const void *d_entries, size_t m);
/* The same from n_blocks all-gathered fixed-capacity blocks, each FSX_SHARD_BLOCK_BYTES of
 * header (int64 entry count first) then cap entries, as fsx_blocklist_export_device fills
 * them (entries beyond cap are left out: a missing entry only sends its packets to their
 * owner, which decides them exactly). No host read. */
int fsx_blocklist_replica_blocks_device(fsx_ctx *ctx, const void *d_blocks, uint32_t n_blocks, size_t cap);
/* Owner side: m received records -> header records + len + ts for the batch entry points
 * (same source key, family, frame length, timestamp and L4 destination port). */
int fsx_shard_unpack_device(fsx_ctx *ctx, const void *d_records, size_t m, uint8_t *d_hdr,
                            uint32_t *d_len, uint64_t *d_ts);
/* Same for m compact 16-byte IPv4 records. */
int fsx_shard_unpack16_device(fsx_ctx *ctx, const void *d_records, size_t m, uint8_t *d_hdr,
                              uint32_t *d_len, uint64_t *d_ts);
/* Owner side, record mode: the batch pipeline straight on n received exchange records
 * of rec_bytes each (FSX_SHARD_RECORD_BYTES or FSX_SHARD_RECORD16_BYTES; one format per
 * call), in their order — verdicts and map state exactly as fsx_verdict_batch_device /
 * fsx_process_batch_device on the header records fsx_shard_unpack_device would build,
 * without building them. */
int fsx_verdict_records_device(fsx_ctx *ctx, const void *d_records, size_t n, uint32_t rec_bytes,
                               uint8_t *d_verdict);
int fsx_process_records_device(fsx_ctx *ctx, const void *d_records, size_t n, uint32_t rec_bytes,
                               uint8_t *d_verdict, uint8_t *d_keys16, uint8_t *d_family,
                               float *d_features, float *d_prob, uint8_t *d_malicious,
                               size_t flow_cap);
/* Origin side: d_verdict[d_send_idx[i]] = d_ret[i] for the m returned verdicts. */
int fsx_shard_scatter_device(fsx_ctx *ctx, const uint8_t *d_ret, const uint32_t *d_send_idx,
                             size_t m, uint8_t *d_verdict);
/* The same for a FSX_SHARD_REGIONS pack: d_ret holds the m returned verdicts owner by owner
 * (d_counts[o] of owner o, the pack's counts), d_send_idx the pack's regions of `region`
 * entries (its n). */
int fsx_shard_scatter_regions_device(fsx_ctx *ctx, const uint8_t *d_ret, const uint32_t *d_send_idx,
                                     size_t m, size_t region, const uint64_t *d_counts, uint32_t n_shards,
                                     uint8_t *d_verdict);

/* ---- pcap ingest (SURVEY.md §8 f). Classic pcap records (the 24-byte file header is
 * the caller's): FSX_PCAP_NANOSECONDS for magic 0xA1B23C4D, FSX_PCAP_SWAPPED when the
 * magic reads byte-swapped. The frame length is the record's original length (what
 * data_end - data is in XDP, src/fsx_kern.c:123). */
#define FSX_PCAP_NANOSECONDS 1u
#define FSX_PCAP_SWAPPED 2u
/* Host only: index up to cap complete records of buf[0, size): data offset, captured
 * and original length, timestamp in ns; *consumed = bytes of the indexed records. */
int fsx_pcap_index(const uint8_t *buf, size_t size, uint32_t flags, uint64_t *data_off,
                   uint32_t *caplen, uint32_t *origlen, uint64_t *ts_ns, size_t cap,
                   size_t *n_out, size_t *consumed);
/* Device: 64-byte header records (first min(caplen, 64) bytes, zero padded) of n indexed
 * records from an HBM copy of the pcap bytes. */
int fsx_pcap_records_device(fsx_ctx *ctx, const uint8_t *d_buf, const uint64_t *d_data_off,
                            const uint32_t *d_caplen, size_t n, uint8_t *d_hdr);

/* Facts about the last batch (after fsx_sync): info[0] IP packets, [1] distinct
 * source IPs, [2] sources new to the maps, [3] any IPv6, [4] non-monotone clock,
 * [5] max frame length, [6] max timestamp, [7] allowed, [8] dropped, [9] packets
 * dropped by a prefix rule (counted in [8], not in [0]), [10] 1 when (ts, len) travelled with the sort as payload
 * words (timestamps within 2^40 ns of the batch minimum, frame lengths < 2^24), 0 when
 * they were gathered by index, [11] IP packets of non-heavy sources (the entries the
 * later sort passes covered), [12] sources evicted before the batch
 * (FSX_FLAG_EVICT_IDLE), [13] 1 when the heavy sources' verdicts and flow rows were
 * computed outside the sort, 0 on the run path, [14] / [15] sources admitted
 * / transient (FSX_FLAG_OVERFLOW_ADMIT), [16] / [17] fixed-window batches since fsx_open
 * (not cleared by fsx_reset) whose heavy sources took the unsorted path / the run path,
 * [18] 1 when the batch took the home-ordered inserts (FSX_FLAG_ORDERED_INSERTS).
 * Returns the number of entries written. */
int fsx_last_batch_info(fsx_ctx *ctx, uint64_t *info, int cap);

/* Per-kernel device timing for the benchmark: while enabled, every batch records a
 * HIP event after each kernel on the context stream. fsx_last_timings returns, per
 * kernel name, the mean device time per batch and the launches per batch over all
 * batches since the previous call (then resets). */
int fsx_enable_timing(fsx_ctx *ctx, int on);
int fsx_last_timings(fsx_ctx *ctx, float *ms_per_batch, float *launches_per_batch,
                     char *names, int cap, int name_len, int *count);

#ifdef __cplusplus
}
#endif
#endif /* FSX_HIP_H */
