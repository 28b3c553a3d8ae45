/*
 * fsx_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * Plain-C restatement of FlowSentryX's packet-verdict path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker. It is
 * never linked into libfsx_hip.so and nothing on the product path calls it.
 *
 * Restated reference (paths relative to the FlowSentryX tree):
 *   parse            src/parsing_helper.h:49-66 (parse_ethhdr), :69-107 (parse_ip6hdr),
 *                    :111-136 (parse_ip4hdr); dispatch src/fsx_kern.c:123-148
 *   maps             src/fsx_kern.c:56-94, value layouts src/fsx_struct.h:11-22
 *   fixed window     src/fsx_kern.c:150-346 (blacklist :159-216, ip_stats :225-284,
 *                    threshold + blacklist insert :308-336, allowed :340-346)
 *   quantized model  model/model.py:124-137 forward, decision model/model.py:206,
 *                    weights src/model_weights.pth; arithmetic of torch 2.10's
 *                    x86/fbgemm quantized kernels (quantize by multiplying with the
 *                    fp32 inverse scale; requantize as (acc + bias/(s_in*s_w)) * M
 *                    with cvtps_epi32 overflow -> INT32_MIN; quantized sigmoid with
 *                    output qparams (1/256, 0)).
 *   build-defined    sliding window, token bucket, flow features: DESIGN.md §4-§5
 *                    (no reference code exists: README.md:155-162, src/fsx_kern_ml.c:1-16);
 *                    prefix blocklists DESIGN.md §4.3 (the reference's TODO.md:251 defers
 *                    LPM; BPF_MAP_TYPE_LPM_TRIE key/lookup semantics).
 *
 * Pinning: parse is checked against the reference's own
 * parsing_helper.h compiled by oracle/Makefile into oracle/_ref/; the fixed window
 * against the known-answer behaviours recorded from the reference program
 * (tests/golden/kat_fixed_window.json); scoring against vectors
 * produced by torch with the reference weights (tests/golden/make_score_vectors.py).
 * Sliding window, token bucket, features, prefix rules: parity unpinned (no reference).
 *
 * Semantics are sequential, single-CPU, arrival order. Maps never evict: an insert
 * into a full map sets the context error (the reference LRU would evict an
 * unspecified entry, SURVEY.md §7 "LRU eviction is not reproducible").
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../flowsentryx_amd/csrc/fsx_synth_common.h"

#define XDP_DROP 1
#define XDP_PASS 2

enum { CLS_DROP_PARSE = 0, CLS_PASS_NONIP = 1, CLS_V4 = 2, CLS_V6 = 3 };

/* ------------------------------------------------------------------ parse */
/* Returns the class; writes the source-address key (4 or 16 raw bytes). */
int fsxo_parse(const uint8_t *f, uint32_t len, uint8_t key[16]) {
    /* parse_ethhdr: 14-byte bound check, returns h_proto (no VLAN handling) */
    if (len < 14) return CLS_DROP_PARSE;
    uint16_t proto = (uint16_t)((f[12] << 8) | f[13]);
    if (proto != 0x86DD && proto != 0x0800) return CLS_PASS_NONIP;
    if (proto == 0x86DD) {
        /* parse_ip6hdr: 40-byte bound check; key = saddr (bytes 22..37) */
        if (len < 14 + 40) return CLS_DROP_PARSE;
        memcpy(key, f + 22, 16);
        return CLS_V6;
    }
    /* parse_ip4hdr: fixed 20-byte bound, IHL/version never checked; key = saddr */
    if (len < 14 + 20) return CLS_DROP_PARSE;
    memcpy(key, f + 26, 4);
    memset(key + 4, 0, 12);
    return CLS_V4;
}

/* ------------------------------------------------------------------ maps */
typedef struct omap {
    size_t cap, count, max_entries;
    uint32_t klen, vlen;
    uint8_t *used;
    uint8_t *keys;
    uint8_t *vals;
} omap;

static uint64_t omap_hash(const uint8_t *k, uint32_t klen) {
    uint64_t h = 0x12345678ull;
    for (uint32_t i = 0; i < klen; i += 4) {
        uint32_t w;
        memcpy(&w, k + i, 4);
        h = fsx_splitmix64(h ^ w);
    }
    return h;
}

static int omap_init(omap *m, size_t max_entries, uint32_t klen, uint32_t vlen) {
    size_t cap = 16;
    while (cap < max_entries * 2 + 2) cap <<= 1;
    m->cap = cap; m->count = 0; m->max_entries = max_entries;
    m->klen = klen; m->vlen = vlen;
    m->used = (uint8_t *)calloc(cap, 1);
    m->keys = (uint8_t *)calloc(cap, klen);
    m->vals = (uint8_t *)calloc(cap, vlen);
    return (m->used && m->keys && m->vals) ? 0 : -ENOMEM;
}

static void omap_free(omap *m) { free(m->used); free(m->keys); free(m->vals); }

static void omap_clear(omap *m) { memset(m->used, 0, m->cap); m->count = 0; }

static void *omap_lookup(omap *m, const uint8_t *k) {
    size_t i = omap_hash(k, m->klen) & (m->cap - 1);
    while (m->used[i]) {
        if (!memcmp(m->keys + i * m->klen, k, m->klen)) return m->vals + i * m->vlen;
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}

/* BPF_ANY update; returns 0 or -ENOSPC. */
static int omap_update(omap *m, const uint8_t *k, const void *v) {
    size_t i = omap_hash(k, m->klen) & (m->cap - 1);
    while (m->used[i]) {
        if (!memcmp(m->keys + i * m->klen, k, m->klen)) {
            memcpy(m->vals + i * m->vlen, v, m->vlen);
            return 0;
        }
        i = (i + 1) & (m->cap - 1);
    }
    if (m->count >= m->max_entries) return -ENOSPC;
    m->used[i] = 1;
    memcpy(m->keys + i * m->klen, k, m->klen);
    memcpy(m->vals + i * m->vlen, v, m->vlen);
    m->count++;
    return 0;
}

/* Backward-shift deletion for linear probing. */
static int omap_delete(omap *m, const uint8_t *k) {
    size_t mask = m->cap - 1;
    size_t i = omap_hash(k, m->klen) & mask;
    while (m->used[i]) {
        if (!memcmp(m->keys + i * m->klen, k, m->klen)) break;
        i = (i + 1) & mask;
    }
    if (!m->used[i]) return -ENOENT;
    m->used[i] = 0;
    m->count--;
    size_t j = i;
    for (;;) {
        j = (j + 1) & mask;
        if (!m->used[j]) break;
        size_t h = omap_hash(m->keys + j * m->klen, m->klen) & mask;
        /* can the entry at j move to the hole at i? */
        int move = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
        if (move) {
            m->used[i] = 1;
            memcpy(m->keys + i * m->klen, m->keys + j * m->klen, m->klen);
            memcpy(m->vals + i * m->vlen, m->vals + j * m->vlen, m->vlen);
            m->used[j] = 0;
            i = j;
        }
    }
    return 0;
}

static size_t omap_dump(omap *m, uint8_t *keys, uint8_t *vals, size_t cap) {
    size_t n = 0;
    for (size_t i = 0; i < m->cap; ++i) {
        if (!m->used[i]) continue;
        if (n < cap) {
            if (keys) memcpy(keys + n * m->klen, m->keys + i * m->klen, m->klen);
            if (vals) memcpy(vals + n * m->vlen, m->vals + i * m->vlen, m->vlen);
        }
        n++;
    }
    return n;
}

/* ------------------------------------------------------------------ context */
typedef struct fsxo_config {
    uint64_t pps_threshold, bps_threshold, window_ns, block_ns, max_entries;
    uint64_t tb_rate, tb_burst;
    int32_t limiter;
    int32_t flags;      /* FSXO_EVICT_IDLE (include/fsx_hip.h FSX_FLAG_EVICT_IDLE) */
} fsxo_config;

/* Opt-in overflow policy, build-defined (parity unpinned like the
 * reference's LRU): before a fixed-window batch of n packets, when the tracked sources
 * plus n exceed max_entries, every idle source is evicted. Idle at now0 = the batch's
 * smallest timestamp: its window has expired (no ip_stats entry, or now0 - track_time >
 * window, the reset test of src/fsx_kern.c:245), it holds no live blacklist entry (none,
 * till 0, or now0 > till, src/fsx_kern.c:189-204) and no token-bucket state. A tracked
 * source is one the GPU table holds a slot for: every source that reached the per-source
 * maps (after the prefix rules) or was written by a map update; map deletes do not
 * untrack it. */
#define FSXO_EVICT_IDLE 4
/* Opt-in overflow policy FSX_FLAG_OVERFLOW_ADMIT (include/fsx_hip.h, DESIGN.md §2.2;
 * build-defined, parity unpinned): in arrival order, a source that is not tracked when its
 * first packet of the batch reaches the per-source maps is admitted (tracked, the maps as
 * usual) while fewer than max_entries sources are tracked, else it is transient for the
 * batch: its packets run against maps of their own (c->tr) that start empty with the batch
 * and are never visible; stats_map counts every verdict. */
#define FSXO_OVERFLOW_ADMIT 8

typedef struct ip_stats { uint64_t pps, bps, track_time; } ip_stats;  /* fsx_struct.h:17-22 */
typedef struct tb_state { uint64_t tokens, last; } tb_state;

enum { MAP_STATS = 0, MAP_V4_STATS = 1, MAP_V6_STATS = 2, MAP_V4_BL = 3, MAP_V6_BL = 4,
       MAP_V4_TB = 5, MAP_V6_TB = 6, MAP_V4_PREFIX = 7, MAP_V6_PREFIX = 8 };
#define PREFIX_MAX_ENTRIES 65536

typedef struct sw_log { uint64_t *t; uint32_t *l; size_t n, cap; } sw_log;

typedef struct fsxo_ctx {
    fsxo_config cfg;
    omap m[7];
    /* prefix blocklists: {u32 prefixlen; addr bytes, bits past prefixlen zero} -> till */
    omap pfx[2];
    uint32_t pfx_len_cnt[2][129];
    uint64_t allowed, dropped;      /* stats_map, fsx_struct.h:11-15 */
    int err;
    /* sliding window logs, indexed by a side map key -> slot */
    omap swidx[2];
    /* FSXO_EVICT_IDLE: tracked sources per family (key -> unused byte) */
    omap src[2];
    uint64_t evicted_last;
    /* FSXO_OVERFLOW_ADMIT: the batch's transient sources' maps, and the batch's counts */
    struct fsxo_ctx *tr;
    uint64_t admitted_last, transient_last;
    sw_log *logs;
    size_t nlogs, caplogs;
} fsxo_ctx;

void fsxo_config_default(fsxo_config *c) {
    c->pps_threshold = 1000;        /* src/fsx_kern.c:309 */
    c->bps_threshold = 125000000;   /* src/fsx_kern.c:310 */
    c->window_ns = 1000000000ull;   /* src/fsx_kern.c:245 */
    c->block_ns = 10000000000ull;   /* src/fsx_kern.c:308,317 */
    c->max_entries = 100000;        /* src/fsx_struct.h:7 */
    c->tb_rate = 1000;              /* nano-tokens per ns = 1000 tokens/s */
    c->tb_burst = 1000;             /* tokens */
    c->limiter = 0;
    c->flags = 0;
}

fsxo_ctx *fsxo_open(const fsxo_config *cfg) {
    fsxo_ctx *c = (fsxo_ctx *)calloc(1, sizeof(*c));
    if (!c) return NULL;
    c->cfg = *cfg;
    size_t me = cfg->max_entries;
    int r = 0;
    r |= omap_init(&c->m[MAP_STATS], 1, 4, 16);
    r |= omap_init(&c->m[MAP_V4_STATS], me, 4, 24);
    r |= omap_init(&c->m[MAP_V6_STATS], me, 16, 24);
    r |= omap_init(&c->m[MAP_V4_BL], me, 4, 8);
    r |= omap_init(&c->m[MAP_V6_BL], me, 16, 8);
    r |= omap_init(&c->m[MAP_V4_TB], me, 4, 16);
    r |= omap_init(&c->m[MAP_V6_TB], me, 16, 16);
    r |= omap_init(&c->swidx[0], me, 4, 8);
    r |= omap_init(&c->swidx[1], me, 16, 8);
    r |= omap_init(&c->pfx[0], PREFIX_MAX_ENTRIES, 8, 8);
    r |= omap_init(&c->pfx[1], PREFIX_MAX_ENTRIES, 20, 8);
    if (cfg->flags & (FSXO_EVICT_IDLE | FSXO_OVERFLOW_ADMIT)) {
        r |= omap_init(&c->src[0], me, 4, 1);
        r |= omap_init(&c->src[1], me, 16, 1);
    }
    if (r) return NULL;
    return c;
}

static void sw_free_logs(fsxo_ctx *c) {
    for (size_t i = 0; i < c->nlogs; ++i) { free(c->logs[i].t); free(c->logs[i].l); }
    free(c->logs);
    c->logs = NULL; c->nlogs = c->caplogs = 0;
}

void fsxo_close(fsxo_ctx *c) {
    if (!c) return;
    for (int i = 0; i < 7; ++i) omap_free(&c->m[i]);
    omap_free(&c->swidx[0]); omap_free(&c->swidx[1]);
    omap_free(&c->pfx[0]); omap_free(&c->pfx[1]);
    omap_free(&c->src[0]); omap_free(&c->src[1]);
    sw_free_logs(c);
    if (c->tr) fsxo_close(c->tr);
    free(c);
}

void fsxo_reset(fsxo_ctx *c) {
    for (int i = 0; i < 7; ++i) omap_clear(&c->m[i]);
    omap_clear(&c->swidx[0]); omap_clear(&c->swidx[1]);
    if (c->src[0].used) { omap_clear(&c->src[0]); omap_clear(&c->src[1]); }
    c->evicted_last = 0;
    c->admitted_last = c->transient_last = 0;
    sw_free_logs(c);   /* (the prefix blocklists stay: configuration, fsx_hip.h) */
    c->allowed = c->dropped = 0;
    c->err = 0;
}

int fsxo_error(const fsxo_ctx *c) { return c->err; }

void fsxo_get_stats(const fsxo_ctx *c, uint64_t out[2]) { out[0] = c->allowed; out[1] = c->dropped; }

/* FSXO_EVICT_IDLE / FSXO_OVERFLOW_ADMIT: the source (family v6, key) is tracked from now on. */
static void src_track(fsxo_ctx *c, int v6, const uint8_t *key) {
    if (!(c->cfg.flags & (FSXO_EVICT_IDLE | FSXO_OVERFLOW_ADMIT))) return;
    static const uint8_t one = 1;
    if (omap_lookup(&c->src[v6], key)) return;
    /* one capacity for both families, as the device table's */
    if (c->src[0].count + c->src[1].count >= c->cfg.max_entries || omap_update(&c->src[v6], key, &one))
        c->err = -ENOSPC;
}

static omap *map_of(fsxo_ctx *c, int map_id) {
    if (map_id < 1 || map_id > 6) return NULL;
    return &c->m[map_id];
}

/* ------------------------------------------------------------------ prefix rules */
/* Canonical rule key: prefixlen, then the address with every bit past prefixlen
 * cleared (network bit order: byte b holds bits 8b..8b+7, most significant first). */
static void prefix_canon(uint32_t plen, const uint8_t *addr, int alen, uint8_t *out) {
    memcpy(out, &plen, 4);
    for (int b = 0; b < alen; ++b) {
        int bits = (int)plen - 8 * b;
        uint8_t m = bits >= 8 ? 0xFF : bits <= 0 ? 0 : (uint8_t)(0xFF << (8 - bits));
        out[4 + b] = addr[b] & m;
    }
}

/* Longest-prefix match of addr over the rules of length <= maxlen; NULL if none. */
static uint64_t *prefix_match(fsxo_ctx *c, int v6, const uint8_t *addr, uint32_t maxlen) {
    const int alen = v6 ? 16 : 4;
    uint8_t k[20];
    for (int L = (int)maxlen; L >= 0; --L) {
        if (!c->pfx_len_cnt[v6][L]) continue;
        prefix_canon((uint32_t)L, addr, alen, k);
        uint64_t *v = (uint64_t *)omap_lookup(&c->pfx[v6], k);
        if (v) return v;
    }
    return NULL;
}

static int prefix_op(fsxo_ctx *c, int op, int map_id, const void *key, const void *val, void *out) {
    const int v6 = map_id == MAP_V6_PREFIX, alen = v6 ? 16 : 4;
    uint32_t plen;
    memcpy(&plen, key, 4);
    if (plen > (uint32_t)(8 * alen)) return -EINVAL;
    const uint8_t *addr = (const uint8_t *)key + 4;
    if (op == 0) {
        uint64_t *v = prefix_match(c, v6, addr, plen);
        if (!v) return -ENOENT;
        memcpy(out, v, 8);
        return 0;
    }
    uint8_t k[20];
    prefix_canon(plen, addr, alen, k);
    omap *m = &c->pfx[v6];
    if (op == 2) {
        int r = omap_delete(m, k);
        if (!r) c->pfx_len_cnt[v6][plen]--;
        return r;
    }
    int existed = omap_lookup(m, k) != NULL;
    int r = omap_update(m, k, val);
    if (!r && !existed) c->pfx_len_cnt[v6][plen]++;
    return r;
}

int fsxo_map_lookup(fsxo_ctx *c, int map_id, const void *key, void *val) {
    if (map_id == MAP_STATS) {
        uint64_t s[2] = {c->allowed, c->dropped};
        memcpy(val, s, 16);
        return 0;
    }
    if (map_id == MAP_V4_PREFIX || map_id == MAP_V6_PREFIX) return prefix_op(c, 0, map_id, key, NULL, val);
    omap *m = map_of(c, map_id);
    if (!m) return -EINVAL;
    void *v = omap_lookup(m, (const uint8_t *)key);
    if (!v) return -ENOENT;
    memcpy(val, v, m->vlen);
    return 0;
}

int fsxo_map_update(fsxo_ctx *c, int map_id, const void *key, const void *val) {
    if (map_id == MAP_STATS) {
        uint64_t s[2];
        memcpy(s, val, 16);
        c->allowed = s[0]; c->dropped = s[1];
        return 0;
    }
    if (map_id == MAP_V4_PREFIX || map_id == MAP_V6_PREFIX) return prefix_op(c, 1, map_id, key, val, NULL);
    omap *m = map_of(c, map_id);
    if (!m) return -EINVAL;
    int r = omap_update(m, (const uint8_t *)key, val);
    if (!r) src_track(c, map_id == MAP_V6_STATS || map_id == MAP_V6_BL || map_id == MAP_V6_TB, key);
    return r;
}

int fsxo_map_delete(fsxo_ctx *c, int map_id, const void *key) {
    if (map_id == MAP_V4_PREFIX || map_id == MAP_V6_PREFIX) return prefix_op(c, 2, map_id, key, NULL, NULL);
    omap *m = map_of(c, map_id);
    if (!m) return -EINVAL;
    return omap_delete(m, (const uint8_t *)key);
}

size_t fsxo_map_dump(fsxo_ctx *c, int map_id, void *keys, void *vals, size_t cap) {
    omap *m = map_id == MAP_V4_PREFIX ? &c->pfx[0] : map_id == MAP_V6_PREFIX ? &c->pfx[1] : map_of(c, map_id);
    if (!m) return 0;
    return omap_dump(m, (uint8_t *)keys, (uint8_t *)vals, cap);
}

/* ------------------------------------------------------------------ fixed window */
/* One packet through fsx(), src/fsx_kern.c:96-347, with now = ts. */
static int fixed_window_packet(fsxo_ctx *c, int v6, const uint8_t *key, uint32_t len,
                               uint64_t now) {
    omap *bl = &c->m[v6 ? MAP_V6_BL : MAP_V4_BL];
    omap *st = &c->m[v6 ? MAP_V6_STATS : MAP_V4_STATS];
    const fsxo_config *k = &c->cfg;

    /* :159-216 blacklist check */
    uint64_t *till = (uint64_t *)omap_lookup(bl, key);
    if (till != NULL && *till > 0) {
        if (now > *till) {
            omap_delete(bl, key);                       /* :193-204 */
        } else {
            c->dropped++;                               /* :208-211 */
            return XDP_DROP;                            /* :214 */
        }
    }
    /* :222-284 ip_stats */
    uint64_t pps = 0, bps = 0;
    ip_stats *s = (ip_stats *)omap_lookup(st, key);
    if (s) {
        if (now - s->track_time > k->window_ns) {       /* :245, u64 wraparound */
            s->pps = 0; s->bps = 0; s->track_time = now;
        } else {
            s->pps += 1;                                /* :258 */
            s->bps += len;                              /* :259 */
            pps = s->pps; bps = s->bps;                 /* :261-262 */
        }
    } else {
        ip_stats nw = {1, len, now};                    /* :267-271 */
        pps = nw.pps; bps = nw.bps;
        if (omap_update(st, key, &nw)) c->err = -ENOSPC;
    }
    /* :312 threshold */
    if (pps > k->pps_threshold || bps > k->bps_threshold) {
        uint64_t t = now + k->block_ns;                 /* :317 */
        if (omap_update(bl, key, &t)) c->err = -ENOSPC;
        c->dropped++;                                   /* :332 */
        return XDP_DROP;
    }
    c->allowed++;                                       /* :342 */
    return XDP_PASS;
}

/* ------------------------------------------------------------------ sliding window */
/* Build-defined. Per source IP, over non-blacklisted packets:
 *   - blacklist check exactly as the fixed window (shared blacklist maps);
 *   - entries leave the IP's log of counted packets from the oldest while
 *     now - t_oldest >= W (u64); then the packet is appended;
 *   - count = |log|, bytes = sum of lengths in the log (packet included);
 *   - count > P or bytes > B: blacklist until now + BLK, clear the log, DROP.
 *   - else PASS.
 * ipv{4,6}_stats_map mirror {count, bytes, oldest t in log} after each packet. */
static sw_log *sw_log_of(fsxo_ctx *c, int v6, const uint8_t *key) {
    uint64_t *slot = (uint64_t *)omap_lookup(&c->swidx[v6], key);
    if (slot) return &c->logs[*slot];
    if (c->nlogs == c->caplogs) {
        size_t nc = c->caplogs ? c->caplogs * 2 : 1024;
        sw_log *nl = (sw_log *)realloc(c->logs, nc * sizeof(sw_log));
        if (!nl) { c->err = -ENOMEM; return NULL; }
        c->logs = nl; c->caplogs = nc;
    }
    uint64_t idx = c->nlogs++;
    memset(&c->logs[idx], 0, sizeof(sw_log));
    if (omap_update(&c->swidx[v6], key, &idx)) { c->err = -ENOSPC; return NULL; }
    return &c->logs[idx];
}

static int sliding_window_packet(fsxo_ctx *c, int v6, const uint8_t *key, uint32_t len,
                                 uint64_t now) {
    omap *bl = &c->m[v6 ? MAP_V6_BL : MAP_V4_BL];
    omap *st = &c->m[v6 ? MAP_V6_STATS : MAP_V4_STATS];
    const fsxo_config *k = &c->cfg;
    uint64_t *till = (uint64_t *)omap_lookup(bl, key);
    if (till != NULL && *till > 0) {
        if (now > *till) omap_delete(bl, key);
        else { c->dropped++; return XDP_DROP; }
    }
    sw_log *lg = sw_log_of(c, v6, key);
    if (!lg) return XDP_DROP;
    /* drop expired entries from the oldest: while now - t_oldest >= W (u64) */
    size_t head = 0;
    while (head < lg->n && now - lg->t[head] >= k->window_ns) head++;
    if (head) {
        memmove(lg->t, lg->t + head, (lg->n - head) * sizeof(uint64_t));
        memmove(lg->l, lg->l + head, (lg->n - head) * sizeof(uint32_t));
        lg->n -= head;
    }
    if (lg->n == lg->cap) {
        size_t nc = lg->cap ? lg->cap * 2 : 8;
        uint64_t *nt = (uint64_t *)realloc(lg->t, nc * sizeof(uint64_t));
        uint32_t *nlen = (uint32_t *)realloc(lg->l, nc * sizeof(uint32_t));
        if (!nt || !nlen) { c->err = -ENOMEM; return XDP_DROP; }
        lg->t = nt; lg->l = nlen; lg->cap = nc;
    }
    lg->t[lg->n] = now; lg->l[lg->n] = len; lg->n++;
    uint64_t bytes = 0;
    for (size_t i = 0; i < lg->n; ++i) bytes += lg->l[i];
    uint64_t cnt = lg->n;
    ip_stats s = {cnt, bytes, lg->t[0]};
    if (cnt > k->pps_threshold || bytes > k->bps_threshold) {
        uint64_t t = now + k->block_ns;
        if (omap_update(bl, key, &t)) c->err = -ENOSPC;
        lg->n = 0;
        if (omap_update(st, key, &s)) c->err = -ENOSPC;
        c->dropped++;
        return XDP_DROP;
    }
    if (omap_update(st, key, &s)) c->err = -ENOSPC;
    c->allowed++;
    return XDP_PASS;
}

/* ------------------------------------------------------------------ token bucket */
/* Build-defined. State per IP {tokens (nano-tokens), last (ns)}.
 * Capacity C = burst * 1e9, cost 1e9 per packet, refill rate nano-tokens per ns.
 *   - blacklist check exactly as the fixed window (static rules still apply);
 *   - new IP: tokens = C, last = now;
 *   - y = min(C, tokens + (now - last) * rate) (u64 wrap of now-last as the
 *     reference's window test; saturating multiply/add), last = now;
 *   - y >= 1e9: tokens = y - 1e9, PASS; else tokens = 0, DROP (the partial token is
 *     discarded: x' = max(0, y - 1e9), a clamp-add map, so the GPU evaluates the
 *     recurrence as a scan); no blacklist insertions.
 * Capacity burst * 1e9 must stay <= 2^61 (fsx_open rejects larger bursts). */
#define TB_COST 1000000000ull
static int token_bucket_packet(fsxo_ctx *c, int v6, const uint8_t *key, uint32_t len,
                               uint64_t now) {
    (void)len;
    omap *bl = &c->m[v6 ? MAP_V6_BL : MAP_V4_BL];
    omap *tbm = &c->m[v6 ? MAP_V6_TB : MAP_V4_TB];
    const fsxo_config *k = &c->cfg;
    uint64_t *till = (uint64_t *)omap_lookup(bl, key);
    if (till != NULL && *till > 0) {
        if (now > *till) omap_delete(bl, key);
        else { c->dropped++; return XDP_DROP; }
    }
    uint64_t cap = k->tb_burst * TB_COST;
    tb_state *s = (tb_state *)omap_lookup(tbm, key);
    tb_state ns;
    uint64_t y;
    if (!s) {
        y = cap;
    } else {
        uint64_t dt = now - s->last;
        uint64_t add;
        if (k->tb_rate && dt > (UINT64_MAX / k->tb_rate)) add = UINT64_MAX;
        else add = dt * k->tb_rate;
        y = s->tokens + add;
        if (y < s->tokens) y = UINT64_MAX;
        if (y > cap) y = cap;
    }
    int v;
    if (y >= TB_COST) { ns.tokens = y - TB_COST; v = XDP_PASS; c->allowed++; }
    else { ns.tokens = 0; v = XDP_DROP; c->dropped++; }
    ns.last = now;
    if (omap_update(tbm, key, &ns)) c->err = -ENOSPC;
    return v;
}

/* ------------------------------------------------------------------ batch */
static int one_packet(fsxo_ctx *c, const uint8_t *hdr, uint32_t len, uint64_t ts) {
    uint8_t key[16];
    int cls = fsxo_parse(hdr, len, key);
    if (cls == CLS_DROP_PARSE) return XDP_DROP;        /* src/fsx_kern.c:124-127,139-140,146-147 */
    if (cls == CLS_PASS_NONIP) return XDP_PASS;        /* src/fsx_kern.c:128-131 */
    int v6 = cls == CLS_V6;
    /* prefix blocklist first: the longest matching rule decides */
    const uint64_t *till = prefix_match(c, v6, key, v6 ? 128 : 32);
    if (till && *till > 0 && ts <= *till) {
        c->dropped++;
        return XDP_DROP;
    }
    fsxo_ctx *m = c;   /* the maps this packet runs against */
    if ((c->cfg.flags & FSXO_OVERFLOW_ADMIT) && !omap_lookup(&c->src[v6], key)) {
        if (c->src[0].count + c->src[1].count < c->cfg.max_entries) {
            c->admitted_last++;                        /* admitted: tracked from now on */
        } else {                                       /* transient for this batch */
            m = c->tr;
            if (!omap_lookup(&m->src[v6], key)) {
                static const uint8_t one = 1;
                if (omap_update(&m->src[v6], key, &one)) c->err = -ENOSPC;
                c->transient_last++;
            }
        }
    }
    if (m == c) src_track(c, v6, key);
    int v;
    switch (c->cfg.limiter) {
    case 1: v = sliding_window_packet(m, v6, key, len, ts); break;
    case 2: v = token_bucket_packet(m, v6, key, len, ts); break;
    default: v = fixed_window_packet(m, v6, key, len, ts); break;
    }
    if (m != c) {   /* the transient maps' verdict counts go to stats_map */
        c->allowed += m->allowed; c->dropped += m->dropped;
        m->allowed = m->dropped = 0;
        if (m->err) c->err = m->err;
    }
    return v;
}

/* FSXO_EVICT_IDLE, before a batch of n packets with smallest timestamp now0. */
static void evict_idle(fsxo_ctx *c, size_t n, uint64_t now0) {
    c->evicted_last = 0;
    if (c->src[0].count + c->src[1].count + n <= c->cfg.max_entries) return;
    for (int v6 = 0; v6 < 2; ++v6) {
        omap *src = &c->src[v6];
        omap *st = &c->m[v6 ? MAP_V6_STATS : MAP_V4_STATS];
        omap *bl = &c->m[v6 ? MAP_V6_BL : MAP_V4_BL];
        omap *tb = &c->m[v6 ? MAP_V6_TB : MAP_V4_TB];
        /* the idle keys first (a delete moves entries of the map it walks) */
        uint8_t *gone = (uint8_t *)malloc(src->count * src->klen + 1);
        size_t ng = 0;
        for (size_t i = 0; i < src->cap; ++i) {
            if (!src->used[i]) continue;
            const uint8_t *k = src->keys + i * src->klen;
            const ip_stats *s = (const ip_stats *)omap_lookup(st, k);
            const uint64_t *till = (const uint64_t *)omap_lookup(bl, k);
            int live = (s && !(now0 - s->track_time > c->cfg.window_ns)) ||
                       (till && *till > 0 && !(now0 > *till)) || omap_lookup(tb, k) != NULL;
            if (!live) memcpy(gone + ng++ * src->klen, k, src->klen);
        }
        for (size_t j = 0; j < ng; ++j) {
            const uint8_t *k = gone + j * src->klen;
            omap_delete(src, k);
            omap_delete(st, k);
            omap_delete(bl, k);
        }
        free(gone);
        c->evicted_last += ng;
    }
}

uint64_t fsxo_evicted_last(const fsxo_ctx *c) { return c->evicted_last; }
void fsxo_admit_last(const fsxo_ctx *c, uint64_t out[2]) { out[0] = c->admitted_last; out[1] = c->transient_last; }

int fsxo_batch(fsxo_ctx *c, const uint8_t *hdr, const uint32_t *len, const uint64_t *ts,
               size_t n, uint8_t *verdict) {
    if ((c->cfg.flags & FSXO_EVICT_IDLE) && c->cfg.limiter == 0 && n) {
        uint64_t now0 = ts[0];
        for (size_t i = 1; i < n; ++i) now0 = ts[i] < now0 ? ts[i] : now0;
        evict_idle(c, n, now0);
    }
    if (c->cfg.flags & FSXO_OVERFLOW_ADMIT) {   /* fresh transient maps for this batch */
        c->admitted_last = c->transient_last = 0;
        if (c->tr && c->tr->cfg.max_entries < n) { fsxo_close(c->tr); c->tr = NULL; }
        if (!c->tr) {
            fsxo_config tc = c->cfg;
            tc.flags = FSXO_OVERFLOW_ADMIT;   /* (its src maps: the batch's transient sources) */
            tc.max_entries = n > 1024 ? n : 1024;
            c->tr = fsxo_open(&tc);
            if (!c->tr) return -ENOMEM;
        } else {
            fsxo_reset(c->tr);
        }
    }
    for (size_t i = 0; i < n; ++i)
        verdict[i] = (uint8_t)one_packet(c, hdr + i * 64, len[i], ts[i]);
    return c->err;
}

/* Parse only (for the golden parse vectors). */
void fsxo_parse_batch(const uint8_t *hdr, const uint32_t *len, size_t n, uint8_t *cls,
                      uint8_t *keys16) {
    for (size_t i = 0; i < n; ++i) cls[i] = (uint8_t)fsxo_parse(hdr + i * 64, len[i], keys16 + i * 16);
}

/* ------------------------------------------------------------------ sharded runner */
/* CPU baseline: T threads, one context each, IP-disjoint shards (owner = hash(key)
 * mod T). Each thread scans the whole stream and processes the packets it owns, so
 * the per-IP arrival order — and hence every verdict — equals the 1-thread run. */
typedef struct shard_arg {
    const fsxo_config *cfg;
    const uint8_t *hdr; const uint32_t *len; const uint64_t *ts;
    size_t n; uint8_t *verdict; int tid, nthreads;
    uint64_t allowed, dropped; int err;
} shard_arg;

static void *shard_main(void *p) {
    shard_arg *a = (shard_arg *)p;
    fsxo_ctx *c = fsxo_open(a->cfg);
    if (!c) { a->err = -ENOMEM; return NULL; }
    for (size_t i = 0; i < a->n; ++i) {
        uint8_t key[16];
        const uint8_t *h = a->hdr + i * 64;
        int cls = fsxo_parse(h, a->len[i], key);
        if (cls <= CLS_PASS_NONIP) {
            if (a->tid == 0) a->verdict[i] = cls == CLS_DROP_PARSE ? XDP_DROP : XDP_PASS;
            continue;
        }
        uint64_t hk = omap_hash(key, cls == CLS_V6 ? 16 : 4) ^ (uint64_t)cls;
        if ((int)(fsx_splitmix64(hk) % (uint64_t)a->nthreads) != a->tid) continue;
        a->verdict[i] = (uint8_t)one_packet(c, h, a->len[i], a->ts[i]);
    }
    a->allowed = c->allowed; a->dropped = c->dropped; a->err = c->err;
    fsxo_close(c);
    return NULL;
}

int fsxo_batch_sharded(const fsxo_config *cfg, const uint8_t *hdr, const uint32_t *len,
                       const uint64_t *ts, size_t n, uint8_t *verdict, int nthreads,
                       uint64_t stats_out[2]) {
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    shard_arg args[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; ++t) {
        shard_arg a = {cfg, hdr, len, ts, n, verdict, t, nthreads, 0, 0, 0};
        args[t] = a;
        pthread_create(&th[t], NULL, shard_main, &args[t]);
    }
    uint64_t al = 0, dr = 0;
    int err = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        al += args[t].allowed; dr += args[t].dropped;
        if (args[t].err) err = args[t].err;
    }
    stats_out[0] = al; stats_out[1] = dr;
    return err;
}

/* Persistent sharded runner (full-size parity checks in bench.py and the large GPU
 * tests): T contexts on IP-disjoint shards (the owner rule of shard_main) that keep
 * their maps across batches, so map dumps, stats and state carry equal one sequential
 * context's. Each shard's maps hold ceil(1.25 * max_entries / T) + 4096 sources (the hash
 * spreads sources evenly): -ENOSPC is not reproduced at max_entries exactly. Prefix
 * rules go to every shard; per-source map updates to the source's owner. */
typedef struct fsxo_shards { int T; fsxo_ctx *c[256]; } fsxo_shards;

static int shard_of(int v6, const uint8_t *key, int T) {
    const uint64_t hk = omap_hash(key, v6 ? 16 : 4) ^ (uint64_t)(v6 ? CLS_V6 : CLS_V4);
    return (int)(fsx_splitmix64(hk) % (uint64_t)T);
}

void fsxo_shards_close(fsxo_shards *h) {
    if (!h) return;
    for (int t = 0; t < h->T; ++t) fsxo_close(h->c[t]);
    free(h);
}

fsxo_shards *fsxo_shards_open(const fsxo_config *cfg, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (cfg->flags & FSXO_OVERFLOW_ADMIT) nthreads = 1;   /* admission follows the global arrival order */
    fsxo_shards *h = (fsxo_shards *)calloc(1, sizeof(*h));
    if (!h) return NULL;
    fsxo_config k = *cfg;
    if (nthreads > 1) k.max_entries = (5 * cfg->max_entries / 4 + nthreads - 1) / nthreads + 4096;
    h->T = nthreads;
    for (int t = 0; t < nthreads; ++t)
        if (!(h->c[t] = fsxo_open(&k))) { fsxo_shards_close(h); return NULL; }
    return h;
}

void fsxo_shards_reset(fsxo_shards *h) { for (int t = 0; t < h->T; ++t) fsxo_reset(h->c[t]); }

int fsxo_shards_map_update(fsxo_shards *h, int map_id, const void *key, const void *val) {
    if (map_id == MAP_V4_PREFIX || map_id == MAP_V6_PREFIX) {
        for (int t = 0; t < h->T; ++t) {
            int r = fsxo_map_update(h->c[t], map_id, key, val);
            if (r) return r;
        }
        return 0;
    }
    if (map_id < 1 || map_id > 6) return -EINVAL;
    const int v6 = map_id == MAP_V6_STATS || map_id == MAP_V6_BL || map_id == MAP_V6_TB;
    return fsxo_map_update(h->c[shard_of(v6, (const uint8_t *)key, h->T)], map_id, key, val);
}

typedef struct shards_arg {
    fsxo_ctx *c; const uint8_t *hdr; const uint32_t *len; const uint64_t *ts;
    size_t n; uint8_t *verdict; int tid, T;
} shards_arg;

static void *shards_main(void *p) {
    shards_arg *a = (shards_arg *)p;
    for (size_t i = 0; i < a->n; ++i) {
        uint8_t key[16];
        const uint8_t *f = a->hdr + i * 64;
        const int cls = fsxo_parse(f, a->len[i], key);
        if (cls <= CLS_PASS_NONIP) {
            if (a->tid == 0) a->verdict[i] = cls == CLS_DROP_PARSE ? XDP_DROP : XDP_PASS;
            continue;
        }
        if (shard_of(cls == CLS_V6, key, a->T) != a->tid) continue;
        a->verdict[i] = (uint8_t)one_packet(a->c, f, a->len[i], a->ts[i]);
    }
    return NULL;
}

int fsxo_shards_batch(fsxo_shards *h, const uint8_t *hdr, const uint32_t *len, const uint64_t *ts,
                      size_t n, uint8_t *verdict) {
    pthread_t th[256];
    shards_arg args[256];
    for (int t = 0; t < h->T; ++t) {
        shards_arg a = {h->c[t], hdr, len, ts, n, verdict, t, h->T};
        args[t] = a;
        pthread_create(&th[t], NULL, shards_main, &args[t]);
    }
    int err = 0;
    for (int t = 0; t < h->T; ++t) {
        pthread_join(th[t], NULL);
        if (h->c[t]->err) err = h->c[t]->err;
    }
    return err;
}

void fsxo_shards_stats(const fsxo_shards *h, uint64_t out[2]) {
    out[0] = out[1] = 0;
    for (int t = 0; t < h->T; ++t) { out[0] += h->c[t]->allowed; out[1] += h->c[t]->dropped; }
}

/* The shards' entries of map_id, concatenated (keys / vals may be NULL: count only). */
size_t fsxo_shards_dump(fsxo_shards *h, int map_id, void *keys, void *vals, size_t cap) {
    size_t n = 0;
    if (map_id == MAP_V4_PREFIX || map_id == MAP_V6_PREFIX)   /* identical on every shard */
        return fsxo_map_dump(h->c[0], map_id, keys, vals, cap);
    omap *m0 = map_of(h->c[0], map_id);
    if (!m0) return 0;
    for (int t = 0; t < h->T; ++t) {
        const size_t left = cap > n ? cap - n : 0;
        n += fsxo_map_dump(h->c[t], map_id, keys ? (uint8_t *)keys + n * m0->klen : NULL,
                           vals ? (uint8_t *)vals + n * m0->vlen : NULL, left);
    }
    return n;
}

/* ------------------------------------------------------------------ scoring */
typedef struct fsxo_q8_model {
    int8_t weight[8];
    float weight_scale, bias, in_scale;
    int32_t in_zero_point;
    float out_scale;
    int32_t out_zero_point;
} fsxo_q8_model;

/* cvtps_epi32: round-half-even; NaN / out of range -> INT32_MIN */
static int32_t cvt_ps_epi32(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
    return (int32_t)rintf(v);
}

/* quantize_per_tensor to quint8, fbgemm QuantizeAvx2 (the path every N x 8 input
 * takes): t = min_ps(x * fp32(1/scale), 2147483520) (NaN -> 2147483520),
 * r = cvtps_epi32(t) + zp (wrapping int32 add), clamp to [0, 255]. */
static int q8_quantize(float x, float inv, int zp) {
    const float lim = 2147483520.0f;
    float v = x * inv;
    float t = v < lim ? v : lim;
    int32_t r = (int32_t)((uint32_t)cvt_ps_epi32(t) + (uint32_t)zp);
    return r < 0 ? 0 : (r > 255 ? 255 : r);
}


/* Quantized sigmoid table: output quint8 with scale 1/256, zp 0. */
void fsxo_sigmoid_lut(float out_scale, int32_t out_zp, uint8_t lut[256]) {
    for (int q = 0; q < 256; ++q) {
        float x = (float)(q - out_zp) * out_scale;
        float s = 1.0f / (1.0f + expf(-x));
        float r = rintf(s * 256.0f);
        lut[q] = (uint8_t)(r > 255.0f ? 255.0f : (r < 0.0f ? 0.0f : r));
    }
}

/* Requantized linear output lq in [0,255] (fbgemm ReQuantizeOutput, float bias). */
int fsxo_q8_linear(const fsxo_q8_model *m, const float *x, int32_t *acc_out) {
    float inv = 1.0f / m->in_scale;
    int32_t acc = 0;
    for (int i = 0; i < 8; ++i) {
        int q = q8_quantize(x[i], inv, m->in_zero_point);
        acc += (q - m->in_zero_point) * (int32_t)m->weight[i];
    }
    if (acc_out) *acc_out = acc;
    float ats = m->in_scale * m->weight_scale;
    float M = ats / m->out_scale;
    float raw = (float)acc + m->bias / ats;
    int64_t r = (int64_t)cvt_ps_epi32(raw * M) + m->out_zero_point;
    return (int)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

void fsxo_score(const fsxo_q8_model *m, const float *feat, size_t n, float *p,
                uint8_t *dec, uint8_t *lq_out) {
    uint8_t lut[256];
    fsxo_sigmoid_lut(m->out_scale, m->out_zero_point, lut);
    for (size_t i = 0; i < n; ++i) {
        int lq = fsxo_q8_linear(m, feat + i * 8, NULL);
        float pr = (float)lut[lq] * 0.00390625f;
        if (p) p[i] = pr;
        if (dec) dec[i] = pr > 0.5f;                    /* model/model.py:206 */
        if (lq_out) lq_out[i] = (uint8_t)lq;
    }
}

/* ------------------------------------------------------------------ flow features */
/* Build-defined: per source IP over the batch's IP packets (any
 * verdict), in arrival order: n packets, lengths L_i, times t_i (ns).
 *   destination_port       L4 dst port of the first packet (UDP/TCP at IHL offset for
 *                          IPv4, fixed 54 for IPv6; 0 if not TCP/UDP or beyond 64 B)
 *   packet_length_mean     S1/n                      (S1 = sum L, S2 = sum L^2)
 *   packet_length_std      sqrt(var)
 *   packet_length_variance var = (n*S2 - S1^2) / (n*(n-1)), 0 if n < 2 (sample)
 *   average_packet_size    S1/n
 *   fwd_iat_mean           sum(d)/(n-1) in µs, d_i = t_i - t_{i-1} (ns), 0 if n < 2
 *   fwd_iat_std            sample std of d in µs, 0 if n < 3
 *   fwd_iat_max            max d in µs
 * Integer sums are exact (unsigned __int128); each float is computed in double from
 * them with the operation order written above, then rounded to fp32. */
typedef unsigned __int128 u128;

static double u128_to_double(u128 v) { return (double)v; }

static void finish_features(uint64_t n, u128 s1, u128 s2, u128 d1, u128 d2, uint64_t dmax,
                            uint32_t dport, float out[8]) {
    double dn = (double)n;
    double mean = u128_to_double(s1) / dn;
    double var = 0.0;
    if (n >= 2) {
        u128 num = (u128)n * s2 - s1 * s1;  /* >= 0 by Cauchy-Schwarz */
        var = u128_to_double(num) / (dn * (dn - 1.0));
    }
    double iat_mean = 0.0, iat_var = 0.0;
    if (n >= 2) iat_mean = u128_to_double(d1) / (double)(n - 1) / 1000.0;
    if (n >= 3) {
        uint64_t m = n - 1;
        u128 num = (u128)m * d2 - d1 * d1;
        iat_var = u128_to_double(num) / ((double)m * ((double)m - 1.0)) / 1000000.0;
    }
    out[0] = (float)dport;
    out[1] = (float)mean;
    out[2] = (float)sqrt(var);
    out[3] = (float)var;
    out[4] = (float)mean;
    out[5] = (float)iat_mean;
    out[6] = (float)sqrt(iat_var);
    out[7] = (float)((double)dmax / 1000.0);
}

uint32_t fsxo_dst_port(const uint8_t *f, uint32_t len) {
    uint16_t proto = (uint16_t)((f[12] << 8) | f[13]);
    uint32_t off;
    uint8_t l4;
    if (proto == 0x0800) {
        if (len < 34) return 0;
        off = 14u + 4u * (f[14] & 0x0Fu);
        l4 = f[23];
    } else if (proto == 0x86DD) {
        if (len < 54) return 0;
        off = 54;
        l4 = f[20];
    } else return 0;
    if (l4 != 6 && l4 != 17) return 0;
    if (off + 4 > len || off + 4 > 64) return 0;
    return ((uint32_t)f[off + 2] << 8) | f[off + 3];
}

typedef struct feat_acc {
    uint64_t n, last_t, dmax;
    u128 s1, s2, d1, d2;
    uint32_t dport;
    uint8_t fam;
    uint8_t key[16];
} feat_acc;

/* Returns number of flows (distinct source IPs, order of first appearance). */
/* max_sources bounds the distinct sources (0: n); more sources than that stop the scan
 * and return (size_t)-1. */
size_t fsxo_flow_features(const uint8_t *hdr, const uint32_t *len, const uint64_t *ts,
                          size_t n, size_t cap, uint8_t *keys16, uint8_t *family,
                          float *features, size_t max_sources) {
    omap idx[2];
    size_t me = max_sources ? max_sources : n + 1;
    omap_init(&idx[0], me, 4, 8);
    omap_init(&idx[1], me, 16, 8);
    feat_acc *acc = (feat_acc *)calloc(me + 1, sizeof(feat_acc));
    size_t nf = 0;
    for (size_t i = 0; i < n; ++i) {
        uint8_t key[16];
        const uint8_t *h = hdr + i * 64;
        int cls = fsxo_parse(h, len[i], key);
        if (cls < CLS_V4) continue;
        int v6 = cls == CLS_V6;
        uint64_t *slot = (uint64_t *)omap_lookup(&idx[v6], key);
        feat_acc *a;
        if (!slot) {
            if (nf == me) { nf = (size_t)-1; break; }
            uint64_t s = nf++;
            omap_update(&idx[v6], key, &s);
            a = &acc[s];
            a->fam = v6 ? 6 : 4;
            memcpy(a->key, key, 16);
            a->dport = fsxo_dst_port(h, len[i]);
        } else {
            a = &acc[*slot];
            uint64_t d = ts[i] - a->last_t;
            a->d1 += d; a->d2 += (u128)d * d;
            if (d > a->dmax) a->dmax = d;
        }
        a->n++;
        a->s1 += len[i];
        a->s2 += (u128)len[i] * len[i];
        a->last_t = ts[i];
    }
    for (size_t f = 0; nf != (size_t)-1 && f < nf && f < cap; ++f) {
        feat_acc *a = &acc[f];
        if (keys16) memcpy(keys16 + f * 16, a->key, 16);
        if (family) family[f] = a->fam;
        if (features) finish_features(a->n, a->s1, a->s2, a->d1, a->d2, a->dmax, a->dport, features + f * 8);
    }
    free(acc);
    omap_free(&idx[0]);
    omap_free(&idx[1]);
    return nf;
}

/* ------------------------------------------------------------------ synth */
/* CPU twin of the device generator (same header, same stream). */
int fsxo_synth(const fsx_synth_params *P, double zipf_s, uint64_t j0, size_t count,
               uint8_t *hdr, uint32_t *len, uint64_t *ts) {
    uint32_t *prob = NULL, *alias = NULL;
    if (P->mode == FSX_SYNTH_ZIPF_V4) {
        prob = (uint32_t *)malloc((size_t)P->n_ips * 4);
        alias = (uint32_t *)malloc((size_t)P->n_ips * 4);
        if (!prob || !alias || fsx_zipf_alias_build(P->n_ips, zipf_s, prob, alias)) {
            free(prob); free(alias);
            return -ENOMEM;
        }
    }
    for (size_t i = 0; i < count; ++i)
        fsx_synth_packet(P, prob, alias, j0 + i, hdr + i * 64, len + i, ts + i);
    free(prob); free(alias);
    return 0;
}

int fsxo_zipf_alias(uint32_t n, double s, uint32_t *prob, uint32_t *alias) {
    return fsx_zipf_alias_build(n, s, prob, alias);
}
