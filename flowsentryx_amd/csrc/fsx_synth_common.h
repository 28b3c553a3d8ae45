/*
 * fsx_synth_common.h — counter-based synthetic packet-stream generator, shared by
 * the device generator (fsx_synth.hip -> libfsx_synth.so) and the CPU oracle
 * (oracle/fsx_oracle.c), so both produce byte-identical streams.
 *
 * This is benchmark / test input plumbing (SURVEY.md §8 d "Generator"), not part of
 * the verdict path. Every packet j is a pure function of (params, j): the stream can
 * be generated in any order, on any device, in shards.
 *
 * Record layout (the ABI of include/fsx_hip.h): 64-byte header record holding the
 * first min(len, 64) frame bytes (zero padded), u32 frame length, u64 ts (ns).
 *
 * Workloads (BASELINE.json configs):
 *   FSX_SYNTH_ZIPF_V4   Ethernet/IPv4/UDP flood, src IP ~ Zipf(s) over n_ips ranks
 *                       (configs 1, 2, 4).
 *   FSX_SYNTH_CARPET    every packet a fresh spoofed source: pct_v6 % IPv6/UDP,
 *                       pct_vlan % 802.1Q-tagged IPv4 (PASS per parse), rest IPv4
 *                       (config 5).
 * Timestamps: ts_j = t0 + j*step + jitter_j, jitter_j in [0, step), step =
 * duration/n, so the stream is strictly increasing in arrival order.
 * Frame length: uniform in [len_min, len_max].
 * Must be compiled with -ffp-contract=off (alias-table construction uses doubles).
 */
#ifndef FSX_SYNTH_COMMON_H
#define FSX_SYNTH_COMMON_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FSX_HD __host__ __device__ __forceinline__
#else
#define FSX_HD static inline
#endif

enum { FSX_SYNTH_ZIPF_V4 = 0, FSX_SYNTH_CARPET = 1 };

typedef struct fsx_synth_params {
    uint64_t n;            /* packets in the whole stream */
    uint64_t seed;
    uint64_t t0_ns;
    uint64_t duration_ns;
    uint32_t n_ips;        /* Zipf domain size (ZIPF_V4) */
    uint32_t mode;
    uint32_t len_min, len_max;
    uint32_t pct_v6, pct_vlan; /* CARPET mix, percent */
    uint32_t ip_salt;
    uint32_t pad;
} fsx_synth_params;

FSX_HD uint64_t fsx_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* Random word k of packet j. */
FSX_HD uint64_t fsx_synth_rand(uint64_t seed, uint64_t j, uint32_t k) {
    return fsx_splitmix64(seed ^ fsx_splitmix64(j * 8ull + k));
}

/* murmur3 fmix32: a bijection on 32-bit words. */
FSX_HD uint32_t fsx_fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu;
    h ^= h >> 13; h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

FSX_HD void fsx_put_be16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* Sample a Zipf rank from a Walker/Vose alias table (prob = 2^32-scaled). */
FSX_HD uint32_t fsx_alias_sample(uint64_t r, uint32_t n, const uint32_t *prob,
                                 const uint32_t *alias) {
    uint32_t i = (uint32_t)(((r >> 32) * (uint64_t)n) >> 32);
    uint32_t coin = (uint32_t)r;
    return coin < prob[i] ? i : alias[i];
}

/* Source address of Zipf rank `rank` (distinct ranks -> distinct addresses). */
FSX_HD uint32_t fsx_synth_ip4_of_rank(uint32_t rank, uint32_t salt) {
    return fsx_fmix32(rank ^ salt);
}

/* Generate packet j: writes hdr[64], *len, *ts. */
FSX_HD void fsx_synth_packet(const fsx_synth_params *P, const uint32_t *prob,
                             const uint32_t *alias, uint64_t j, uint8_t *hdr,
                             uint32_t *len_out, uint64_t *ts_out) {
    uint64_t r0 = fsx_synth_rand(P->seed, j, 0);
    uint64_t r1 = fsx_synth_rand(P->seed, j, 1);
    uint64_t r2 = fsx_synth_rand(P->seed, j, 2);
    uint64_t step = P->n ? P->duration_ns / P->n : 0;
    uint64_t jit = step ? (r1 >> 11) % step : 0;
    *ts_out = P->t0_ns + j * step + jit;
    uint32_t span = P->len_max - P->len_min + 1u;
    uint32_t L = P->len_min + (uint32_t)((r2 >> 16) % span);
    *len_out = L;

    for (int i = 0; i < 64; ++i) hdr[i] = 0;
    /* Ethernet: dst 02:00:00:00:00:01, src 02:<random> */
    hdr[0] = 0x02; hdr[5] = 0x01;
    hdr[6] = 0x02;
    hdr[7] = (uint8_t)(r2 >> 0); hdr[8] = (uint8_t)(r2 >> 8);
    hdr[9] = (uint8_t)(r2 >> 56); hdr[10] = (uint8_t)(r2 >> 48); hdr[11] = (uint8_t)(r2 >> 40);

    uint32_t kind = 0; /* 0 v4, 1 v6, 2 vlan-v4 */
    uint32_t ip4 = 0;
    if (P->mode == FSX_SYNTH_ZIPF_V4) {
        uint32_t rank = fsx_alias_sample(r0, P->n_ips, prob, alias);
        ip4 = fsx_synth_ip4_of_rank(rank, P->ip_salt);
    } else {
        uint32_t pick = (uint32_t)((r0 >> 40) % 100u);
        kind = pick < P->pct_v6 ? 1u : (pick < P->pct_v6 + P->pct_vlan ? 2u : 0u);
        ip4 = fsx_fmix32((uint32_t)j ^ P->ip_salt) ^ (uint32_t)(j >> 32);
    }
    uint16_t sport = (uint16_t)(1024u + (uint32_t)((r1 >> 48) % 60000u));
    uint16_t dport;
    switch ((r0 >> 8) & 7u) {
    case 0: dport = 53; break;
    case 1: dport = 80; break;
    case 2: dport = 123; break;
    case 3: dport = 443; break;
    case 4: dport = 1900; break;
    case 5: dport = 11211; break;
    case 6: dport = 19; break;
    default: dport = 389; break;
    }

    uint8_t *l3;
    uint32_t l3off;
    if (kind == 2) {
        fsx_put_be16(hdr + 12, 0x8100);
        fsx_put_be16(hdr + 14, (uint32_t)(r1 & 0x0FFFu));
        fsx_put_be16(hdr + 16, 0x0800);
        l3off = 18;
    } else if (kind == 1) {
        fsx_put_be16(hdr + 12, 0x86DD);
        l3off = 14;
    } else {
        fsx_put_be16(hdr + 12, 0x0800);
        l3off = 14;
    }
    l3 = hdr + l3off;
    if (kind == 1) {
        uint32_t plen = L > 54 ? L - 54 : 0;
        l3[0] = 0x60; l3[1] = 0; l3[2] = 0; l3[3] = 0;
        fsx_put_be16(l3 + 4, plen);
        l3[6] = 17; l3[7] = 64;
        /* src 2001:db8:<32 random>::<64-bit bijective id> ; dst 2001:db8::1 */
        uint64_t id = fsx_splitmix64(j ^ ((uint64_t)P->ip_salt << 32));
        l3[8] = 0x20; l3[9] = 0x01; l3[10] = 0x0d; l3[11] = 0xb8;
        for (int i = 0; i < 4; ++i) l3[12 + i] = (uint8_t)(r2 >> (8 * i + 24));
        for (int i = 0; i < 8; ++i) l3[16 + i] = (uint8_t)(id >> (56 - 8 * i));
        /* dst at l3+24..39: bytes 38..53 of the frame; record keeps bytes < 64 */
        l3[24] = 0x20; l3[25] = 0x01; l3[26] = 0x0d; l3[27] = 0xb8;
        l3[39] = 0x01;
        /* UDP at 54 */
        fsx_put_be16(hdr + 54, sport);
        fsx_put_be16(hdr + 56, dport);
        fsx_put_be16(hdr + 58, plen);
    } else {
        uint32_t tot = L > l3off ? L - l3off : 0;
        l3[0] = 0x45; l3[1] = 0;
        fsx_put_be16(l3 + 2, tot & 0xFFFFu);
        fsx_put_be16(l3 + 4, (uint32_t)(r1 >> 32) & 0xFFFFu);
        l3[6] = 0x40; l3[7] = 0;
        l3[8] = 64; l3[9] = 17;
        /* source address, network byte order of ip4 */
        l3[12] = (uint8_t)(ip4 >> 24); l3[13] = (uint8_t)(ip4 >> 16);
        l3[14] = (uint8_t)(ip4 >> 8); l3[15] = (uint8_t)ip4;
        l3[16] = 10; l3[17] = 0; l3[18] = 0; l3[19] = 1;
        uint8_t *l4 = l3 + 20;
        fsx_put_be16(l4 + 0, sport);
        fsx_put_be16(l4 + 2, dport);
        fsx_put_be16(l4 + 4, tot > 20 ? (tot - 20) & 0xFFFFu : 0);
    }
    /* Bytes past the frame end are not part of the frame. */
    for (uint32_t i = L; i < 64; ++i) hdr[i] = 0;
}

#include <math.h>
#include <stdlib.h>
/* Vose alias table for Zipf(s) over ranks 0..n-1 (p_r ∝ (r+1)^-s). Host only.
 * Returns 0 or -1 on allocation failure. */
static inline int fsx_zipf_alias_build(uint32_t n, double s, uint32_t *prob,
                                       uint32_t *alias) {
    double *p = (double *)malloc((size_t)n * sizeof(double));
    uint32_t *small = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    uint32_t *large = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    if (!p || !small || !large) { free(p); free(small); free(large); return -1; }
    double sum = 0.0;
    for (uint32_t i = 0; i < n; ++i) { p[i] = pow((double)i + 1.0, -s); sum += p[i]; }
    uint32_t ns = 0, nl = 0;
    for (uint32_t i = 0; i < n; ++i) {
        p[i] = p[i] * (double)n / sum;
        if (p[i] < 1.0) small[ns++] = i; else large[nl++] = i;
    }
    while (ns && nl) {
        uint32_t l = small[--ns], g = large[--nl];
        prob[l] = (uint32_t)(p[l] * 4294967296.0);
        alias[l] = g;
        p[g] = (p[g] + p[l]) - 1.0;
        if (p[g] < 1.0) small[ns++] = g; else large[nl++] = g;
    }
    while (nl) { uint32_t g = large[--nl]; prob[g] = 0xFFFFFFFFu; alias[g] = g; }
    while (ns) { uint32_t l = small[--ns]; prob[l] = 0xFFFFFFFFu; alias[l] = l; }
    free(p); free(small); free(large);
    return 0;
}

#endif /* FSX_SYNTH_COMMON_H */
