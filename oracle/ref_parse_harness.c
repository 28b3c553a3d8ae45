/*
 * ref_parse_harness.c — TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libref_parse.so).
 *
 * Compiles the reference's OWN header parsers, FlowSentryX src/parsing_helper.h
 * (parse_ethhdr :49-66, parse_ip6hdr :69-107, parse_ip4hdr :111-136), straight
 * from the read-only reference tree with the system's linux uapi headers, and
 * drives them with the dispatch of src/fsx_kern.c:123-148 (restated below, since
 * fsx_kern.c itself needs libbpf's bpf_helpers.h, absent here, and a BPF backend).
 * Used only to generate / re-check tests/golden/parse_vectors.npz and to pin the
 * oracle's restated parse (oracle/fsx_oracle.c fsxo_parse). Never shipped.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <arpa/inet.h>

#include <parsing_helper.h>   /* -I <reference>/src */
#include <fsx_struct.h>

#ifndef ETH_P_IP
#define ETH_P_IP 0x0800
#endif
#ifndef ETH_P_IPV6
#define ETH_P_IPV6 0x86DD
#endif

/* class: 0 DROP (parse failure), 1 PASS (non-IP), 2 IPv4, 3 IPv6 */
static int ref_parse_one(const uint8_t *rec, uint32_t len, uint8_t key[16]) {
    uint8_t buf[4096];
    memset(buf, 0, sizeof(buf));
    memcpy(buf, rec, 64);
    uint32_t span = len > sizeof(buf) ? (uint32_t)sizeof(buf) : len; /* only bounds at 14/34/54 matter */
    void *data = buf, *data_end = buf + span;
    struct hdr_cursor nh;
    struct ethhdr *eth;
    struct iphdr *ip4 = NULL;
    struct ipv6hdr *ip6 = NULL;
    nh.pos = data;
    int nh_type = parse_ethhdr(&nh, data_end, &eth);
    memset(key, 0, 16);
    if (nh_type == -1) return 0;
    if (nh_type != htons(ETH_P_IPV6) && nh_type != htons(ETH_P_IP)) return 1;
    if (nh_type == htons(ETH_P_IPV6)) {
        if (parse_ip6hdr(&nh, data_end, &ip6) == -1) return 0;
        memcpy(key, &ip6->saddr, 16);
        return 3;
    }
    if (parse_ip4hdr(&nh, data_end, &ip4) == -1) return 0;
    memcpy(key, &ip4->saddr, 4);
    return 2;
}

void ref_parse_batch(const uint8_t *hdr, const uint32_t *len, size_t n, uint8_t *cls,
                     uint8_t *keys16) {
    for (size_t i = 0; i < n; ++i)
        cls[i] = (uint8_t)ref_parse_one(hdr + i * 64, len[i], keys16 + i * 16);
}

size_t ref_sizeof_stats(void) { return sizeof(struct stats); }
size_t ref_sizeof_ip_stats(void) { return sizeof(struct ip_stats); }
