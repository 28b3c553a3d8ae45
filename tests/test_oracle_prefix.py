"""Prefix blocklists in the CPU oracle: known answers worked by hand.

Build-defined feature (the reference defers LPM, TODO.md:251): the semantics are those
of a BPF_MAP_TYPE_LPM_TRIE consulted before the per-source maps — parity unpinned
against the reference, pinned here by hand-computed cases.
"""
import numpy as np

from flowsentryx_amd import synth
from flowsentryx_amd.lib import prefix_key

NEVER = 2**64 - 1


def v4(a, b, c, d):
    return bytes([a, b, c, d])


def frames4(srcs, t0=10**9, dt=1000):
    hdr = synth.records([synth.frame_ipv4_udp(s, 100) for s in srcs])
    ln = np.full(len(srcs), 100, np.uint32)
    ts = (t0 + dt * np.arange(len(srcs))).astype(np.uint64)
    return hdr, ln, ts


def test_longest_match_and_exception(oracle):
    o = oracle.Oracle(pps_threshold=10**6)
    o.map_update(7, prefix_key(v4(10, 0, 0, 0), 8), NEVER)         # 10/8 blocked
    o.map_update(7, prefix_key(v4(10, 1, 0, 0), 16), 0)            # 10.1/16 exception
    o.map_update(7, prefix_key(v4(10, 1, 2, 0), 24), NEVER)        # 10.1.2/24 blocked again
    srcs = [v4(10, 9, 9, 9), v4(10, 1, 9, 9), v4(10, 1, 2, 3), v4(11, 0, 0, 1)]
    v = o.batch(*frames4(srcs))
    assert list(v) == [1, 2, 1, 2]
    assert o.stats() == (2, 2)
    # rule-dropped sources never reach the per-source maps
    assert set(o.map_dump(1)) == {v4(10, 1, 9, 9), v4(11, 0, 0, 1)}


def test_expiry_and_canonical_keys(oracle):
    o = oracle.Oracle(pps_threshold=10**6)
    # address bits past the prefix are ignored: the stored key is canonical
    o.map_update(7, prefix_key(v4(192, 168, 77, 5), 20), 10**9 + 1500)
    assert o.map_dump(7) == {prefix_key(v4(192, 168, 64, 0), 20): 10**9 + 1500}
    v = o.batch(*frames4([v4(192, 168, 79, 1)] * 3))   # t = 1e9, +1000, +2000
    assert list(v) == [1, 1, 2]                         # till is inclusive, then expired
    # LPM lookup: the longest rule with length <= the key's prefixlen
    assert o.map_lookup(7, prefix_key(v4(192, 168, 70, 70), 32)) == 10**9 + 1500
    assert o.map_lookup(7, prefix_key(v4(192, 168, 70, 70), 19)) is None
    assert o.map_delete(7, prefix_key(v4(192, 168, 64, 9), 20)) == 0
    assert o.map_dump(7) == {}


def test_ipv6_prefix_and_zero_length(oracle):
    o = oracle.Oracle(pps_threshold=10**6)
    net = bytes.fromhex("20010db8000000000000000000000000")
    o.map_update(8, prefix_key(net, 32), NEVER)
    a = bytes.fromhex("20010db8ffff00000000000000000001")
    b = bytes.fromhex("20010db9000000000000000000000001")
    hdr = synth.records([synth.frame_ipv6_udp(a, 100), synth.frame_ipv6_udp(b, 100)])
    v = o.batch(hdr, np.full(2, 100, np.uint32), np.array([10**9, 10**9 + 5], np.uint64))
    assert list(v) == [1, 2]
    # a /0 rule matches every address of its family only
    o.map_update(7, prefix_key(v4(0, 0, 0, 0), 0), NEVER)
    v = o.batch(*frames4([v4(1, 2, 3, 4)], t0=2 * 10**9))
    assert list(v) == [1]
    v = o.batch(hdr[1:], np.full(1, 100, np.uint32), np.array([2 * 10**9], np.uint64))
    assert list(v) == [2]
