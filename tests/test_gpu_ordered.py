"""GPU: home-ordered inserts (DESIGN.md §3 "Home-ordered inserts").

A batch on this path writes each IP packet's home-ordered source hash instead of probing
the source index, sorts, separates the sources that share a key hash (IPv6 / mixed-family
runs: k_ord_fix, k_ord_long) and finds / inserts one slot per segment in home order
(k_ord_resolve). Everything must equal the oracle exactly as on the probing path: verdicts,
stats_map and the map dumps (src/fsx_kern.c:150-346), over carried batches, with the rule
table, IPv6 hash collisions, repeated sources, a table that fills up (rollback) and the
host's automatic choice after a flood."""
import errno

import numpy as np
import pytest

from test_gpu_parity import assert_same_state, gpu_ctx, rand_stream
from test_gpu_scale import THREADS, _same_state, _verdicts_equal, carpet_rules

pytestmark = pytest.mark.gpu


def _flags(*names):
    from flowsentryx_amd import lib
    f = 0
    for nm in names:
        f |= getattr(lib, nm)
    return f


def test_ordered_carpet_slices_with_rule_table(native, oracle):
    """Config-5 carpet (every packet a new source; 60% IPv4 / 30% IPv6 / 10% 802.1Q) with a
    scaled rule table, two carried batches, both on the home-ordered path."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 22)
    n = int(p.n)
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    rules = carpet_rules(hdr, np.random.default_rng(56), 4096, 2048, 4096, 512)
    me = n + (1 << 16)
    o = oracle.ShardedOracle(THREADS, max_entries=me)
    with native.FsxContext(max_batch=n, max_entries=me, flags=_flags("FLAG_ORDERED_INSERTS")) as c:
        for m, entries in rules.items():
            c.map_update_batch(m, entries)
            for k, v in entries.items():
                o.map_update(m, k, v)
        for a, b in ((0, n // 2), (n // 2, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
            info = c.last_batch_info()
            assert info["ordered_inserts"] == 1 and info["new_sources"] > 0
        _same_state(c, o, (1, 2, 3, 4))


def test_ordered_config2_stream(native, oracle):
    """The config-2 Zipf stream (sources repeated up to ~10^5 times: long key-hash runs of one
    IPv4 source) forced onto the home-ordered path, carried over two batches."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    n = 1 << 21
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cfg = dict(max_entries=1 << 20)
    o = oracle.ShardedOracle(THREADS, **cfg)
    with native.FsxContext(max_batch=n, flags=_flags("FLAG_ORDERED_INSERTS"), **cfg) as c:
        for a, b in ((0, 1_234_567), (1_234_567, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
            assert c.last_batch_info()["ordered_inserts"] == 1
        _same_state(c, o, (1, 2, 3, 4))


def test_ordered_ipv6_key_hash_collisions(native, oracle):
    """FSX_FLAG_TEST_V6_COLLIDE gives every IPv6 source the same home slot, so on a 2^21-slot
    table ~160K IPv6 sources share 2^11 key hashes: runs of ~80 sources (k_ord_long) and short
    mixed runs (k_ord_fix) are regrouped by address."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 19)
    n = int(p.n)
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cfg = dict(max_entries=1 << 20)
    o = oracle.Oracle(flags=1, **cfg)
    with native.FsxContext(max_batch=n, flags=_flags("FLAG_ORDERED_INSERTS", "FLAG_TEST_V6_COLLIDE"), **cfg) as c:
        for a, b in ((0, n // 3), (n // 3, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
            assert c.last_batch_info()["ordered_inserts"] == 1
        _same_state(c, o, (1, 2, 3, 4))


def test_ordered_repeated_ipv6_source(native, oracle):
    """One IPv6 source repeated 3000 times inside a carpet slice: a key-hash run far longer
    than k_ord_long's regroup limit, all one source (checked, nothing moved); it exceeds
    pps_threshold and is blacklisted mid-batch."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 20)
    n = int(p.n)
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    hdr = hdr.copy()
    ln = ln.copy()
    v6 = np.nonzero((hdr[:, 12] == 0x86) & (hdr[:, 13] == 0xDD))[0]
    rng = np.random.default_rng(9)
    src = v6[0]
    dst = np.sort(rng.choice(np.arange(1, n), 3000, replace=False))
    hdr[dst] = hdr[src]
    ln[dst] = ln[src]
    cfg = dict(max_entries=1 << 21)
    o = oracle.ShardedOracle(THREADS, **cfg)
    with native.FsxContext(max_batch=n, flags=_flags("FLAG_ORDERED_INSERTS"), **cfg) as c:
        _verdicts_equal(c.verdict_batch(hdr, ln, ts), o.batch(hdr, ln, ts))
        assert c.last_batch_info()["ordered_inserts"] == 1
        _same_state(c, o, (1, 2, 3, 4))
        assert o.stats()[1] > 0   # (the repeated source was blacklisted)


def test_ordered_long_mixed_ipv6_run(native, oracle):
    """A key-hash run far longer than k_ord_long's LDS regroup (kOrdLong = 512) that holds many
    sources (a heavy IPv6 source sharing its 32-bit key hash with flood sources):
    under FSX_FLAG_TEST_V6_COLLIDE ~77 IPv6 carpet sources share each key hash, and one of them
    is repeated 3000 times. The run is separated source by source (ord_extract) instead of
    failing the batch; verdicts, stats and maps equal the oracle, the source is blacklisted."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 19)
    n = int(p.n)
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    hdr = hdr.copy()
    ln = ln.copy()
    v6 = np.nonzero((hdr[:, 12] == 0x86) & (hdr[:, 13] == 0xDD))[0]
    rng = np.random.default_rng(19)
    src = v6[3]
    dst = np.sort(rng.choice(np.arange(v6[3] + 1, n), 3000, replace=False))
    hdr[dst] = hdr[src]
    ln[dst] = ln[src]
    cfg = dict(max_entries=1 << 20)
    o = oracle.Oracle(flags=1, **cfg)
    with native.FsxContext(max_batch=n, flags=_flags("FLAG_ORDERED_INSERTS", "FLAG_TEST_V6_COLLIDE"), **cfg) as c:
        _verdicts_equal(c.verdict_batch(hdr, ln, ts), o.batch(hdr, ln, ts))
        assert c.last_batch_info()["ordered_inserts"] == 1
        _same_state(c, o, (1, 2, 3, 4))
        assert o.stats()[1] > 0   # (the repeated source was blacklisted)


def test_ordered_inserts_follow_a_flood(native, oracle):
    """Without the flag the host chooses: a batch after a flood (new sources > half of its IP
    packets) takes the home-ordered path, a batch after a stream of known sources does not."""
    from flowsentryx_amd import synth
    p5, s5 = synth.config_params(5, n=1 << 20)
    h5, l5, t5 = oracle.synth(p5, s5, 0, 1 << 20)
    p2, s2 = synth.config_params(2)
    h2, l2, t2 = oracle.synth(p2, s2, 0, 1 << 20)
    t2 = t2 + np.uint64(int(t5[-1]))
    cfg = dict(max_entries=1 << 21)
    o = oracle.ShardedOracle(THREADS, **cfg)
    batches = [(h5[:1 << 19], l5[:1 << 19], t5[:1 << 19]), (h5[1 << 19:], l5[1 << 19:], t5[1 << 19:]),
               (h2[:1 << 19], l2[:1 << 19], t2[:1 << 19]), (h2[1 << 19:], l2[1 << 19:], t2[1 << 19:]),
               (h2[1 << 19:], l2[1 << 19:], t2[1 << 19:] + np.uint64(10**10))]
    got = []
    with native.FsxContext(max_batch=1 << 19, **cfg) as c:
        for h, ln, ts in batches:
            _verdicts_equal(c.verdict_batch(h, ln, ts), o.batch(h, ln, ts))
            got.append(c.last_batch_info()["ordered_inserts"])
        _same_state(c, o, (1, 2, 3, 4))
    # the first carpet half: no history yet; the second: after a flood; the first config-2
    # half: after a flood too (its new sources make it one as well); the last: known sources
    assert got[0] == 0 and got[1] == 1 and got[-1] == 0, got


def test_ordered_table_full_rolls_back(native, oracle):
    """A home-ordered batch whose new sources exceed max_entries fails with ENOSPC and
    changes nothing; the next batches equal an oracle that never saw it."""
    from flowsentryx_amd import lib, synth
    rng = np.random.default_rng(61)
    cfg = dict(pps_threshold=5, window_ns=100_000, block_ns=300_000, max_entries=300)
    h1, l1, t1 = rand_stream(rng, 3000, 60, dt_max=200, v6_frac=0.3)   # (<= 120 sources)
    t1 = t1 + np.uint64(10**6)
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 77, i // 256, i % 256]), 90) for i in range(400)])
    tb = t1[-1] + np.arange(1, 401, dtype=np.uint64)
    h3, l3, t3 = rand_stream(rng, 3000, 60, dt_max=200, v6_frac=0.3)
    t3 = t3 + tb[-1]
    okw = {k: v for k, v in cfg.items() if k != "max_entries"}
    o = oracle.Oracle(max_entries=1 << 12, **okw)
    with gpu_ctx(native, max_batch=4096, flags=lib.FLAG_ORDERED_INSERTS, **cfg) as c:
        assert np.array_equal(c.verdict_batch(h1, l1, t1), o.batch(h1, l1, t1))
        assert c.last_batch_info()["ordered_inserts"] == 1
        before = {m: c.map_dump(m) for m in (1, 2, 3, 4)}
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(big, np.full(400, 90, np.uint32), tb)
        assert e.value.code == -errno.ENOSPC
        assert {m: c.map_dump(m) for m in (1, 2, 3, 4)} == before
        assert np.array_equal(c.verdict_batch(h3, l3, t3), o.batch(h3, l3, t3))
        assert_same_state(c, o)
