"""GPU parity at the BASELINE configs' own shapes (through the C ABI, bit-exact against
the oracle): the reference-generated parse vectors, the config-2 stream under all three
limiters, a config-4 share from the 16M-source population (a table of more than 2^24
slots), a 2^24-packet config-5 carpet slice with a 64K-entry rule table, and flow
features of sources spanning hundreds of flow tiles.

The large cases check with the sharded oracle (oracle.ShardedOracle: the sequential
oracle on IP-disjoint host threads, equal to it by tests/test_oracle_sharded.py) and
compare full map dumps as sorted arrays."""
import os

import numpy as np
import pytest

from kat import GOLDEN
from test_gpu_parity import _check_flows, _process_batch_device

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _same_state(c, o, maps):
    from oracle import pyoracle
    assert c.stats() == o.stats()
    for m in maps:
        g, r = c.map_arrays(m), o.map_arrays(m)
        assert g[0].shape[0] == r[0].shape[0], (m, g[0].shape[0], r[0].shape[0])
        assert pyoracle.same_map(g, r), m


def _verdicts_equal(vg, vo):
    bad = np.nonzero(vg != vo)[0]
    assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"


def test_reference_parse_vectors_through_gpu(native):
    """tests/golden/parse_vectors.npz (made by the reference's own parsing_helper.h,
    src/parsing_helper.h:49-136) through fsx_verdict_batch: short frames DROP, non-IP
    PASS, every IP record counted under exactly the key the reference parser extracts
    (ipv4/ipv6_stats_map dumps: per key the packet count and byte sum)."""
    g = np.load(GOLDEN / "parse_vectors.npz")
    hdr, ln, cls, keys = g["hdr"], g["len"], g["cls"], g["keys"]
    n = len(ln)
    ts = (10**9 + np.arange(n)).astype(np.uint64)   # one window, far below any limit
    with native.FsxContext(max_entries=1 << 13, max_batch=8192, pps_threshold=1 << 40,
                           bps_threshold=1 << 60) as c:
        v = c.verdict_batch(hdr, ln, ts)
        assert np.array_equal(v[cls == 0], np.full((cls == 0).sum(), 1, np.uint8))
        assert np.array_equal(v[cls >= 1], np.full((cls >= 1).sum(), 2, np.uint8))
        for fam, klen, mid in ((2, 4, 1), (3, 16, 2)):
            want = {}
            first = {}
            for i in np.nonzero(cls == fam)[0]:
                k = keys[i, :klen].tobytes()
                p, b = want.get(k, (0, 0))
                want[k] = (p + 1, b + int(ln[i]))
                first.setdefault(k, int(ts[i]))
            got = c.map_dump(mid)
            assert set(got) == set(want), mid
            for k, (p, b) in want.items():
                assert got[k] == (p, b, first[k]), (mid, k.hex())
        assert c.stats() == (int((cls >= 2).sum()), 0)


@pytest.mark.parametrize("limiter", [0, 1, 2])
def test_config2_stream_all_limiters(native, oracle, limiter):
    """The config-2 generator stream (1M Zipf(1.1) sources), a 2M-packet slice, under
    the fixed window (src/fsx_kern.c:150-346), the sliding window and the token bucket
    (DESIGN.md §4), carried over two batches."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    n = 1 << 21
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cfg = dict(limiter=limiter, max_entries=1 << 20)
    if limiter == 2:
        cfg.update(tb_rate=2000, tb_burst=50)
    o = oracle.ShardedOracle(THREADS, **cfg)
    cut = 1_234_567
    with native.FsxContext(max_batch=n, **cfg) as c:
        for a, b in ((0, cut), (cut, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
        _same_state(c, o, (3, 4, 5, 6) if limiter == 2 else (1, 2, 3, 4))


def test_config4_share_16m_population(native, oracle):
    """BASELINE config 4's source population (16M Zipf(1.1) sources, 1B packets over 120 s):
    the first 8M packets of the stream, max_entries = 16M (a 2^25-slot table: 25-bit source
    ids, the heavy-source sort with an 8-bit first bucket, 128 heavy sources and two 9-bit light
    passes),
    fixed window with state carried."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    n = 1 << 23
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    o = oracle.ShardedOracle(THREADS, max_entries=16 << 20)
    with native.FsxContext(max_batch=n, max_entries=16 << 20) as c:
        for a, b in ((0, n // 2), (n // 2, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
        info = c.last_batch_info()
        assert info["sources"] > 1 << 19   # (about 630K distinct sources per 4M packets)
        _same_state(c, o, (1, 2, 3, 4))


def carpet_rules(hdr, rng, n_exact4=24576, n_exact6=8192, n_pfx4=30720, n_pfx6=2048):
    """A 64K-entry user rule table for a carpet stream (BASELINE config 5, README.md:72-74):
    exact blacklist entries on stream sources (maps 3 / 4; till UINT64_MAX = static block,
    every 8th one till = 0 = ignored), random IPv4 /24 prefixes and IPv6 /48 prefixes of
    stream sources (maps 7 / 8)."""
    from flowsentryx_amd.lib import prefix_key
    v4 = np.nonzero((hdr[:, 12] == 0x08) & (hdr[:, 13] == 0x00))[0]
    v6 = np.nonzero((hdr[:, 12] == 0x86) & (hdr[:, 13] == 0xDD))[0]
    rules = {3: {}, 4: {}, 7: {}, 8: {}}
    for j, i in enumerate(rng.choice(v4, n_exact4, replace=False)):
        rules[3][hdr[i, 26:30].tobytes()] = 0 if j % 8 == 0 else 2**64 - 1
    for j, i in enumerate(rng.choice(v6, n_exact6, replace=False)):
        rules[4][hdr[i, 22:38].tobytes()] = 0 if j % 8 == 0 else 2**64 - 1
    for a in rng.integers(0, 2**32, n_pfx4, dtype=np.uint64):
        rules[7][prefix_key(int(a).to_bytes(4, "big"), 24)] = 2**64 - 1
    for i in rng.choice(v6, n_pfx6, replace=False):
        rules[8][prefix_key(hdr[i, 22:38].tobytes(), 48)] = 2**64 - 1
    return rules


def test_config5_carpet_slice_with_rule_table(native, oracle):
    """BASELINE config 5 scaled slice (SURVEY.md §8 d: oracle parity on 2^24 packets):
    every packet a fresh spoofed source, 60% IPv4 / 30% IPv6 / 10% 802.1Q (PASS per
    parse), plus a 64K-entry rule table (exact + prefix)."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 24)
    n = int(p.n)
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    rules = carpet_rules(hdr, np.random.default_rng(55))
    me = n + (1 << 16)
    o = oracle.ShardedOracle(THREADS, max_entries=me)
    with native.FsxContext(max_batch=n, max_entries=me) as c:
        for m, entries in rules.items():
            c.map_update_batch(m, entries)
            for k, v in entries.items():
                o.map_update(m, k, v)
        vg = c.verdict_batch(hdr, ln, ts)
        vo = o.batch(hdr, ln, ts)
        _verdicts_equal(vg, vo)
        info = c.last_batch_info()
        assert info["prefix_rule_drops"] > 0 and info["any_ipv6"] == 1
        _same_state(c, o, (1, 2, 3, 4))


def test_flow_features_sources_of_many_tiles(native, oracle):
    """Sources of >= 300K packets (k_flow_combine's four-partials loop needs a source
    spanning >= 194 flow tiles): config-1 population over 4M packets, where the Zipf head
    has ~0.7M packets."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(1, n=1 << 22)
    hdr, ln, ts = oracle.synth(p, s, 0, p.n)
    counts = np.unique(hdr[:, 26:30].copy().view(np.uint32).reshape(-1), return_counts=True)[1]
    assert counts.max() >= 300_000
    _check_flows(native, oracle, hdr, ln, ts, cfg={"max_batch": 1 << 22})


@pytest.mark.parametrize("max_entries", [6 << 20, 16 << 20], ids=["ids24", "ids25"])
def test_wide_ids_full_path(native, oracle, max_entries):
    """Tables of 2^24 / 2^25 slots take the 3-pass heavy-source sort (DESIGN.md §3 "Two 9-bit
    light passes": pass 0's 8-bit bucket, then two light passes of 9 + 8 / 9 + 9 bits with
    512-digit tiles, 16-bit digit words and the digit bases from the tile scan): verdicts,
    features and q8 scores of two carried batches of the config-4 population against the
    oracle."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    n = 1 << 21
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cut = 777_777
    _process_batch_device(native, oracle, [(hdr[:cut], ln[:cut], ts[:cut]), (hdr[cut:], ln[cut:], ts[cut:])],
                          max_entries=max_entries)


@pytest.mark.parametrize("limiter", [1, 2], ids=["sliding", "token"])
@pytest.mark.parametrize("max_entries", [6 << 20, 16 << 20], ids=["ids24", "ids25"])
def test_wide_ids_limiters(native, oracle, limiter, max_entries):
    """The sliding window and the token bucket on tables of 2^24 / 2^25 slots (24- / 25-bit
    source ids: the plain sort, three 8-bit passes for 24 bits, 8 + 8 + 9 bits for 25 — the
    last with 512-digit tiles, 16-bit digit words and bases from the tile scan; each pass's
    digits read by the next pass's tile histogram; DESIGN.md §3 "Wider ids", §8): the config-4
    population over two carried batches, verdicts and every map against the oracle."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    n = 1 << 21
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cfg = dict(limiter=limiter, max_entries=max_entries)
    if limiter == 2:
        cfg.update(tb_rate=2000, tb_burst=50)
    o = oracle.ShardedOracle(THREADS, **cfg)
    cut = 777_777
    with native.FsxContext(max_batch=n, **cfg) as c:
        for a, b in ((0, cut), (cut, n)):
            _verdicts_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
        _same_state(c, o, (3, 4, 5, 6) if limiter == 2 else (1, 2, 3, 4))


def test_wide_ids_flow_features(native, oracle):
    """Flow-only batches on a 2^25-slot table (the per-batch id table has the table's 25-bit
    ids): the plain sort in three passes of 8 + 8 + 9 bits, features of the
    config-4 population against the oracle."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    hdr, ln, ts = oracle.synth(p, s, 0, 1 << 21)
    _check_flows(native, oracle, hdr, ln, ts, cfg={"max_batch": 1 << 21, "max_entries": 16 << 20})


def _wide_cfg(limiter):
    cfg = dict(limiter=limiter, max_entries=16 << 20)
    if limiter == 2:
        cfg.update(tb_rate=2000, tb_burst=50)
    return cfg


@pytest.mark.parametrize("limiter", [0, 1, 2], ids=["fixed", "sliding", "token"])
def test_wide_ids_edge_batches(native, oracle, limiter):
    """The 9-bit plans at their edges (DESIGN.md §3 "Two 9-bit light passes"): on a 2^25-slot
    table, carried batches of 1, 100, 4095, 4097 and 70000 packets (one to 18 sort tiles), a
    batch of three sources (light passes over next to nothing), IPv6, non-IP and short frames
    mixed in, and a batch whose clock steps back (the run path) — verdicts and every map
    against the oracle."""
    from test_gpu_parity import rand_stream
    rng = np.random.default_rng(77)
    cfg = _wide_cfg(limiter)
    o = oracle.ShardedOracle(THREADS, **cfg)
    batches, t = [], 10**9
    for n, ips in ((1, 1), (100, 30), (4095, 500), (4097, 3000), (70000, 20000), (50000, 3)):
        hdr, ln, ts = rand_stream(rng, n, ips, v6_frac=0.2, nonip_frac=0.02, short_frac=0.01, t0=t)
        t = int(ts[-1]) + 1
        batches.append((hdr, ln, ts))
    hdr, ln, ts = rand_stream(rng, 30000, 2000, t0=t + 10**6)
    ts[15000:] -= np.uint64(10**6)   # (the clock steps back mid-batch)
    batches.append((hdr, ln, ts))
    with native.FsxContext(max_batch=70000, **cfg) as c:
        for hdr, ln, ts in batches:
            _verdicts_equal(c.verdict_batch(hdr, ln, ts), o.batch(hdr, ln, ts))
        _same_state(c, o, (3, 4, 5, 6) if limiter == 2 else (1, 2, 3, 4))


@pytest.mark.parametrize("limiter", [1, 2], ids=["sliding", "token"])
def test_wide_ids_limiters_pipelined(native, oracle, limiter):
    """The sliding window and the token bucket on a 2^25-slot table with pipelined batches
    (the heavy-source sort with two 9-bit light passes in each front set): three
    uneven carried batches of the config-4 population, one sync at the end, verdicts and every
    map against the oracle."""
    import torch
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    n = 1 << 20
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cuts = [0, 250_000, 250_001, n]
    cfg = _wide_cfg(limiter)
    o = oracle.ShardedOracle(THREADS, **cfg)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).cuda()
    with native.FsxContext(max_batch=n, **cfg) as c:
        c.set_pipeline(True)
        outs = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            d = dict(h=dev(hdr[a:b]), l=dev(ln[a:b]), t=dev(ts[a:b]),
                     v=torch.empty(b - a, dtype=torch.uint8, device="cuda"))
            c.verdict_batch_device(d["h"].data_ptr(), d["l"].data_ptr(), d["t"].data_ptr(), b - a,
                                   d["v"].data_ptr())
            d["vo"] = o.batch(hdr[a:b], ln[a:b], ts[a:b])
            outs.append(d)
        c.sync()
        for d in outs:
            _verdicts_equal(d["v"].cpu().numpy(), d["vo"])
        _same_state(c, o, (3, 4, 5, 6) if limiter == 2 else (1, 2, 3, 4))
