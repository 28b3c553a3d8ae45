"""GPU parity: libfsx_hip.so (through the C ABI) against the CPU oracle.

Bit-exact: verdict arrays, stats_map, and every entry of the four per-IP maps.
Inputs are seeded synthetic streams at sizes the oracle finishes in seconds, the
golden known-answer tests, and edge cases (short frames, non-IP, IPv6 hash
collisions, non-monotone clocks, block < window, byte-limit triggers, full maps).
"""
import errno
import zlib
import json

import numpy as np
import pytest

from kat import GOLDEN, build_case, expected_maps, load_kats

pytestmark = pytest.mark.gpu

MAPS = (1, 2, 3, 4)


def gpu_ctx(native, **kw):
    kw.setdefault("max_batch", 1 << 20)
    kw.setdefault("max_entries", 1 << 18)
    return native.FsxContext(**kw)


def assert_same_state(c, o):
    assert c.stats() == o.stats()
    for m in MAPS:
        g, r = c.map_dump(m), o.map_dump(m)
        assert len(g) == len(r), (m, len(g), len(r))
        assert g == r, m


def run_both(native, oracle, batches, cfg=None, oracle_cfg=None):
    cfg = cfg or {}
    okw = {k: v for k, v in cfg.items() if k in ("pps_threshold", "bps_threshold", "window_ns",
                                                    "block_ns", "max_entries")}
    okw.setdefault("max_entries", cfg.get("max_entries", 1 << 18))
    o = oracle.Oracle(**okw)
    with gpu_ctx(native, **cfg) as c:
        for hdr, ln, ts in batches:
            vg = c.verdict_batch(hdr, ln, ts)
            vo = o.batch(hdr, ln, ts)
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
        assert_same_state(c, o)


def rand_stream(rng, n, n_ips, dt_max=2000, v6_frac=0.0, nonip_frac=0.0, short_frac=0.0,
                len_lo=60, len_hi=1514, t0=10**9):
    from flowsentryx_amd import synth
    ips4 = rng.integers(0, 2**32, n_ips, dtype=np.uint64).astype(np.uint32)
    ips6 = rng.integers(0, 256, (n_ips, 16), dtype=np.uint8)
    w = 1.0 / np.arange(1, n_ips + 1) ** 1.1
    pick = rng.choice(n_ips, n, p=w / w.sum())
    kind = rng.random(n)
    frames = []
    ln = rng.integers(len_lo, len_hi + 1, n).astype(np.uint32)
    for i in range(n):
        k = kind[i]
        if k < nonip_frac:
            frames.append(synth.frame_raw(0x0806, bytes(46), 60))
        elif k < nonip_frac + v6_frac:
            frames.append(synth.frame_ipv6_udp(ips6[pick[i]].tobytes(), int(ln[i])))
        else:
            frames.append(synth.frame_ipv4_udp(int(ips4[pick[i]]).to_bytes(4, "big"), int(ln[i])))
        if rng.random() < short_frac:
            ln[i] = rng.integers(0, 54)
    ts = t0 + np.cumsum(rng.integers(0, dt_max + 1, n)).astype(np.uint64)
    return synth.records(frames), ln, ts


# ------------------------------------------------------------------ known answers
@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_known_answers(native, case):
    hdr, ln, ts, exp = build_case(case)
    with gpu_ctx(native, max_entries=1000, max_batch=8192) as c:
        v = c.verdict_batch(hdr, ln, ts)
        assert np.array_equal(v, exp), np.nonzero(v != exp)[0][:10]
        assert list(c.stats()) == case["stats"]
        for mid, entries in expected_maps(case).items():
            dump = c.map_dump(mid)
            for k, val in entries.items():
                assert dump.get(k) == val, (mid, k, dump.get(k), val)


def test_known_answers_one_packet_per_batch(native):
    """Cross-batch state carry: the KAT stream fed one packet per call."""
    case = load_kats()[1]
    hdr, ln, ts, exp = build_case(case)
    with gpu_ctx(native, max_entries=1000, max_batch=16) as c:
        out = [c.verdict_batch(hdr[i:i + 1], ln[i:i + 1], ts[i:i + 1])[0] for i in range(len(exp))]
    assert np.array_equal(np.array(out, dtype=np.uint8), exp)


# ------------------------------------------------------------------ random streams
CFGS = {
    "default": {},
    "tight": {"pps_threshold": 7, "window_ns": 200_000, "block_ns": 1_000_000},
    "block_lt_window": {"pps_threshold": 5, "window_ns": 1_000_000, "block_ns": 50_000},
    "block_zero": {"pps_threshold": 3, "window_ns": 100_000, "block_ns": 0},
    "bytes_limit": {"pps_threshold": 50, "bps_threshold": 9_000, "window_ns": 500_000,
                    "block_ns": 2_000_000},
    "pps_zero": {"pps_threshold": 0, "window_ns": 100_000, "block_ns": 300_000},
}


@pytest.mark.parametrize("name", list(CFGS))
def test_random_ipv4(native, oracle, name):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    hdr, ln, ts = rand_stream(rng, 40000, 300, dt_max=400)
    run_both(native, oracle, [(hdr, ln, ts)], CFGS[name])


@pytest.mark.parametrize("name", ["default", "tight", "block_lt_window"])
def test_random_mixed_families(native, oracle, name):
    rng = np.random.default_rng(11 + len(name))
    hdr, ln, ts = rand_stream(rng, 30000, 500, dt_max=300, v6_frac=0.4, nonip_frac=0.05,
                              short_frac=0.03)
    run_both(native, oracle, [(hdr, ln, ts)], CFGS[name])


@pytest.mark.parametrize("name", ["tight", "block_lt_window", "bytes_limit"])
def test_state_carry_across_batches(native, oracle, name):
    rng = np.random.default_rng(5)
    hdr, ln, ts = rand_stream(rng, 30000, 200, dt_max=300, v6_frac=0.2)
    cuts = [0, 1, 2, 777, 5000, 5001, 17000, 29999, 30000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    run_both(native, oracle, batches, CFGS[name])


def test_non_monotone_clock(native, oracle):
    rng = np.random.default_rng(8)
    hdr, ln, ts = rand_stream(rng, 20000, 100, dt_max=200)
    sw = rng.choice(len(ts), 3000, replace=False)
    ts[sw] = ts[sw] - rng.integers(0, 50000, sw.size).astype(np.uint64)
    ts[5] = np.uint64(2**64 - 5)   # u64 wraparound in now - track_time
    run_both(native, oracle, [(hdr, ln, ts)], CFGS["tight"])


def test_ipv6_forced_collisions(native, oracle):
    """FSX_FLAG_TEST_V6_COLLIDE: every IPv6 source starts probing the per-batch id table
    at IPv4 10.0.0.1's slot, so all of them (and 10.0.0.1) share one long probe chain."""
    rng = np.random.default_rng(21)
    from flowsentryx_amd import synth
    hdr, ln, ts = rand_stream(rng, 20000, 50, dt_max=300, v6_frac=0.5)
    extra = synth.records([synth.frame_ipv4_udp(bytes([10, 0, 0, 1]), 100)] * 500)
    hdr = np.concatenate([hdr, extra])
    ln = np.concatenate([ln, np.full(500, 100, np.uint32)])
    ts = np.concatenate([ts, ts[-1] + np.arange(1, 501, dtype=np.uint64)])
    run_both(native, oracle, [(hdr, ln, ts)], dict(CFGS["tight"], flags=1))


def test_many_ipv6_sources(native, oracle):
    """2^17 distinct IPv6 + 2^17 IPv4 sources in one batch (a half-full id table)."""
    rng = np.random.default_rng(3)
    n = 1 << 17
    from flowsentryx_amd import synth
    hdr = np.zeros((2 * n, 64), np.uint8)
    for i in range(n):
        hdr[i] = np.frombuffer(synth.frame_ipv6_udp(rng.bytes(16), 100), np.uint8)
    k4 = rng.integers(0, 2**32, n, dtype=np.uint64)
    for i in range(n):
        hdr[n + i] = np.frombuffer(synth.frame_ipv4_udp(int(k4[i]).to_bytes(4, "big"), 100), np.uint8)
    perm = rng.permutation(2 * n)
    hdr = hdr[perm]
    ln = np.full(2 * n, 100, np.uint32)
    ts = (10**9 + np.arange(2 * n) * 10).astype(np.uint64)
    run_both(native, oracle, [(hdr, ln, ts)], {"max_entries": 1 << 19})


def test_config1_stream(native, oracle):
    """BASELINE config 1: 1M-packet IPv4/UDP flood, 1024 Zipf sources over 5 s."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(1)
    hdr, ln, ts = oracle.synth(p, s, 0, p.n)
    run_both(native, oracle, [(hdr, ln, ts)], {"max_entries": 4096})


def test_carpet_stream(native, oracle):
    """BASELINE config 5 shape (scaled): unique spoofed v4/v6 sources + VLAN + rule table."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=200_000)
    hdr, ln, ts = oracle.synth(p, s, 0, p.n)
    rng = np.random.default_rng(4)
    o = oracle.Oracle(max_entries=1 << 19)
    with gpu_ctx(native, max_entries=1 << 19) as c:
        # user rule table: static blocks (till = UINT64_MAX) and ignored entries (till = 0)
        ip_rows = np.nonzero(hdr[:, 12] == 0x08)[0][:2000]
        for j, i in enumerate(ip_rows):
            key = hdr[i, 26:30].tobytes()
            till = (2**64 - 1) if j % 2 == 0 else 0
            c.map_update(3, key, till)
            o.map_update(3, key, till)
        vg = c.verdict_batch(hdr, ln, ts)
        vo = o.batch(hdr, ln, ts)
        assert np.array_equal(vg, vo)
        assert_same_state(c, o)


def test_table_full_reports_enospc(native):
    from flowsentryx_amd import lib, synth
    hdr = synth.records([synth.frame_ipv4_udp(bytes([10, 9, i // 256, i % 256]), 80) for i in range(600)])
    with gpu_ctx(native, max_entries=500, max_batch=1024) as c:
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(hdr, np.full(600, 80, np.uint32), np.arange(600, dtype=np.uint64) + 5)
        assert e.value.code == -errno.ENOSPC


@pytest.mark.parametrize("limiter", [0, 1, 2])
def test_failed_batch_rolls_back(native, oracle, limiter):
    """A batch that would exceed max_entries changes nothing (its new sources are rolled
    back out of the source index): the next batches equal an oracle that never saw it."""
    from flowsentryx_amd import lib, synth
    rng = np.random.default_rng(60 + limiter)
    cfg = dict(pps_threshold=5, window_ns=100_000, block_ns=300_000, max_entries=300, limiter=limiter,
               tb_rate=300_000, tb_burst=4)
    h1, l1, t1 = rand_stream(rng, 3000, 120, dt_max=200)
    t1 = t1 + np.uint64(10**6)
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 77, i // 256, i % 256]), 90) for i in range(400)])
    tb = t1[-1] + np.arange(1, 401, dtype=np.uint64)
    h3, l3, t3 = rand_stream(rng, 3000, 120, dt_max=200)
    t3 = t3 + tb[-1]
    okw = {k: v for k, v in cfg.items() if k != "max_entries"}
    o = oracle.Oracle(max_entries=1 << 12, **okw)
    with gpu_ctx(native, max_batch=4096, **cfg) as c:
        assert np.array_equal(c.verdict_batch(h1, l1, t1), o.batch(h1, l1, t1))
        before = {m: c.map_dump(m) for m in (1, 2, 3, 4, 5, 6)}
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(big, np.full(400, 90, np.uint32), tb)
        assert e.value.code == -errno.ENOSPC
        assert {m: c.map_dump(m) for m in (1, 2, 3, 4, 5, 6)} == before
        assert np.array_equal(c.verdict_batch(h3, l3, t3), o.batch(h3, l3, t3))
        assert c.stats() == o.stats()
        for m in ((1, 2, 3, 4) if limiter < 2 else (3, 4, 5, 6)):
            assert c.map_dump(m) == o.map_dump(m), m


def test_mirror_cleared_on_rollback_and_reset(native, oracle):
    """Tables of >= 2^18 slots probe IPv4 sources on the 2-byte mirror of the source index
    (DESIGN.md §3). A rolled-back batch's sources, and every source after fsx_reset, must not
    match a stale mirror entry: the next batches re-send rolled-back and surviving sources and
    equal an oracle that never saw the failed batch; after a reset, one that starts empty."""
    from flowsentryx_amd import lib, synth
    rng = np.random.default_rng(77)
    cfg = dict(CFGS["tight"], max_entries=70_000)
    h1, l1, t1 = rand_stream(rng, 20000, 3000, dt_max=200)
    t1 = t1 + np.uint64(10**6)
    nb = 70_000
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 77 + (i >> 16), (i >> 8) & 255, i & 255]), 90)
                         for i in range(nb)])
    tb = t1[-1] + np.arange(1, nb + 1, dtype=np.uint64)
    # next batch: the first batch's sources again, plus 1000 of the rolled-back ones
    pick = rng.integers(0, 1000, 4000)
    h3 = np.concatenate([h1, big[pick]])
    l3 = np.concatenate([l1, np.full(pick.size, 90, np.uint32)])
    t3 = tb[-1] + np.arange(1, h3.shape[0] + 1, dtype=np.uint64) * 7
    perm = rng.permutation(h3.shape[0])
    h3, l3 = h3[perm], l3[perm]
    o = oracle.Oracle(max_entries=1 << 18, **{k: v for k, v in cfg.items() if k != "max_entries"})
    with gpu_ctx(native, max_batch=1 << 17, **cfg) as c:
        assert np.array_equal(c.verdict_batch(h1, l1, t1), o.batch(h1, l1, t1))
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(big, np.full(nb, 90, np.uint32), tb)
        assert e.value.code == -errno.ENOSPC
        assert np.array_equal(c.verdict_batch(h3, l3, t3), o.batch(h3, l3, t3))
        assert_same_state(c, o)
        c.reset()
        o2 = oracle.Oracle(max_entries=1 << 18, **{k: v for k, v in cfg.items() if k != "max_entries"})
        assert np.array_equal(c.verdict_batch(h3, l3, t3), o2.batch(h3, l3, t3))
        assert_same_state(c, o2)


def test_map_syscalls(native):
    from flowsentryx_amd import lib
    with gpu_ctx(native, max_entries=64, max_batch=64) as c:
        k4, k6 = bytes([1, 2, 3, 4]), bytes(range(16))
        assert c.map_lookup(lib.MAP_IPV4_STATS, k4) is None
        c.map_update(lib.MAP_IPV4_STATS, k4, (5, 6, 7))
        assert c.map_lookup(lib.MAP_IPV4_STATS, k4) == (5, 6, 7)
        with pytest.raises(lib.FsxError) as e:
            c.map_update(lib.MAP_IPV4_STATS, k4, (1, 1, 1), lib.BPF_NOEXIST)
        assert e.value.code == -errno.EEXIST
        with pytest.raises(lib.FsxError) as e:
            c.map_update(lib.MAP_IPV6_BLACKLIST, k6, 9, lib.BPF_EXIST)
        assert e.value.code == -errno.ENOENT
        c.map_update(lib.MAP_IPV6_BLACKLIST, k6, 9)
        assert c.map_lookup(lib.MAP_IPV6_BLACKLIST, k6) == 9
        assert c.map_lookup(lib.MAP_IPV4_BLACKLIST, k4) is None
        assert c.map_delete(lib.MAP_IPV4_STATS, k4)
        assert not c.map_delete(lib.MAP_IPV4_STATS, k4)
        assert c.map_dump(lib.MAP_IPV6_BLACKLIST) == {k6: 9}
        c.map_update(lib.MAP_STATS, 0, (3, 4))
        assert c.stats() == (3, 4)
        c.reset()
        assert c.stats() == (0, 0) and c.map_dump(lib.MAP_IPV6_BLACKLIST) == {}


def test_empty_batch(native):
    with gpu_ctx(native) as c:
        v = c.verdict_batch(np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint64))
        assert v.size == 0 and c.stats() == (0, 0)


# ------------------------------------------------------------------ device entry + synth
def test_device_synth_and_device_batch(native, oracle):
    import torch
    from flowsentryx_amd import synth
    p, s = synth.config_params(2, n=1 << 20)
    n = int(p.n)
    d_hdr = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_len = torch.empty(n, dtype=torch.int32, device="cuda")
    d_ts = torch.empty(n, dtype=torch.int64, device="cuda")
    d_v = torch.empty(n, dtype=torch.uint8, device="cuda")
    synth.generate_device(p, s, 0, n, d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr())
    torch.cuda.synchronize()
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    assert np.array_equal(d_hdr.cpu().numpy().reshape(n, 64), hdr)
    assert np.array_equal(d_len.cpu().numpy().view(np.uint32), ln)
    assert np.array_equal(d_ts.cpu().numpy().view(np.uint64), ts)
    with gpu_ctx(native, max_entries=1 << 20, max_batch=n) as c:
        c.verdict_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n, d_v.data_ptr())
        c.sync()
        vo = oracle.Oracle(max_entries=1 << 20).batch(hdr, ln, ts)
        assert np.array_equal(d_v.cpu().numpy(), vo)
        info = c.last_batch_info()   # the heavy-source sort took the Zipf head out early
        assert 0 < info["light_packets"] < info["ip_packets"] * 0.6


# ------------------------------------------------------------------ heavy-source sort
def _uniform_stream(rng, n, n_ips, dt_max=50):
    from flowsentryx_amd import synth
    ips = rng.integers(0, 2**32, n_ips, dtype=np.uint64).astype(np.uint32)
    pick = rng.integers(0, n_ips, n)
    ln = rng.integers(60, 1515, n).astype(np.uint32)
    frames = [synth.frame_ipv4_udp(int(ips[j]).to_bytes(4, "big"), int(ln[i]))
              for i, j in enumerate(pick)]
    ts = 10**9 + np.cumsum(rng.integers(0, dt_max + 1, n)).astype(np.uint64)
    return synth.records(frames), ln, ts


@pytest.mark.parametrize("name", ["default", "tight"])
def test_heavy_sort_mixed_families(native, oracle, name):
    """Heavy IPv4 and IPv6 sources (DESIGN.md §3 heavy-source sort) across uneven batches."""
    rng = np.random.default_rng(41)
    hdr, ln, ts = rand_stream(rng, 200000, 3000, dt_max=40, v6_frac=0.5, nonip_frac=0.02,
                              short_frac=0.01)
    cuts = [0, 3, 70000, 70001, 200000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    run_both(native, oracle, batches, CFGS[name])


def test_heavy_sort_more_candidates_than_buckets(native, oracle):
    """400 equally heavy sources: 128 of them get their own first-pass bucket, the rest
    go through the light passes; same results either way."""
    rng = np.random.default_rng(42)
    hdr, ln, ts = _uniform_stream(rng, 120000, 400)
    with gpu_ctx(native) as c:
        vg = c.verdict_batch(hdr, ln, ts)
        info = c.last_batch_info()
        assert 0 < info["light_packets"] < info["ip_packets"]
    o = oracle.Oracle(max_entries=1 << 18)
    assert np.array_equal(vg, o.batch(hdr, ln, ts))
    run_both(native, oracle, [(hdr, ln, ts)], CFGS["tight"])


# ------------------------------------------------------------------ scoring
def _model(native, d):
    m = native.FsxQ8Model()
    for i, w in enumerate(d["weight"]):
        m.weight[i] = int(w)
    for k in ("weight_scale", "bias", "in_scale", "out_scale"):
        setattr(m, k, d[k])
    m.in_zero_point = d["in_zero_point"]
    m.out_zero_point = d["out_zero_point"]
    return m


def test_score_reference_model(native):
    g = np.load(GOLDEN / "score_vectors.npz")
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    with gpu_ctx(native) as c:
        c.load_q8_model(_model(native, ref))
        p, d = c.score(g["x_ref"])
    assert np.array_equal(p.view(np.uint32), g["p_ref"].view(np.uint32))
    assert np.array_equal(d, (g["p_ref"] > 0.5).astype(np.uint8))


def test_score_random_models(native):
    g = np.load(GOLDEN / "score_vectors.npz")
    models = json.loads((GOLDEN / "score_random_models.json").read_text())
    with gpu_ctx(native) as c:
        for i, m in enumerate(models):
            c.load_q8_model(_model(native, m))
            p, _ = c.score(g["rand_x"][i])
            assert np.array_equal(p.view(np.uint32), g["rand_p"][i].view(np.uint32)), i


# ------------------------------------------------------------------ flow features + scoring
def _sorted_flows(keys, fam, feat):
    order = sorted(range(len(fam)), key=lambda i: (int(fam[i]), keys[i].tobytes()))
    return keys[order], fam[order], feat[order]


def _check_flows(native, oracle, hdr, ln, ts, cfg=None):
    ko, fo, xo = oracle.flow_features(hdr, ln, ts)
    with gpu_ctx(native, **(cfg or {})) as c:
        kg, fg, xg = c.flow_features(hdr, ln, ts)
    assert len(fg) == len(fo)
    ko, fo, xo = _sorted_flows(ko, fo, xo)
    kg, fg, xg = _sorted_flows(kg, fg, xg)
    assert np.array_equal(fg, fo) and np.array_equal(kg, ko)
    bad = np.nonzero((xg.view(np.uint32) != xo.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:5], xg[bad[:3]], xo[bad[:3]])


def test_flow_features_random(native, oracle):
    rng = np.random.default_rng(31)
    hdr, ln, ts = rand_stream(rng, 60000, 700, dt_max=5000, v6_frac=0.3, nonip_frac=0.02,
                              short_frac=0.01)
    _check_flows(native, oracle, hdr, ln, ts)


def test_flow_features_header_variants(native, oracle):
    """The per-source port column on unusual headers: every IPv4 IHL 0..15 (the port's
    offset 14 + 4 IHL, past the 64-byte record for IHL > 12), TCP / UDP / other protocols,
    frames too short for the port, IPv6 with and without room for it; each source's first
    packet decides its port."""
    import struct
    from flowsentryx_amd import synth
    rng = np.random.default_rng(77)
    frames, lens = [], []
    for i in range(3000):
        src = bytes([10, 20, (i // 7) % 256, (i // 7) // 256 + 1])
        if i % 5 == 4:
            L = int(rng.choice([40, 54, 57, 58, 60, 100, 1500]))
            f = bytearray(synth.frame_ipv6_udp(bytes([0x20, 1]) + src + bytes(10), L,
                                              dport=int(rng.integers(0, 65536))))
            f[20] = int(rng.choice([6, 17, 58]))
        else:
            L = int(rng.choice([20, 33, 34, 37, 38, 41, 64, 80, 1500]))
            ihl = int(rng.integers(0, 16))
            f = bytearray(synth.frame_ipv4_udp(src, L, dport=int(rng.integers(0, 65536)), ihl_byte=0x40 | ihl))
            # a port word at every candidate offset, so a wrong offset reads different bytes
            for w in range(16, 62, 2):
                if w not in (26, 28):
                    f[w:w + 2] = struct.pack("!H", int(rng.integers(0, 65536)))
            f[23] = int(rng.choice([6, 17, 1]))
        frames.append(bytes(f[:64]))
        lens.append(L)
    hdr = synth.records(frames)
    ln = np.array(lens, dtype=np.uint32)
    ts = np.cumsum(rng.integers(1, 1000, len(ln))).astype(np.uint64)
    _check_flows(native, oracle, hdr, ln, ts)


def test_flow_features_heavy_sources(native, oracle):
    """Config-1 stream: 1024 Zipf sources over 1M packets, so the heavy sources span
    hundreds of flow tiles (exercises the cross-tile combine)."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(1)
    hdr, ln, ts = oracle.synth(p, s, 0, p.n)
    _check_flows(native, oracle, hdr, ln, ts)


def test_flow_features_long_spans(native, oracle):
    """Config-1 sources over 4M packets: the top source has ~750K packets (~730 flow tiles),
    so k_flow_combine's four-partials-per-lane loop (sources spanning >= 194 tiles) runs,
    not only its remainder loop."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(1, n=1 << 22)
    hdr, ln, ts = oracle.synth(p, s, 0, int(p.n))
    _, counts = np.unique(hdr[:, 26:30].copy().view(np.uint32), return_counts=True)
    assert counts.max() >= 194 * 1024
    _check_flows(native, oracle, hdr, ln, ts, cfg=dict(max_batch=1 << 22))


def _process_batch_device(native, oracle, batches, max_entries=1 << 20):
    """Verdicts + per-source features + q8 scores of each batch in one device call on one
    context (maps carried), against the oracle's verdicts and its per-batch flow rows."""
    import torch
    from flowsentryx_amd import fsx_load
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    o = oracle.Oracle(max_entries=max_entries)
    cap = max(len(b[0]) for b in batches)
    dev = lambda a: torch.from_numpy(a.view(np.uint8).reshape(-1)).cuda()
    d_v = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_k = torch.empty(cap * 16, dtype=torch.uint8, device="cuda")
    d_f = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(cap * 8, dtype=torch.float32, device="cuda")
    d_p = torch.empty(cap, dtype=torch.float32, device="cuda")
    d_d = torch.empty(cap, dtype=torch.uint8, device="cuda")
    with gpu_ctx(native, max_entries=max_entries, max_batch=cap) as c:
        c.load_q8_model(fsx_load.model_from_dict(ref))
        for hdr, ln, ts in batches:
            n = len(ln)
            d_hdr, d_len, d_ts = dev(hdr), dev(ln), dev(ts)
            c.process_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                                   d_v.data_ptr(), d_k.data_ptr(), d_f.data_ptr(), d_x.data_ptr(),
                                   d_p.data_ptr(), d_d.data_ptr(), cap)
            c.sync()
            m = c.last_batch_info()["sources"]
            assert np.array_equal(d_v[:n].cpu().numpy(), o.batch(hdr, ln, ts))
            kg = d_k.cpu().numpy().reshape(cap, 16)[:m]
            fg = d_f.cpu().numpy()[:m]
            xg = d_x.cpu().numpy().reshape(cap, 8)[:m]
            pg = d_p.cpu().numpy()[:m]
            ko, fo, xo = oracle.flow_features(hdr, ln, ts)
            assert m == len(fo)
            order_g = sorted(range(m), key=lambda i: (int(fg[i]), kg[i].tobytes()))
            order_o = sorted(range(m), key=lambda i: (int(fo[i]), ko[i].tobytes()))
            assert np.array_equal(kg[order_g], ko[order_o])
            assert np.array_equal(xg[order_g].view(np.uint32), xo[order_o].view(np.uint32))
            po, _, _ = oracle.score(ref, xo[order_o])
            assert np.array_equal(pg[order_g].view(np.uint32), po.view(np.uint32))


def test_process_batch_device(native, oracle):
    """Full path on device: verdicts + per-source features + q8 scores in one call (the
    fixed-window walkers finish the light sources' rows, the flow tiles the heavy ones)."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2, n=1 << 19)
    _process_batch_device(native, oracle, [oracle.synth(p, s, 0, int(p.n))])


@pytest.mark.parametrize("case", ["mixed", "gather", "jitter", "carry", "all_heavy", "nonip_only"])
def test_fused_flows(native, oracle, case):
    """The full path with the heavy-source machinery (light-only heads, heavy runs appended,
    heavy verdict lists, chunked heavy flow sums): mixed families with short / long / heavy
    sources, the gather path (no payload words), non-monotone clocks (exact wave replay,
    wrapped inter-arrival times), maps carried across batches, a stream whose sources are all
    heavy (no light entries) and one without IP packets."""
    from flowsentryx_amd import synth
    rng = np.random.default_rng(0xF10 + len(case))
    if case == "all_heavy":
        batches = [rand_stream(rng, 60_000, 40, dt_max=300, v6_frac=0.2)]
    elif case == "nonip_only":
        batches = [rand_stream(rng, 5_000, 10, dt_max=300, nonip_frac=1.0)]
    elif case == "mixed":
        batches = [rand_stream(rng, 300_000, 3000, dt_max=400, v6_frac=0.3, nonip_frac=0.03, short_frac=0.01)]
    elif case == "gather":
        p, s = synth.config_params(2, n=1 << 18)
        batches = [_with_far_nonip(*oracle.synth(p, s, 0, int(p.n)), 1 << 40)]
    elif case == "jitter":
        hdr, ln, ts = rand_stream(rng, 200_000, 1500, dt_max=300)
        sw = rng.choice(len(ts), len(ts) // 10, replace=False)
        ts[sw] = ts[sw] - rng.integers(0, 5000, sw.size).astype(np.uint64)
        batches = [(hdr, ln, ts)]
    else:
        p, s = synth.config_params(2, n=3 << 17)
        hdr, ln, ts = oracle.synth(p, s, 0, int(p.n))
        cut = [0, 100_000, 250_000, len(ln)]
        batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cut[:-1], cut[1:])]
    _process_batch_device(native, oracle, batches)


# ------------------------------------------------------------------ payload fallback
def _with_far_nonip(hdr, ln, ts, dt):
    """Append one ARP frame dt ns after the last packet: it takes no part in the
    limiter or the flows, but widens the batch's timestamp range."""
    from flowsentryx_amd import synth
    arp = synth.records([synth.frame_raw(0x0806, bytes(46), 60)])
    return (np.concatenate([hdr, arp]), np.concatenate([ln, np.array([60], np.uint32)]),
            np.concatenate([ts, np.array([int(ts[-1]) + dt], np.uint64)]))


@pytest.mark.parametrize("dt,payload", [(1, 1), ((1 << 40) - 10**9, 1), (1 << 40, 0)])
def test_sorted_payload_and_gather_paths(native, oracle, dt, payload):
    """Both ways of reading (ts, len) in sorted order: payload words carried by the
    sort (timestamps within 2^40 ns of the minimum) and the gather fallback."""
    rng = np.random.default_rng(77)
    hdr, ln, ts = rand_stream(rng, 40000, 400, dt_max=400, v6_frac=0.25, t0=10**12)
    hdr, ln, ts = _with_far_nonip(hdr, ln, ts, dt)
    for name in ("tight", "bytes_limit"):
        o = oracle.Oracle(**{k: v for k, v in CFGS[name].items()}, max_entries=1 << 18)
        with gpu_ctx(native, **CFGS[name]) as c:
            vg = c.verdict_batch(hdr, ln, ts)
            info = c.last_batch_info()
            assert info["sorted_payload"] == payload
            assert np.array_equal(vg, o.batch(hdr, ln, ts))
            assert_same_state(c, o)
    _check_flows(native, oracle, hdr, ln, ts)


def test_gather_path_large_frame_len(native, oracle):
    """A frame length >= 2^24 disables the payload words (len field is 24 bits)."""
    rng = np.random.default_rng(78)
    hdr, ln, ts = rand_stream(rng, 20000, 300, dt_max=400)
    ln[100] = 1 << 24
    for name in ("tight", "bytes_limit"):
        o = oracle.Oracle(**CFGS[name], max_entries=1 << 18)
        with gpu_ctx(native, **CFGS[name]) as c:
            vg = c.verdict_batch(hdr, ln, ts)
            assert c.last_batch_info()["sorted_payload"] == 0
            assert np.array_equal(vg, o.batch(hdr, ln, ts))
            assert_same_state(c, o)
    _check_flows(native, oracle, hdr, ln, ts)


# ------------------------------------------------------------------ batched map updates
@pytest.mark.parametrize("limiter,maps", [(0, (1, 2, 3, 4)), (1, (1, 2, 3, 4)), (2, (3, 4, 5, 6))])
def test_map_update_batch_restores_state(native, oracle, limiter, maps):
    """A restart: every map of one context dumped and batch-imported into a fresh one
    (stats_map with map_update); the next batch then gives identical verdicts, maps and
    stats on both (state carry through export/import, SURVEY §8 f row 1)."""
    rng = np.random.default_rng(51 + limiter)
    hdr, ln, ts = rand_stream(rng, 40000, 400, dt_max=300, v6_frac=0.3)
    cfg = dict(CFGS["tight"], limiter=limiter, max_entries=1 << 14)
    if limiter == 2:
        cfg = dict(limiter=2, tb_rate=300_000, tb_burst=4, max_entries=1 << 14)
    from flowsentryx_amd.lib import prefix_key
    maps = maps + (7, 8)   # with prefix rules: configuration travels too
    with gpu_ctx(native, **cfg) as a, gpu_ctx(native, **cfg) as b:
        for i in range(0, 2000, 97):
            a.map_update(7, prefix_key(bytes(hdr[i, 26:30]), 24 + i % 9), 2**64 - 1 if i % 3 else 0)
        a.map_update(8, prefix_key(bytes(16), 1), 2**64 - 1)
        a.verdict_batch(hdr[:20000], ln[:20000], ts[:20000])
        for m in maps:
            b.map_update_batch(m, a.map_dump(m))
        b.map_update(0, 0, a.stats())
        for m in maps:
            assert b.map_dump(m) == a.map_dump(m), m
        if limiter != 1:   # (the sliding window's carried logs are not map state)
            va = a.verdict_batch(hdr[20000:], ln[20000:], ts[20000:])
            vb = b.verdict_batch(hdr[20000:], ln[20000:], ts[20000:])
            assert np.array_equal(va, vb)
            assert a.stats() == b.stats()
            for m in maps:
                assert b.map_dump(m) == a.map_dump(m), m


def test_map_update_batch_all_or_nothing(native):
    from flowsentryx_amd import lib
    with gpu_ctx(native, max_entries=100, max_batch=1024) as c:
        c.map_update(3, bytes([1, 2, 3, 4]), 77)
        rules = {bytes([10, 0, i // 256, i % 256]): 2**64 - 1 for i in range(150)}
        with pytest.raises(lib.FsxError) as e:
            c.map_update_batch(3, rules)
        assert e.value.code == -errno.ENOSPC
        assert c.map_dump(3) == {bytes([1, 2, 3, 4]): 77}
        few = dict(list(rules.items())[:60])
        c.map_update_batch(3, few)
        assert c.map_dump(3) == {**few, bytes([1, 2, 3, 4]): 77}
        v6 = {bytes(range(i, i + 16)): (5, 6 + i, 7) for i in range(30)}
        c.map_update_batch(2, v6)
        assert c.map_dump(2) == v6
