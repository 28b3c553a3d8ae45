"""GPU parity of the build-defined limiters against the CPU oracle.

The reference only names a token bucket and a sliding window (README.md:155-162), so
these are parity-unpinned: the oracle (oracle/fsx_oracle.c) restates the in-repo spec
sequentially, the GPU evaluates it in parallel (a segmented clamp-add scan for the
token bucket), and the two must agree bit-exactly: verdicts, stats_map, the blacklist
maps and the per-source limiter state maps.
"""
import zlib

import numpy as np
import pytest

from test_gpu_parity import rand_stream

pytestmark = pytest.mark.gpu

TB = 2
ORACLE_KEYS = ("pps_threshold", "bps_threshold", "window_ns", "block_ns", "max_entries",
               "tb_rate", "tb_burst", "limiter")


def run_limiter(native, oracle, batches, cfg, maps, rules=()):
    cfg = dict(cfg)
    cfg.setdefault("max_entries", 1 << 16)
    okw = {k: v for k, v in cfg.items() if k in ORACLE_KEYS}
    o = oracle.Oracle(**okw)
    with native.FsxContext(max_batch=1 << 20, **cfg) as c:
        for mid, key, val in rules:
            c.map_update(mid, key, val)
            o.map_update(mid, key, val)
        for hdr, ln, ts in batches:
            vg = c.verdict_batch(hdr, ln, ts)
            vo = o.batch(hdr, ln, ts)
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
        assert c.stats() == o.stats()
        for m in maps:
            g, r = c.map_dump(m), o.map_dump(m)
            assert len(g) == len(r), (m, len(g), len(r))
            assert g == r, m
        return c.stats()


TB_MAPS = (3, 4, 5, 6)
TB_CFGS = {
    "default": {},                                         # 1000 tok/s, burst 1000
    "mixed": {"tb_rate": 300_000, "tb_burst": 4},          # heavy sources alternate
    "slow": {"tb_rate": 20_000, "tb_burst": 2},
    "no_refill": {"tb_rate": 0, "tb_burst": 3},
    "burst_zero": {"tb_rate": 10**6, "tb_burst": 0},      # capacity < cost: all drop
    "saturating": {"tb_rate": 1 << 40, "tb_burst": 1},
    "max_burst": {"tb_rate": 1 << 20, "tb_burst": 2305843009},
}


@pytest.fixture(params=["sorted", "unsorted_heavy"])
def tb_path(request, monkeypatch):
    """Both token-bucket paths: every packet through the heavy-source sort (the default), and
    the heavy sources outside the sort (FSX_TB_UNSORTED=1; small batches pick up
    to 128 heavy sources too, and the run-path refusals — capacity below one token, a clock step
    back, blacklisted heavy sources — take the run path with tagged heavy packets)."""
    if request.param == "unsorted_heavy":
        monkeypatch.setenv("FSX_TB_UNSORTED", "1")
    else:
        monkeypatch.delenv("FSX_TB_UNSORTED", raising=False)
    return request.param


@pytest.mark.parametrize("name", list(TB_CFGS))
def test_token_bucket_random(native, oracle, name, tb_path):
    rng = np.random.default_rng(zlib.crc32(b"tb" + name.encode()))
    hdr, ln, ts = rand_stream(rng, 60000, 300, dt_max=400)
    st = run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=TB, **TB_CFGS[name]), TB_MAPS)
    if name == "burst_zero":
        assert st[0] == 0
    if name == "mixed":
        assert st[0] > 1000 and st[1] > 1000


def test_token_bucket_mixed_families(native, oracle, tb_path):
    rng = np.random.default_rng(21)
    hdr, ln, ts = rand_stream(rng, 40000, 600, dt_max=300, v6_frac=0.4, nonip_frac=0.05,
                              short_frac=0.03)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=TB, **TB_CFGS["mixed"]), TB_MAPS)


def test_token_bucket_state_carry(native, oracle, tb_path):
    rng = np.random.default_rng(22)
    hdr, ln, ts = rand_stream(rng, 30000, 200, dt_max=300, v6_frac=0.2)
    cuts = [0, 1, 2, 777, 4096, 4097, 17000, 29999, 30000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    run_limiter(native, oracle, batches, dict(limiter=TB, **TB_CFGS["mixed"]), TB_MAPS)


def test_token_bucket_heavy_source(native, oracle, tb_path):
    """One source with most packets of a 300k-packet batch: a segment spanning ~60 scan
    tiles, alternating verdicts inside one tile."""
    rng = np.random.default_rng(23)
    hdr, ln, ts = rand_stream(rng, 300000, 8, dt_max=100)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=TB, tb_rate=4_000_000, tb_burst=7),
                TB_MAPS)


def test_token_bucket_non_monotone_clock(native, oracle, tb_path):
    rng = np.random.default_rng(24)
    hdr, ln, ts = rand_stream(rng, 20000, 100, dt_max=200)
    sw = rng.choice(len(ts), 3000, replace=False)
    ts[sw] = ts[sw] - rng.integers(0, 50000, sw.size).astype(np.uint64)
    ts[7] = np.uint64(2**64 - 3)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=TB, **TB_CFGS["mixed"]), TB_MAPS)


def test_token_bucket_with_rules_and_state_updates(native, oracle, tb_path):
    """Static and expiring blacklist rules apply before the bucket (src/fsx_kern.c:159-216
    semantics); user-written bucket states are honoured."""
    rng = np.random.default_rng(25)
    hdr, ln, ts = rand_stream(rng, 30000, 60, dt_max=300)
    srcs = sorted({bytes(hdr[i, 26:30]) for i in range(0, 30000, 97)})
    t_mid = int(ts[15000])
    rules = []
    for i, k in enumerate(srcs[:24]):
        if i % 4 == 0:
            rules.append((3, k, 2**64 - 1))          # static block
        elif i % 4 == 1:
            rules.append((3, k, t_mid))              # expires mid-batch
        elif i % 4 == 2:
            rules.append((3, k, 0))                  # till = 0: ignored (:189)
        else:
            rules.append((5, k, (123_456_789, int(ts[0]) - 10)))  # preset bucket state
    batches = [(hdr[:15000], ln[:15000], ts[:15000]), (hdr[15000:], ln[15000:], ts[15000:])]
    run_limiter(native, oracle, batches, dict(limiter=TB, **TB_CFGS["mixed"]), TB_MAPS, rules)


def test_token_bucket_rejects_oversized_burst(native):
    with pytest.raises(native.FsxError):
        native.FsxContext(limiter=TB, tb_burst=2305843010)


# ------------------------------------------------------------------ sliding window
SW = 1
SW_MAPS = (1, 2, 3, 4)
SW_CFGS = {
    "default": {},
    "tight": {"pps_threshold": 7, "window_ns": 200_000, "block_ns": 1_000_000},
    "block_lt_window": {"pps_threshold": 5, "window_ns": 1_000_000, "block_ns": 50_000},
    "block_zero": {"pps_threshold": 3, "window_ns": 100_000, "block_ns": 0},
    "bytes_limit": {"pps_threshold": 50, "bps_threshold": 9_000, "window_ns": 500_000,
                    "block_ns": 2_000_000},
    "pps_zero": {"pps_threshold": 0, "window_ns": 100_000, "block_ns": 300_000},
    "window_zero": {"pps_threshold": 3, "window_ns": 0, "block_ns": 100_000},
}


@pytest.mark.parametrize("name", list(SW_CFGS))
def test_sliding_window_random(native, oracle, name):
    rng = np.random.default_rng(zlib.crc32(b"sw" + name.encode()))
    hdr, ln, ts = rand_stream(rng, 60000, 300, dt_max=400)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=SW, **SW_CFGS[name]), SW_MAPS)


@pytest.mark.parametrize("name", ["tight", "block_lt_window", "bytes_limit"])
def test_sliding_window_heavy_sources(native, oracle, name):
    """Few sources, long segments: the wave walkers (epoch scan on monotone clocks; the
    exact replay when a byte trigger is possible)."""
    rng = np.random.default_rng(31)
    hdr, ln, ts = rand_stream(rng, 200000, 6, dt_max=60)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=SW, **SW_CFGS[name]), SW_MAPS)


@pytest.mark.parametrize("name", ["default", "tight", "block_lt_window"])
def test_sliding_window_mixed_families(native, oracle, name):
    rng = np.random.default_rng(32 + len(name))
    hdr, ln, ts = rand_stream(rng, 40000, 500, dt_max=300, v6_frac=0.4, nonip_frac=0.05,
                              short_frac=0.03)
    run_limiter(native, oracle, [(hdr, ln, ts)], dict(limiter=SW, **SW_CFGS[name]), SW_MAPS)


@pytest.mark.parametrize("name", ["tight", "block_lt_window", "bytes_limit"])
def test_sliding_window_state_carry(native, oracle, name):
    """Carried logs across uneven batch cuts (down to one packet), including sources
    idle for many windows (their logs are pruned by the batch clock)."""
    rng = np.random.default_rng(33)
    hdr, ln, ts = rand_stream(rng, 60000, 40, dt_max=200, v6_frac=0.2)
    cuts = [0, 1, 2, 777, 4096, 4097, 17000, 30000, 45000, 59999, 60000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    run_limiter(native, oracle, batches, dict(limiter=SW, **SW_CFGS[name]), SW_MAPS)


def test_sliding_window_long_sources_across_batches(native, oracle):
    """Heavy sources whose logs (up to P entries) are carried into the next batch and
    consumed by the wave walker."""
    rng = np.random.default_rng(34)
    hdr, ln, ts = rand_stream(rng, 240000, 5, dt_max=40)
    cfg = dict(limiter=SW, pps_threshold=900, window_ns=1_000_000, block_ns=400_000)
    cuts = [0, 50000, 50001, 120000, 240000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    run_limiter(native, oracle, batches, cfg, SW_MAPS)


def test_sliding_window_non_monotone_clock(native, oracle):
    rng = np.random.default_rng(35)
    hdr, ln, ts = rand_stream(rng, 40000, 30, dt_max=200)
    sw = rng.choice(len(ts), 5000, replace=False)
    ts[sw] = ts[sw] - rng.integers(0, 50000, sw.size).astype(np.uint64)
    ts[9] = np.uint64(2**64 - 7)
    batches = [(ts_[0], ts_[1], ts_[2]) for ts_ in
               ((hdr[:20000], ln[:20000], ts[:20000]), (hdr[20000:], ln[20000:], ts[20000:]))]
    run_limiter(native, oracle, batches, dict(limiter=SW, **SW_CFGS["tight"]), SW_MAPS)


def test_sliding_window_rules(native, oracle):
    rng = np.random.default_rng(36)
    hdr, ln, ts = rand_stream(rng, 30000, 60, dt_max=300)
    srcs = sorted({bytes(hdr[i, 26:30]) for i in range(0, 30000, 97)})
    t_mid = int(ts[15000])
    rules = []
    for i, k in enumerate(srcs[:24]):
        rules.append((3, k, [2**64 - 1, t_mid, 0][i % 3]))
    batches = [(hdr[:15000], ln[:15000], ts[:15000]), (hdr[15000:], ln[15000:], ts[15000:])]
    run_limiter(native, oracle, batches, dict(limiter=SW, **SW_CFGS["tight"]), SW_MAPS, rules)


def test_sliding_window_rejects_large_threshold(native):
    with pytest.raises(native.FsxError):
        native.FsxContext(limiter=SW, pps_threshold=1 << 24)
