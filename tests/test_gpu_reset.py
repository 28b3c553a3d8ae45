"""GPU: clear-free fsx_reset (DESIGN.md §3 "Clear-free reset").

A reset moves the table to its next generation instead of clearing it: a slot's tag word
carries the generation, and a line of an older one reads as empty. Each case leaves the
table full of the previous generation's lines — the same sources again, so their probes land
on slots that still hold their own old state — and checks verdicts, stats_map and every map
dump against an oracle that was reset for real; for all three limiters, both families, the
prefix-rule path (heavy sources inserted lazily), map updates into stale slots, and the
16-bit generation wrap (the table then cleared for real).
"""
import numpy as np
import pytest

from test_gpu_parity import rand_stream

pytestmark = pytest.mark.gpu

KEYS = ("pps_threshold", "bps_threshold", "window_ns", "block_ns", "max_entries", "tb_rate", "tb_burst",
        "limiter")


def _check(c, o, maps):
    assert c.stats() == o.stats()
    for m in maps:
        g, r = c.map_dump(m), o.map_dump(m)
        assert len(g) == len(r), (m, len(g), len(r))
        assert g == r, m


def _batches(seed, n=60000, n_ips=3000):
    rng = np.random.default_rng(seed)
    h1, l1, t1 = rand_stream(rng, n, n_ips, dt_max=300, v6_frac=0.3, nonip_frac=0.02, short_frac=0.01)
    h2, l2, t2 = rand_stream(rng, n, n_ips, dt_max=300, v6_frac=0.3)
    return [(h1, l1, t1), (h2, l2, t2 + t1[-1]), (h1, l1, t1 + t1[-1] + t2[-1])]   # (3rd: 1st's sources)


@pytest.mark.parametrize("limiter,maps", [(0, (1, 2, 3, 4)), (1, (1, 2, 3, 4)), (2, (3, 4, 5, 6))])
def test_reset_reads_old_generation_as_empty(native, oracle, limiter, maps):
    cfg = dict(limiter=limiter, pps_threshold=40, window_ns=200_000, block_ns=1_000_000,
               tb_rate=300_000, tb_burst=4, max_entries=1 << 14)
    o = oracle.Oracle(**{k: v for k, v in cfg.items() if k in KEYS})
    with native.FsxContext(max_batch=1 << 17, **cfg) as c:
        for j, (h, ln, t) in enumerate(_batches(31 + limiter)):
            if j:
                c.reset()
                o.reset()
            assert np.array_equal(c.verdict_batch(h, ln, t), o.batch(h, ln, t)), j
            _check(c, o, maps)
        # a map update after a reset lands in a stale slot of the same key
        key = bytes(_batches(31 + limiter)[0][0][5, 26:30])
        c.reset()
        o.reset()
        assert c.map_dump(3) == {} and c.map_dump(1) == {}
        c.map_update(3, key, 123)
        o.map_update(3, key, 123)
        _check(c, o, maps)


def test_reset_with_prefix_rules_heavy_lazy(native, oracle):
    """Prefix rules: the heavy sources are inserted lazily by the parse and adopted by the
    run-path heavy walker — over stale lines of their own after a reset."""
    from flowsentryx_amd.lib import prefix_key
    cfg = dict(pps_threshold=40, window_ns=200_000, block_ns=1_000_000, max_entries=1 << 14)
    o = oracle.Oracle(**cfg)
    b = _batches(41, n=120000, n_ips=2000)
    with native.FsxContext(max_batch=1 << 17, **cfg) as c:
        rule = prefix_key(bytes([b[0][0][7, 26], 0, 0, 0]), 8)   # one /8 of the stream's sources
        c.map_update(7, rule, 2**64 - 1)
        o.map_update(7, rule, 2**64 - 1)
        for j, (h, ln, t) in enumerate(b):
            if j:
                c.reset()
                o.reset()
            assert np.array_equal(c.verdict_batch(h, ln, t), o.batch(h, ln, t)), j
            _check(c, o, (1, 2, 3, 4))


def test_reset_generation_wrap(native, oracle):
    """65536 resets wrap the 16-bit table generation: the table is cleared for real then, so
    lines of the generation that comes round again do not come back."""
    cfg = dict(pps_threshold=40, window_ns=200_000, block_ns=1_000_000, max_entries=1 << 12)
    o = oracle.Oracle(**cfg)
    b = _batches(43, n=8000, n_ips=500)
    with native.FsxContext(max_batch=1 << 14, **cfg) as c:
        h, ln, t = b[0]
        assert np.array_equal(c.verdict_batch(h, ln, t), o.batch(h, ln, t))
        for _ in range(65536):   # (host-side only: no batch between them)
            c.reset()
        o.reset()
        h, ln, t = b[1]
        assert np.array_equal(c.verdict_batch(h, ln, t), o.batch(h, ln, t))
        _check(c, o, (1, 2, 3, 4))
