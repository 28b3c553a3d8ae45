"""GPU: FSX_FLAG_OVERFLOW_ADMIT (include/fsx_hip.h) against the oracle's
restatement (oracle/fsx_oracle.c): floods beyond max_entries keep getting verdicts. In
arrival order, a new source is admitted (tracked, the maps as usual) while fewer than
max_entries sources are tracked, else it is transient for its batch (fresh state that is
never visible). Verdicts, stats_map, every map entry and the admitted / transient counts,
bit-exact — under all three limiters, at the reference's MAX_TRACK_IPS = 100000
(src/fsx_struct.h:7) on a BASELINE config-5 carpet slice."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ADMIT = 8   # FSX_FLAG_OVERFLOW_ADMIT


def _check(native, oracle, batches, cfg, maps=(1, 2, 3, 4), rules=None, expect=None, pipeline=False):
    from oracle import pyoracle
    o = oracle.Oracle(flags=oracle.OVERFLOW_ADMIT, **cfg)
    cap = max(len(b[1]) for b in batches)
    got_counts = []
    with native.FsxContext(flags=ADMIT, max_batch=cap, **cfg) as c:
        for m, entries in (rules or {}).items():
            c.map_update_batch(m, entries)
            for k, v in entries.items():
                o.map_update(m, k, v)
        if pipeline:
            c.set_pipeline(True)
        for hdr, ln, ts in batches:
            vg = c.verdict_batch(hdr, ln, ts)
            vo = o.batch(hdr, ln, ts)
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
            info = c.last_batch_info()
            counts = (info["admitted"], info["transient"])
            assert counts == o.admit_last(), (counts, o.admit_last())
            got_counts.append(counts)
        assert c.stats() == o.stats()
        for m in maps:
            g, r = c.map_arrays(m), o.map_arrays(m)
            assert g[0].shape[0] == r[0].shape[0], (m, g[0].shape[0], r[0].shape[0])
            assert pyoracle.same_map(g, r), m
    if expect:
        expect(got_counts)
    return got_counts


def _carpet(oracle, n, j0=0):
    from flowsentryx_amd import synth
    p, s = synth.config_params(5, n=1 << 24)
    return oracle.synth(p, s, j0, n)


@pytest.mark.parametrize("limiter", [0, 1, 2], ids=["fixed", "sliding", "token"])
def test_config5_carpet_at_max_track_ips(native, oracle, limiter):
    """Two consecutive 2^22-packet batches of the config-5 carpet (every packet a fresh
    spoofed source, IPv4 / IPv6 / 802.1Q) at max_entries = 100000: the first 100000 new
    sources are admitted, every later one is transient, every packet gets a verdict."""
    n = 1 << 22
    hdr, ln, ts = _carpet(oracle, 2 * n)
    cfg = dict(max_entries=100_000, limiter=limiter)
    if limiter == 2:
        cfg.update(tb_rate=2000, tb_burst=3)
    maps = (3, 4, 5, 6) if limiter == 2 else (1, 2, 3, 4)

    def expect(counts):
        assert counts[0][0] == 100_000 and counts[0][1] > 3_000_000
        assert counts[1][0] == 0 and counts[1][1] > 3_000_000
    _check(native, oracle, [(hdr[:n], ln[:n], ts[:n]), (hdr[n:], ln[n:], ts[n:])], cfg, maps, expect=expect)


def test_config5_carpet_with_rule_table(native, oracle):
    """The carpet with a user rule table (exact + prefix rules, test_gpu_scale.carpet_rules):
    rule-dropped sources take no room."""
    from test_gpu_scale import carpet_rules
    n = 1 << 22
    hdr, ln, ts = _carpet(oracle, n)
    rules = carpet_rules(hdr, np.random.default_rng(7), 4096, 1024, 4096, 256)
    _check(native, oracle, [(hdr, ln, ts)], dict(max_entries=100_000), rules=rules)


def test_zipf_flood_beyond_capacity_with_heavy_sources(native, oracle):
    """The config-2 population (1M Zipf sources) at max_entries = 50000 over two batches:
    heavy sources admitted early, the tail largely transient; blacklists of admitted
    sources carry, transient ones restart every batch."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    hdr, ln, ts = oracle.synth(p, s, 0, 1 << 21)
    h = 1 << 20
    _check(native, oracle, [(hdr[:h], ln[:h], ts[:h]), (hdr[h:], ln[h:], ts[h:])], dict(max_entries=50_000))


def test_pipelined_admission(native, oracle):
    """Pipelined calls (admission batches run whole on the context stream)."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    hdr, ln, ts = oracle.synth(p, s, 0, 3 << 18)
    k = 1 << 18
    _check(native, oracle, [(hdr[i * k:(i + 1) * k], ln[i * k:(i + 1) * k], ts[i * k:(i + 1) * k]) for i in range(3)],
           dict(max_entries=20_000), pipeline=True)


def test_transient_flood_source_small(native, oracle):
    """max_entries 1: A admitted, B transient in both batches (P passes per batch, its
    blacklist not carried); the maps hold A only."""
    from flowsentryx_amd import synth
    P = 3
    a, b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    frames = [synth.frame_ipv4_udp(a)] + [synth.frame_ipv4_udp(b)] * (P + 3)
    hdr = synth.records(frames)
    ln = np.full(len(frames), 100, np.uint32)
    batches = [(hdr, ln, (10**9 * (k + 1) + np.arange(len(frames))).astype(np.uint64)) for k in range(2)]
    counts = _check(native, oracle, batches, dict(max_entries=1, pps_threshold=P))
    assert counts == [(1, 1), (0, 1)]
