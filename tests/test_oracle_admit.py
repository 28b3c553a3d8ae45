"""CPU: FSX_FLAG_OVERFLOW_ADMIT in the oracle (oracle/fsx_oracle.c; include/fsx_hip.h,
DESIGN.md §2.2) against a direct Python transcription of the policy over the reference's
fixed window (src/fsx_kern.c:150-346): in arrival order, an untracked source is admitted
while fewer than max_entries sources are tracked, else it is transient for the batch (maps
of its own that start empty with the batch and are never visible).

Build-defined (the reference's LRU_HASH eviction is not reproducible): parity unpinned."""
import numpy as np
import pytest

from test_gpu_parity import rand_stream
from test_oracle_limiters import _src

U64 = (1 << 64) - 1


def spec_admit_fixed(batches, P, B, W, BLK, max_entries):
    """-> per batch (verdicts, (admitted, transient)), final stats, ip_stats, blacklist."""
    st, bl, tracked = {}, {}, set()
    allowed = dropped = 0
    out = []

    def packet(s, L, now, st_, bl_):
        nonlocal allowed, dropped
        till = bl_.get(s)
        if till is not None and till > 0:
            if now > till:
                del bl_[s]
            else:
                dropped += 1
                return 1
        if s in st_:
            pps, bps, tt = st_[s]
            if ((now - tt) & U64) > W:
                st_[s] = (0, 0, now)
                cp, cb = 0, 0
            else:
                st_[s] = (pps + 1, bps + L, tt)
                cp, cb = pps + 1, bps + L
        else:
            st_[s] = (1, L, now)
            cp, cb = 1, L
        if cp > P or cb > B:
            bl_[s] = (now + BLK) & U64
            dropped += 1
            return 1
        allowed += 1
        return 2

    for hdr, ln, ts in batches:
        tst, tbl, trans = {}, {}, set()
        adm = 0
        v = []
        for i in range(len(ln)):
            s = _src(hdr[i], int(ln[i]))
            if s == "drop":
                v.append(1)
                continue
            if s == "pass":
                v.append(2)
                continue
            if s not in tracked and s not in trans:
                if len(tracked) < max_entries:
                    tracked.add(s)
                    adm += 1
                else:
                    trans.add(s)
            if s in trans:
                v.append(packet(s, int(ln[i]), int(ts[i]), tst, tbl))
            else:
                v.append(packet(s, int(ln[i]), int(ts[i]), st, bl))
        out.append((np.array(v, np.uint8), (adm, len(trans))))
    return out, (allowed, dropped), st, bl


@pytest.mark.parametrize("max_entries,P", [(3, 4), (17, 6), (40, 2), (1000, 5)])
def test_admission_matches_spec(oracle, max_entries, P):
    rng = np.random.default_rng(max_entries * 7 + P)
    cfg = dict(pps_threshold=P, bps_threshold=1 << 40, window_ns=3000, block_ns=9000)
    batches = []
    t0 = 0
    for k in range(3):
        hdr, ln, ts = rand_stream(rng, 3000, 60, dt_max=30, v6_frac=0.25, nonip_frac=0.03, short_frac=0.02)
        ts = ts + np.uint64(t0)
        t0 = int(ts[-1]) + 1
        batches.append((hdr, ln, ts))
    want, stats, st, bl = spec_admit_fixed(batches, P, cfg["bps_threshold"], cfg["window_ns"], cfg["block_ns"],
                                           max_entries)
    o = oracle.Oracle(flags=oracle.OVERFLOW_ADMIT, max_entries=max_entries, **cfg)
    for (hdr, ln, ts), (v, counts) in zip(batches, want):
        assert np.array_equal(o.batch(hdr, ln, ts), v)
        assert o.admit_last() == counts
    assert o.stats() == stats
    for fam, mid in ((4, 1), (6, 2)):
        got = o.map_dump(mid)
        exp = {k: vv for (f, k), vv in st.items() if f == fam}
        assert got == exp
    for fam, mid in ((4, 3), (6, 4)):
        got = o.map_dump(mid)
        exp = {k: vv for (f, k), vv in bl.items() if f == fam}
        assert got == exp


def test_transient_state_lives_for_one_batch(oracle):
    """max_entries 1: A is admitted; B floods (P + 3 packets per batch) and is transient in
    both batches, so it passes P packets in each of them (its blacklist entry of the first
    batch is not carried) while A's state carries."""
    from flowsentryx_amd import synth
    P = 3
    a, b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    frames = [synth.frame_ipv4_udp(a)] + [synth.frame_ipv4_udp(b)] * (P + 3)
    hdr = synth.records(frames)
    ln = np.full(len(frames), 100, np.uint32)
    o = oracle.Oracle(flags=oracle.OVERFLOW_ADMIT, max_entries=1, pps_threshold=P)
    for k in range(2):
        ts = (10**9 * (k + 1) + np.arange(len(frames))).astype(np.uint64)
        v = o.batch(hdr, ln, ts)
        assert list(v) == [2] + [2] * P + [1] * 3
        assert o.admit_last() == ((1, 1) if k == 0 else (0, 1))
    assert set(o.map_dump(1)) == {a}
    assert o.map_dump(3) == {}
    assert o.stats() == (2 * (P + 1), 6)


def test_rule_dropped_sources_are_never_admitted(oracle):
    """A source whose packets a prefix rule drops never reaches the per-source maps: it
    takes no admission room (DESIGN.md §4.3 order: rules first)."""
    from flowsentryx_amd import lib, synth
    a, b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    hdr = synth.records([synth.frame_ipv4_udp(a), synth.frame_ipv4_udp(b)])
    ln = np.full(2, 100, np.uint32)
    o = oracle.Oracle(flags=oracle.OVERFLOW_ADMIT, max_entries=1)
    o.map_update(lib.MAP_IPV4_PREFIX, lib.prefix_key(a, 32), 2**64 - 1)
    v = o.batch(hdr, ln, np.array([5, 6], np.uint64))
    assert list(v) == [1, 2]
    assert o.admit_last() == (1, 0)
    assert set(o.map_dump(1)) == {b}


def test_admission_with_idle_eviction(oracle):
    """FSX_FLAG_EVICT_IDLE first (an idle source leaves), then admission."""
    from flowsentryx_amd import synth
    srcs = [bytes([10, 0, 0, i]) for i in range(1, 5)]
    o = oracle.Oracle(flags=oracle.OVERFLOW_ADMIT | oracle.EVICT_IDLE, max_entries=2, window_ns=100)
    hdr = synth.records([synth.frame_ipv4_udp(srcs[0]), synth.frame_ipv4_udp(srcs[1])])
    o.batch(hdr, np.full(2, 100, np.uint32), np.array([10, 11], np.uint64))
    assert o.admit_last() == (2, 0)
    # s0 idle at t = 500 (window 100 expired), s1 too: both evicted, s2 and s3 admitted
    hdr = synth.records([synth.frame_ipv4_udp(srcs[2]), synth.frame_ipv4_udp(srcs[3])])
    o.batch(hdr, np.full(2, 100, np.uint32), np.array([500, 501], np.uint64))
    assert o.evicted_last() == 2 and o.admit_last() == (2, 0)
    assert set(o.map_dump(1)) == {srcs[2], srcs[3]}
