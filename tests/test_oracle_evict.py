"""FSX_FLAG_EVICT_IDLE in the oracle (oracle/fsx_oracle.c evict_idle):
the build-defined overflow policy, restated on hand-made streams whose evictions are
worked out by hand. Parity unpinned (the reference's LRU_HASH eviction is kernel code)."""
import errno

import numpy as np
import pytest

from flowsentryx_amd import synth

S = 1_000_000_000


def pkts(rows):
    """rows: (ipv4 last byte, ts ns[, len]) -> hdr, len, ts."""
    frames = [synth.frame_ipv4_udp(bytes([10, 0, 0, r[0]]), r[2] if len(r) > 2 else 100) for r in rows]
    return (synth.records(frames), np.array([r[2] if len(r) > 2 else 100 for r in rows], np.uint32),
            np.array([r[1] for r in rows], np.uint64))


def key(b):
    return bytes([10, 0, 0, b])


def test_idle_sources_evicted_live_kept(oracle):
    o = oracle.Oracle(max_entries=4, pps_threshold=2, flags=oracle.EVICT_IDLE)
    # A (1) exceeds 2 pps at t=0 and is blacklisted till 10 s; B, C seen once at t=0
    o.batch(*pkts([(1, 0), (1, 1), (1, 2), (2, 3), (3, 4)]))
    assert o.evicted_last() == 0 and o.map_lookup(3, key(1)) == 2 + 10 * S
    # D at 2.5 s: 3 tracked + 1 packet = 4 <= 4, no eviction
    o.batch(*pkts([(4, int(2.5 * S))]))
    assert o.evicted_last() == 0
    # E, F at 3 s: 4 + 2 > 4 -> B, C idle (window from t=0 expired, no blacklist) go;
    # A keeps a live blacklist entry; D's window (2.5 s) is still open
    v = o.batch(*pkts([(5, 3 * S), (6, 3 * S + 1)]))
    assert o.evicted_last() == 2
    assert list(v) == [2, 2]
    assert set(o.map_dump(1)) == {key(1), key(4), key(5), key(6)}
    assert set(o.map_dump(3)) == {key(1)}


def test_window_boundary_is_the_reset_test(oracle):
    """now0 - track_time == window is not expired (src/fsx_kern.c:245 uses >)."""
    o = oracle.Oracle(max_entries=2, flags=oracle.EVICT_IDLE)
    o.batch(*pkts([(1, 0), (2, 1)]))
    with pytest.raises(RuntimeError):     # 2 + 1 > 2, but A (S - 0 > S? no) and B are live:
        o.batch(*pkts([(3, S)]))          # nothing to evict, the map overflows
    assert o.evicted_last() == 0
    o2 = oracle.Oracle(max_entries=2, flags=oracle.EVICT_IDLE)
    o2.batch(*pkts([(1, 0), (2, 1)]))
    o2.batch(*pkts([(3, S + 1)]))         # A: S + 1 - 0 > S -> idle; B: S + 1 - 1 = S -> kept
    assert o2.evicted_last() == 1
    assert set(o2.map_dump(1)) == {key(2), key(3)}


def test_expired_blacklist_and_deleted_entries(oracle):
    o = oracle.Oracle(max_entries=3, flags=oracle.EVICT_IDLE)
    o.map_update(3, key(7), 5 * S)            # blacklist entry only, till 5 s
    o.map_update(1, key(8), (0, 0, 0))        # stats entry, window from t=0
    o.map_update(3, key(9), 0)                # till 0: never live
    o.map_delete(1, key(8))                   # deleted: still tracked, idle
    o.batch(*pkts([(1, 4 * S)]))              # 3 + 1 > 3: 8 and 9 go, 7 (till 5 s) stays
    assert o.evicted_last() == 2
    assert set(o.map_dump(3)) == {key(7)}
    o.batch(*pkts([(2, 6 * S)]))              # 2 + 1 <= 3
    assert o.evicted_last() == 0
    o.batch(*pkts([(3, 6 * S)]))              # 3 + 1 > 3: 7 (expired at 6 s) and 1 go
    assert o.evicted_last() == 2
    assert set(o.map_dump(1)) == {key(2), key(3)} and o.map_dump(3) == {}


def test_without_flag_nothing_is_evicted(oracle):
    o = oracle.Oracle(max_entries=2)
    o.batch(*pkts([(1, 0), (2, 1)]))
    with pytest.raises(RuntimeError):
        o.batch(*pkts([(3, 5 * S)]))
    assert o.evicted_last() == 0


def test_flag_rejected_for_other_limiters():
    """fsx_open refuses FSX_FLAG_EVICT_IDLE outside the fixed window (before any device
    call, so this runs without a GPU)."""
    from flowsentryx_amd import build, lib
    build.build_all(only_missing=True)
    for lim in (lib.LIMIT_SLIDING_WINDOW, lib.LIMIT_TOKEN_BUCKET):
        with pytest.raises(lib.FsxError) as e:
            lib.FsxContext(limiter=lim, flags=lib.FLAG_EVICT_IDLE, max_batch=1024)
        assert e.value.code == -errno.EINVAL


def test_families_share_the_capacity(oracle):
    """Like the device table, IPv4 and IPv6 sources count against one max_entries."""
    o = oracle.Oracle(max_entries=3, flags=oracle.EVICT_IDLE)
    v6 = synth.records([synth.frame_ipv6_udp(bytes([0x20, 1] + [0] * 13 + [i]), 100) for i in (1, 2)])
    o.batch(v6, np.full(2, 100, np.uint32), np.array([0, 1], np.uint64))
    o.batch(*pkts([(1, 2)]))
    with pytest.raises(RuntimeError):
        o.batch(*pkts([(2, 3)]))      # 3 + 1 > 3, nothing idle: the fourth source overflows
