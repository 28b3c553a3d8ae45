"""FSX_FLAG_EVICT_IDLE on the GPU against the oracle's restatement:
verdicts, stats_map, per-batch eviction counts and the map contents, bit-exact.
Parity unpinned (build-defined policy; the reference's LRU_HASH eviction is kernel code)."""
import errno

import numpy as np
import pytest

from test_gpu_parity import rand_stream
from test_oracle_evict import S, key, pkts

pytestmark = pytest.mark.gpu

MAPS = (1, 2, 3, 4)


def same_state(c, o):
    assert c.stats() == o.stats()
    for m in MAPS:
        assert c.map_dump(m) == o.map_dump(m), m


def run_both(native, oracle, batches, updates=(), pipeline=False, **cfg):
    o = oracle.Oracle(flags=oracle.EVICT_IDLE, **cfg)
    evicted = []
    with native.FsxContext(flags=native.FLAG_EVICT_IDLE, max_batch=1 << 17, **cfg) as c:
        if pipeline:
            c.set_pipeline(True)
        for mid, k, v in updates:
            c.map_update(mid, k, v)
            o.map_update(mid, k, v)
        for hdr, ln, ts in batches:
            vg = c.verdict_batch(hdr, ln, ts)
            vo = o.batch(hdr, ln, ts)
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
            c.sync()
            ev = c.last_batch_info()["evicted"]
            assert ev == o.evicted_last()
            evicted.append(ev)
        same_state(c, o)
    return evicted


def test_hand_made_sequence(native, oracle):
    batches = [pkts([(1, 0), (1, 1), (1, 2), (2, 3), (3, 4)]), pkts([(4, int(2.5 * S))]),
               pkts([(5, 3 * S), (6, 3 * S + 1)])]
    assert run_both(native, oracle, batches, max_entries=4, pps_threshold=2) == [0, 0, 2]


def test_blacklist_only_and_deleted_entries(native, oracle):
    ups = [(3, key(7), 5 * S), (1, key(8), (0, 0, 0)), (3, key(9), 0)]
    batches = [pkts([(1, 4 * S)]), pkts([(2, 6 * S)]), pkts([(3, 6 * S)])]
    o = oracle.Oracle(flags=oracle.EVICT_IDLE, max_entries=3)
    with native.FsxContext(flags=native.FLAG_EVICT_IDLE, max_batch=1024, max_entries=3) as c:
        for mid, k, v in ups:
            c.map_update(mid, k, v)
            o.map_update(mid, k, v)
        c.map_delete(1, key(8))
        o.map_delete(1, key(8))
        for b in batches:
            assert np.array_equal(c.verdict_batch(*b), o.batch(*b))
            assert c.last_batch_info()["evicted"] == o.evicted_last()
        same_state(c, o)


def test_overflow_with_nothing_idle_is_enospc(native):
    from flowsentryx_amd import lib
    with native.FsxContext(flags=native.FLAG_EVICT_IDLE, max_batch=1024, max_entries=2) as c:
        c.verdict_batch(*pkts([(1, 0), (2, 1)]))
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(*pkts([(3, S)]))
        assert e.value.code == -errno.ENOSPC
        # the failed batch changed nothing; an idle moment later the batch fits
        v = c.verdict_batch(*pkts([(3, 3 * S)]))
        assert list(v) == [2] and c.last_batch_info()["evicted"] == 2


@pytest.mark.parametrize("pipeline", [False, True])
def test_config2_stream_at_max_track_ips(native, oracle, pipeline):
    """The config-2 source population (1M Zipf(1.1) sources, 30 s) at 1/16 of its packet
    rate, in 64 batches of 65536 packets, with the reference's MAX_TRACK_IPS = 100000:
    about 12K sources are evicted before every batch from the fourth on."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    p.n = 4 << 20
    B = 1 << 16
    batches = [oracle.synth(p, s, b, B) for b in range(0, p.n, B)]
    ev = run_both(native, oracle, batches, pipeline=pipeline, max_entries=100000)
    assert sum(ev) > 500000 and ev[0] == 0


def test_mixed_families_with_gaps(native, oracle):
    rng = np.random.default_rng(31)
    hdr, ln, ts = rand_stream(rng, 60000, 3000, dt_max=40, v6_frac=0.4, nonip_frac=0.05)
    # six batches 0.4 ms apart in time, window 1 ms: sources of three batches back go idle;
    # up to 3488 sources tracked (both families share max_entries)
    cuts = np.linspace(0, len(ts), 7).astype(int)
    batches = []
    for j, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        t = ts[a:b] - ts[a] + np.uint64(10**9 + j * 400_000)
        batches.append((hdr[a:b], ln[a:b], t))
    ev = run_both(native, oracle, batches, max_entries=4000, pps_threshold=20, window_ns=1_000_000,
                  block_ns=500_000)
    assert sum(ev) > 0
