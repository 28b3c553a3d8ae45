"""Pipelined batches (include/fsx_hip.h fsx_set_pipeline, DESIGN.md §3 "Pipelined batches").

The front of batch k + 1 (heavy pick, parse, sort) runs while the tail of batch k (walkers,
verdicts, flows) is still on the device, with alternating front buffers. Checked bit-exactly
against the oracle fed the same batches in order: every batch's verdicts (each batch keeps
its own output buffer; nothing is read before fsx_sync), its flow rows, stats_map and every
map entry at the end; map syscalls between pipelined batches; a failed batch cancelling
the one after it.
"""
import errno
import json

import numpy as np
import pytest

from kat import GOLDEN
from test_gpu_parity import MAPS, assert_same_state, rand_stream

pytestmark = pytest.mark.gpu


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).cuda()


def _flows_of(d, m):
    k = d["k"].cpu().numpy().reshape(-1, 16)[:m]
    f = d["f"].cpu().numpy()[:m]
    x = d["x"].cpu().numpy().reshape(-1, 8)[:m]
    p = d["p"].cpu().numpy()[:m]
    o = sorted(range(m), key=lambda i: (int(f[i]), k[i].tobytes()))
    return k[o], f[o], x[o], p[o]


def _run(native, oracle, batches, flows=True, between=None, max_entries=1 << 20):
    """All batches launched back to back on a pipelined context (one sync at the end),
    then each batch's verdicts / flow rows and the final maps against the oracle."""
    import torch
    from flowsentryx_amd import fsx_load
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    o = oracle.Oracle(max_entries=max_entries)
    cap = max(len(b[1]) for b in batches)
    bufs = []
    with native.FsxContext(max_batch=cap, max_entries=max_entries) as c:
        c.load_q8_model(fsx_load.model_from_dict(ref))
        c.set_pipeline(True)
        for j, (hdr, ln, ts) in enumerate(batches):
            n = len(ln)
            d = dict(h=_dev(torch, hdr), l=_dev(torch, ln), t=_dev(torch, ts),
                     v=torch.empty(n, dtype=torch.uint8, device="cuda"))
            if flows:
                d.update(k=torch.empty(n * 16, dtype=torch.uint8, device="cuda"),
                         f=torch.empty(n, dtype=torch.uint8, device="cuda"),
                         x=torch.empty(n * 8, dtype=torch.float32, device="cuda"),
                         p=torch.empty(n, dtype=torch.float32, device="cuda"),
                         d=torch.empty(n, dtype=torch.uint8, device="cuda"))
                c.process_batch_device(d["h"].data_ptr(), d["l"].data_ptr(), d["t"].data_ptr(), n,
                                       d["v"].data_ptr(), d["k"].data_ptr(), d["f"].data_ptr(),
                                       d["x"].data_ptr(), d["p"].data_ptr(), d["d"].data_ptr(), n)
            else:
                c.verdict_batch_device(d["h"].data_ptr(), d["l"].data_ptr(), d["t"].data_ptr(), n,
                                       d["v"].data_ptr())
            bufs.append(d)
            d["vo"] = o.batch(hdr, ln, ts)
            if between:
                between(j, c, o)
            if flows:
                d["fo"] = oracle.flow_features(hdr, ln, ts)
        c.sync()
        for j, d in enumerate(bufs):
            vg = d["v"].cpu().numpy()
            bad = np.nonzero(vg != d["vo"])[0]
            assert bad.size == 0, f"batch {j}: {bad.size} verdicts differ, first at {bad[:8]}"
        if flows:
            # rows of the last batch (every batch writes its own buffers; rows counted by
            # the last batch's facts), and of every batch by their own count
            for j, d in enumerate(bufs):
                ko, fo, xo = d["fo"]
                m = len(fo)
                kg, fg, xg, pg = _flows_of(d, m)
                oo = sorted(range(m), key=lambda i: (int(fo[i]), ko[i].tobytes()))
                assert np.array_equal(kg, ko[oo]), j
                assert np.array_equal(xg.view(np.uint32), xo[oo].view(np.uint32)), j
                po, _, _ = oracle.score(ref, xo[oo])
                assert np.array_equal(pg.view(np.uint32), po.view(np.uint32)), j
            assert c.last_batch_info()["sources"] == len(bufs[-1]["fo"][1])
        assert_same_state(c, o)


def _config2_batches(oracle, n, cuts):
    from flowsentryx_amd import synth
    p, s = synth.config_params(2, n=n)
    hdr, ln, ts = oracle.synth(p, s, 0, int(p.n))
    return [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]


def test_pipelined_config2_flows(native, oracle):
    """Four uneven batches of a config-2 stream (the heavy-source path active), features +
    scores, maps carried, launched back to back."""
    n = 1 << 20
    _run(native, oracle, _config2_batches(oracle, n, [0, 300_000, 300_001, 700_000, n]))


def test_pipelined_replayed_stream(native, oracle):
    """The warm streaming case of bench.py: the same batch shifted by its duration, 5 times."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(2, n=1 << 19)
    hdr, ln, ts = oracle.synth(p, s, 0, int(p.n))
    batches = [(hdr, ln, ts + np.uint64(k * int(p.duration_ns))) for k in range(5)]
    _run(native, oracle, batches)


def test_pipelined_mixed_families_verdicts(native, oracle):
    """Mixed IPv4 / IPv6 / non-IP / short frames, a jittered (non-monotone) batch between
    monotone ones, verdicts only, many small batches."""
    rng = np.random.default_rng(0x919E)
    hdr, ln, ts = rand_stream(rng, 240_000, 2500, dt_max=60, v6_frac=0.3, nonip_frac=0.02,
                              short_frac=0.01)
    sw = rng.choice(np.arange(100_000, 140_000), 3000, replace=False)
    ts[sw] -= rng.integers(0, 4000, sw.size).astype(np.uint64)
    cuts = [0, 1, 5000, 60_000, 100_000, 140_000, 141_000, 240_000]
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    _run(native, oracle, batches, flows=False, max_entries=1 << 18)


def test_pipelined_map_ops_between_batches(native, oracle):
    """A map update and a lookup between pipelined batches see (and order after) the batches
    enqueued before them."""
    from flowsentryx_amd import lib
    batches = _config2_batches(oracle, 1 << 19, [0, 200_000, 400_000, 1 << 19])
    key = batches[1][0][5, 26:30].tobytes()   # a source of the stream, blacklisted by hand

    def between(j, c, o):
        if j == 0:
            till = int(batches[1][2][0]) + 10**12
            c.map_update(lib.MAP_IPV4_BLACKLIST, key, till)
            o.map_update(lib.MAP_IPV4_BLACKLIST, key, till)
            assert c.map_lookup(lib.MAP_IPV4_BLACKLIST, key) == till
    _run(native, oracle, batches, between=between)


def test_pipelined_failed_batch_cancels_next(native, oracle):
    """A batch that overflows max_entries fails; the batch launched after it is cancelled; the
    error surfaces at sync and neither changes any map; the context then carries on."""
    from flowsentryx_amd import lib, synth
    import torch
    rng = np.random.default_rng(77)
    cfg = dict(pps_threshold=5, window_ns=100_000, block_ns=300_000)
    h1, l1, t1 = rand_stream(rng, 3000, 120, dt_max=200)
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 77, i // 256, i % 256]), 90) for i in range(400)])
    lb = np.full(400, 90, np.uint32)
    tb = t1[-1] + np.arange(1, 401, dtype=np.uint64)
    h3, l3, t3 = rand_stream(rng, 3000, 120, dt_max=200)
    t3 = t3 + tb[-1]
    h4, l4, t4 = rand_stream(rng, 3000, 120, dt_max=200)
    t4 = t4 + t3[-1]
    o = oracle.Oracle(max_entries=1 << 12, **cfg)
    keep = []

    def launch(c, h, l, t):
        d = [_dev(torch, h), _dev(torch, l), _dev(torch, t), torch.empty(len(l), dtype=torch.uint8, device="cuda")]
        keep.append(d)
        c.verdict_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(l), d[3].data_ptr())
        return d[3]

    with native.FsxContext(max_batch=4096, max_entries=300, **cfg) as c:
        c.set_pipeline(True)
        v1 = launch(c, h1, l1, t1)
        c.sync()
        assert np.array_equal(v1.cpu().numpy(), o.batch(h1, l1, t1))
        before = {m: c.map_dump(m) for m in MAPS}
        s_before = c.stats()
        launch(c, big, lb, tb)          # fails: 400 new sources > 300 - 120
        launch(c, h3, l3, t3)           # cancelled by the device
        with pytest.raises(lib.FsxError) as e:
            c.sync()
        assert e.value.code == -errno.ENOSPC
        assert {m: c.map_dump(m) for m in MAPS} == before
        assert c.stats() == s_before
        v4 = launch(c, h4, l4, t4)
        c.sync()
        assert np.array_equal(v4.cpu().numpy(), o.batch(h4, l4, t4))
        assert_same_state(c, o)


def test_pipelined_failure_found_by_a_later_call(native, oracle):
    """Four calls in a row: the fourth finds the first one's failure (it waits for the batch
    three back before reusing its buffers), returns its error and enqueues nothing; the two
    batches in between were cancelled on the device and are rolled back too."""
    from flowsentryx_amd import lib, synth
    import torch
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 78, i // 256, i % 256]), 90) for i in range(400)])
    ln = np.full(400, 90, np.uint32)
    ts = np.arange(1, 401, dtype=np.uint64) + 10**9
    d = [_dev(torch, big), _dev(torch, ln), _dev(torch, ts), torch.empty(400, dtype=torch.uint8, device="cuda")]
    with native.FsxContext(max_batch=4096, max_entries=300) as c:
        c.set_pipeline(True)
        args = (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 400, d[3].data_ptr())
        c.verdict_batch_device(*args)
        c.verdict_batch_device(*args)
        c.verdict_batch_device(*args)
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch_device(*args)
        assert e.value.code == -errno.ENOSPC
        c.sync()   # nothing left in flight
        assert len(c.map_dump(lib.MAP_IPV4_STATS)) == 0


@pytest.mark.parametrize("limiter", [1, 2])
def test_pipelined_other_limiters(native, oracle, limiter):
    """Sliding window and token bucket with pipelining on: each batch runs whole on the
    context stream, in order, without a host synchronization per call (device-side
    cancellation after a failure, as for the split fixed window)."""
    import torch
    rng = np.random.default_rng(0x51 + limiter)
    cfg = dict(pps_threshold=20, window_ns=200_000, block_ns=500_000, limiter=limiter,
               tb_rate=50_000, tb_burst=8)
    hdr, ln, ts = rand_stream(rng, 150_000, 800, dt_max=80, v6_frac=0.2, nonip_frac=0.01)
    cuts = [0, 20_000, 20_001, 90_000, 150_000]
    o = oracle.Oracle(max_entries=1 << 16, **cfg)
    maps = (3, 4, 5, 6) if limiter == 2 else MAPS
    outs = []
    with native.FsxContext(max_batch=1 << 17, max_entries=1 << 16, **cfg) as c:
        c.set_pipeline(True)
        for a, b in zip(cuts[:-1], cuts[1:]):
            d = [_dev(torch, hdr[a:b]), _dev(torch, ln[a:b]), _dev(torch, ts[a:b]),
                 torch.empty(b - a, dtype=torch.uint8, device="cuda")]
            c.verdict_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), b - a, d[3].data_ptr())
            outs.append((d, o.batch(hdr[a:b], ln[a:b], ts[a:b])))
        c.sync()
        for j, (d, vo) in enumerate(outs):
            assert np.array_equal(d[3].cpu().numpy(), vo), j
        assert c.stats() == o.stats()
        for m in maps:
            assert c.map_dump(m) == o.map_dump(m), m


def test_pipelined_host_pointer_batches(native, oracle):
    """fsx_verdict_batch (host buffers, staged) on a pipelined context: the copy back waits
    for the batch's deferred tail."""
    rng = np.random.default_rng(0x4057)
    hdr, ln, ts = rand_stream(rng, 120_000, 900, dt_max=100, v6_frac=0.2)
    o = oracle.Oracle(max_entries=1 << 18)
    with native.FsxContext(max_batch=1 << 17, max_entries=1 << 18) as c:
        c.set_pipeline(True)
        for a, b in ((0, 50_000), (50_000, 50_001), (50_001, 120_000)):
            assert np.array_equal(c.verdict_batch(hdr[a:b], ln[a:b], ts[a:b]), o.batch(hdr[a:b], ln[a:b], ts[a:b]))
        assert_same_state(c, o)


def test_pipelined_wide_ids(native, oracle):
    """Pipelined batches on a 2^25-slot table (the heavy-source sort with two 9-bit light
    passes, DESIGN.md §3: heavy runs and light entries in pass 0's buffer, 512-digit tiles and
    tile-scan bases in each front set): three uneven batches of the config-4 population with
    features + scores."""
    from flowsentryx_amd import synth
    p, s = synth.config_params(4)
    n = 1 << 20
    hdr, ln, ts = oracle.synth(p, s, 0, n)
    cuts = [0, 250_000, 250_001, n]
    _run(native, oracle, [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])],
         max_entries=16 << 20)


def test_pipelined_reset_and_import_between_batches(native, oracle):
    """fsx_reset (a new index epoch: the IPv4 mirror is cleared) and a batched map import
    between pipelined batches: the next batch's early prologue (heavy-source pick, which may
    insert into the index) must run after them, not beside them."""
    from flowsentryx_amd import lib
    batches = _config2_batches(oracle, 1 << 19, [0, 150_000, 300_000, 420_000, 1 << 19])
    keys = [bytes(batches[2][0][i, 26:30]) for i in range(0, 2000, 7)]   # sources of the stream
    entries = {k: (3, 77_000, int(batches[2][2][0])) for k in keys}

    def between(j, c, o):
        if j == 0:
            c.reset()
            o.reset()
        elif j == 1:
            c.map_update_batch(lib.MAP_IPV4_STATS, entries)
            for k, v in entries.items():
                o.map_update(lib.MAP_IPV4_STATS, k, v)
    _run(native, oracle, batches, between=between)


def test_pipelined_sliding_window_history_full(native, oracle):
    """Split sliding-window batches check their history room in their tail (after the
    previous tail set it): logs that keep every packet (huge thresholds, 10 s window) fill
    the history buffer; the batch that does not fit fails with -ENOSPC, it and the batches
    after it are rolled back, and the state equals an unpipelined context's that stopped at
    the same batch and the oracle's over the batches before it."""
    import torch
    from flowsentryx_amd import lib
    rng = np.random.default_rng(0x415)
    B = 1 << 15
    cfg = dict(limiter=1, pps_threshold=10**6, bps_threshold=10**12, window_ns=10**10, block_ns=10**9,
               max_entries=1 << 16, max_batch=B)
    hdr, ln, ts = rand_stream(rng, 12 * B, 3000, dt_max=100)
    batches = [(hdr[k * B:(k + 1) * B], ln[k * B:(k + 1) * B], ts[k * B:(k + 1) * B]) for k in range(12)]
    failed = None
    with native.FsxContext(**cfg) as cu:
        for j, b in enumerate(batches):
            try:
                cu.verdict_batch(*b)
            except lib.FsxError as e:
                assert e.code == -errno.ENOSPC
                failed = j
                break
        assert failed is not None and failed >= 2, failed
        o = oracle.Oracle(**{k: v for k, v in cfg.items() if k != "max_batch"})
        for b in batches[:failed]:
            o.batch(*b)
        with native.FsxContext(**cfg) as cp:
            cp.set_pipeline(True)
            d = [(_dev(torch, h), _dev(torch, l), _dev(torch, t), torch.empty(B, dtype=torch.uint8, device="cuda"))
                 for h, l, t in batches]
            raised = False
            for x in d:
                try:
                    cp.verdict_batch_device(x[0].data_ptr(), x[1].data_ptr(), x[2].data_ptr(), B, x[3].data_ptr())
                except lib.FsxError as e:
                    assert e.code == -errno.ENOSPC
                    raised = True
                    break
            if not raised:
                with pytest.raises(lib.FsxError) as e:
                    cp.sync()
                assert e.value.code == -errno.ENOSPC
            cp.sync()
            assert cp.stats() == cu.stats() == o.stats()
            for m in MAPS:
                assert cp.map_dump(m) == cu.map_dump(m) == o.map_dump(m), m


def test_pipelined_sliding_window_history_full_then_fits(native, oracle):
    """the batch after a split sliding-window batch that fails its history check
    in its tail must not run, even when it would fit by itself (here: a small batch after a
    large one that overflows). Its k_batch_check may run before the failure is known, so
    the tail of every later split batch cancels itself (TableState::tail_fail): the state
    equals an unpipelined context's that stopped at the failed batch, and the oracle's over
    the batches before it."""
    import torch
    from flowsentryx_amd import lib
    rng = np.random.default_rng(0x416)
    B = 1 << 15   # history buffer: max(2 B, 64K) = 65536 entries
    cfg = dict(limiter=1, pps_threshold=10**6, bps_threshold=10**12, window_ns=10**10, block_ns=10**9,
               max_entries=1 << 16, max_batch=B)
    sizes = [B, 20000, B, 4096, 2048]   # 32768 + 20000 fit; + 32768 overflows; + 4096 would fit
    hdr, ln, ts = rand_stream(rng, sum(sizes), 3000, dt_max=100)
    cuts = np.cumsum([0] + sizes)
    batches = [(hdr[a:b], ln[a:b], ts[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    with native.FsxContext(**cfg) as cu:
        failed = None
        for j, b in enumerate(batches):
            try:
                cu.verdict_batch(*b)
            except lib.FsxError as e:
                assert e.code == -errno.ENOSPC
                failed = j
                break
        assert failed == 2, failed
        o = oracle.Oracle(**{k: v for k, v in cfg.items() if k != "max_batch"})
        for b in batches[:failed]:
            o.batch(*b)
        for rep in range(3):   # (the race depends on timing: a few tries, each from empty maps)
            with native.FsxContext(**cfg) as cp:
                cp.set_pipeline(True)
                d = [(_dev(torch, h), _dev(torch, l), _dev(torch, t), torch.empty(len(l), dtype=torch.uint8, device="cuda"))
                     for h, l, t in batches]
                raised = False
                for x, b in zip(d, batches):
                    try:
                        cp.verdict_batch_device(x[0].data_ptr(), x[1].data_ptr(), x[2].data_ptr(), len(b[1]),
                                                x[3].data_ptr())
                    except lib.FsxError as e:
                        assert e.code == -errno.ENOSPC
                        raised = True
                        break
                if not raised:
                    with pytest.raises(lib.FsxError) as e:
                        cp.sync()
                    assert e.value.code == -errno.ENOSPC
                cp.sync()
                assert cp.stats() == cu.stats() == o.stats(), rep
                for m in MAPS:
                    assert cp.map_dump(m) == cu.map_dump(m) == o.map_dump(m), (rep, m)
                # after the rollback the context works on: the small batch now runs and fits
                cp.verdict_batch(*batches[3])
                cp.sync()


@pytest.mark.parametrize("same_batch,resets", [(False, 1), (True, 1), (False, 2)])
def test_pipelined_reset_every_batch(native, oracle, same_batch, resets):
    """fsx_reset after every pipelined batch (the bench's cold leg): each reset swaps in the
    spare table set (slots, scalars, index) and clears it on the device after the tails that
    last used it, without a host synchronization and without ordering the next front after
    the last tail (DESIGN.md §3 "Pipelined resets"). Every batch equals the oracle from empty
    maps; the final maps are the last batch's; features + scores of every batch."""
    batches = _config2_batches(oracle, 1 << 19, [0, 150_000, 300_000, 420_000, 1 << 19])
    if same_batch:
        batches = [batches[1]] * 5

    def between(j, c, o):
        if j < len(batches) - 1:
            for _ in range(resets):   # (two in a row: the second swaps the sets back)
                c.reset()
            o.reset()
    _run(native, oracle, batches, between=between)


def test_pipelined_reset_into_recycled_spare(native, oracle, monkeypatch):
    """The spare table set may come from recycled device memory: with
    FSX_TEST_SPARE_POISON its slots are filled at allocation with live-looking lines of the
    very table generation the first pipelined reset moves to (state + blacklist entries). The
    allocation zeroes it, so after the swap-in verdicts, stats_map and every map dump equal
    the oracle's from empty maps — no phantom source."""
    monkeypatch.setenv("FSX_TEST_SPARE_POISON", "1")
    batches = _config2_batches(oracle, 1 << 18, [0, 100_000, 200_000, 1 << 18])

    def between(j, c, o):
        if j < len(batches) - 1:
            c.reset()
            o.reset()
    _run(native, oracle, batches, between=between)


def test_pipelined_failed_batch_then_reset(native, oracle):
    """A batch fails (max_entries) and the caller resets before its error is seen: the batch
    after the reset runs on fresh tables and is not cancelled; the error surfaces at sync;
    the maps are those of the batch after the reset alone."""
    from flowsentryx_amd import lib, synth
    import torch
    rng = np.random.default_rng(79)
    cfg = dict(pps_threshold=5, window_ns=100_000, block_ns=300_000)
    h1, l1, t1 = rand_stream(rng, 3000, 120, dt_max=200)
    big = synth.records([synth.frame_ipv4_udp(bytes([10, 77, i // 256, i % 256]), 90) for i in range(400)])
    lb = np.full(400, 90, np.uint32)
    tb = t1[-1] + np.arange(1, 401, dtype=np.uint64)
    h3, l3, t3 = rand_stream(rng, 3000, 120, dt_max=200, v6_frac=0.3)
    t3 = t3 + tb[-1]
    keep = []

    def launch(c, h, l, t):
        d = [_dev(torch, h), _dev(torch, l), _dev(torch, t), torch.empty(len(l), dtype=torch.uint8, device="cuda")]
        keep.append(d)
        c.verdict_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(l), d[3].data_ptr())
        return d[3]

    with native.FsxContext(max_batch=4096, max_entries=300, **cfg) as c:
        c.set_pipeline(True)
        launch(c, h1, l1, t1)
        launch(c, big, lb, tb)          # fails: 400 new sources > 300 - 120
        c.reset()                       # (pipelined: no wait, the spare tables swapped in)
        v3 = launch(c, h3, l3, t3)
        with pytest.raises(lib.FsxError) as e:
            c.sync()
        assert e.value.code == -errno.ENOSPC
        o = oracle.Oracle(max_entries=1 << 12, **cfg)
        assert np.array_equal(v3.cpu().numpy(), o.batch(h3, l3, t3))
        assert_same_state(c, o)
        v4 = launch(c, h3, l3, t3 + t3[-1])   # (the same 225 sources: no new ones)
        c.sync()
        assert np.array_equal(v4.cpu().numpy(), o.batch(h3, l3, t3 + t3[-1]))
        assert_same_state(c, o)
