"""GPU: heavy sources outside the sort (DESIGN.md §3 "Heavy sources outside the sort").

The fixed and sliding windows' heavy sources are walked by rank over the arrival order
(select / rank over the tagged verdict bytes) and their flow rows come from per-tile sums,
when k_hmode finds the batch eligible; otherwise k_heavy_gather builds their runs and the run path
takes over. Both paths, bit-exact against the oracle: verdicts, stats_map, every map entry,
and the per-source features + q8 scores (src/fsx_kern.c:150-346, model/model.py:132-137)."""
import json

import numpy as np
import pytest

from kat import GOLDEN

pytestmark = pytest.mark.gpu


def _run(native, oracle, batches, cfg, prepare=None, want_path=None, pipeline=False, cap=None,
         maps=(1, 2, 3, 4)):
    """Each batch through fsx_process_batch_device on one context (maps carried); after each
    one: verdicts, flow rows and (at the end) stats + maps against the oracle. Returns the
    heavy_unsorted flag of every batch."""
    import torch
    from flowsentryx_amd import fsx_load
    from oracle import pyoracle
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    o = oracle.Oracle(**cfg)
    cap = cap or max(len(b[1]) for b in batches)   # (also sizes the sliding-window history: 2 x cap)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).cuda()
    out = dict(v=torch.empty(cap, dtype=torch.uint8, device="cuda"),
               k=torch.empty(cap * 16, dtype=torch.uint8, device="cuda"),
               f=torch.empty(cap, dtype=torch.uint8, device="cuda"),
               x=torch.empty(cap * 8, dtype=torch.float32, device="cuda"),
               p=torch.empty(cap, dtype=torch.float32, device="cuda"),
               d=torch.empty(cap, dtype=torch.uint8, device="cuda"))
    paths = []
    with native.FsxContext(max_batch=cap, **cfg) as c:
        c.load_q8_model(fsx_load.model_from_dict(ref))
        if prepare:
            prepare(c, o)
        if pipeline:
            c.set_pipeline(True)
        for hdr, ln, ts in batches:
            n = len(ln)
            d_hdr, d_len, d_ts = dev(hdr), dev(ln), dev(ts)
            c.process_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n, out["v"].data_ptr(),
                                   out["k"].data_ptr(), out["f"].data_ptr(), out["x"].data_ptr(),
                                   out["p"].data_ptr(), out["d"].data_ptr(), cap)
            c.sync()
            info = c.last_batch_info()
            paths.append(info["heavy_unsorted"])
            vo = o.batch(hdr, ln, ts)
            bad = np.nonzero(out["v"][:n].cpu().numpy() != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
            m = info["sources"]
            kg = out["k"].cpu().numpy().reshape(cap, 16)[:m]
            fg = out["f"].cpu().numpy()[:m]
            xg = out["x"].cpu().numpy().reshape(cap, 8)[:m]
            pg = out["p"].cpu().numpy()[:m]
            ko, fo, xo = oracle.flow_features(hdr, ln, ts)
            assert m == len(fo)
            og = sorted(range(m), key=lambda i: (int(fg[i]), kg[i].tobytes()))
            oo = sorted(range(m), key=lambda i: (int(fo[i]), ko[i].tobytes()))
            assert np.array_equal(kg[og], ko[oo])
            bad = np.nonzero((xg[og].view(np.uint32) != xo[oo].view(np.uint32)).any(axis=1))[0]
            assert bad.size == 0, (bad[:4], xg[og][bad[:2]], xo[oo][bad[:2]])
            po, _, _ = oracle.score(ref, xo[oo])
            assert np.array_equal(pg[og].view(np.uint32), po.view(np.uint32))
        assert c.stats() == o.stats()
        for mid in maps:
            g, r = c.map_arrays(mid), o.map_arrays(mid)
            assert g[0].shape[0] == r[0].shape[0], mid
            assert pyoracle.same_map(g, r), mid
    if want_path is not None:
        assert paths == want_path, paths
    return paths


def _config2(oracle, n, j0=0):
    from flowsentryx_amd import synth
    p, s = synth.config_params(2)
    return oracle.synth(p, s, j0, n)


CFG = dict(max_entries=1 << 20)   # a 2^21-slot table: the heavy-source sort with verdict lists


@pytest.mark.parametrize("max_entries", [1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 23, 1 << 24])
def test_unsorted_heavy_path_config2_slices(native, oracle, max_entries):
    """Two carried 1M-packet slices of the config-2 stream (heads blacklisted across the
    cut): both batches on the unsorted path, everything equal to the oracle. Tables of 2^20
    to 2^25 slots: 6-, 7- and 8-bit light digits, two light passes up to 23-bit ids and three
    for 24 / 25 (an 8-bit light pass once overwrote the heavy buckets' pass-0 tile rows the
    walker reads)."""
    hdr, ln, ts = _config2(oracle, 1 << 21)
    cut = 1 << 20
    _run(native, oracle, [(hdr[:cut], ln[:cut], ts[:cut]), (hdr[cut:], ln[cut:], ts[cut:])],
         dict(CFG, max_entries=max_entries), want_path=[1, 1])


def test_corrupted_heavy_row_fails_not_hangs(native, oracle, monkeypatch):
    """round 5's aliasing bug (ff010e0) corrupted the heavy sources'
    pass-0 tile-count rows and the rank view's search never ended. With the rows overwritten
    through a test hook (FSX_TEST_HEAVY_ROW_CORRUPT), the bounded searches (fsx_search.h)
    flag ERR_HEAVY_VIEW and the batch fails with -EIO; a fresh context afterwards is exact."""
    import errno
    from flowsentryx_amd import lib
    hdr, ln, ts = _config2(oracle, 1 << 20)
    monkeypatch.setenv("FSX_TEST_HEAVY_ROW_CORRUPT", "1")
    with native.FsxContext(max_batch=1 << 20, **CFG) as c:
        with pytest.raises(lib.FsxError) as e:
            c.verdict_batch(hdr, ln, ts)
        assert e.value.code == -errno.EIO
        assert "rank view" in str(e.value)
    monkeypatch.delenv("FSX_TEST_HEAVY_ROW_CORRUPT")
    _run(native, oracle, [(hdr, ln, ts)], CFG, want_path=[1])


def test_unsorted_heavy_path_pipelined(native, oracle):
    """The same slices pipelined (the tail of one batch beside the next batch's front:
    per-set tile sums and chunk counts)."""
    hdr, ln, ts = _config2(oracle, 3 << 19)
    k = 1 << 19
    _run(native, oracle, [(hdr[i * k:(i + 1) * k], ln[i * k:(i + 1) * k], ts[i * k:(i + 1) * k]) for i in range(3)],
         CFG, pipeline=True)


def test_non_monotone_clock_takes_the_run_path(native, oracle):
    """A timestamp that goes back: k_hmode sends the batch to the run path (k_heavy_gather)."""
    hdr, ln, ts = _config2(oracle, 1 << 20)
    ts = ts.copy()
    ts[500_000], ts[500_001] = ts[500_001], ts[500_000] - 7
    _run(native, oracle, [(hdr, ln, ts)], CFG, want_path=[0])


def test_tile_spanning_2_32_ns_takes_the_run_path(native, oracle):
    """A 5 s gap inside one sort tile (gap squares could pass 2^64 in a tile's u64 sum)."""
    hdr, ln, ts = _config2(oracle, 1 << 20)
    ts = ts.copy()
    ts[300_000:] += 5_000_000_000
    _run(native, oracle, [(hdr, ln, ts)], CFG, want_path=[0])


def test_reachable_byte_trigger_takes_the_run_path(native, oracle):
    """bps_threshold below (pps + 1) x the largest frame: the byte trigger is reachable."""
    hdr, ln, ts = _config2(oracle, 1 << 20)
    cfg = dict(CFG, bps_threshold=300_000)
    _run(native, oracle, [(hdr, ln, ts)], cfg, want_path=[0])


def test_carried_state_off_the_epoch_path(native, oracle):
    """A heavy source whose carried ip_stats cannot take epoch jumps (track_time near
    2^64): the batch takes the run path, the carried entry is honoured exactly."""
    hdr, ln, ts = _config2(oracle, 1 << 20)
    src, cnt = np.unique(hdr[:, 26:30].copy().view(np.uint32).reshape(-1), return_counts=True)
    top = int(src[np.argmax(cnt)]).to_bytes(4, "little")

    def prepare(c, o):
        val = (3, 300, 2**64 - 5)
        c.map_update(1, top, val)
        o.map_update(1, top, val)
    _run(native, oracle, [(hdr, ln, ts)], CFG, prepare=prepare, want_path=[0])


def test_blacklisted_heavy_source_carried(native, oracle):
    """Heavy sources entering the batch blacklisted (map 3 entries, one expiring mid-batch,
    one permanent) on the unsorted path."""
    hdr, ln, ts = _config2(oracle, 1 << 20)
    src, cnt = np.unique(hdr[:, 26:30].copy().view(np.uint32).reshape(-1), return_counts=True)
    order = np.argsort(-cnt)
    a, b = (int(src[order[i]]).to_bytes(4, "little") for i in (0, 3))
    mid = int(ts[len(ts) // 2])

    def prepare(c, o):
        for k, v in ((a, mid), (b, 2**64 - 1)):
            c.map_update(3, k, v)
            o.map_update(3, k, v)
    _run(native, oracle, [(hdr, ln, ts)], CFG, prepare=prepare, want_path=[1])


SW = dict(CFG, limiter=1)   # the sliding window's heavy verdict lists (3-pass sort: 21-bit ids)


@pytest.mark.parametrize("case", ["default", "slices", "slices4", "sparse", "sparse_pipelined", "non_monotone",
                                  "byte_trigger", "blacklisted", "pipelined", "pps_over_staging"])
def test_sliding_window_heavy_lists(native, oracle, case):
    """The sliding window with heavy verdict lists: by default on the heavy-source
    sort (k_walk_sw_heavy over the pass-0 runs). With FSX_FLAG_SW_UNSORTED (A/B), monotone
    clocks and the byte trigger out of reach: k_walk_sw_heavy_sel walks each heavy source by rank over the
    arrival order and stages its final log for the history rebuild (heavy_unsorted = 1 every
    batch, the first one from an empty map included); heavy sources under 1/128 of a batch
    take the run path alone ("sparse": the test flag keeps them in the heavy set). Otherwise (a clock step back — then
    for good —, a reachable byte trigger, pps_threshold above the 4096-entry staging)
    k_heavy_gather builds the runs and k_walk_sw_heavy walks them. Carried over the cuts,
    verdicts / flows / stats / maps bit-exact."""
    n = 1 << 21 if case in ("slices", "slices4", "pipelined", "sparse_pipelined") else 1 << 20
    hdr, ln, ts = _config2(oracle, n)
    from flowsentryx_amd import lib
    cfg, prepare = dict(SW, flags=lib.FLAG_SW_UNSORTED), None
    fast = 1
    if case == "default":
        cfg, fast = dict(SW), 0
    if case == "non_monotone":
        ts = ts.copy()
        ts[500_000], ts[500_001] = ts[500_001], ts[500_000] - 7
        fast = 0
    elif case == "byte_trigger":
        cfg.update(bps_threshold=300_000)
        fast = 0
    elif case.startswith("sparse"):
        cfg.update(flags=lib.FLAG_SW_UNSORTED | lib.FLAG_TEST_SW_SPARSE)
    elif case == "pps_over_staging":
        cfg.update(pps_threshold=4097)
        fast = 0
    elif case == "blacklisted":
        src, cnt = np.unique(hdr[:, 26:30].copy().view(np.uint32).reshape(-1), return_counts=True)
        order = np.argsort(-cnt)
        a, b = (int(src[order[i]]).to_bytes(4, "little") for i in (0, 3))
        mid = int(ts[len(ts) // 2])

        def prepare(c, o):
            for k, v in ((a, mid), (b, 2**64 - 1)):
                c.map_update(3, k, v)
                o.map_update(3, k, v)
    k = {"pipelined": 3, "sparse_pipelined": 3, "slices4": 4}.get(case, 2)
    cuts = [i * n // k for i in range(k + 1)]
    _run(native, oracle, [(hdr[x:y], ln[x:y], ts[x:y]) for x, y in zip(cuts[:-1], cuts[1:])], cfg,
         prepare=prepare, want_path=[fast] * k, pipeline=case.endswith("pipelined"),
         cap=n if case == "slices4" else None)


def test_unsorted_heavy_path_record_mode(native, oracle):
    """The owner side of the sharded path (record mode: 16-byte exchange records read
    directly, their len / ts in context scratch) on the unsorted heavy path: two carried
    config-2 slices through fsx_process_records_device, verdicts / flow rows / stats / maps
    equal to the oracle on the original header records."""
    import torch
    from flowsentryx_amd import fsx_load
    from flowsentryx_amd.shard import HipShardEngine
    from oracle import pyoracle
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    n = 1 << 21
    hdr, ln, ts = _config2(oracle, n)
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hdr.reshape(-1).copy()).to(dev)
    tl = torch.from_numpy(ln.view(np.int32).copy()).to(dev)
    tt = torch.from_numpy(ts.view(np.int64).copy()).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    o = oracle.Oracle(**CFG)
    cut = n // 2
    with native.FsxContext(max_batch=n, **CFG) as c:
        c.load_q8_model(fsx_load.model_from_dict(ref))
        e = HipShardEngine(c, n, dev)
        rec, counts = e.pack(th, tl, tt, n, 1, tv)
        c.sync()
        m, rb = int(counts[0].item()), int(counts[2].item())
        assert m == n and rb == 16   # config 2: every packet an IPv4 packet, in arrival order
        v = torch.zeros(n, dtype=torch.uint8, device=dev)
        out = dict(k=torch.empty(n * 16, dtype=torch.uint8, device=dev),
                   f=torch.empty(n, dtype=torch.uint8, device=dev),
                   x=torch.empty(n * 8, dtype=torch.float32, device=dev),
                   p=torch.empty(n, dtype=torch.float32, device=dev),
                   d=torch.empty(n, dtype=torch.uint8, device=dev))
        for a, b in ((0, cut), (cut, n)):
            c.process_records_device(rec.data_ptr() + a * rb, b - a, rb, v.data_ptr() + a, out["k"].data_ptr(),
                                     out["f"].data_ptr(), out["x"].data_ptr(), out["p"].data_ptr(),
                                     out["d"].data_ptr(), n)
            c.sync()
            info = c.last_batch_info()
            assert info["heavy_unsorted"] == 1
            vo = o.batch(hdr[a:b], ln[a:b], ts[a:b])
            bad = np.nonzero(v[a:b].cpu().numpy() != vo)[0]
            assert bad.size == 0, f"{bad.size} verdicts differ, first at {bad[:8]}"
            rows = info["sources"]
            kg = out["k"].cpu().numpy().reshape(n, 16)[:rows]
            fg = out["f"].cpu().numpy()[:rows]
            xg = out["x"].cpu().numpy().reshape(n, 8)[:rows]
            pg = out["p"].cpu().numpy()[:rows]
            ko, fo, xo = oracle.flow_features(hdr[a:b], ln[a:b], ts[a:b])
            assert rows == len(fo)
            og = sorted(range(rows), key=lambda i: (int(fg[i]), kg[i].tobytes()))
            oo = sorted(range(rows), key=lambda i: (int(fo[i]), ko[i].tobytes()))
            assert np.array_equal(kg[og], ko[oo])
            assert np.array_equal(xg[og].view(np.uint32), xo[oo].view(np.uint32))
            po, _, _ = oracle.score(ref, xo[oo])
            assert np.array_equal(pg[og].view(np.uint32), po.view(np.uint32))
        assert c.stats() == o.stats()
        for mid in (1, 2, 3, 4):
            assert pyoracle.same_map(c.map_arrays(mid), o.map_arrays(mid)), mid


TB = dict(CFG, limiter=2)   # token bucket, default rate / burst (1000 tokens/s, burst 1000)


@pytest.mark.parametrize("case", ["slices", "pipelined", "mixed_rate", "blacklisted", "non_monotone", "sorted"])
def test_token_bucket_unsorted_heavy(native, oracle, case, monkeypatch):
    """Token bucket with the heavy sources outside the sort (round 6, opt-in
    FSX_TB_UNSORTED=1: measured slower than the heavy-source sort): their packets' verdicts
    come from per-tile clamp-add maps, a scan over the tiles per source and a replay in arrival
    order (launch_tb_heavy); the sort carries the light entries only. Config-2 slices carried
    over the cuts — the heavy sources rate-limited — verdicts, flow rows, stats and the
    blacklist + token maps bit-exact against the oracle, heavy_unsorted every batch (the first
    from empty maps: every heavy source new, starting full). A heavy source with a live
    blacklist entry, or a clock step back, sends the batch to the run path (heavy runs gathered
    into the sort's buffer, DROPs stored, the passed ones untagged); "sorted": the default."""
    n = 1 << 21 if case in ("slices", "pipelined") else 1 << 20
    hdr, ln, ts = _config2(oracle, n)
    cfg, prepare, fast = dict(TB), None, 1
    if case == "mixed_rate":
        cfg.update(tb_rate=300_000, tb_burst=4)
    elif case == "non_monotone":
        ts = ts.copy()
        ts[500_000], ts[500_001] = ts[500_001], ts[500_000] - 7
        fast = 0
    elif case == "blacklisted":
        src, cnt = np.unique(hdr[:, 26:30].copy().view(np.uint32).reshape(-1), return_counts=True)
        order = np.argsort(-cnt)
        a, b = (int(src[order[i]]).to_bytes(4, "little") for i in (0, 3))
        mid = int(ts[len(ts) // 4])

        def prepare(c, o):
            for k, v in ((a, mid), (b, 2**64 - 1)):
                c.map_update(3, k, v)
                o.map_update(3, k, v)
        fast = 0
    k = 3 if case == "pipelined" else 2
    cuts = [i * n // k for i in range(k + 1)]
    want = [fast] * k
    if case == "non_monotone":
        want = [0, 1]   # (the step back is in the first slice; the token bucket's maps need no
                        # monotone clock across batches — the flow sums refuse only that batch)
    if case == "sorted":
        monkeypatch.delenv("FSX_TB_UNSORTED", raising=False)
        want = None
    else:
        monkeypatch.setenv("FSX_TB_UNSORTED", "1")
    _run(native, oracle, [(hdr[x:y], ln[x:y], ts[x:y]) for x, y in zip(cuts[:-1], cuts[1:])], cfg,
         prepare=prepare, want_path=want, pipeline=case == "pipelined", maps=(3, 4, 5, 6))
