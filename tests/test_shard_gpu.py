"""GPU: the sharded path's HIP kernels (fsx_shard.hip) and the protocol end to end.

* pack / unpack / scatter against the CPU engine's numpy restatement of the 32-byte
  and compact 16-byte record layouts (records, per-owner counts and send order
  byte-identical);
* 2 and 3 ranks on the one GPU of the box (gloo carries the exchange through host
  memory; RCCL refuses two ranks on one device) with libfsx_hip.so owners: verdicts,
  stats_map and map dumps equal one sequential oracle over the whole stream.
"""
import numpy as np
import pytest
import torch

from shard_cpu import CpuShardEngine, REC_DTYPE, REC16_DTYPE, records_to_headers, widen
from test_gpu_parity import rand_stream
from test_shard_cpu import BASE, run_sharded

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("regions", [False, True])
@pytest.mark.parametrize("v6_frac,rec_bytes", [(0.4, 32), (0.0, 16)])
def test_pack_unpack_scatter_match_restatement(native, oracle, v6_frac, rec_bytes, regions):
    """regions: FSX_SHARD_REGIONS (owner o's records at o * n; compact records placed by
    k_shard_place16 in one pass with a look-back over the tiles) — the same records per
    owner, in the same order, as the contiguous layout and the restatement."""
    rng = np.random.default_rng(41)
    hdr, ln, ts = rand_stream(rng, 20000, 500, dt_max=300, v6_frac=v6_frac, nonip_frac=0.05,
                              short_frac=0.05)
    n, G = hdr.shape[0], 5
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hdr.reshape(-1).copy()).to(dev)
    tl = torch.from_numpy(ln.view(np.int32).copy()).to(dev)
    tt = torch.from_numpy(ts.view(np.int64).copy()).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    from flowsentryx_amd.shard import HipShardEngine
    with native.FsxContext(max_batch=1 << 15, max_entries=4096) as c:
        e = HipShardEngine(c, n, dev)
        e.regions = regions
        rec, counts = e.pack(th, tl, tt, n, G, tv)
        c.sync()
        cpu = CpuShardEngine(oracle, max_entries=4096)
        cv = torch.zeros(n, dtype=torch.uint8)
        crec, ccounts = cpu.pack(torch.from_numpy(hdr.reshape(-1).copy()),
                                 torch.from_numpy(ln.view(np.int32).copy()),
                                 torch.from_numpy(ts.view(np.int64).copy()), n, G, cv)
        m = int(ccounts[:G].sum())
        assert counts.cpu().tolist() == ccounts.tolist()
        assert int(ccounts[G + 1]) == rec_bytes
        sc = [int(x) for x in ccounts[:G]]
        rec = torch.cat(e.send_views(rec, sc, rec_bytes, 0))
        sidx = torch.cat(e.send_views(e.send_idx.view(torch.uint8), sc, 4, 0)).view(torch.int32)
        assert np.array_equal(rec.cpu().numpy(), crec.numpy())
        assert np.array_equal(sidx.cpu().numpy().astype(np.int64), cpu.send_idx)
        ipmask = np.zeros(n, dtype=bool)
        ipmask[cpu.send_idx] = True
        assert np.array_equal(tv.cpu().numpy()[~ipmask], cv.numpy()[~ipmask])
        # unpack: same parse, keys, lengths, timestamps, dst ports as the restatement
        hdr_o, ln_o, ts_o, _ = e._owner_buffers(m)
        c.shard_unpack_device(rec.data_ptr(), m, hdr_o.data_ptr(), ln_o.data_ptr(), ts_o.data_ptr(),
                              rec_bytes)
        c.sync()
        gh = hdr_o[:m * 64].cpu().numpy().reshape(m, 64)
        crec32 = widen(crec.numpy().view(REC16_DTYPE)) if rec_bytes == 16 else crec.numpy().view(REC_DTYPE)
        eh, el, et = records_to_headers(crec32)
        assert np.array_equal(gh, eh)
        assert np.array_equal(ln_o[:m].cpu().numpy().view(np.uint32), el)
        assert np.array_equal(ts_o[:m].cpu().numpy().view(np.uint64), et)
        gc, gk = oracle.parse(gh, el)
        oc, ok = oracle.parse(hdr[cpu.send_idx], ln[cpu.send_idx])
        assert np.array_equal(gc, oc) and np.array_equal(gk, ok)
        assert np.array_equal(oracle.dst_port(gh, el), oracle.dst_port(hdr[cpu.send_idx], ln[cpu.send_idx]))
        # scatter
        ret = torch.from_numpy(rng.integers(1, 3, m).astype(np.uint8)).to(dev)
        e.scatter(ret, m, tv)
        c.sync()
        assert np.array_equal(tv.cpu().numpy()[cpu.send_idx], ret.cpu().numpy())


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_hip_owners(tmp_path, world):
    spec = dict(BASE, v6_frac=0.2, nonip_frac=0.03, short_frac=0.02, seed=13,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096),
                owner_batch=4096)
    run_sharded(tmp_path, world, spec, engine="hip")


@pytest.mark.parametrize("world,v6", [(2, 0.0), (3, 0.3)])
def test_sharded_flow_features_equal_one_gpu(tmp_path, world, v6):
    """Per-source features + q8 scores under sharding: every owner accumulates its sources
    over the batch's sub-batches (fsx_flows_begin / fsx_flows_end); the replica still drops
    blacklisted packets at their arrival rank, whose flow partials merge into the owners'
    sums first; the union of the rows equals the 1-GPU rows over each whole global batch,
    bit for bit."""
    spec = dict(BASE, v6_frac=v6, nonip_frac=0.03, short_frac=0.02, seed=29 + world, flows=True,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096),
                owner_batch=4096)
    res = run_sharded(tmp_path, world, spec, engine="hip")
    assert res["filtered"] > 0 and res["partials"] > 0   # dropped at arrival, still in the features
    # one host read per global batch with the filter and the flows on:
    # replica, filter decision and flow partials stay on the device
    assert res["host_reads"] == len(BASE["cuts"]) - 1, res["host_reads"]


def test_sharded_flow_features_small_replica(tmp_path):
    """The flow partials travel in fixed blocks of the replica's per-owner capacity: with a
    capacity of 2 the owners' other blacklisted sources stay out of the replica, their
    packets reach the owner, and the rows still equal the 1-GPU rows."""
    spec = dict(BASE, v6_frac=0.1, seed=37, flows=True, blk_cap=2,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096),
                owner_batch=4096)
    res = run_sharded(tmp_path, 2, spec, engine="hip")
    assert res["filtered"] > 0 and res["blk_cap"] > 2


@pytest.mark.parametrize("filt", [True, False])
def test_sharded_flow_features_heavy_path(tmp_path, filt):
    """The same with a table of 2^17 slots, so every owner runs the heavy-source sort, the
    heavy verdict lists and the heavy runs' flow sums (k_flow_heavy) in accumulate mode; with
    and without the replica filter (without it every packet reaches its owner)."""
    spec = dict(BASE, n_ips=600, v6_frac=0.2, nonip_frac=0.02, seed=41, flows=True, filter=filt,
                cfg=dict(pps_threshold=40, window_ns=2_000_000, block_ns=5_000_000, max_entries=1 << 16),
                owner_batch=1 << 15)
    res = run_sharded(tmp_path, 2, spec, engine="hip")
    assert (res["filtered"] > 0) == filt


def test_sharded_hip_owners_limiters(tmp_path):
    for lim, maps, extra in ((1, [1, 2, 3, 4], dict(pps_threshold=5, window_ns=1_000_000,
                                                     block_ns=50_000)),
                             (2, [3, 4, 5, 6], dict(tb_rate=300_000, tb_burst=4))):
        spec = dict(BASE, seed=17 + lim, maps=maps, cfg=dict(limiter=lim, max_entries=4096, **extra))
        run_sharded(tmp_path, 2, spec, engine="hip")


@pytest.mark.parametrize("v6_frac", [0.0, 0.3])
def test_record_mode_equals_header_mode(native, oracle, v6_frac):
    """The owner's record mode (fsx_process_records_device) against the pipeline on the
    header records fsx_shard_unpack_device builds: verdicts, maps, stats and per-source
    features / scores identical, over two batches (state carry)."""
    from flowsentryx_amd.shard import HipShardEngine
    from test_gpu_parity import MAPS
    rng = np.random.default_rng(43)
    hdr, ln, ts = rand_stream(rng, 60000, 700, dt_max=200, v6_frac=v6_frac, nonip_frac=0.03,
                              short_frac=0.02)
    n = hdr.shape[0]
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hdr.reshape(-1).copy()).to(dev)
    tl = torch.from_numpy(ln.view(np.int32).copy()).to(dev)
    tt = torch.from_numpy(ts.view(np.int64).copy()).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    cfg = dict(max_batch=1 << 16, max_entries=1 << 15, pps_threshold=7, window_ns=200_000,
               block_ns=1_000_000)
    with native.FsxContext(**cfg) as ca, native.FsxContext(**cfg) as cb:
        from flowsentryx_amd import fsx_load
        from pathlib import Path
        model = fsx_load.load_weights(Path(__file__).parent / "golden" / "model_weights.json")
        ca.load_q8_model(model)
        cb.load_q8_model(model)
        e = HipShardEngine(ca, n, dev)
        rec, counts = e.pack(th, tl, tt, n, 1, tv)
        ca.sync()
        m, rb = int(counts[0].item()), int(counts[2].item())
        assert rb == (32 if v6_frac else 16)
        hb, lb, tsb, _ = e._owner_buffers(m)
        cb.shard_unpack_device(rec.data_ptr(), m, hb.data_ptr(), lb.data_ptr(), tsb.data_ptr(), rb)
        cb.sync()
        outs = {}
        for name, ctx in (("rec", ca), ("hdr", cb)):
            v = torch.zeros(m, dtype=torch.uint8, device=dev)
            keys = torch.zeros(m * 16, dtype=torch.uint8, device=dev)
            fam = torch.zeros(m, dtype=torch.uint8, device=dev)
            feat = torch.zeros(m * 8, dtype=torch.float32, device=dev)
            prob = torch.zeros(m, dtype=torch.float32, device=dev)
            dec = torch.zeros(m, dtype=torch.uint8, device=dev)
            for a, b in ((0, m // 3), (m // 3, m)):   # two batches: state carries
                args = (v.data_ptr() + a, keys.data_ptr(), fam.data_ptr(), feat.data_ptr(),
                        prob.data_ptr(), dec.data_ptr(), m)
                if name == "rec":
                    ctx.process_records_device(rec.data_ptr() + a * rb, b - a, rb, *args)
                else:
                    ctx.process_batch_device(hb.data_ptr() + a * 64, lb.data_ptr() + a * 4,
                                             tsb.data_ptr() + a * 8, b - a, *args)
                ctx.sync()
            ns = ctx.last_batch_info()["sources"]
            # per-source rows come in table-slot order, which depends on insertion races:
            # compare them keyed by source
            kk, ff = keys[:ns * 16].cpu().numpy().reshape(ns, 16), fam[:ns].cpu().numpy()
            fe = feat[:ns * 8].cpu().numpy().reshape(ns, 8)
            pr, de = prob[:ns].cpu().numpy(), dec[:ns].cpu().numpy()
            rows = {(int(ff[j]), kk[j].tobytes()): (fe[j].tobytes(), float(pr[j]), int(de[j]))
                    for j in range(ns)}
            outs[name] = (v.cpu().numpy(), rows, ctx.stats(), {mid: ctx.map_dump(mid) for mid in MAPS})
        assert np.array_equal(outs["rec"][0], outs["hdr"][0])
        assert outs["rec"][1] == outs["hdr"][1]
        assert outs["rec"][2] == outs["hdr"][2]
        assert outs["rec"][3] == outs["hdr"][3]
        # and the verdicts equal the oracle on the original stream's IP packets
        o = oracle.Oracle(max_entries=1 << 15, pps_threshold=7, window_ns=200_000, block_ns=1_000_000)
        idx = e.send_idx[:m].cpu().numpy().astype(np.int64)
        vo = o.batch(hdr[idx], ln[idx], ts[idx])
        assert np.array_equal(outs["rec"][0], vo)


@pytest.mark.parametrize("flows", [False, True])
def test_record_batches_split_pipelined(native, oracle, flows):
    """Record batches split like header batches (fsx_set_pipeline 1: each tail beside the
    next batch's front, the len / ts of every front set in its own buffers): five record
    batches enqueued back to back without a synchronization, each batch's verdicts copied
    on another stream after fsx_stream_wait_batches(all=0) following the NEXT call (the last
    after all=1) — every copy, the maps and stats equal the oracle over the whole stream."""
    from flowsentryx_amd.shard import HipShardEngine
    from test_gpu_parity import MAPS, assert_same_state
    rng = np.random.default_rng(47)
    hdr, ln, ts = rand_stream(rng, 150000, 900, dt_max=150, v6_frac=0.0, nonip_frac=0.02, short_frac=0.01)
    n = hdr.shape[0]
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hdr.reshape(-1).copy()).to(dev)
    tl = torch.from_numpy(ln.view(np.int32).copy()).to(dev)
    tt = torch.from_numpy(ts.view(np.int64).copy()).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    cfg = dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000)
    with native.FsxContext(max_batch=1 << 18, max_entries=1 << 15, **cfg) as c:
        e = HipShardEngine(c, n, dev)      # (pipeline mode 1)
        rec, counts = e.pack(th, tl, tt, n, 1, tv)
        c.sync()
        m, rb = int(counts[0].item()), int(counts[2].item())
        assert rb == 16
        cuts = [0, m // 7, 2 * m // 7, m // 2, 4 * m // 5, m]
        v = torch.zeros(m, dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(dev)
        got = torch.zeros(m, dtype=torch.uint8, device=dev)
        fo = None
        if flows:
            fo = [torch.zeros(m * 16, dtype=torch.uint8, device=dev), torch.zeros(m, dtype=torch.uint8, device=dev),
                  torch.zeros(m * 8, dtype=torch.float32, device=dev), torch.zeros(m, dtype=torch.float32, device=dev),
                  torch.zeros(m, dtype=torch.uint8, device=dev)]
            from flowsentryx_amd import fsx_load
            from pathlib import Path
            c.load_q8_model(fsx_load.load_weights(Path(__file__).parent / "golden" / "model_weights.json"))

        def copy_back(j, all_batches):
            a, b = cuts[j], cuts[j + 1]
            c.stream_wait_batches(side.cuda_stream, all_batches)
            with torch.cuda.stream(side):
                got[a:b].copy_(v[a:b])

        for j in range(len(cuts) - 1):
            a, b = cuts[j], cuts[j + 1]
            if flows:
                c.process_records_device(rec.data_ptr() + a * rb, b - a, rb, v.data_ptr() + a,
                                         *[x.data_ptr() for x in fo], m)
            else:
                c.verdict_records_device(rec.data_ptr() + a * rb, b - a, rb, v.data_ptr() + a)
            if j:
                copy_back(j - 1, False)
        copy_back(len(cuts) - 2, True)
        side.synchronize()
        c.sync()
        idx = e.send_idx[:m].cpu().numpy().astype(np.int64)
        o = oracle.Oracle(max_entries=1 << 15, **cfg)
        vo = np.concatenate([o.batch(hdr[idx[a:b]], ln[idx[a:b]], ts[idx[a:b]])
                             for a, b in zip(cuts[:-1], cuts[1:])])
        assert np.array_equal(got.cpu().numpy(), vo)
        assert np.array_equal(v.cpu().numpy(), vo)
        assert_same_state(c, o)
