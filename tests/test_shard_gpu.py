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


@pytest.mark.parametrize("v6_frac,rec_bytes", [(0.4, 32), (0.0, 16)])
def test_pack_unpack_scatter_match_restatement(native, oracle, v6_frac, rec_bytes):
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
        assert np.array_equal(rec[:m * rec_bytes].cpu().numpy(), crec.numpy())
        assert np.array_equal(e.send_idx[:m].cpu().numpy().astype(np.int64), cpu.send_idx)
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


def test_sharded_hip_owners_limiters(tmp_path):
    for lim, maps, extra in ((1, [1, 2, 3, 4], dict(pps_threshold=5, window_ns=1_000_000,
                                                     block_ns=50_000)),
                             (2, [3, 4, 5, 6], dict(tb_rate=300_000, tb_burst=4))):
        spec = dict(BASE, seed=17 + lim, maps=maps, cfg=dict(limiter=lim, max_entries=4096, **extra))
        run_sharded(tmp_path, 2, spec, engine="hip")
