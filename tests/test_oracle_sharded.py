"""CPU: the persistent sharded oracle (fsxo_shards_*, the full-size checker of bench.py
and the large GPU tests) equals the sequential oracle — verdicts, stats_map and every
map entry — for all three limiters, across batches, with exact and prefix rules.
Also the product's .pth weight loader against the committed JSON export."""
import json
from pathlib import Path

import numpy as np
import pytest

from test_gpu_parity import CFGS, rand_stream

GOLDEN = Path(__file__).resolve().parent / "golden"
REF_PTH = Path("/root/reference/src/model_weights.pth")


def _maps(limiter):
    return (3, 4, 5, 6, 7, 8) if limiter == 2 else (1, 2, 3, 4, 7, 8)


@pytest.mark.parametrize("limiter", [0, 1, 2])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_sharded_equals_sequential(oracle, limiter, threads):
    rng = np.random.default_rng(90 + limiter)
    hdr, ln, ts = rand_stream(rng, 30000, 400, dt_max=300, v6_frac=0.3, nonip_frac=0.03,
                              short_frac=0.02)
    cfg = dict(CFGS["tight"], limiter=limiter, max_entries=1 << 14)
    if limiter == 2:
        cfg = dict(limiter=2, tb_rate=300_000, tb_burst=4, max_entries=1 << 14)
    seq = oracle.Oracle(**cfg)
    sh = oracle.ShardedOracle(threads, **cfg)
    from flowsentryx_amd.lib import prefix_key
    for i in range(0, 3000, 101):   # exact rules and prefix rules on stream sources
        if hdr[i, 12] == 0x08 and hdr[i, 13] == 0:
            k = bytes(hdr[i, 26:30])
            for o in (seq, sh):
                o.map_update(3, k, 2**64 - 1 if i % 2 else 0)
                o.map_update(7, prefix_key(k, 24 + i % 9), 2**64 - 1)
    for a, b in ((0, 11111), (11111, 11112), (11112, 30000)):
        v1 = seq.batch(hdr[a:b], ln[a:b], ts[a:b])
        v2 = sh.batch(hdr[a:b], ln[a:b], ts[a:b])
        assert np.array_equal(v1, v2)
    assert seq.stats() == sh.stats()
    for m in _maps(limiter):
        want = seq.map_dump(m)
        k, v = sh.map_arrays(m)
        got = {k[i].tobytes(): (tuple(int(x) for x in v[i]) if v.shape[1] > 1 else int(v[i, 0]))
               for i in range(len(k))}
        assert got == want, m
    sh.reset()
    assert sh.stats() == (0, 0) and sh.map_arrays(1)[0].shape[0] == 0


def test_sort_map_arrays_orders_bytes(oracle):
    keys = np.array([[2, 0, 0, 1], [1, 255, 0, 0], [1, 0, 0, 9]], dtype=np.uint8)
    vals = np.array([[3], [2], [1]], dtype=np.uint64)
    k, v = oracle.sort_map_arrays(keys, vals)
    assert k.tolist() == [[1, 0, 0, 9], [1, 255, 0, 0], [2, 0, 0, 1]]
    assert v.reshape(-1).tolist() == [1, 2, 3]
    assert oracle.same_map((keys, vals), (keys[::-1], vals[::-1]))
    assert not oracle.same_map((keys, vals), (keys, vals + 1))


@pytest.mark.skipif(not REF_PTH.exists(), reason="reference tree absent (GPU box)")
def test_pth_loader_matches_json_export():
    """flowsentryx_amd.fsx_load.load_weights on the reference's model_weights.pth
    (torch.load(weights_only=True), src/fsx_load.py:17) gives the same fsx_q8_model as
    the committed JSON export (tests/golden/make_score_vectors.py)."""
    from flowsentryx_amd import fsx_load
    a = fsx_load.load_weights(REF_PTH)
    b = fsx_load.load_weights(GOLDEN / "model_weights.json")
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    assert list(a.weight) == list(b.weight) == ref["weight"]
    for f in ("weight_scale", "bias", "in_scale", "out_scale"):
        assert np.float32(getattr(a, f)) == np.float32(getattr(b, f)) == np.float32(ref[f]), f
    assert a.in_zero_point == b.in_zero_point == ref["in_zero_point"]
    assert a.out_zero_point == b.out_zero_point == ref["out_zero_point"]
