"""CPU (gloo, world_size 2 and 3): the sharded protocol of flowsentryx_amd/shard.py with
the CPU engine (oracle owners) equals one sequential oracle over the whole stream —
verdicts, stats_map and every map entry (SURVEY.md §8 e: the result must be exactly the
1-GPU result)."""
import json
import socket

import pytest
import torch.multiprocessing as mp

import shard_worker


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_sharded(tmp_path, world, spec, engine="cpu"):
    out = tmp_path / "result.json"
    mp.start_processes(shard_worker.worker, args=(world, _port(), spec, str(out), engine),
                       nprocs=world, start_method="spawn")
    res = json.loads(out.read_text())
    assert res["ok"], res["msg"]
    return res


BASE = dict(n=24000, n_ips=300, seed=7, maps=[1, 2, 3, 4],
            cuts=[0, 5000, 5001, 16000, 24000], chunks=3)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fixed_window(tmp_path, world):
    spec = dict(BASE, cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000,
                               max_entries=4096))
    res = run_sharded(tmp_path, world, spec)
    assert res["filtered"] > 0      # the replicated blocklist dropped packets at arrival
    # one host read per global batch with the filter on
    assert res["host_reads"] == len(BASE["cuts"]) - 1, res["host_reads"]


def test_sharded_replica_capacity_overflow(tmp_path):
    """A replica capacity of 2 entries per owner: the owners' other blacklisted sources are
    left out of the replica (their packets go to the owner, which decides them), the result
    stays exact, and the capacity grows for the next batch from the one host read."""
    spec = dict(BASE, blk_cap=2, cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000,
                                          max_entries=4096))
    res = run_sharded(tmp_path, 2, spec)
    assert res["blk_cap"] > 2 and res["host_reads"] == len(BASE["cuts"]) - 1


def test_sharded_without_blocklist_filter_one_chunk(tmp_path):
    spec = dict(BASE, chunks=1, filter=False,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096))
    res = run_sharded(tmp_path, 2, spec)
    assert res["filtered"] == 0


def test_sharded_non_monotone_clock_disables_filter(tmp_path):
    """Sub-batches whose clock goes back skip the replica (exactness first)."""
    spec = dict(BASE, seed=23, dt_max=40, cfg=dict(pps_threshold=5, window_ns=100_000,
                                                   block_ns=400_000, max_entries=4096),
                jitter=3000)
    run_sharded(tmp_path, 2, spec)


def test_sharded_mixed_families_sliding_window(tmp_path):
    spec = dict(BASE, v6_frac=0.3, nonip_frac=0.05, short_frac=0.03, seed=9,
                cfg=dict(limiter=1, pps_threshold=5, window_ns=1_000_000, block_ns=50_000,
                         max_entries=4096))
    run_sharded(tmp_path, 2, spec)


def test_sharded_token_bucket(tmp_path):
    spec = dict(BASE, seed=11, maps=[3, 4, 5, 6],
                cfg=dict(limiter=2, tb_rate=300_000, tb_burst=4, max_entries=4096))
    run_sharded(tmp_path, 2, spec)


def test_sharded_mixed_record_formats(tmp_path):
    """A few IPv6 sources: pieces without one ship 16-byte records, the others 32-byte
    records, in the same sub-batch (the format travels in the counts' low bit)."""
    spec = dict(BASE, v6_frac=0.0007, seed=29, n_ips=60,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096))
    res = run_sharded(tmp_path, 2, spec)
    assert set(res["formats"]) == {16, 32}, res["formats"]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_without_blocklist_filter_all_packs_first(tmp_path, world):
    """Filter off (as with flow features): every sub-batch is packed first and one exchange of
    all their counts precedes the record exchanges (shard.py _exchange_all), mixed record
    formats and families included."""
    spec = dict(BASE, chunks=4, filter=False, v6_frac=0.001, seed=31, n_ips=80,
                cfg=dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096))
    res = run_sharded(tmp_path, world, spec)
    assert res["filtered"] == 0
