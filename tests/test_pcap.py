"""pcap ingest/export (SURVEY.md §8 f row 2): round trips through the writer and the
library's record index, both timestamp resolutions and byte orders, truncated tails,
and replay through the orchestrator's reader against the oracle (GPU)."""
import struct

import numpy as np
import pytest

from flowsentryx_amd import pcap
from test_gpu_parity import rand_stream


def _stream(n=3000, seed=3):
    rng = np.random.default_rng(seed)
    return rand_stream(rng, n, 50, dt_max=5000, v6_frac=0.3, nonip_frac=0.05, short_frac=0.05)


def _expected_records(hdr, ln, snap=64):
    cl = np.minimum(ln, snap)
    out = hdr.copy()
    out[np.arange(64)[None, :] >= cl[:, None]] = 0
    return out


@pytest.mark.parametrize("ns", [True, False])
def test_roundtrip(tmp_path, ns):
    hdr, ln, ts = _stream()
    if not ns:
        ts = ts - ts % 1000           # microsecond files hold whole microseconds
    p = tmp_path / "a.pcap"
    pcap.write(p, hdr, ln, ts, nanoseconds=ns)
    h2, l2, t2 = pcap.read(p)
    assert np.array_equal(h2, _expected_records(hdr, ln))
    assert np.array_equal(l2, ln) and np.array_equal(t2, ts)
    # batched reading covers the same records
    parts = list(pcap.read_batches(p, 777))
    assert sum(len(x[1]) for x in parts) == len(ln)
    assert np.array_equal(np.concatenate([x[0] for x in parts]), h2)


def test_swapped_byte_order_and_truncated_tail(tmp_path):
    hdr, ln, ts = _stream(200, 5)
    p = tmp_path / "le.pcap"
    pcap.write(p, hdr, ln, ts, nanoseconds=True)
    raw = p.read_bytes()
    # rewrite as big-endian: file header + every record header byte-swapped
    fh = struct.unpack("<IHHiIII", raw[:24])
    out = bytearray(struct.pack(">IHHiIII", *fh))
    pos = 24
    while pos < len(raw):
        sec, frac, cl, ol = struct.unpack("<IIII", raw[pos:pos + 16])
        out += struct.pack(">IIII", sec, frac, cl, ol) + raw[pos + 16:pos + 16 + cl]
        pos += 16 + cl
    q = tmp_path / "be.pcap"
    q.write_bytes(bytes(out[:-5]))                 # last record cut short: not returned
    h2, l2, t2 = pcap.read(q)
    assert len(l2) == len(ln) - 1
    assert np.array_equal(h2, _expected_records(hdr, ln)[:-1])
    assert np.array_equal(l2, ln[:-1]) and np.array_equal(t2, ts[:-1])


def test_full_snaplen_frames(tmp_path):
    """Captures longer than 64 bytes: the header record is the first 64 bytes."""
    hdr, ln, ts = _stream(300, 9)
    p = tmp_path / "s.pcap"
    pcap.write(p, hdr, ln, ts, snaplen=64)
    raw = bytearray(p.read_bytes())
    # re-write with 100-byte captures (64 known bytes + 36 bytes of junk payload)
    out = bytearray(raw[:24])
    pos = 24
    while pos < len(raw):
        sec, frac, cl, ol = struct.unpack("<IIII", raw[pos:pos + 16])
        data = bytes(raw[pos + 16:pos + 16 + cl])
        ext = data + bytes([0xAB]) * (100 - cl) if cl == 64 and ol >= 100 else data
        out += struct.pack("<IIII", sec, frac, len(ext), ol) + ext
        pos += 16 + cl
    q = tmp_path / "big.pcap"
    q.write_bytes(bytes(out))
    h2, l2, _ = pcap.read(q)
    assert np.array_equal(h2, _expected_records(hdr, ln))


def test_rejects_non_pcap(tmp_path):
    q = tmp_path / "x.pcap"
    q.write_bytes(b"\x0a\x0d\x0d\x0a" + bytes(40))   # pcapng section header block
    with pytest.raises(ValueError):
        pcap.read(q)


@pytest.mark.gpu
def test_device_ingest_and_replay(tmp_path, native, oracle):
    import torch
    from flowsentryx_amd import fsx_load
    hdr, ln, ts = _stream(20000, 11)
    p = tmp_path / "r.pcap"
    pcap.write(p, hdr, ln, ts)
    cfg = dict(pps_threshold=7, window_ns=200_000, block_ns=1_000_000, max_entries=4096)
    with native.FsxContext(max_batch=1 << 15, **cfg) as c:
        dh, dl, dt = pcap.to_device(p, c)
        assert np.array_equal(dh.cpu().numpy().reshape(-1, 64), _expected_records(hdr, ln))
        assert np.array_equal(dl.cpu().numpy().view(np.uint32), ln)
        assert np.array_equal(dt.cpu().numpy().view(np.uint64), ts)
    o = oracle.Oracle(**cfg)
    with native.FsxContext(max_batch=4096, **cfg) as c:
        got = np.concatenate([v for v, _ in fsx_load.replay_pcap(c, p, 4096)])
        exp = o.batch(_expected_records(hdr, ln), ln, ts)
        assert np.array_equal(got, exp)
        assert c.stats() == o.stats()
