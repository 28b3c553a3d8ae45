"""pcap ingest and export (SURVEY.md §8 f, row 2).

Classic pcap (magic 0xA1B2C3D4 µs / 0xA1B23C4D ns, either byte order, link type 1
Ethernet) <-> the batch layout of include/fsx_hip.h: 64-byte header records (the first
min(caplen, 64) frame bytes, zero padded), frame length (the record's original length:
data_end - data of the reference's XDP program, src/fsx_kern.c:123) and arrival time in
ns (what the reference's bpf_ktime_get_ns() returns, src/fsx_kern.c:150).

Reading: libfsx_hip.so's host function fsx_pcap_index walks the record headers (the one
sequential step); the records are then gathered on the host with numpy
(`read_batches`) or on the GPU from an HBM copy of the file bytes (`to_device`,
fsx_pcap_records_device). Writing: vectorised numpy, snap length 64 by default (the
header record is all the data plane reads).
"""
from __future__ import annotations

import ctypes as C
import mmap
import struct
from pathlib import Path

import numpy as np

from . import lib

MAGIC_US = 0xA1B2C3D4
MAGIC_NS = 0xA1B23C4D
LINKTYPE_ETHERNET = 1
PCAP_NANOSECONDS = 1
PCAP_SWAPPED = 2


def _sig():
    L = lib.load_library()
    f = L.fsx_pcap_index
    if getattr(f, "_fsx_sig", False):
        return L
    vp, sz = C.c_void_p, C.c_size_t
    f.restype = C.c_int
    f.argtypes = [vp, sz, C.c_uint32, vp, vp, vp, vp, sz, C.POINTER(sz), C.POINTER(sz)]
    f._fsx_sig = True
    g = L.fsx_pcap_records_device
    g.restype = C.c_int
    g.argtypes = [vp, vp, vp, vp, sz, vp]
    return L


def parse_file_header(b: bytes) -> tuple[int, int, int]:
    """-> (flags, snaplen, linktype) of a 24-byte pcap file header."""
    if len(b) < 24:
        raise ValueError("truncated pcap file header")
    (m,) = struct.unpack("<I", b[:4])
    table = {MAGIC_US: 0, MAGIC_NS: PCAP_NANOSECONDS,
             0xD4C3B2A1: PCAP_SWAPPED, 0x4D3CB2A1: PCAP_NANOSECONDS | PCAP_SWAPPED}
    if m not in table:
        raise ValueError(f"not a classic pcap file (magic 0x{m:08x})")
    flags = table[m]
    endian = ">" if flags & PCAP_SWAPPED else "<"
    _, _, _, _, snaplen, linktype = struct.unpack(endian + "HHiIII", b[4:24])
    if linktype != LINKTYPE_ETHERNET:
        raise ValueError(f"link type {linktype} is not Ethernet")
    return flags, snaplen, linktype


def index(buf, flags: int, cap: int):
    """Index up to cap complete records of the record bytes buf -> (data offsets,
    caplen, origlen, ts_ns, bytes consumed)."""
    L = _sig()
    a = np.frombuffer(buf, dtype=np.uint8)
    off = np.empty(cap, dtype=np.uint64)
    cl = np.empty(cap, dtype=np.uint32)
    ol = np.empty(cap, dtype=np.uint32)
    ts = np.empty(cap, dtype=np.uint64)
    n, used = C.c_size_t(), C.c_size_t()
    rc = L.fsx_pcap_index(a.ctypes.data if a.size else None, a.size, flags, off.ctypes.data,
                          cl.ctypes.data, ol.ctypes.data, ts.ctypes.data, cap, C.byref(n),
                          C.byref(used))
    if rc:
        raise lib.FsxError(rc, "fsx_pcap_index")
    k = n.value
    return off[:k], cl[:k], ol[:k], ts[:k], used.value


def gather_records(buf, off: np.ndarray, caplen: np.ndarray) -> np.ndarray:
    """Host: 64-byte zero-padded header records of indexed records."""
    a = np.frombuffer(buf, dtype=np.uint8)
    n = off.size
    cols = np.arange(64, dtype=np.uint64)
    pos = off[:, None] + cols[None, :]
    valid = cols[None, :] < np.minimum(caplen, 64)[:, None]
    pos = np.where(valid, pos, 0).astype(np.int64)
    out = a[pos] if a.size else np.zeros((n, 64), dtype=np.uint8)
    return np.where(valid, out, 0).astype(np.uint8).reshape(n, 64)


def read_batches(path: str | Path, batch: int = 1 << 20):
    """Yield (hdr[n, 64], len[n], ts[n]) batches of a pcap file (memory-mapped)."""
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            flags, _, _ = parse_file_header(mm[:24])
            pos = 24
            while True:
                view = memoryview(mm)[pos:]
                off, cl, ol, ts, used = index(view, flags, batch)
                if off.size == 0:
                    view.release()
                    break
                hdr = gather_records(view, off, cl)
                view.release()
                yield hdr, ol.copy(), ts.copy()
                pos += used
        finally:
            mm.close()


def read(path: str | Path):
    """The whole file as one batch."""
    parts = list(read_batches(path, 1 << 22))
    if not parts:
        return np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint64)
    return (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]),
            np.concatenate([p[2] for p in parts]))


def write(path: str | Path, hdr, length, ts, nanoseconds: bool = True, snaplen: int = 64):
    """Write header records as a classic pcap (caplen = min(len, snaplen, 64))."""
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    n = hdr.shape[0]
    cl = np.minimum(length, min(snaplen, 64)).astype(np.uint32)
    sec = (ts // 1_000_000_000).astype(np.uint32)
    frac = ts % 1_000_000_000
    if not nanoseconds:
        frac = frac // 1000
    rh = np.zeros((n, 4), dtype="<u4")
    rh[:, 0], rh[:, 1], rh[:, 2], rh[:, 3] = sec, frac.astype(np.uint32), cl, length
    magic = MAGIC_NS if nanoseconds else MAGIC_US
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", magic, 2, 4, 0, 0, snaplen, LINKTYPE_ETHERNET))
        rec_sz = 16 + cl.astype(np.int64)
        total = int(rec_sz.sum())
        out = np.zeros(total, dtype=np.uint8)
        starts = np.concatenate([[0], np.cumsum(rec_sz)[:-1]]).astype(np.int64)
        out[(starts[:, None] + np.arange(16)[None, :]).reshape(-1)] = rh.view(np.uint8).reshape(-1)
        cols = np.arange(64)
        m = cols[None, :] < cl[:, None]
        dst = (starts[:, None] + 16 + cols[None, :])[m]
        out[dst] = hdr[m]
        f.write(out.tobytes())


def to_device(path: str | Path, ctx: lib.FsxContext, device=None):
    """Parse a pcap on the GPU: the file bytes go to HBM once, the host only walks the
    record headers, k_pcap_records builds the header records there. Returns device
    tensors (hdr uint8 [n*64], len int32 [n], ts int64 [n])."""
    import torch

    dev = device or torch.device("cuda", int(ctx.config.device))
    raw = Path(path).read_bytes()
    flags, _, _ = parse_file_header(raw[:24])
    body = memoryview(raw)[24:]
    off, cl, ol, ts, _ = index(body, flags, len(raw) // 16 + 1)
    n = off.size
    d_buf = torch.frombuffer(bytearray(body), dtype=torch.uint8).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_cl = torch.from_numpy(cl.view(np.int32)).to(dev)
    d_hdr = torch.empty(max(n, 1) * 64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    L = _sig()
    rc = L.fsx_pcap_records_device(ctx._h, d_buf.data_ptr(), d_off.data_ptr(), d_cl.data_ptr(), n,
                                   d_hdr.data_ptr())
    if rc:
        raise lib.FsxError(rc, "fsx_pcap_records_device")
    ctx.sync()
    return (d_hdr[:n * 64], torch.from_numpy(ol.view(np.int32).copy()).to(dev),
            torch.from_numpy(ts.view(np.int64).copy()).to(dev))
