"""Synthetic packet streams (BASELINE.json configs) and single-frame builders.

`generate_device` drives libfsx_synth.so (device generator); the CPU twin lives in
oracle/ (same fsx_synth_common.h), so a stream generated on either side is
byte-identical. `frame_*` build individual 64-byte header records for tests.
"""
from __future__ import annotations

import ctypes as C
import struct
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent

SYNTH_ZIPF_V4 = 0
SYNTH_CARPET = 1


class SynthParams(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("seed", C.c_uint64),
        ("t0_ns", C.c_uint64),
        ("duration_ns", C.c_uint64),
        ("n_ips", C.c_uint32),
        ("mode", C.c_uint32),
        ("len_min", C.c_uint32),
        ("len_max", C.c_uint32),
        ("pct_v6", C.c_uint32),
        ("pct_vlan", C.c_uint32),
        ("ip_salt", C.c_uint32),
        ("pad", C.c_uint32),
    ]


def config_params(config: int, n: int | None = None) -> tuple[SynthParams, float]:
    """Generator parameters of BASELINE.json configs[config-1] (SURVEY.md §8 d)."""
    p = SynthParams()
    p.t0_ns = 1_000_000_000
    p.len_min, p.len_max = 60, 1514
    p.ip_salt = 0x5A17
    zipf_s = 1.1
    if config == 1:
        p.n, p.n_ips, p.duration_ns, p.mode = 1 << 20, 1024, 5_000_000_000, SYNTH_ZIPF_V4
    elif config == 2:
        p.n, p.n_ips, p.duration_ns, p.mode = 64 << 20, 1 << 20, 30_000_000_000, SYNTH_ZIPF_V4
    elif config == 3:
        # features + scores of 4M per-IP flows extracted from a packet stream (SURVEY §8 d
        # config 3): 64M packets from 4M sources drawn uniformly (Zipf exponent 0), so every
        # source is seen (16 packets per source on average)
        p.n, p.n_ips, p.duration_ns, p.mode = 64 << 20, 4 << 20, 30_000_000_000, SYNTH_ZIPF_V4
        zipf_s = 0.0
    elif config == 4:
        p.n, p.n_ips, p.duration_ns, p.mode = 1 << 30, 16 << 20, 120_000_000_000, SYNTH_ZIPF_V4
    elif config == 5:
        p.n, p.n_ips, p.duration_ns, p.mode = 1 << 28, 0, 60_000_000_000, SYNTH_CARPET
        p.pct_v6, p.pct_vlan = 30, 10
    else:
        raise ValueError(f"no packet stream for config {config}")
    p.seed = 0xF5A0 + config
    if n is not None:
        # keep the packet rate of the full config: shorter duration for fewer packets
        p.duration_ns = max(1, p.duration_ns * n // p.n)
        p.n = n
    return p, zipf_s


_synth = None


def _lib():
    global _synth
    if _synth is None:
        path = _PKG / "libfsx_synth.so"
        if not path.exists():
            raise RuntimeError(f"{path} not built: run `python -m flowsentryx_amd.build`")
        lib = C.CDLL(str(path))
        lib.fsx_synth_generate.restype = C.c_int
        lib.fsx_synth_generate.argtypes = [C.POINTER(SynthParams), C.c_double, C.c_uint64,
                                           C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]
        _synth = lib
    return _synth


def generate_device(params: SynthParams, zipf_s: float, j0: int, count: int, d_hdr: int,
                    d_len: int, d_ts: int, stream: int | None = None) -> None:
    rc = _lib().fsx_synth_generate(C.byref(params), zipf_s, j0, count, d_hdr, d_len, d_ts, stream)
    if rc != 0:
        raise RuntimeError(f"fsx_synth_generate failed: {rc}")


# ----------------------------------------------------------------- frame builders
def _pad64(b: bytes, length: int) -> bytes:
    b = b[: min(64, length)]
    return b + bytes(64 - len(b))


def eth(proto: int, src_mac: bytes = b"\x02\x00\x00\x00\x00\x02") -> bytes:
    return b"\x02\x00\x00\x00\x00\x01" + src_mac + struct.pack("!H", proto)


def frame_ipv4_udp(src: bytes, length: int = 100, dport: int = 53, sport: int = 4242,
                   ihl_byte: int = 0x45) -> bytes:
    """64-byte record of an Ethernet/IPv4/UDP frame of `length` bytes from `src`."""
    tot = max(0, length - 14)
    ip = bytes([ihl_byte, 0]) + struct.pack("!HHHBBH", tot & 0xFFFF, 1, 0x4000, 64, 17, 0)
    ip += bytes(src) + bytes([10, 0, 0, 1])
    udp = struct.pack("!HHHH", sport, dport, max(0, tot - 20) & 0xFFFF, 0)
    return _pad64(eth(0x0800) + ip + udp, length)


def frame_ipv6_udp(src: bytes, length: int = 120, dport: int = 443, sport: int = 4242) -> bytes:
    plen = max(0, length - 54)
    ip6 = bytes([0x60, 0, 0, 0]) + struct.pack("!HBB", plen & 0xFFFF, 17, 64) + bytes(src)
    ip6 += bytes.fromhex("20010db8000000000000000000000001")
    udp = struct.pack("!HHHH", sport, dport, plen & 0xFFFF, 0)
    return _pad64(eth(0x86DD) + ip6 + udp, length)


def frame_raw(proto: int, payload: bytes, length: int) -> bytes:
    return _pad64(eth(proto) + payload, length)


def records(frames: list[bytes]) -> np.ndarray:
    return np.frombuffer(b"".join(frames), dtype=np.uint8).reshape(-1, 64).copy()
