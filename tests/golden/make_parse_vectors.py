"""Generate tests/golden/parse_vectors.npz with the REFERENCE's own parsers.

Runs only in the build container (needs /root/reference): oracle/Makefile compiles
FlowSentryX src/parsing_helper.h (parse_ethhdr / parse_ip6hdr / parse_ip4hdr) from
the read-only tree into oracle/_ref/libref_parse.so, driven with the dispatch of
src/fsx_kern.c:123-148. The committed .npz is data (frames + expected class/key);
tests compare the oracle restatement and the GPU parse against it.
"""
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import pyoracle  # noqa: E402
from flowsentryx_amd import synth  # noqa: E402

subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
rng = np.random.default_rng(20241220)
frames, lens = [], []


def add(rec: bytes, length: int):
    frames.append(np.frombuffer(rec, dtype=np.uint8))
    lens.append(length)


# edge cases of SURVEY.md §4 and around every bound (14 / 34 / 54 bytes)
src4 = bytes([198, 51, 100, 7])
src6 = bytes.fromhex("20010db8aaaabbbbccccddddeeeeffff")
for L in [0, 1, 12, 13, 14, 15, 20, 33, 34, 35, 60, 64, 65, 1514, 9000, 65535, 2**32 - 1]:
    add(synth.frame_ipv4_udp(src4, L), L)
for L in [13, 14, 40, 53, 54, 55, 64, 120, 1514]:
    add(synth.frame_ipv6_udp(src6, L), L)
for proto in [0x0806, 0x8100, 0x88A8, 0x0000, 0xFFFF, 0x0801, 0x86DC, 0x0008, 0xDD86]:
    for L in [13, 14, 60]:
        add(synth.frame_raw(proto, bytes(range(50)), L), L)
# EtherType 0x0800 carrying a version-6 / IHL-15 header: still IPv4 (IHL never checked)
add(synth.frame_ipv4_udp(src4, 60, ihl_byte=0x6F), 60)
add(synth.frame_ipv4_udp(src4, 34, ihl_byte=0x00), 34)
# VLAN-tagged IPv4 -> non-IP EtherType at bytes 12-13
add(synth.frame_raw(0x8100, b"\x00\x05\x08\x00" + synth.frame_ipv4_udp(src4, 60)[14:], 64), 64)
# random records: random bytes with IP-ish EtherTypes and random lengths
for _ in range(4000):
    rec = rng.integers(0, 256, 64, dtype=np.uint8)
    pick = rng.integers(0, 4)
    if pick == 0:
        rec[12:14] = (0x08, 0x00)
    elif pick == 1:
        rec[12:14] = (0x86, 0xDD)
    L = int(rng.choice([rng.integers(0, 80), rng.integers(0, 2000), rng.integers(0, 2**32)]))
    add(rec.tobytes(), L)

hdr = np.stack(frames).astype(np.uint8)
length = np.array(lens, dtype=np.uint32)
cls, keys = pyoracle.ref_parse(hdr, length)
out = Path(__file__).with_name("parse_vectors.npz")
np.savez_compressed(out, hdr=hdr, len=length, cls=cls, keys=keys)
print(f"wrote {out}: {len(lens)} records; classes {np.bincount(cls, minlength=4).tolist()}")
