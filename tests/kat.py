"""Test support: expand tests/golden/kat_fixed_window.json into packet arrays."""
from __future__ import annotations

import ipaddress
import json
from pathlib import Path

import numpy as np

from flowsentryx_amd import synth

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_kats():
    return json.loads((GOLDEN / "kat_fixed_window.json").read_text())["cases"]


def addr_bytes(s: str) -> bytes:
    return ipaddress.ip_address(s).packed


def build_case(case: dict, restatement: bool = True):
    frames, lens, tss, exp = [], [], [], []
    t = 1_000_000_000
    for run in case.get("runs", []):
        src = addr_bytes(run["src"])
        mk = synth.frame_ipv4_udp if run["family"] == 4 else synth.frame_ipv6_udp
        e = run["expect"]
        for i in range(run["count"]):
            frames.append(mk(src, run["len"]))
            lens.append(run["len"])
            tss.append(run["t0"] + i * run["dt"])
            exp.append(e[i] if isinstance(e, list) else e)
    for f in case.get("frames", []):
        if f.get("restatement_only") and not restatement:
            continue
        k = f["kind"]
        if k == "ipv4":
            rec = synth.frame_ipv4_udp(addr_bytes(f["src"]), f["len"])
        elif k == "ipv6":
            rec = synth.frame_ipv6_udp(addr_bytes(f["src"]), f["len"])
        elif k == "ipv4_v6ihl15":
            rec = synth.frame_ipv4_udp(addr_bytes(f["src"]), f["len"], ihl_byte=0x6F)
        else:
            rec = synth.frame_raw(f["proto"], bytes(range(46)), f["len"])
        frames.append(rec)
        lens.append(f["len"])
        tss.append(t)
        t += 1000
        exp.append(f["expect"])
    hdr = synth.records(frames)
    return (hdr, np.array(lens, dtype=np.uint32), np.array(tss, dtype=np.uint64),
            np.array(exp, dtype=np.uint8))


MAP_IDS = {"ipv4_stats_map": 1, "ipv6_stats_map": 2, "ipv4_blacklist_map": 3,
           "ipv6_blacklist_map": 4}


def expected_maps(case: dict):
    out = {}
    for name, entries in case.get("maps", {}).items():
        out[MAP_IDS[name]] = {addr_bytes(k): (tuple(v) if isinstance(v, list) else v)
                              for k, v in entries.items()}
    return out
