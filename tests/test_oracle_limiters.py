"""CPU: the oracle's build-defined limiters (oracle/fsx_oracle.c) against a direct
Python transcription of the spec in DESIGN.md §4 (the reference only names these
limiters, README.md:155-162: parity unpinned, so the spec text is the contract).

Small seeded streams; pure-Python loops.
"""
import numpy as np
import pytest

from test_gpu_parity import rand_stream

U64 = (1 << 64) - 1
COST = 10**9


def _src(hdr_row, length):
    et = (int(hdr_row[12]) << 8) | int(hdr_row[13])
    if length < 14:
        return "drop"
    if et == 0x86DD:
        return "drop" if length < 54 else (6, bytes(hdr_row[22:38]))
    if et == 0x0800:
        return "drop" if length < 34 else (4, bytes(hdr_row[26:30]))
    return "pass"


def spec_token_bucket(hdr, ln, ts, rate, burst, rules=None):
    """DESIGN.md §4.2, one packet at a time."""
    cap = burst * COST
    bl = dict(rules or {})
    tb = {}
    out, allowed, dropped = [], 0, 0
    for i in range(len(ln)):
        s = _src(hdr[i], int(ln[i]))
        if s == "drop":
            out.append(1)
            continue
        if s == "pass":
            out.append(2)
            continue
        now = int(ts[i])
        till = bl.get(s)
        if till is not None and till > 0:
            if now > till:
                del bl[s]
            else:
                out.append(1)
                dropped += 1
                continue
        if s not in tb:
            y = cap
        else:
            tok, last = tb[s]
            add = min(((now - last) & U64) * rate, U64)
            y = min(min(tok + add, U64), cap)
        if y >= COST:
            tb[s] = (y - COST, now)
            out.append(2)
            allowed += 1
        else:
            tb[s] = (0, now)
            out.append(1)
            dropped += 1
    return np.array(out, dtype=np.uint8), (allowed, dropped), tb, bl


@pytest.mark.parametrize("rate,burst", [(1000, 1000), (300_000, 4), (0, 3), (10**6, 0),
                                        (1 << 40, 1)])
def test_oracle_token_bucket_matches_spec(oracle, rate, burst):
    rng = np.random.default_rng(rate % 97 + burst)
    hdr, ln, ts = rand_stream(rng, 4000, 40, dt_max=400, v6_frac=0.3, nonip_frac=0.05,
                              short_frac=0.02)
    ts[100] = ts[100] - np.uint64(5000)           # a step back in time
    o = oracle.Oracle(limiter=2, tb_rate=rate, tb_burst=burst, max_entries=1 << 12)
    k0 = bytes(hdr[3, 26:30]) if _src(hdr[3], int(ln[3])) not in ("drop", "pass") else None
    rules = {}
    if k0 is not None and _src(hdr[3], int(ln[3]))[0] == 4:
        rules[(4, k0)] = int(ts[2000])
        o.map_update(3, k0, int(ts[2000]))
    v = o.batch(hdr, ln, ts)
    exp, st, tb, bl = spec_token_bucket(hdr, ln, ts, rate, burst, rules)
    assert np.array_equal(v, exp)
    assert o.stats() == st
    d4, d6 = o.map_dump(5), o.map_dump(6)
    assert {(4, k): val for k, val in d4.items()} | {(6, k): val for k, val in d6.items()} == tb
    assert {(4, k): val for k, val in o.map_dump(3).items()} == {k: t for k, t in bl.items()
                                                                  if k[0] == 4}


def spec_sliding_window(hdr, ln, ts, P, B, W, BLK, rules=None):
    """DESIGN.md §4.1, one packet at a time, explicit per-source logs."""
    bl = dict(rules or {})
    logs, st = {}, {}
    out, allowed, dropped = [], 0, 0
    for i in range(len(ln)):
        s = _src(hdr[i], int(ln[i]))
        if s in ("drop", "pass"):
            out.append(1 if s == "drop" else 2)
            continue
        now = int(ts[i])
        till = bl.get(s)
        if till is not None and till > 0:
            if now > till:
                del bl[s]
            else:
                out.append(1)
                dropped += 1
                continue
        log = logs.setdefault(s, [])
        while log and ((now - log[0][0]) & U64) >= W:
            log.pop(0)
        log.append((now, int(ln[i])))
        cnt, byt = len(log), sum(x[1] for x in log)
        st[s] = (cnt, byt, log[0][0])
        if cnt > P or byt > B:
            bl[s] = (now + BLK) & U64
            log.clear()
            out.append(1)
            dropped += 1
        else:
            out.append(2)
            allowed += 1
    return np.array(out, dtype=np.uint8), (allowed, dropped), st, bl


@pytest.mark.parametrize("P,B,W,BLK", [(1000, 125_000_000, 10**9, 10**10), (7, 10**9, 200_000, 10**6),
                                       (5, 10**9, 10**6, 50_000), (3, 10**9, 100_000, 0),
                                       (50, 9000, 500_000, 2 * 10**6), (0, 10**9, 10**5, 3 * 10**5),
                                       (3, 10**9, 0, 10**5)])
def test_oracle_sliding_window_matches_spec(oracle, P, B, W, BLK):
    rng = np.random.default_rng(P + W % 1000)
    hdr, ln, ts = rand_stream(rng, 4000, 40, dt_max=400, v6_frac=0.3, nonip_frac=0.05,
                              short_frac=0.02)
    ts[100] = ts[100] - np.uint64(5000)
    o = oracle.Oracle(limiter=1, pps_threshold=P, bps_threshold=B, window_ns=W, block_ns=BLK,
                      max_entries=1 << 12)
    v = o.batch(hdr[:2500], ln[:2500], ts[:2500])
    v = np.concatenate([v, o.batch(hdr[2500:], ln[2500:], ts[2500:])])
    exp, st, stats, bl = spec_sliding_window(hdr, ln, ts, P, B, W, BLK)
    assert np.array_equal(v, exp)
    assert o.stats() == st
    got = {(4, k): val for k, val in o.map_dump(1).items()}
    got |= {(6, k): val for k, val in o.map_dump(2).items()}
    assert got == stats
    gbl = {(4, k): val for k, val in o.map_dump(3).items()}
    gbl |= {(6, k): val for k, val in o.map_dump(4).items()}
    assert gbl == bl
