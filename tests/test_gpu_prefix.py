"""GPU parity of the prefix blocklists (FSX_MAP_IPV4_PREFIX / _IPV6_PREFIX)
against the CPU oracle: verdicts, stats_map and every map (the prefix maps included) under
all three limiters, rule changes between batches, the map syscalls' LPM semantics, the
owner's record mode, and the flow features of the packets that reach the per-source path.
Build-defined semantics (the reference defers LPM, TODO.md:251): parity unpinned against
the reference itself; hand-worked cases pin the oracle (tests/test_oracle_prefix.py).
"""
import errno

import numpy as np
import pytest

from test_gpu_parity import CFGS, gpu_ctx, rand_stream

pytestmark = pytest.mark.gpu

NEVER = 2**64 - 1
ALL_MAPS = (1, 2, 3, 4, 7, 8)


def _ips(hdr, ln):
    """(family, address bytes) of every IPv4 / IPv6 frame (the parse rules)."""
    out = []
    for h, L in zip(hdr, ln):
        proto = int(h[12]) << 8 | int(h[13])
        if proto == 0x0800 and L >= 34:
            out.append((4, bytes(h[26:30])))
        elif proto == 0x86DD and L >= 54:
            out.append((6, bytes(h[22:38])))
        else:
            out.append(None)
    return out


def _rules(rng, ips, n, t_lo, t_hi):
    """Random prefixes around the stream's sources: mixed lengths, exceptions (till 0),
    rules that expire inside the stream's time span and permanent ones."""
    from flowsentryx_amd.lib import prefix_key
    srcs = sorted({x for x in ips if x is not None})
    out = {}
    for _ in range(n):
        fam, a = srcs[rng.integers(len(srcs))]
        bits = 32 if fam == 4 else 128
        plen = int(rng.integers(0, bits + 1)) if rng.random() < 0.2 else \
            int(rng.integers(bits // 2, bits + 1))
        r = rng.random()
        till = 0 if r < 0.2 else NEVER if r < 0.6 else int(rng.integers(t_lo, t_hi))
        out[(7 if fam == 4 else 8, prefix_key(a, plen))] = till
    return out


def _install(ctx, rules, batched=False):
    if batched:
        for m in (7, 8):
            ctx.map_update_batch(m, {k: v for (mm, k), v in rules.items() if mm == m})
    else:
        for (m, k), v in rules.items():
            ctx.map_update(m, k, v)


def _assert_same(c, o, maps=ALL_MAPS):
    assert c.stats() == o.stats()
    for m in maps:
        g, r = c.map_dump(m), o.map_dump(m)
        assert g == r, (m, len(g), len(r))


@pytest.mark.parametrize("limiter", [0, 1, 2])
def test_prefix_rules_random(native, oracle, limiter):
    rng = np.random.default_rng(70 + limiter)
    hdr, ln, ts = rand_stream(rng, 90000, 900, dt_max=300, v6_frac=0.3, nonip_frac=0.02,
                              short_frac=0.01)
    ips = _ips(hdr, ln)
    t0, t1 = int(ts[0]), int(ts[-1])
    cfg = dict(CFGS["tight"], limiter=limiter, max_entries=1 << 15)
    okw = dict(CFGS["tight"], limiter=limiter, max_entries=1 << 15)
    if limiter == 2:
        cfg = okw = dict(limiter=2, tb_rate=300_000, tb_burst=4, max_entries=1 << 15)
    maps = (3, 4, 5, 6, 7, 8) if limiter == 2 else ALL_MAPS
    o = oracle.Oracle(**okw)
    with gpu_ctx(native, **cfg) as c:
        rules = _rules(rng, ips, 60, t0, t1)
        _install(c, rules, batched=True)
        for (m, k), v in rules.items():
            o.map_update(m, k, v)
        drops = 0
        for b, (a, z) in enumerate(((0, 30000), (30000, 60000), (60000, 90000))):
            vg = c.verdict_batch(hdr[a:z], ln[a:z], ts[a:z])
            vo = o.batch(hdr[a:z], ln[a:z], ts[a:z])
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"batch {b}: {bad.size} verdicts differ, first at {bad[:8]}"
            drops += c.last_batch_info()["prefix_rule_drops"]
            _assert_same(c, o, maps)
            # rule changes between batches: deletes, new rules, a changed till
            keys = list(rules)
            for j in rng.choice(len(keys), 8, replace=False):
                m, k = keys[j]
                assert c.map_delete(m, k) and o.map_delete(m, k) == 0
                del rules[keys[j]]
            more = _rules(rng, ips, 10, t0, t1)
            _install(c, more)
            for (m, k), v in more.items():
                o.map_update(m, k, v)
            rules.update(more)
    assert drops > 0


def test_prefix_map_syscalls(native, oracle):
    from flowsentryx_amd import lib
    from flowsentryx_amd.lib import prefix_key
    rng = np.random.default_rng(7)
    o = oracle.Oracle()
    with gpu_ctx(native, max_batch=1024) as c:
        for _ in range(300):
            fam = 4 if rng.random() < 0.5 else 6
            a = rng.integers(0, 4, 4 if fam == 4 else 16, dtype=np.uint8).tobytes()
            plen = int(rng.integers(0, (32 if fam == 4 else 128) + 1))
            m = 7 if fam == 4 else 8
            till = int(rng.integers(1, 2**63))
            c.map_update(m, prefix_key(a, plen), till)
            o.map_update(m, prefix_key(a, plen), till)
        assert c.map_dump(7) == o.map_dump(7) and c.map_dump(8) == o.map_dump(8)
        for _ in range(500):   # longest-prefix-match lookups, capped by the key's prefixlen
            fam = 4 if rng.random() < 0.5 else 6
            a = rng.integers(0, 4, 4 if fam == 4 else 16, dtype=np.uint8).tobytes()
            plen = int(rng.integers(0, (32 if fam == 4 else 128) + 1))
            m = 7 if fam == 4 else 8
            assert c.map_lookup(m, prefix_key(a, plen)) == o.map_lookup(m, prefix_key(a, plen))
        k = next(iter(c.map_dump(7)))
        with pytest.raises(lib.FsxError) as e:
            c.map_update(7, k, 5, flags=lib.BPF_NOEXIST)
        assert e.value.code == -errno.EEXIST
        with pytest.raises(lib.FsxError) as e:
            c.map_update(7, prefix_key(bytes(4), 33), 5)
        assert e.value.code == -errno.EINVAL
        assert c.map_delete(7, k) and not c.map_delete(7, k)
        # batched import is all or nothing at FSX_PREFIX_MAX_ENTRIES
        big = {prefix_key(i.to_bytes(4, "big"), 32): NEVER for i in range(lib.PREFIX_MAX_ENTRIES)}
        before = c.map_dump(7)
        with pytest.raises(lib.FsxError) as e:
            c.map_update_batch(7, big)
        assert e.value.code == -errno.ENOSPC
        assert c.map_dump(7) == before
        c.reset()   # per-source state only: the rules are configuration
        assert c.map_dump(7) == before
        for k in before:
            assert c.map_delete(7, k)
        assert c.map_dump(7) == {}


def test_prefix_drops_whole_batch(native, oracle):
    """A /0 rule per family: every IP packet is dropped before the sort (an empty
    per-source pass), non-IP frames pass, short frames drop uncounted."""
    from flowsentryx_amd.lib import prefix_key
    rng = np.random.default_rng(9)
    hdr, ln, ts = rand_stream(rng, 20000, 300, v6_frac=0.4, nonip_frac=0.05, short_frac=0.02)
    o = oracle.Oracle()
    with gpu_ctx(native) as c:
        for m, z in ((7, bytes(4)), (8, bytes(16))):
            c.map_update(m, prefix_key(z, 0), NEVER)
            o.map_update(m, prefix_key(z, 0), NEVER)
        vg = c.verdict_batch(hdr, ln, ts)
        assert np.array_equal(vg, o.batch(hdr, ln, ts))
        info = c.last_batch_info()
        assert info["ip_packets"] == 0 and info["prefix_rule_drops"] == info["dropped"] > 0
        _assert_same(c, o)


def test_prefix_rules_record_mode(native, oracle):
    """The owner's record mode (sharded path) applies the rules like the header path."""
    import torch
    from flowsentryx_amd.shard import HipShardEngine
    rng = np.random.default_rng(11)
    hdr, ln, ts = rand_stream(rng, 40000, 500, dt_max=200, v6_frac=0.3, nonip_frac=0.03)
    n = hdr.shape[0]
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hdr.reshape(-1).copy()).to(dev)
    tl = torch.from_numpy(ln.view(np.int32).copy()).to(dev)
    tt = torch.from_numpy(ts.view(np.int64).copy()).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    cfg = dict(max_batch=1 << 16, max_entries=1 << 15, pps_threshold=7, window_ns=200_000,
               block_ns=1_000_000)
    rules = _rules(rng, _ips(hdr, ln), 50, int(ts[0]), int(ts[-1]))
    with native.FsxContext(**cfg) as ca, native.FsxContext(**cfg) as cb:
        _install(ca, rules)
        e = HipShardEngine(ca, n, dev)
        rec, counts = e.pack(th, tl, tt, n, 1, tv)
        ca.sync()
        m, rb = int(counts[0].item()), int(counts[2].item())
        hb, lb, tsb, _ = e._owner_buffers(m)
        cb.shard_unpack_device(rec.data_ptr(), m, hb.data_ptr(), lb.data_ptr(), tsb.data_ptr(), rb)
        cb.sync()
        v = torch.zeros(m, dtype=torch.uint8, device=dev)
        ca.verdict_records_device(rec.data_ptr(), m, rb, v.data_ptr())
        ca.sync()
        h_np = hb.cpu().numpy().reshape(-1, 64)[:m]
        l_np = lb.cpu().numpy().view(np.uint32)[:m]
        t_np = tsb.cpu().numpy().view(np.uint64)[:m]
    o = oracle.Oracle(max_entries=1 << 15, pps_threshold=7, window_ns=200_000, block_ns=1_000_000)
    for (mm, k), val in rules.items():
        o.map_update(mm, k, val)
    assert np.array_equal(v.cpu().numpy(), o.batch(h_np, l_np, t_np))


def _rule_dropped(rules, ips, ts):
    """Independent LPM restatement (bit strings) for the feature filter."""
    def bits(a):
        return "".join(f"{x:08b}" for x in a)
    table = {}
    for (m, k), till in rules.items():
        plen = int.from_bytes(k[:4], "little")
        table[(4 if m == 7 else 6, bits(k[4:])[:plen])] = till
    out = np.zeros(len(ips), bool)
    for i, x in enumerate(ips):
        if x is None:
            continue
        b = bits(x[1])
        for L in range(len(b), -1, -1):
            till = table.get((x[0], b[:L]))
            if till is not None:
                out[i] = 0 < int(ts[i]) <= till
                break
    return out


def test_prefix_rules_and_flow_features(native, oracle):
    """process_batch_device with rules: the features cover the packets that reach the
    per-source path (rule-dropped packets are not part of any flow)."""
    import torch
    from test_gpu_parity import _sorted_flows
    rng = np.random.default_rng(13)
    hdr, ln, ts = rand_stream(rng, 30000, 400, dt_max=500, v6_frac=0.3, nonip_frac=0.02)
    n = hdr.shape[0]
    ips = _ips(hdr, ln)
    rules = _rules(rng, ips, 40, int(ts[0]), int(ts[-1]))
    dev = lambda a: torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).cuda()
    d_hdr, d_len, d_ts = dev(hdr), dev(ln), dev(ts)
    d_v = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_k = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    d_f = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(n * 8, dtype=torch.float32, device="cuda")
    with gpu_ctx(native, max_batch=n) as c:
        _install(c, rules)
        c.process_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                               d_v.data_ptr(), d_k.data_ptr(), d_f.data_ptr(), d_x.data_ptr(),
                               None, None, n)
        c.sync()
        m = c.last_batch_info()["sources"]
    o = oracle.Oracle(max_entries=1 << 18)
    for (mm, k), val in rules.items():
        o.map_update(mm, k, val)
    assert np.array_equal(d_v.cpu().numpy(), o.batch(hdr, ln, ts))
    keep = ~_rule_dropped(rules, ips, ts)
    assert keep.sum() < n
    ko, fo, xo = oracle.flow_features(hdr[keep], ln[keep], ts[keep])
    assert m == len(fo)
    kg = d_k.cpu().numpy().reshape(n, 16)[:m]
    fg = d_f.cpu().numpy()[:m]
    xg = d_x.cpu().numpy().reshape(n, 8)[:m]
    kg, fg, xg = _sorted_flows(kg, fg, xg)
    ko, fo, xo = _sorted_flows(ko, fo, xo)
    assert np.array_equal(fg, fo) and np.array_equal(kg, ko)
    assert np.array_equal(xg.view(np.uint32), xo.view(np.uint32))


@pytest.mark.parametrize("cover", ["some", "top"])
def test_prefix_rules_unsorted_heavy_path(native, oracle, cover):
    """Prefix rules on the unsorted-heavy path: the pick leaves every source
    whose /24 a rule touches light, so the heavy sources are resolved in the pick and every
    batch still takes the unsorted path (heavy_unsorted). Rules on the most popular sources —
    permanent, expiring inside the batch and exceptions — across three carried batches, against
    the oracle. "top": every one of the 16 most popular sources is under a rule (the heavy set
    is the next ones down)."""
    from collections import Counter
    from flowsentryx_amd.lib import prefix_key
    rng = np.random.default_rng(91)
    hdr, ln, ts = rand_stream(rng, 90000, 600, dt_max=300, v6_frac=0.2)
    ips = _ips(hdr, ln)
    t0, t1 = int(ts[0]), int(ts[-1])
    top = [s for s, _ in Counter(x for x in ips if x is not None).most_common(16)]
    rules = {}
    for j, (fam, a) in enumerate(top if cover == "top" else top[::3]):
        bits = 32 if fam == 4 else 128
        plen = (bits, bits - 4, 24 if fam == 4 else 64)[j % 3]
        till = (2**64 - 1, (t0 + t1) // 2, 0)[j % 3] if cover == "top" else (2**64 - 1, (t0 + t1) // 2)[j % 2]
        rules[(7 if fam == 4 else 8, prefix_key(a, plen))] = till
    cfg = dict(CFGS["tight"], max_entries=1 << 18)   # (>= 2^17 slots: the heavy-source sort)
    o = oracle.Oracle(**cfg)
    for (m, k), v in rules.items():
        o.map_update(m, k, v)
    with gpu_ctx(native, **cfg) as c:
        _install(c, rules, batched=True)
        for b, (a, z) in enumerate(((0, 30000), (30000, 60000), (60000, 90000))):
            vg = c.verdict_batch(hdr[a:z], ln[a:z], ts[a:z])
            vo = o.batch(hdr[a:z], ln[a:z], ts[a:z])
            bad = np.nonzero(vg != vo)[0]
            assert bad.size == 0, f"batch {b}: {bad.size} verdicts differ, first at {bad[:8]}"
            info = c.last_batch_info()
            assert info["heavy_unsorted"] == 1, (b, info)
            assert info["prefix_rule_drops"] > 0
            _assert_same(c, o)
