"""CPU engine of the sharded protocol (flowsentryx_amd/shard.py) for gloo tests.

TEST INFRASTRUCTURE: the per-owner limiter is the CPU oracle, the exchange records are
built with numpy in the 16- and 32-byte layouts of include/fsx_hip.h, owners come from the
library's host function fsx_shard_owner. The protocol code under test is the product's.
"""
import contextlib

import numpy as np
import torch

from flowsentryx_amd import lib

REC_DTYPE = np.dtype([("key", "<u4", 4), ("ts", "<u8"), ("len", "<u4"), ("dport", "<u2"),
                      ("family", "u1"), ("pad", "u1")])
assert REC_DTYPE.itemsize == lib.SHARD_RECORD_BYTES
REC16_DTYPE = np.dtype([("key", "<u4"), ("len", "<u2"), ("dport", "<u2"), ("ts", "<u8")])
assert REC16_DTYPE.itemsize == lib.SHARD_RECORD16_BYTES


def widen(rec16: np.ndarray) -> np.ndarray:
    r = np.zeros(rec16.shape[0], dtype=REC_DTYPE)
    r["key"][:, 0] = rec16["key"]
    r["ts"] = rec16["ts"]
    r["len"] = rec16["len"]
    r["dport"] = rec16["dport"]
    r["family"] = 4
    return r


def records_to_headers(rec: np.ndarray):
    """Header records that parse to the records' source, family, length and dst port."""
    m = rec.shape[0]
    hdr = np.zeros((m, 64), dtype=np.uint8)
    key = rec["key"].copy().view(np.uint8).reshape(m, 16)
    v6 = rec["family"] == 6
    dp = rec["dport"].astype(np.uint32)
    hdr[:, 12] = np.where(v6, 0x86, 0x08)
    hdr[:, 13] = np.where(v6, 0xDD, 0x00)
    hdr[~v6, 14] = 0x45
    hdr[~v6, 23] = 17
    hdr[~v6, 26:30] = key[~v6, :4]
    hdr[~v6, 36] = (dp[~v6] >> 8) & 0xFF
    hdr[~v6, 37] = dp[~v6] & 0xFF
    hdr[v6, 20] = 17
    hdr[v6, 22:38] = key[v6]
    hdr[v6, 56] = (dp[v6] >> 8) & 0xFF
    hdr[v6, 57] = dp[v6] & 0xFF
    return hdr, rec["len"].copy(), rec["ts"].copy()


class CpuShardEngine:
    def __init__(self, oracle, **cfg):
        self.oracle = oracle
        self.o = oracle.Oracle(**cfg)
        self.send_idx = np.zeros(0, dtype=np.int64)
        self.send_idxs = {}   # per pipeline slot
        self.replica = {}

    def stream_ctx(self):
        return contextlib.nullcontext()

    def comm_ctx(self):
        return contextlib.nullcontext()

    def comm_event(self):
        return None

    def return_ctx(self, all_batches):
        return contextlib.nullcontext()

    @staticmethod
    def send_views(rec, sc, rb, slot):
        return list(rec[:sum(sc) * rb].split([c * rb for c in sc]))

    @staticmethod
    def drop_first(slot, sent):
        return sent

    def engine_wait(self, ev):
        pass

    def keep(self, t):
        pass

    @staticmethod
    def _np(hdr, length, ts, n):
        return (hdr.numpy().reshape(-1, 64)[:n], length.numpy().view(np.uint32)[:n],
                ts.numpy().view(np.uint64)[:n])

    def direct(self, hdr, length, ts, n, verdict):
        h, l, t = self._np(hdr, length, ts, n)
        verdict[:n] = torch.from_numpy(self.o.batch(h, l, t))

    def clock(self, ts, n):
        t = ts.numpy().view(np.uint64)[:n]
        if n == 0:
            return torch.tensor([-1, 0, 0], dtype=torch.int64)
        dec = int(np.any(t[1:] < t[:-1]))
        return torch.tensor(np.array([t.min(), t.max(), dec], dtype=np.uint64).view(np.int64))

    def clocks(self, ts, bounds):
        return torch.cat([self.clock(ts[a:], b - a) for a, b in zip(bounds[:-1], bounds[1:])])

    def blocklist_buffer(self, cap):
        ent, m = self.export_blocklist()
        buf = torch.zeros(32 + cap * 32, dtype=torch.uint8)
        buf[:8] = torch.from_numpy(np.array([m], dtype=np.int64).view(np.uint8))
        k = min(m, cap)
        buf[32:32 + k * 32] = ent[:k * 32]
        return buf

    @staticmethod
    def filter_plan(clocks, G, k):
        """The replica filter's decision per sub-batch (fsx_shard_filter_plan_device restated)."""
        c = clocks.numpy().view(np.uint64).reshape(G, k, 3)
        out, prev_hi = [], None
        for j in range(k):
            ok, last, lo, hi = True, None, None, None
            for r in range(G):
                mn, mx, dec = (int(x) for x in c[r, j])
                if dec:
                    ok = False
                if mx == 0 and mn == 2**64 - 1:   # empty piece
                    continue
                if last is not None and mn < last:
                    ok = False
                last = mx
                lo = mn if lo is None else min(lo, mn)
                hi = mx if hi is None else max(hi, mx)
            if ok and prev_hi is not None and lo is not None and lo < prev_hi:
                ok = False
            out.append(1 if ok else 0)
            if hi is not None:
                prev_hi = hi if prev_hi is None else max(prev_hi, hi)
        return torch.tensor(out, dtype=torch.int32)

    def load_replica_blocks(self, blocks, G, cap):
        b = blocks.numpy().reshape(G, 32 + cap * 32)
        self.replica = {}
        for r in range(G):
            m = min(int(b[r, :8].view(np.int64)[0]), cap)
            for e in b[r, 32:32 + m * 32].view(self.BLK_DTYPE):
                fam = 6 if e["tag"] == 2 else 4
                self.replica[(fam, e["key"].tobytes()[:16 if fam == 6 else 4])] = int(e["till"])

    def pack(self, hdr, length, ts, n, G, verdict, filt=None, slot=0, drop_rec=False):
        # (filt: the plan's word for this sub-batch; drop_rec: the HIP engine's flow partials of
        # replica drops; no flows on the CPU engine)
        filt = filt is not None and int(filt[0]) != 0
        h, l, t = self._np(hdr, length, ts, n)
        cls, keys = self.oracle.parse(h, l)
        v = verdict.numpy()
        v[:n][cls == 0] = 1
        v[:n][cls == 1] = 2
        filtered = 0
        if filt:
            for i in np.nonzero(cls >= 2)[0]:
                k = (6 if cls[i] == 3 else 4, keys[i].tobytes()[:16 if cls[i] == 3 else 4])
                till = self.replica.get(k)
                if till is not None and till > 0 and not int(t[i]) > till:
                    cls[i] = 9          # dropped here, counted by the protocol
                    v[i] = 1
                    filtered += 1
        ip = np.nonzero((cls >= 2) & (cls <= 3))[0]
        fam = np.where(cls[ip] == 3, 6, 4).astype(np.uint8)
        own = np.array([lib.shard_owner(keys[i].tobytes(), int(f), G) for i, f in zip(ip, fam)],
                       dtype=np.int64)
        order = np.argsort(own, kind="stable")
        ip, fam = ip[order], fam[order]
        rec = np.zeros(ip.size, dtype=REC_DTYPE)
        rec["key"] = keys[ip].view("<u4").reshape(-1, 4)
        rec["ts"] = t[ip]
        rec["len"] = l[ip]
        rec["dport"] = self.oracle.dst_port(h[ip], l[ip]).astype(np.uint16)
        rec["family"] = fam
        self.send_idx = ip
        self.send_idxs[slot] = ip
        counts = np.bincount(own, minlength=G).astype(np.int64)
        compact = not np.any(fam == 6) and not np.any(rec["len"] > 0xFFFF)
        if compact:
            r16 = np.zeros(ip.size, dtype=REC16_DTYPE)
            for f in ("key", "len", "dport", "ts"):
                r16[f] = rec[f][:, 0] if f == "key" else rec[f]
            rec = r16
        rb = lib.SHARD_RECORD16_BYTES if compact else lib.SHARD_RECORD_BYTES
        counts = np.concatenate([counts, [filtered, rb]]).astype(np.int64)
        return torch.from_numpy(rec.view(np.uint8).copy()), torch.from_numpy(counts)

    BLK_DTYPE = np.dtype([("key", "<u4", 4), ("till", "<u8"), ("tag", "<u4"), ("pad", "<u4")])

    def export_blocklist(self):
        rows = []
        for mid, tag, klen in ((3, 1, 4), (4, 2, 16)):
            for k, till in self.o.map_dump(mid).items():
                if till > 0:
                    rows.append((np.frombuffer(k.ljust(16, b"\0"), dtype="<u4"), till, tag, 0))
        a = np.zeros(len(rows), dtype=self.BLK_DTYPE)
        for i, r in enumerate(rows):
            a[i] = r
        return torch.from_numpy(a.view(np.uint8).copy()), len(rows)

    def load_replica(self, entries, m):
        a = entries.numpy()[:m * 32].view(self.BLK_DTYPE)
        self.replica = {}
        for e in a:
            fam = 6 if e["tag"] == 2 else 4
            k = e["key"].tobytes()[:16 if fam == 6 else 4]
            self.replica[(fam, k)] = int(e["till"])

    def recv_buffer(self, nbytes):
        return torch.empty(max(1, nbytes), dtype=torch.uint8)

    def owner_batch(self, recv, segs, slot=0):
        b = recv.numpy()
        parts = []
        for off, cnt, rb in segs:
            seg = b[off:off + cnt * rb]
            parts.append(widen(seg.view(REC16_DTYPE)) if rb == lib.SHARD_RECORD16_BYTES
                         else seg.view(REC_DTYPE))
        rec = np.concatenate(parts) if parts else np.zeros(0, dtype=REC_DTYPE)
        m = rec.shape[0]
        h, l, t = records_to_headers(rec)
        v = self.o.batch(h, l, t) if m else np.zeros(1, dtype=np.uint8)
        return torch.from_numpy(v)

    def scatter(self, ret, m, verdict, slot=0):
        verdict.numpy()[self.send_idxs[slot]] = ret.numpy()[:m]

    def stats(self):
        return torch.tensor(self.o.stats(), dtype=torch.int64)
