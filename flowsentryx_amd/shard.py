"""Hash(src IP) sharding of the verdict path over G ranks (SURVEY.md §8 e).

The reference is one XDP program per host (src/fsx_kern.c:96-97) whose state is all
per source IP (src/fsx_kern.c:56-94) plus two summed counters. So the path shards with
no shared state: every rank holds a contiguous slice of each arrival batch, every
source has ONE owner rank (include/fsx_hip.h fsx_shard_owner), and the owner runs the
unchanged batch pipeline on all of that source's packets:

  1. pack      parse the local slice, partition its IP packets by owner into 16-byte
               IPv4 records (32-byte when the slice has an IPv6 source or a frame of 64 KiB
               or more; stable: arrival order), verdicts for packets that never reach a
               limiter (short frames DROP, non-IP PASS)
  2. all-to-all of the per-owner counts (record format in the low bit), then of the
     records (RCCL over xGMI)
  3. owner     the batch pipeline straight on the received records (record mode; when
               senders used both record sizes: records -> header records first) — maps,
               verdicts, optionally flow features + MLP scores of the owned sources
  4. all-to-all of the verdicts back (1 byte per packet), scatter to arrival positions
  5. all-gather of every owner's live blacklist entries (the replicated blocklist);
     the next sub-batch's pack drops packets of replica-blacklisted sources locally
     (now <= till: the owner would drop them without touching any state,
     src/fsx_kern.c:189-215) — taken only when that sub-batch's clock is non-decreasing
     in global order (one all-gather of {min, max, decreases} per rank), which is exactly
     the condition under which no earlier packet can have deleted the entry
  6. stats_map = all-reduce(sum) of the owners' counters + the locally dropped packets
  7. with flow features (HipShardEngine.enable_flows): every owner accumulates its sources'
     sums over the batch's sub-batches (fsx_flows_begin / fsx_flows_end) and writes one row
     per owned source at the end of the batch — the row the 1-GPU run over the whole batch
     gives. The packets a replica drops at arrival (5) still count in their source's
     features: the pack keeps them as records, the arrival rank turns them into one flow
     partial per source (fsx_flow_partials_records_device: exact sums, first / last
     timestamp), the partials go to the owners (one small all-to-all) and merge into the
     owner's sums (fsx_flows_merge_device, sender ranks in order) before the owner's own
     records of that sub-batch. Exact because a replica drops a source's packets exactly
     while now <= till, and the filter is only used where the clock is non-decreasing in
     global order: the dropped packets of a source are the first of its packets in the
     sub-batch, and in rank order

A global batch is cut into `chunks` sub-batches; in sub-batch i every rank contributes
the i-th piece of its slice, and the global order of a sub-batch is rank 0's piece,
then rank 1's, ... (the arrival shard "chunk j on rank j mod G" of SURVEY.md §8 d
config 4). Pieces are concatenated in rank order on the owner, so every source's
packets arrive there in global arrival order and the sharded result equals the 1-GPU
run over the same order (tests/test_shard_*.py check this bit-exactly).

The protocol is written against an engine (pack / owner_batch / scatter / stats): the
HIP engine below drives libfsx_hip.so on device tensors; tests drive the same protocol
with a CPU engine over gloo.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from . import lib

REC = lib.SHARD_RECORD_BYTES


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    """all_to_all_single; device tensors go through host memory on a gloo group."""
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


class HipShardEngine:
    """One rank's side of the sharded path on libfsx_hip.so (device tensors)."""

    def __init__(self, ctx: lib.FsxContext, max_local: int, device: torch.device):
        self.ctx = ctx
        self.device = device
        # one stream for the library's kernels and torch's copies / collectives (a real
        # stream: a NULL handle would give the context its own stream back)
        self.stream = torch.cuda.Stream(device)
        ctx.set_stream(self.stream.cuda_stream)
        # owner batches back to back without a host synchronization per call (errors surface
        # at the next synchronization; each batch whole on the engine stream)
        ctx.set_pipeline(2)
        # collectives run from a second stream, so the exchange of sub-batch j + 1 overlaps
        # the owner pipeline of sub-batch j (ShardedDataPlane)
        self.comm = torch.cuda.Stream(device)
        self.max_local = max_local
        self.owner_cap = int(ctx.config.max_batch)
        # per-sub-batch buffers by pipeline slot (allocated on first use, sized for the piece)
        self.recs, self.send_idxs, self.countss = {}, {}, {}
        self.rec = self.send_idx = self.counts = None
        self.clock3 = torch.empty(3, dtype=torch.int64, device=device)
        self.blk = torch.empty(1024 * lib.SHARD_BLOCK_BYTES, dtype=torch.uint8, device=device)
        self.blk_count = torch.empty(1, dtype=torch.int64, device=device)
        self._oh = None  # owner-side header/len/ts buffers, grown on demand
        self._ov = {}             # owner-side verdicts per slot
        self.flows = None
        # arrival side of the replica filter with flows: a flow-only context for the partials
        # of the replica-dropped packets, its output buffers per pipeline slot
        self.pctx = None
        self.pctx_entries = 0
        self.pbufs, self.pcnts = {}, {}
        self.owner_calls = 0      # batch-pipeline calls of this rank (per-kernel timings are per call)

    # -- streams of the pipelined plane (the CPU engine has none)
    @contextlib.contextmanager
    def comm_ctx(self):
        """Collectives on the comm stream, after all work enqueued on the engine stream."""
        self.comm.wait_stream(self.stream)
        with torch.cuda.stream(self.comm):
            yield

    def comm_event(self):
        """An event after the work enqueued on the comm stream so far."""
        ev = torch.cuda.Event()
        ev.record(self.comm)
        return ev

    def engine_wait(self, ev):
        """The engine stream continues after `ev` (a comm_event)."""
        self.stream.wait_event(ev)

    def keep(self, t: torch.Tensor):
        """t (allocated on the comm stream) is also used by the engine stream: its memory
        is not reused before the engine stream's work so far has finished."""
        if t.is_cuda:
            t.record_stream(self.stream)

    @contextlib.contextmanager
    def stream_ctx(self):
        """Run a protocol step on the engine stream, ordered after the caller's stream
        (which produced the inputs) and before it (which consumes the verdicts)."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            yield
        cur.wait_stream(self.stream)

    def _owner_buffers(self, m: int):
        if self._oh is None or self._oh[0].numel() < m * 64:
            cap = max(m, 1)
            self._oh = (torch.empty(cap * 64, dtype=torch.uint8, device=self.device),
                        torch.empty(cap, dtype=torch.int32, device=self.device),
                        torch.empty(cap, dtype=torch.int64, device=self.device),
                        torch.empty(cap, dtype=torch.uint8, device=self.device))
        return self._oh

    def enable_flows(self, cap: int):
        """Per owned source of every global batch: key, family, the eight features, q8
        probability and decision, over ALL of the source's packets of the batch (its
        sub-batches accumulate, fsx_flows_begin / fsx_flows_end); rows[0] = row count."""
        d = self.device
        self.flows = dict(keys=torch.empty(cap * 16, dtype=torch.uint8, device=d),
                          fam=torch.empty(cap, dtype=torch.uint8, device=d),
                          feat=torch.empty(cap * 8, dtype=torch.float32, device=d),
                          prob=torch.empty(cap, dtype=torch.float32, device=d),
                          dec=torch.empty(cap, dtype=torch.uint8, device=d),
                          rows=torch.zeros(1, dtype=torch.int64, device=d), cap=cap)

    def flows_begin(self):
        if self.flows is not None:
            self.ctx.flows_begin()

    def flows_end(self):
        """The batch's rows into self.flows (asynchronous; rows[0] = their count)."""
        if self.flows is None:
            return
        f = self.flows
        self.ctx.flows_end(f["keys"].data_ptr(), f["fam"].data_ptr(), f["feat"].data_ptr(),
                           f["prob"].data_ptr(), f["dec"].data_ptr(), f["cap"], f["rows"].data_ptr())

    def direct(self, hdr, length, ts, n, verdict):
        """G == 1: the batch pipeline straight on the local slice."""
        self._run(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, verdict.data_ptr())

    def _owner_verdicts(self, m: int, slot: int) -> torch.Tensor:
        if self._ov.get(slot) is None or self._ov[slot].numel() < m:
            self._ov[slot] = torch.empty(max(m, 1), dtype=torch.uint8, device=self.device)
        return self._ov[slot]

    def _run_records(self, rec, n, rb, v):
        self.owner_calls += 1
        if self.flows is None:
            self.ctx.verdict_records_device(rec, n, rb, v)
        else:
            f = self.flows
            self.ctx.process_records_device(rec, n, rb, v, f["keys"].data_ptr(), f["fam"].data_ptr(),
                                            f["feat"].data_ptr(), f["prob"].data_ptr(), f["dec"].data_ptr(),
                                            f["cap"])

    def _run(self, h, l, t, n, v):
        self.owner_calls += 1
        if self.flows is None:
            self.ctx.verdict_batch_device(h, l, t, n, v)
        else:
            f = self.flows
            self.ctx.process_batch_device(h, l, t, n, v, f["keys"].data_ptr(), f["fam"].data_ptr(),
                                          f["feat"].data_ptr(), f["prob"].data_ptr(), f["dec"].data_ptr(),
                                          f["cap"])

    def clock(self, ts, n) -> torch.Tensor:
        self.ctx.shard_clock_device(ts.data_ptr(), n, self.clock3.data_ptr())
        return self.clock3

    def clocks(self, ts, bounds) -> torch.Tensor:
        """{min, max, decreases} of every piece [bounds[j], bounds[j+1]) (int64 [3 * pieces])."""
        k = len(bounds) - 1
        out = torch.empty(3 * k, dtype=torch.int64, device=self.device)
        for j in range(k):
            a, b = bounds[j], bounds[j + 1]
            self.ctx.shard_clock_device(ts.data_ptr() + 8 * a, b - a, out.data_ptr() + 24 * j)
        return out

    def blocklist_buffer(self, cap: int) -> torch.Tensor:
        """This rank's live blacklist entries for one all-gather: 32 header bytes (int64
        entry count first) then up to cap 32-byte entries; no host synchronization."""
        B = lib.SHARD_BLOCK_BYTES
        buf = torch.empty(B + cap * B, dtype=torch.uint8, device=self.device)
        self.ctx.blocklist_export_device(buf.data_ptr() + B, cap, buf.data_ptr())
        return buf

    def pack(self, hdr, length, ts, n, G, verdict, filt=False, slot=0, drop_rec=False):
        """-> records, counts[G + 2] (counts[G]: packets dropped by the replica,
        counts[G + 1]: record bytes, 16 or 32), in pipeline slot `slot`. drop_rec: the
        dropped packets' records follow the owners' runs."""
        if n > self.max_local:
            raise ValueError(f"local slice of {n} packets exceeds {self.max_local}")
        flags = lib.SHARD_COMPACT | (lib.SHARD_FILTER_BLOCKLIST if filt else 0)
        if filt and drop_rec:
            flags |= lib.SHARD_DROP_RECORDS
        if slot not in self.recs or self.send_idxs[slot].numel() < max(1, n):
            m = max(1, n)
            self.recs[slot] = torch.empty(m * REC, dtype=torch.uint8, device=self.device)
            self.send_idxs[slot] = torch.empty(m, dtype=torch.int32, device=self.device)
            self.countss[slot] = torch.empty(lib.MAX_SHARDS + 2, dtype=torch.int64, device=self.device)
        rec, idx, cnt = self.recs[slot], self.send_idxs[slot], self.countss[slot]
        self.rec, self.send_idx, self.counts = rec, idx, cnt   # (tests read the last pack)
        self.ctx.shard_pack_device(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, G,
                                   verdict.data_ptr(), rec.data_ptr(), idx.data_ptr(), cnt.data_ptr(),
                                   flags)
        return rec, cnt[:G + 2]

    def partials(self, rec, first, m, rb, G, cap, slot=0):
        """Flow partials of the m replica-dropped records from record index `first` of a pack
        buffer: G runs of cap partials (source -> run of its owner) and counts[G]; enqueued
        on the engine stream (no host synchronization)."""
        if self.pctx is None or self.pctx_entries < cap:
            if self.pctx is not None:
                self.pctx.sync()
                self.pctx.close()
            ent = max(1024, 2 * cap)
            self.pctx = lib.FsxContext(max_batch=max(1, self.max_local), max_entries=ent,
                                       device=self.device.index or 0)
            self.pctx.set_stream(self.stream.cuda_stream)
            self.pctx_entries = ent
        B = lib.FLOW_PARTIAL_BYTES
        if self.pbufs.get(slot) is None or self.pbufs[slot].numel() < G * cap * B:
            self.pbufs[slot] = torch.empty(max(1, G * cap * B), dtype=torch.uint8, device=self.device)
            self.pcnts[slot] = torch.empty(G, dtype=torch.int64, device=self.device)
        buf, cnt = self.pbufs[slot], self.pcnts[slot]
        self.pctx.flow_partials_records_device(rec.data_ptr() + first * rb, m, rb, G, buf.data_ptr(), cap,
                                               cnt.data_ptr())
        return buf, cnt

    def merge(self, parts: torch.Tensor, m: int):
        """Merge m received partials (one sender's, distinct sources) into the owner's sums."""
        if m:
            self.ctx.flows_merge_device(parts.data_ptr(), m)

    def export_blocklist(self) -> tuple[torch.Tensor, int]:
        """This rank's live blacklist entries (32-byte records) and their count."""
        while True:
            cap = self.blk.numel() // lib.SHARD_BLOCK_BYTES
            self.ctx.blocklist_export_device(self.blk.data_ptr(), cap, self.blk_count.data_ptr())
            m = int(self.blk_count.item())
            if m <= cap:
                return self.blk, m
            self.blk = torch.empty(2 * m * lib.SHARD_BLOCK_BYTES, dtype=torch.uint8,
                                   device=self.device)

    def load_replica(self, entries: torch.Tensor, m: int):
        self.ctx.blocklist_replica_device(entries.data_ptr(), m)

    def recv_buffer(self, nbytes: int) -> torch.Tensor:
        return torch.empty(max(1, nbytes), dtype=torch.uint8, device=self.device)

    def owner_batch(self, recv: torch.Tensor, segs, slot: int = 0) -> torch.Tensor:
        """The limiter over the received records, in received order: segs = [(byte
        offset, records, record bytes)] per sender (chunked by the context's max_batch:
        state carries across chunks exactly as across batches)."""
        m = sum(c for _, c, _ in segs)
        fmts = {rb for _, c, rb in segs if c}
        if len(fmts) == 1:
            # one record format: the pipeline reads the received records directly
            rb = fmts.pop()
            v = self._owner_verdicts(m, slot)
            for a in range(0, m, self.owner_cap):
                b = min(m, a + self.owner_cap)
                self._run_records(recv.data_ptr() + a * rb, b - a, rb, v.data_ptr() + a)
            return v[:max(m, 1)]
        hdr, ln, ts, _ = self._owner_buffers(m)
        v = self._owner_verdicts(m, slot)
        r = 0
        for off, cnt, rb in segs:
            if cnt:
                self.ctx.shard_unpack_device(recv.data_ptr() + off, cnt, hdr.data_ptr() + r * 64,
                                             ln.data_ptr() + r * 4, ts.data_ptr() + r * 8, rb)
            r += cnt
        for a in range(0, m, self.owner_cap):
            b = min(m, a + self.owner_cap)
            self._run(hdr.data_ptr() + a * 64, ln.data_ptr() + a * 4, ts.data_ptr() + a * 8,
                      b - a, v.data_ptr() + a)
        return v[:max(m, 1)]

    def scatter(self, ret: torch.Tensor, m: int, verdict, slot: int = 0):
        if m:
            self.ctx.shard_scatter_device(ret.data_ptr(), self.send_idxs[slot].data_ptr(), m,
                                          verdict.data_ptr())

    def stats(self) -> torch.Tensor:
        a, d = self.ctx.stats()
        return torch.tensor([a, d], dtype=torch.int64, device=self.device)


def _all_gather(t: torch.Tensor, G: int, group=None) -> torch.Tensor:
    """[G * numel] concatenation of every rank's equally sized t."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        out = torch.empty(G * t.numel(), dtype=t.dtype)
        dist.all_gather_into_tensor(out, t.cpu().contiguous(), group=group)
        return out.to(t.device)
    out = torch.empty(G * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


class ShardedDataPlane:
    """The sharded verdict path of one rank (one process per GPU)."""

    def __init__(self, engine, group=None, blocklist_filter: bool = True):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.filter = blocklist_filter and self.world > 1
        self.filtered = 0          # packets dropped at their arrival rank by the replica
        self.last_exchange = None
        self.formats = set()       # record sizes received (16 / 32)
        self.blk_cap = 1024        # blocklist entries per rank of one all-gather (grows)
        self.rep_size = 0          # entries of the last replica (bounds the dropped sources)
        self.partials_sent = 0     # flow partials sent for replica-dropped packets

    def verdict_batch(self, hdr, length, ts, n: int, verdict, chunks: int = 1, bounds=None):
        """Verdicts for this rank's slice (arrival order) of one global batch; every rank
        calls it once per batch with its own slice, cut into `chunks` equal sub-batch
        pieces (or at the explicit local cut points `bounds`, chunks + 1 of them).

        Sub-batches run as a two-stage software pipeline: the pack and record exchange of
        sub-batch j + 1 (collectives on the engine's comm stream) overlap the owner
        pipeline of sub-batch j; buffers alternate between two slots."""
        with self.engine.stream_ctx():
            flows = getattr(self.engine, "flows", None) is not None
            if self.world == 1:
                self.engine.direct(hdr, length, ts, n, verdict)
                if flows:   # one call: its rows are the batch's rows
                    f = self.engine.flows
                    f["rows"].fill_(-1)   # (count: ctx.last_batch_info()["sources"])
                return
            # with flow features the replica-dropped packets reach their owner as flow
            # partials (step 7 of the module doc)
            filt_on = self.filter
            if flows:
                self.engine.flows_begin()
            if filt_on:
                self._sync_blocklist()   # maps may have changed since the last batch
            if bounds is None:
                bounds = [n * i // chunks for i in range(chunks + 1)]
            k = len(bounds) - 1
            if not filt_on:
                # no replica filter: every pack is independent of the owners, so all of them
                # go first and one exchange of all their counts is the batch's only host
                # synchronization; the record exchanges then overlap the owner work
                pend = self._exchange_all(hdr, length, ts, verdict, bounds)
                sent = recv = 0
                for j in range(k):
                    ms, mr = self._stage_owner(verdict, bounds, j, pend[j], slot=j)
                    pend[j] = None
                    sent, recv = sent + ms, recv + mr
                if flows:
                    self.engine.flows_end()
                self.last_exchange = {"sent": sent, "received": recv, "filtered": self.filtered}
                return
            filt = self._filter_plan(ts, bounds)
            pend = [None] * k
            pend[0] = self._stage_exchange(hdr, length, ts, verdict, bounds, 0, filt[0], flows)
            sent = recv = 0
            for j in range(k):
                if j + 1 < k:   # enqueued before the owner work of j: its exchange overlaps it
                    pend[j + 1] = self._stage_exchange(hdr, length, ts, verdict, bounds, j + 1,
                                                       filt[j + 1], flows)
                ms, mr = self._stage_owner(verdict, bounds, j, pend[j])
                pend[j] = None
                sent, recv = sent + ms, recv + mr
                # the replica packs j + 2 onward filter with (one sub-batch stale: exact for
                # clocks that do not go back between consecutive sub-batches, _filter_plan)
                if filt_on and j + 2 < k:
                    self._sync_blocklist()
            if flows:
                self.engine.flows_end()
            self.last_exchange = {"sent": sent, "received": recv, "filtered": self.filtered}

    def _filter_plan(self, ts, bounds) -> list:
        """Per sub-batch: may its pack drop replica-blacklisted packets? Pack j filters
        with the replica refreshed at the batch start (j = 0, 1) or after the owners of
        sub-batch j - 2 (j >= 2), so it can miss what the owners did in sub-batch j - 1.
        A stale entry only drops packets the owner drops too unless some earlier packet
        deleted it at a later time, so the filter is exact when the clock is
        non-decreasing in global order (rank 0's piece, then rank 1's, ...) inside the
        sub-batch and no packet of an earlier sub-batch of the batch is later than its
        first. One all-gather of {min, max, decreases} of every piece."""
        k = len(bounds) - 1
        c = _all_gather(self.engine.clocks(ts, bounds), self.world, self.group).tolist()
        within, lo, hi = [], [], []
        for j in range(k):
            ok, last, mn_j, mx_j = True, None, None, None
            for r in range(self.world):
                mn, mx, dec = c[3 * (r * k + j): 3 * (r * k + j) + 3]
                if dec:
                    ok = False
                if mx == 0 and mn == -1:      # empty piece ({~0, 0} as int64)
                    continue
                mn, mx = mn & (2**64 - 1), mx & (2**64 - 1)
                if last is not None and mn < last:
                    ok = False
                last = mx
                mn_j = mn if mn_j is None else min(mn_j, mn)
                mx_j = mx if mx_j is None else max(mx_j, mx)
            within.append(ok)
            lo.append(mn_j)
            hi.append(mx_j)
        out = []
        for j in range(k):
            ok = within[j]
            if ok and j >= 1:
                prev = max((h for h in hi[:j] if h is not None), default=None)
                if prev is not None and lo[j] is not None and lo[j] < prev:
                    ok = False
            out.append(ok)
        return out

    def _exchange_all(self, hdr, length, ts, verdict, bounds):
        """Pack every sub-batch j into slot j (engine stream), one all-to-all of all their
        per-owner counts and ONE host read of them (comm stream), then the record exchange
        of every sub-batch; per sub-batch what _stage_exchange returns."""
        G, e = self.world, self.engine
        k = len(bounds) - 1
        packs = [e.pack(hdr[bounds[j] * 64:], length[bounds[j]:], ts[bounds[j]:], bounds[j + 1] - bounds[j],
                        G, verdict[bounds[j]:], False, j) for j in range(k)]
        pend = []
        with e.comm_ctx():
            cnt = torch.stack([c for _, c in packs])                       # [k, G + 2]
            fmt = (cnt[:, G + 1:G + 2] == lib.SHARD_RECORD16_BYTES).to(cnt.dtype)
            send = (cnt[:, :G] * 2 + fmt).t().contiguous()                  # [G, k] by destination
            recv_counts = torch.empty_like(send)                            # [G, k] by source
            _a2a(recv_counts.view(-1), send.view(-1), [k] * G, [k] * G, self.group)
            both = torch.cat([cnt.reshape(-1), recv_counts.view(-1).to(cnt.device)]).tolist()
            base = k * (G + 2)
            for j in range(k):
                cj = both[j * (G + 2):(j + 1) * (G + 2)]
                rw = [int(both[base + r * k + j]) for r in range(G)]
                self.filtered += int(cj[G])
                rb = int(cj[G + 1])
                sc = [int(x) for x in cj[:G]]
                rc = [x >> 1 for x in rw]
                rf = [lib.SHARD_RECORD16_BYTES if x & 1 else lib.SHARD_RECORD_BYTES for x in rw]
                in_b = [x * rb for x in sc]
                out_b = [c * f for c, f in zip(rc, rf)]
                recv = e.recv_buffer(sum(out_b))
                _a2a(recv[:sum(out_b)], packs[j][0][:sum(in_b)], out_b, in_b, self.group)
                arrived = e.comm_event()
                segs, off = [], 0
                for c, f, nb in zip(rc, rf, out_b):
                    segs.append((off, c, f))
                    off += nb
                    if c:
                        self.formats.add(f)
                pend.append((recv, segs, sc, rc, arrived, None))
        return pend

    def _stage_exchange(self, hdr, length, ts, verdict, bounds, j: int, filt: bool, flows: bool = False):
        """Pack sub-batch j (engine stream) and exchange its counts and records (comm stream);
        with flows and the filter, also the flow partials of the replica-dropped packets."""
        G, e = self.world, self.engine
        a, b = bounds[j], bounds[j + 1]
        slot = j % 2
        drop = flows and filt   # (the same on every rank: the filter plan is global)
        recs, counts = e.pack(hdr[a * 64:], length[a:], ts[a:], b - a, G, verdict[a:], filt, slot, drop)
        with e.comm_ctx():
            # per-owner counts with the record format in the low bit; the host reads its
            # own and the received counts together (one synchronization, comm stream)
            send = (counts[:G] * 2 + (counts[G + 1] == lib.SHARD_RECORD16_BYTES).to(counts.dtype)).contiguous()
            recv_counts = torch.empty_like(send)
            ones = [1] * G
            _a2a(recv_counts, send, ones, ones, self.group)
            both = torch.cat([counts.to(recv_counts.device), recv_counts]).tolist()
            cnt, rw = both[:G + 2], [int(x) for x in both[G + 2:]]
            self.filtered += int(cnt[G])
            rb = int(cnt[G + 1])   # this sender's record size (16: compact IPv4 records)
            sc = [int(x) for x in cnt[:G]]
            rc = [x >> 1 for x in rw]
            rf = [lib.SHARD_RECORD16_BYTES if x & 1 else lib.SHARD_RECORD_BYTES for x in rw]
            in_b = [x * rb for x in sc]
            out_b = [c * f for c, f in zip(rc, rf)]
        partial = self._exchange_partials(recs, sum(sc), int(cnt[G]), rb, slot) if drop else None
        with e.comm_ctx():
            recv = e.recv_buffer(sum(out_b))
            _a2a(recv[:sum(out_b)], recs[:sum(in_b)], out_b, in_b, self.group)
        arrived = e.comm_event()      # only these records: the owner work of the previous
        segs, off = [], 0             # sub-batch must not wait for later exchanges
        for c, f, nb in zip(rc, rf, out_b):
            segs.append((off, c, f))
            off += nb
            if c:
                self.formats.add(f)
        return recv, segs, sc, rc, arrived, partial

    def _exchange_partials(self, recs, first: int, m: int, rb: int, slot: int):
        """The flow partials of this rank's m replica-dropped records (engine stream), their
        per-owner counts (all-to-all + one host read) and the partials (all-to-all), on the
        comm stream -> (received partials, per sender)."""
        G, e = self.world, self.engine
        B = lib.FLOW_PARTIAL_BYTES
        cap = max(1, self.rep_size)   # every dropped source is a replica entry
        buf, pcnt = e.partials(recs, first, m, rb, G, cap, slot)
        with e.comm_ctx():
            prc = torch.empty_like(pcnt)
            _a2a(prc, pcnt, [1] * G, [1] * G, self.group)
            both = torch.cat([pcnt, prc]).tolist()
            ps, pr = [int(x) for x in both[:G]], [int(x) for x in both[G:]]
            if max(ps) > cap:
                raise RuntimeError(f"flow partials overflow: {max(ps)} sources for {cap} replica entries")
            send = torch.cat([buf[o * cap * B:(o * cap + ps[o]) * B] for o in range(G)])
            precv = e.recv_buffer(sum(pr) * B)
            _a2a(precv[:sum(pr) * B], send, [x * B for x in pr], [x * B for x in ps], self.group)
        self.partials_sent += sum(ps)
        return precv, pr

    def _stage_owner(self, verdict, bounds, j: int, pend, slot=None):
        """Owner pipeline of sub-batch j (engine stream), verdicts back (comm stream) and
        into arrival positions (engine stream)."""
        G, e = self.world, self.engine
        recv, segs, sc, rc, arrived, partial = pend
        a = bounds[j]
        slot = j % 2 if slot is None else slot
        ms, mr = sum(sc), sum(rc)
        e.engine_wait(arrived)        # the records (and partials) of sub-batch j have arrived
        e.keep(recv)                  # allocated on the comm stream, read on the engine's
        if partial is not None:       # the replica-dropped packets' sums first, senders in order
            precv, pr = partial
            e.keep(precv)
            off = 0
            for r in range(G):
                e.merge(precv[off * lib.FLOW_PARTIAL_BYTES:], pr[r])
                off += pr[r]
        v = e.owner_batch(recv, segs, slot)
        with e.comm_ctx():
            ret = torch.empty(max(ms, 1), dtype=torch.uint8, device=v.device)
            _a2a(ret[:ms], v[:mr], sc, rc, self.group)
        e.engine_wait(e.comm_event())
        e.keep(ret)
        e.scatter(ret, ms, verdict[a:], slot)
        return ms, mr

    def _sync_blocklist(self):
        """All-gather every owner's live blacklist entries into every rank's replica: one
        all-gather of fixed-capacity buffers (entry count in the header), repeated with a
        larger capacity only when some rank overflowed it."""
        G, e = self.world, self.engine
        B = lib.SHARD_BLOCK_BYTES
        while True:
            cap = self.blk_cap
            allb = _all_gather(e.blocklist_buffer(cap), G, self.group)
            per = B + cap * B
            sizes = allb.view(-1)[:G * per].view(G, per)[:, :8].contiguous().view(torch.int64).view(-1).tolist()
            if max(sizes) <= cap:
                break
            self.blk_cap = 2 * max(sizes)
        self.rep_size = sum(sizes)
        parts = [allb[r * per + B: r * per + B + sizes[r] * B] for r in range(G) if sizes[r]]
        if parts:
            e.load_replica(torch.cat(parts), sum(sizes))
        else:
            e.load_replica(allb, 0)

    def stats(self) -> tuple[int, int]:
        """stats_map of the whole sharded data plane: sum over the owners, plus the
        packets the replicas dropped at their arrival ranks."""
        with self.engine.stream_ctx():
            s = self.engine.stats()
            s[1] += self.filtered
            if self.world > 1:
                _all_reduce_sum(s, self.group)
            return int(s[0]), int(s[1])

    def reset(self):
        """Forget the replica-drop count (the owners' maps are reset by the caller)."""
        self.filtered = 0
