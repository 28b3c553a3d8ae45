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
  5. all-gather of every owner's live blacklist entries (the replicated blocklist, once per
     global batch, fixed-capacity blocks whose counts stay on the device); the packs drop
     packets of replica-blacklisted sources locally (now <= till: the owner would drop them
     without touching any state, src/fsx_kern.c:189-215) — for the sub-batches whose
     global clock does not go back up to their end (one all-gather of {min, max,
     decreases} per piece, the decision made on the device), which is exactly the
     condition under which no earlier packet can have deleted the entry
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
     sub-batch, and in rank order. The partials travel in fixed-capacity blocks (the
     replica's per-owner capacity bounds the sources an owner can have dropped) whose
     counts stay on the device

Host synchronization: ONE host read per global batch — every sub-batch is packed first,
then one all-to-all carries all their per-owner record counts (plus the replica-drop
counts and the replica blocks' sizes) and the host reads them together;
torch.distributed.all_to_all_single needs its split sizes on the host. Everything else (the
replica, the filter decision, the flow partials and their merge) stays on the device.

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


_A2A_LISTS = True   # the backend takes list all-to-alls (cleared at the first refusal)


def _a2a_views(out: torch.Tensor, out_splits, ins, group=None):
    """all-to-all of one view per destination (not one contiguous tensor: a regions pack,
    HipShardEngine.send_views) into `out` split by out_splits. RCCL takes the views as they
    are (grouped send / receive); gloo gets them concatenated."""
    global _A2A_LISTS
    if dist.get_backend(group) != "gloo" and _A2A_LISTS:
        try:
            dist.all_to_all(list(out.split(list(out_splits))), list(ins), group=group)
            return
        except (RuntimeError, ValueError):   # (a backend without list all-to-all: one copy)
            _A2A_LISTS = False
    inp = torch.cat(ins) if ins else out[:0]
    _a2a(out, inp, out_splits, [int(x.numel()) for x in ins], group)


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
        # at the next synchronization), split: a record batch's tail (walkers, verdicts, flows)
        # runs on the context's side streams beside the next sub-batch's front, and its
        # verdicts go back after that next call (ShardedDataPlane, fsx_stream_wait_batches)
        ctx.set_pipeline(1)
        # collectives run from a second stream, so the exchange of sub-batch j + 1 overlaps
        # the owner pipeline of sub-batch j (ShardedDataPlane)
        self.comm = torch.cuda.Stream(device)
        self.max_local = max_local
        self.owner_cap = int(ctx.config.max_batch)
        # per-sub-batch buffers by pipeline slot (allocated on first use, sized for the piece)
        self.recs, self.send_idxs, self.countss = {}, {}, {}
        # FSX_SHARD_REGIONS packs (one pass over the headers: owner o's records at o * n); the
        # pieces' n and G per slot for the views and the scatter
        self.regions = True
        self.pack_ng = {}
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

    def return_ctx(self, all_batches: bool):
        """Collectives on the comm stream after the owner batches enqueued so far: the engine
        stream's work and their split tails (all_batches=False: except the last batch's, still
        deferred beside the next call)."""
        self.comm.wait_stream(self.stream)
        self.ctx.stream_wait_batches(self.comm.cuda_stream, all_batches)
        return torch.cuda.stream(self.comm)

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
        # (the engine stream and every split tail, the last one enqueued first)
        self.ctx.stream_wait_batches(cur.cuda_stream, True)

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

    def pack(self, hdr, length, ts, n, G, verdict, filt=None, slot=0, drop_rec=False):
        """-> records, counts[G + 2] (counts[G]: packets dropped by the replica,
        counts[G + 1]: record bytes, 16 or 32), in pipeline slot `slot`. filt: a device word
        (filter_plan), the replica filter applies iff it is nonzero; drop_rec: the dropped
        packets' records follow the owners' runs."""
        if n > self.max_local:
            raise ValueError(f"local slice of {n} packets exceeds {self.max_local}")
        flags = lib.SHARD_COMPACT
        if filt is not None and drop_rec:
            flags |= lib.SHARD_DROP_RECORDS
        if self.regions:
            flags |= lib.SHARD_REGIONS
        m = max(1, n) * ((G + 1) if self.regions else 1)
        if slot not in self.recs or self.send_idxs[slot].numel() < m:
            self.recs[slot] = torch.empty(m * REC, dtype=torch.uint8, device=self.device)
            self.send_idxs[slot] = torch.empty(m, dtype=torch.int32, device=self.device)
            self.countss[slot] = torch.empty(lib.MAX_SHARDS + 2, dtype=torch.int64, device=self.device)
        self.pack_ng[slot] = (n, G)
        rec, idx, cnt = self.recs[slot], self.send_idxs[slot], self.countss[slot]
        self.rec, self.send_idx, self.counts = rec, idx, cnt   # (tests read the last pack)
        if filt is None:
            self.ctx.shard_pack_device(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, G,
                                       verdict.data_ptr(), rec.data_ptr(), idx.data_ptr(), cnt.data_ptr(),
                                       flags)
        else:
            self.ctx.shard_pack_filtered_device(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, G,
                                                filt.data_ptr(), verdict.data_ptr(), rec.data_ptr(),
                                                idx.data_ptr(), cnt.data_ptr(), flags)
        return rec, cnt[:G + 2]

    def send_views(self, rec: torch.Tensor, sc, rb: int, slot: int):
        """The records for each owner (sc[o] of rb bytes): views into its region."""
        if not self.regions:
            return list(rec[:sum(sc) * rb].split([c * rb for c in sc]))
        n = self.pack_ng[slot][0]
        return [rec[o * n * rb:(o * n + c) * rb] for o, c in enumerate(sc)]

    def drop_first(self, slot: int, sent: int) -> int:
        """Record index of the first replica-dropped record (FSX_SHARD_DROP_RECORDS)."""
        n, G = self.pack_ng[slot]
        return G * n if self.regions else sent

    def filter_plan(self, clocks: torch.Tensor, G: int, k: int) -> torch.Tensor:
        """The replica filter's decision per sub-batch from the all-gathered piece clocks
        ([G][k][3]), on the device: int32 [k]."""
        out = torch.empty(k, dtype=torch.int32, device=self.device)
        self.ctx.shard_filter_plan_device(clocks.data_ptr(), G, k, out.data_ptr())
        return out

    def load_replica_blocks(self, blocks: torch.Tensor, G: int, cap: int):
        """The replica from G all-gathered blocklist_buffer(cap) blocks (counts on the device)."""
        self.ctx.blocklist_replica_blocks_device(blocks.data_ptr(), G, cap)

    def partials(self, rec, first, m, rb, G, cap, slot=0):
        """Flow partials of the m replica-dropped records from record index `first` of a pack
        buffer: G runs of cap partials (source -> run of its owner) and counts[G]; enqueued
        on the engine stream (no host synchronization). m = 0: zero counts."""
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
        if m == 0:
            cnt.zero_()
        else:
            self.pctx.flow_partials_records_device(rec.data_ptr() + first * rb, m, rb, G, buf.data_ptr(), cap,
                                                   cnt.data_ptr())
        return buf[:G * cap * B], cnt

    def merge(self, parts: torch.Tensor, m: int):
        """Merge m received partials (one sender's, distinct sources) into the owner's sums."""
        if m:
            self.ctx.flows_merge_device(parts.data_ptr(), m)

    def merge_counted(self, parts: torch.Tensor, cap: int, count: torch.Tensor):
        """Merge one sender's fixed-capacity block: min(count[0], cap) partials (device count)."""
        self.ctx.flows_merge_counted_device(parts.data_ptr(), cap, count.data_ptr())

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
        """ret: the m returned verdicts, owner by owner, into their arrival positions."""
        if not m:
            return
        if self.regions:
            n, G = self.pack_ng[slot]
            self.ctx.shard_scatter_regions_device(ret.data_ptr(), self.send_idxs[slot].data_ptr(), m, n,
                                                  self.countss[slot].data_ptr(), G, verdict.data_ptr())
        else:
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
        self.partials_sent = 0     # flow partials sent for replica-dropped packets
        self.host_reads = 0        # host synchronizations of the data plane (one per global batch)
        self._sc, self._rc = {}, {}  # per sub-batch: records sent to / received from each rank

    def verdict_batch(self, hdr, length, ts, n: int, verdict, chunks: int = 1, bounds=None):
        """Verdicts for this rank's slice (arrival order) of one global batch; every rank
        calls it once per batch with its own slice, cut into `chunks` equal sub-batch
        pieces (or at the explicit local cut points `bounds`, chunks + 1 of them).

        Every sub-batch is packed first (the replica refreshed at the batch start, the
        filter decided on the device), one all-to-all of all their counts is the batch's
        only host read, then the record exchanges (comm stream) overlap the owner pipelines
        of the sub-batches before them."""
        with self.engine.stream_ctx():
            flows = getattr(self.engine, "flows", None) is not None
            if self.world == 1:
                self.engine.direct(hdr, length, ts, n, verdict)
                if flows:   # one call: its rows are the batch's rows
                    f = self.engine.flows
                    f["rows"].fill_(-1)   # (count: ctx.last_batch_info()["sources"])
                return
            if flows:
                self.engine.flows_begin()
            if bounds is None:
                bounds = [n * i // chunks for i in range(chunks + 1)]
            k = len(bounds) - 1
            filt = blk = None
            if self.filter:
                blk = self._refresh_replica()   # maps may have changed since the last batch
                filt = self._filter_plan(ts, bounds)
            pend = self._exchange_all(hdr, length, ts, verdict, bounds, filt, blk, flows)
            sent = recv = 0
            # owner j's verdicts go back after owner j + 1 is enqueued (its split tail runs
            # beside that call's front), the last after its tail is enqueued; the scatters into
            # arrival positions after all of them (every other library call joins the tail)
            back, live = [], []
            for j in range(k):
                calls = getattr(self.engine, "owner_calls", 0)
                ms, mr, v = self._stage_owner(verdict, bounds, j, pend[j], slot=j)
                live.append(pend[j][0])   # (the records: read by the tail on the side streams)
                pend[j] = None
                if back:
                    # (no owner call for sub-batch j: the tail of j - 1 is still deferred)
                    back[-1] = self._return(*back[-1], all_batches=getattr(self.engine, "owner_calls", 0) == calls)
                back.append((j, ms, mr, v))
                sent, recv = sent + ms, recv + mr
            if back:
                back[-1] = self._return(*back[-1], all_batches=True)
            self.engine.engine_wait(self.engine.comm_event())
            for j, ms, ret in back:
                self.engine.keep(ret)
                self.engine.scatter(ret, ms, verdict[bounds[j]:], j)
            del live
            if flows:
                self.engine.flows_end()
            self.last_exchange = {"sent": sent, "received": recv, "filtered": self.filtered}

    def _refresh_replica(self):
        """All-gather every owner's live blacklist entries into every rank's replica: one
        all-gather of fixed-capacity blocks whose entry counts stay on the device (an owner
        with more than blk_cap entries contributes blk_cap of them: its other sources' packets
        go to it and are decided there). -> (the blocks' counts [G] on the device, cap)."""
        G, e = self.world, self.engine
        B = lib.SHARD_BLOCK_BYTES
        cap = self.blk_cap
        allb = _all_gather(e.blocklist_buffer(cap), G, self.group)
        e.load_replica_blocks(allb, G, cap)
        per = B + cap * B
        sizes = allb.view(-1)[:G * per].view(G, per)[:, :8].contiguous().view(torch.int64).view(-1)
        return sizes, cap

    def _filter_plan(self, ts, bounds) -> torch.Tensor:
        """Per sub-batch: may its pack drop replica-blacklisted packets? The replica holds the
        owners' entries as of the batch start. A stale entry only drops packets the owner
        drops too unless some earlier packet deleted it at a later time, so the filter is
        exact when the clock is non-decreasing in global order (rank 0's piece, then rank
        1's, ...) inside the sub-batch and no packet of an earlier sub-batch of the batch is
        later than its first. One all-gather of {min, max, decreases} of every piece; the
        decision on the device (fsx_shard_filter_plan_device) -> int32 [k]."""
        k = len(bounds) - 1
        c = _all_gather(self.engine.clocks(ts, bounds), self.world, self.group)
        return self.engine.filter_plan(c, self.world, k)

    def _exchange_all(self, hdr, length, ts, verdict, bounds, filt=None, blk=None, flows=False):
        """Pack every sub-batch j into slot j (engine stream), one all-to-all of all their
        per-owner counts and ONE host read of them (comm stream), then the record exchange
        of every sub-batch and, with flows and the filter, the flow partials of its
        replica-dropped packets (fixed-capacity blocks); per sub-batch (received records,
        segments, sent / received counts, arrival event, partials)."""
        G, e = self.world, self.engine
        k = len(bounds) - 1
        drop = flows and filt is not None
        packs = [e.pack(hdr[bounds[j] * 64:], length[bounds[j]:], ts[bounds[j]:], bounds[j + 1] - bounds[j],
                        G, verdict[bounds[j]:], None if filt is None else filt[j:j + 1], j, drop)
                 for j in range(k)]
        pend = []
        with e.comm_ctx():
            cnt = torch.stack([c for _, c in packs])                       # [k, G + 2]
            fmt = (cnt[:, G + 1:G + 2] == lib.SHARD_RECORD16_BYTES).to(cnt.dtype)
            send = (cnt[:, :G] * 2 + fmt).t().contiguous()                  # [G, k] by destination
            recv_counts = torch.empty_like(send)                            # [G, k] by source
            _a2a(recv_counts.view(-1), send.view(-1), [k] * G, [k] * G, self.group)
            parts = [cnt.reshape(-1), recv_counts.view(-1).to(cnt.device)]
            if blk is not None:
                parts.append(blk[0].to(cnt.device))
            both = torch.cat(parts).tolist()   # the batch's one host read
        self.host_reads += 1
        base = k * (G + 2)
        if blk is not None:   # an owner overflowed the replica's capacity: larger next batch
            big = max(both[base + G * k: base + G * k + G])
            if big > blk[1]:
                self.blk_cap = max(self.blk_cap, 2 * int(big))
        for j in range(k):
            cj = both[j * (G + 2):(j + 1) * (G + 2)]
            rw = [int(both[base + r * k + j]) for r in range(G)]
            self.filtered += int(cj[G])
            rb = int(cj[G + 1])
            if rb not in (lib.SHARD_RECORD16_BYTES, lib.SHARD_RECORD_BYTES):   # (FSX_SHARD_PACK_ERR)
                raise RuntimeError(f"sharded pack of sub-batch {j} failed on the device (record size {rb})")
            sc = [int(x) for x in cj[:G]]
            rc = [x >> 1 for x in rw]
            rf = [lib.SHARD_RECORD16_BYTES if x & 1 else lib.SHARD_RECORD_BYTES for x in rw]
            in_b = [x * rb for x in sc]
            out_b = [c * f for c, f in zip(rc, rf)]
            with e.comm_ctx():
                recv = e.recv_buffer(sum(out_b))
                _a2a_views(recv[:sum(out_b)], out_b, e.send_views(packs[j][0], sc, rb, j), self.group)
            # with flows and the filter: the flow partials of the replica-dropped packets
            partial = (self._exchange_partials(packs[j][0], e.drop_first(j, sum(sc)), int(cj[G]), rb, blk[1], j)
                       if drop else None)
            segs, off = [], 0
            for c, f, nb in zip(rc, rf, out_b):
                segs.append((off, c, f))
                off += nb
                if c:
                    self.formats.add(f)
            # (only this sub-batch's exchanges: the owner work of the one before must not
            # wait for later ones)
            pend.append((recv, segs, sc, rc, e.comm_event(), partial))
        return pend

    def _exchange_partials(self, recs, first: int, m: int, rb: int, cap: int, slot: int):
        """The flow partials of this rank's m replica-dropped records (engine stream) in G
        runs of cap (a source's owner contributed it to the replica, which holds at most cap
        entries per owner), exchanged as fixed-capacity blocks with their counts (comm
        stream; no host read) -> (received partials [G x cap], received counts [G])."""
        G, e = self.world, self.engine
        B = lib.FLOW_PARTIAL_BYTES
        buf, pcnt = e.partials(recs, first, m, rb, G, cap, slot)
        with e.comm_ctx():
            prc = torch.empty_like(pcnt)
            _a2a(prc, pcnt, [1] * G, [1] * G, self.group)
            precv = e.recv_buffer(G * cap * B)
            _a2a(precv[:G * cap * B], buf, [cap * B] * G, [cap * B] * G, self.group)
        self.partials_sent += m
        return precv, prc, cap

    def _return(self, j: int, ms: int, mr: int, v, all_batches: bool):
        """Sub-batch j's verdicts back to their arrival ranks (comm stream, after its owner
        batches' tails) -> (j, ms, received verdicts)."""
        with self.engine.return_ctx(all_batches):
            ret = torch.empty(max(ms, 1), dtype=torch.uint8, device=v.device)
            _a2a(ret[:ms], v[:mr], self._sc[j], self._rc[j], self.group)
        return j, ms, ret

    def _stage_owner(self, verdict, bounds, j: int, pend, slot=None):
        """Owner pipeline of sub-batch j (engine stream) -> (sent, received, its verdicts in
        received order); _return sends them back."""
        G, e = self.world, self.engine
        recv, segs, sc, rc, arrived, partial = pend
        slot = j % 2 if slot is None else slot
        ms, mr = sum(sc), sum(rc)
        e.engine_wait(arrived)        # the records (and partials) of sub-batch j have arrived
        e.keep(recv)                  # allocated on the comm stream, read on the engine's
        if partial is not None:       # the replica-dropped packets' sums first, senders in order
            precv, prc, cap = partial
            e.keep(precv)
            e.keep(prc)
            B = lib.FLOW_PARTIAL_BYTES
            for r in range(G):
                e.merge_counted(precv[r * cap * B:], cap, prc[r:r + 1])
        v = e.owner_batch(recv, segs, slot)
        self._sc[j], self._rc[j] = sc, rc
        return ms, mr, v

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
