"""Hash(src IP) sharding of the verdict path over G ranks (SURVEY.md §8 e).

The reference is one XDP program per host (src/fsx_kern.c:96-97) whose state is all
per source IP (src/fsx_kern.c:56-94) plus two summed counters. So the path shards with
no shared state: every rank holds a contiguous slice of each arrival batch, every
source has ONE owner rank (include/fsx_hip.h fsx_shard_owner), and the owner runs the
unchanged batch pipeline on all of that source's packets:

  1. pack      parse the local slice, partition its IP packets by owner into 32-byte
               records (stable: arrival order), verdicts for packets that never reach a
               limiter (short frames DROP, non-IP PASS)
  2. all-to-all of the per-owner counts, then of the records (RCCL over xGMI)
  3. owner     records -> header records, the batch pipeline on them (maps, verdicts,
               optionally flow features + MLP scores of the owned sources)
  4. all-to-all of the verdicts back (1 byte per packet), scatter to arrival positions
  5. stats_map = all-reduce(sum) of the owners' counters

Rank slices are concatenated in rank order on the owner, so every source's packets
arrive there in global arrival order and the sharded result equals the 1-GPU run
(tests/test_shard_*.py check this bit-exactly).

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
        self.max_local = max_local
        self.owner_cap = int(ctx.config.max_batch)
        self.rec = torch.empty(max(1, max_local) * REC, dtype=torch.uint8, device=device)
        self.send_idx = torch.empty(max(1, max_local), dtype=torch.int32, device=device)
        self.counts = torch.empty(lib.MAX_SHARDS, dtype=torch.int64, device=device)
        self._oh = None  # owner-side header/len/ts/verdict buffers, grown on demand
        self.flows = None

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
        """Per owned source: key, family, q8 probability and decision of every batch."""
        d = self.device
        self.flows = dict(keys=torch.empty(cap * 16, dtype=torch.uint8, device=d),
                          fam=torch.empty(cap, dtype=torch.uint8, device=d),
                          prob=torch.empty(cap, dtype=torch.float32, device=d),
                          dec=torch.empty(cap, dtype=torch.uint8, device=d), cap=cap)

    def direct(self, hdr, length, ts, n, verdict):
        """G == 1: the batch pipeline straight on the local slice."""
        self._run(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, verdict.data_ptr())

    def _run(self, h, l, t, n, v):
        if self.flows is None:
            self.ctx.verdict_batch_device(h, l, t, n, v)
        else:
            f = self.flows
            self.ctx.process_batch_device(h, l, t, n, v, f["keys"].data_ptr(), f["fam"].data_ptr(),
                                          None, f["prob"].data_ptr(), f["dec"].data_ptr(), f["cap"])

    def pack(self, hdr, length, ts, n, G, verdict):
        if n > self.max_local:
            raise ValueError(f"local slice of {n} packets exceeds {self.max_local}")
        self.ctx.shard_pack_device(hdr.data_ptr(), length.data_ptr(), ts.data_ptr(), n, G,
                                   verdict.data_ptr(), self.rec.data_ptr(),
                                   self.send_idx.data_ptr(), self.counts.data_ptr())
        return self.rec, self.counts[:G]

    def recv_buffer(self, m: int) -> torch.Tensor:
        return torch.empty(max(1, m) * REC, dtype=torch.uint8, device=self.device)

    def owner_batch(self, recv: torch.Tensor, m: int) -> torch.Tensor:
        """The limiter over the m received records, in received order (chunked by the
        context's max_batch: state carries across chunks exactly as across batches)."""
        hdr, ln, ts, v = self._owner_buffers(m)
        if m:
            self.ctx.shard_unpack_device(recv.data_ptr(), m, hdr.data_ptr(), ln.data_ptr(),
                                         ts.data_ptr())
        for a in range(0, m, self.owner_cap):
            b = min(m, a + self.owner_cap)
            self._run(hdr.data_ptr() + a * 64, ln.data_ptr() + a * 4, ts.data_ptr() + a * 8,
                      b - a, v.data_ptr() + a)
        return v[:max(m, 1)]

    def scatter(self, ret: torch.Tensor, m: int, verdict):
        if m:
            self.ctx.shard_scatter_device(ret.data_ptr(), self.send_idx.data_ptr(), m,
                                          verdict.data_ptr())

    def stats(self) -> torch.Tensor:
        a, d = self.ctx.stats()
        return torch.tensor([a, d], dtype=torch.int64, device=self.device)


class ShardedDataPlane:
    """The sharded verdict path of one rank (one process per GPU)."""

    def __init__(self, engine, group=None):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.last_exchange = None

    def verdict_batch(self, hdr, length, ts, n: int, verdict):
        """Verdicts for this rank's slice (arrival order) of one global batch; every rank
        calls it once per batch with its own slice."""
        with self.engine.stream_ctx():
            self._step(hdr, length, ts, n, verdict)

    def _step(self, hdr, length, ts, n: int, verdict):
        G, e = self.world, self.engine
        if G == 1:
            e.direct(hdr, length, ts, n, verdict)
            return
        recs, counts = e.pack(hdr, length, ts, n, G, verdict)
        recv_counts = torch.empty_like(counts)
        ones = [1] * G
        _a2a(recv_counts, counts, ones, ones, self.group)
        sc = [int(x) for x in counts.tolist()]
        rc = [int(x) for x in recv_counts.tolist()]
        ms, mr = sum(sc), sum(rc)
        recv = e.recv_buffer(mr)
        _a2a(recv[:mr * REC], recs[:ms * REC], [x * REC for x in rc], [x * REC for x in sc],
             self.group)
        v = e.owner_batch(recv, mr)
        ret = torch.empty(max(ms, 1), dtype=torch.uint8, device=v.device)
        _a2a(ret[:ms], v[:mr], sc, rc, self.group)
        e.scatter(ret, ms, verdict)
        self.last_exchange = {"sent": sc, "received": rc}

    def stats(self) -> tuple[int, int]:
        """stats_map of the whole sharded data plane: sum over the owners."""
        with self.engine.stream_ctx():
            s = self.engine.stats()
            if self.world > 1:
                _all_reduce_sum(s, self.group)
            return int(s[0]), int(s[1])
