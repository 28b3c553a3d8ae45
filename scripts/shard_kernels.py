"""Single-GPU timing of the sharded path's local kernels on a config-2 batch: pack (parse
+ owner partition into exchange records) for G owners, and the owner-side unpack of the
records a rank would receive. The collectives themselves need a multi-GPU node.
"""
import json
import sys
import time

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from flowsentryx_amd import lib, synth  # noqa: E402
from flowsentryx_amd.shard import HipShardEngine  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    p, s = synth.config_params(2)
    n = int(p.n)
    dev = torch.device("cuda", 0)
    hdr = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    synth.generate_device(p, s, 0, n, hdr.data_ptr(), ln.data_ptr(), ts.data_ptr())
    torch.cuda.synchronize()
    out = {"G": G, "n": n}
    with lib.FsxContext(max_batch=n, max_entries=int(p.n_ips), device=0) as ctx:
        e = HipShardEngine(ctx, n, dev)
        with e.stream_ctx():
            # (pack_contiguous_ms: the owners' runs back to back — parse, then k_shard_pack16
            # from the arrival-order copy; pack_ms: FSX_SHARD_REGIONS, HipShardEngine's, one pass)
            for regions in (False, True):
                e.regions = regions
                for _ in range(2):
                    rec, counts = e.pack(hdr, ln, ts, n, G, v)
                ctx.sync()
                t0 = time.perf_counter()
                for _ in range(5):
                    rec, counts = e.pack(hdr, ln, ts, n, G, v)
                ctx.sync()
                out["pack_ms" if regions else "pack_contiguous_ms"] = (time.perf_counter() - t0) / 5 * 1e3
            e.regions = False   # (the unpack below reads the first m records)
            rec, counts = e.pack(hdr, ln, ts, n, G, v)
            ctx.sync()
            c = counts.tolist()
            rb = int(c[G + 1])
            m = int(sum(c[:G]))
            out["record_bytes"] = rb
            hb, lb, tb, _ = e._owner_buffers(m)
            segs = [(0, m, rb)]
            ctx.shard_unpack_device(rec.data_ptr(), m, hb.data_ptr(), lb.data_ptr(), tb.data_ptr(), rb)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(5):
                ctx.shard_unpack_device(rec.data_ptr(), m, hb.data_ptr(), lb.data_ptr(), tb.data_ptr(), rb)
            ctx.sync()
            out["unpack_ms"] = (time.perf_counter() - t0) / 5 * 1e3
            out["records"] = m
            out["exchange_bytes_per_rank"] = m * rb * (G - 1) // G
            # owner pipeline on all records in arrival order (a G = 1 pack: monotone clock,
            # as every owner's received stream is)
            rec, counts = e.pack(hdr, ln, ts, n, 1, v)
            m = int(counts[0].item())
            ov = torch.empty(m, dtype=torch.uint8, device=dev)
            for mode in ("records", "headers"):
                for it in range(4):
                    if it == 1:
                        ctx.sync()
                        t0 = time.perf_counter()
                    ctx.reset()
                    if mode == "records":
                        ctx.verdict_records_device(rec.data_ptr(), m, rb, ov.data_ptr())
                    else:
                        ctx.shard_unpack_device(rec.data_ptr(), m, hb.data_ptr(), lb.data_ptr(),
                                                tb.data_ptr(), rb)
                        ctx.verdict_batch_device(hb.data_ptr(), lb.data_ptr(), tb.data_ptr(), m,
                                                 ov.data_ptr())
                ctx.sync()
                out[f"owner_{mode}_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    # the owner as the sharded stream runs it: maps carried (no reset), every call the next
    # batch of the stream (the records' timestamps shifted by one duration), calls enqueued
    # back to back (pipeline mode 2, HipShardEngine's), verdicts only and with features +
    # q8 scores (per-source rows)
    from flowsentryx_amd import fsx_load   # noqa: E402
    from pathlib import Path
    model = fsx_load.load_weights(Path(__file__).resolve().parents[1] / "tests" / "golden" / "model_weights.json")
    dur = int(p.duration_ns)
    assert rb == 16
    rec = rec[:m * rb].clone()   # (the engine's pack buffer belongs to the closed context)
    tsw = rec.view(torch.int64)[1::2]   # ShardRecord16.ts (bytes 8..15)
    for flows in (False, True):
        with lib.FsxContext(max_batch=n, max_entries=int(p.n_ips), device=0) as ctx:
            ctx.load_q8_model(model)
            ctx.set_pipeline(2)
            ov = torch.empty(m, dtype=torch.uint8, device=dev)
            cap = int(p.n_ips)
            fo = [torch.empty(cap * 16, dtype=torch.uint8, device=dev), torch.empty(cap, dtype=torch.uint8, device=dev),
                  torch.empty(cap * 8, dtype=torch.float32, device=dev), torch.empty(cap, dtype=torch.float32, device=dev),
                  torch.empty(cap, dtype=torch.uint8, device=dev)]
            K = 6
            per = []
            for it in range(K + 2):
                tsw.add_(dur)
                torch.cuda.synchronize()   # (the shift on torch's stream, before the call)
                t0 = time.perf_counter()
                if flows:
                    ctx.process_records_device(rec.data_ptr(), m, rb, ov.data_ptr(), *[x.data_ptr() for x in fo], cap)
                else:
                    ctx.verdict_records_device(rec.data_ptr(), m, rb, ov.data_ptr())
                ctx.sync()
                per.append((time.perf_counter() - t0) * 1e3)
            el = sorted(per[2:])[len(per[2:]) // 2]   # median of the warm calls
            out["owner_records_warm_flows_ms" if flows else "owner_records_warm_ms"] = el
            out["owner_heavy_unsorted"] = ctx.last_batch_info().get("heavy_unsorted")
    # the owner as HipShardEngine runs it (pipeline mode 1: each record batch's tail beside the
    # next call's front): W + K calls back to back, each on its own copy of the records
    # shifted by one more stream duration, timed over the K calls after the W
    W, K = 3, 8
    base = rec.clone()
    bufs = []
    for i in range(W + K):
        b = base.clone()
        b.view(torch.int64)[1::2].add_((i + 1) * dur)
        bufs.append(b)
    torch.cuda.synchronize()
    for flows in (False, True):
        with lib.FsxContext(max_batch=n, max_entries=int(p.n_ips), device=0) as ctx:
            ctx.load_q8_model(model)
            ctx.set_pipeline(1)
            # (a batch's verdict buffer holds its heavy tags until its tail is done: one each)
            ovs = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in bufs]
            cap = int(p.n_ips)
            fo = [torch.empty(cap * 16, dtype=torch.uint8, device=dev), torch.empty(cap, dtype=torch.uint8, device=dev),
                  torch.empty(cap * 8, dtype=torch.float32, device=dev), torch.empty(cap, dtype=torch.float32, device=dev),
                  torch.empty(cap, dtype=torch.uint8, device=dev)]
            for i, (b, ov) in enumerate(zip(bufs, ovs)):
                if i == W:
                    ctx.sync()
                    t0 = time.perf_counter()
                if flows:
                    ctx.process_records_device(b.data_ptr(), m, rb, ov.data_ptr(), *[x.data_ptr() for x in fo], cap)
                else:
                    ctx.verdict_records_device(b.data_ptr(), m, rb, ov.data_ptr())
            ctx.sync()
            el = (time.perf_counter() - t0) / K * 1e3
            out["owner_records_split_flows_ms" if flows else "owner_records_split_ms"] = el
    del bufs
    out["note"] = ("owner_records_warm*: maps carried, one 64M-record batch per call (records shifted by one "
                   "stream duration per call), median host time of a call through its sync; "
                   "owner_records_split*: the same stream, pipeline mode 1 (HipShardEngine's), "
                   f"{K} calls back to back after {W}, per call")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
