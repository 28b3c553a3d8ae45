"""One rank of a multi-process sharded run (spawned by tests/test_shard_*.py).

Every rank builds the same seeded global stream, takes its contiguous slice of every
global batch, runs flowsentryx_amd.shard.ShardedDataPlane, and rank 0 compares the
gathered verdicts, stats_map and map dumps with ONE sequential oracle over the whole
stream (the 1-GPU semantics)."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def _stream(spec):
    from test_gpu_parity import rand_stream
    rng = np.random.default_rng(spec["seed"])
    hdr, ln, ts = rand_stream(rng, spec["n"], spec["n_ips"], dt_max=spec.get("dt_max", 300),
                              v6_frac=spec.get("v6_frac", 0.0),
                              nonip_frac=spec.get("nonip_frac", 0.0),
                              short_frac=spec.get("short_frac", 0.0))
    if spec.get("jitter"):   # timestamps going back by up to `jitter` ns
        sw = rng.choice(len(ts), len(ts) // 10, replace=False)
        ts[sw] = ts[sw] - rng.integers(0, spec["jitter"], sw.size).astype(np.uint64)
    return hdr, ln, ts


def worker(rank, world, port, spec, out_path, engine_kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle
        from flowsentryx_amd.shard import ShardedDataPlane
        cfg = spec["cfg"]
        hdr, ln, ts = _stream(spec)
        cuts = spec["cuts"]
        if engine_kind == "cpu":
            from shard_cpu import CpuShardEngine
            eng = CpuShardEngine(pyoracle, **cfg)
            dev = torch.device("cpu")
        else:
            torch.cuda.init()                 # torch's runtime first (tests/conftest.py)
            torch.cuda.set_device(0)
            from flowsentryx_amd import lib
            from flowsentryx_amd.shard import HipShardEngine
            dev = torch.device("cuda", 0)
            ctx = lib.FsxContext(max_batch=spec.get("owner_batch", 1 << 16), **cfg)
            eng = HipShardEngine(ctx, max(b - a for a, b in zip(cuts[:-1], cuts[1:])), dev)
            if spec.get("flows"):   # per-source features + q8 scores of every global batch
                from pathlib import Path
                from flowsentryx_amd import fsx_load
                ctx.load_q8_model(fsx_load.load_weights(Path(__file__).parent / "golden" / "model_weights.json"))
                eng.enable_flows(cfg["max_entries"])
        plane = ShardedDataPlane(eng, blocklist_filter=spec.get("filter", True))
        if spec.get("blk_cap"):   # a tiny replica capacity: owners overflow it (entries left out)
            plane.blk_cap = spec["blk_cap"]
        k = spec.get("chunks", 1)
        mine = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            # the batch in k*world pieces; piece j is on rank j % world, in sub-batch j // world
            pb = np.linspace(a, b, k * world + 1).astype(np.int64)
            idx = np.concatenate([np.arange(pb[i * world + rank], pb[i * world + rank + 1])
                                  for i in range(k)]).astype(np.int64)
            local_bounds = [0]
            for i in range(k):
                local_bounds.append(local_bounds[-1] + int(pb[i * world + rank + 1] - pb[i * world + rank]))
            n = idx.size
            th = torch.from_numpy(hdr[idx].reshape(-1).copy()).to(dev)
            tl = torch.from_numpy(ln[idx].view(np.int32).copy()).to(dev)
            tt = torch.from_numpy(ts[idx].view(np.int64).copy()).to(dev)
            tv = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
            plane.verdict_batch(th, tl, tt, n, tv, chunks=k, bounds=local_bounds)
            rows = None
            if spec.get("flows"):
                f = eng.flows
                m = int(f["rows"].item())
                rows = (f["keys"][:m * 16].cpu().numpy().reshape(m, 16).copy(), f["fam"][:m].cpu().numpy().copy(),
                        f["feat"][:m * 8].cpu().numpy().reshape(m, 8).copy(), f["prob"][:m].cpu().numpy().copy())
            mine.append((idx, tv[:n].cpu().numpy().copy(), rows))
        stats = plane.stats()
        if engine_kind == "cpu":
            dumps = {m: eng.o.map_dump(m) for m in spec["maps"]}
        else:
            dumps = {m: ctx.map_dump(m) for m in spec["maps"]}
        got = [None] * world
        dist.all_gather_object(got, (mine, dumps))
        if rank == 0:
            o = pyoracle.Oracle(**cfg)
            ok, msg = True, []
            for bi, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
                exp = o.batch(hdr[a:b], ln[a:b], ts[a:b])
                v = np.zeros(b - a, dtype=np.uint8)
                for r in range(world):
                    ridx, rv, _ = got[r][0][bi]
                    v[ridx - a] = rv
                if not np.array_equal(v, exp):
                    ok = False
                    msg.append(f"batch {bi}: {int((v != exp).sum())} verdicts differ")
                if spec.get("flows"):
                    # the union of the owners' rows = the 1-GPU rows over the whole batch
                    # (features bit-exact, q8 probabilities bit-exact)
                    from pathlib import Path
                    model = json.loads((Path(__file__).parent / "golden" / "model_weights.json").read_text())
                    ko, fo, xo = pyoracle.flow_features(hdr[a:b], ln[a:b], ts[a:b])
                    po, _, _ = pyoracle.score(model, xo)
                    want = {(int(fo[i]), ko[i].tobytes()): (xo[i].tobytes(), po[i].tobytes()) for i in range(len(fo))}
                    have = {}
                    for r in range(world):
                        kk, ff, xx, pp = got[r][0][bi][2]
                        for i in range(len(ff)):
                            key = (int(ff[i]), kk[i].tobytes())
                            if key in have:
                                ok = False
                                msg.append(f"batch {bi}: source {key} has rows on two owners")
                            have[key] = (xx[i].tobytes(), pp[i].tobytes())
                    if have != want:
                        ok = False
                        bad = sum(1 for k_ in want if have.get(k_) != want[k_])
                        msg.append(f"batch {bi}: {len(have)} rows vs {len(want)}, {bad} differ")
            if tuple(stats) != o.stats():
                ok = False
                msg.append(f"stats {stats} != {o.stats()}")
            for m in spec["maps"]:
                union = {}
                for r in range(world):
                    d = got[r][1][m]
                    if set(d) & set(union):
                        ok = False
                        msg.append(f"map {m}: a source on two owners")
                    union.update(d)
                if union != o.map_dump(m):
                    ok = False
                    msg.append(f"map {m}: {len(union)} vs {len(o.map_dump(m))} entries differ")
            with open(out_path, "w") as f:
                json.dump({"ok": ok, "msg": msg, "stats": list(stats),
                           "filtered": plane.filtered, "formats": sorted(plane.formats),
                           "partials": plane.partials_sent, "host_reads": plane.host_reads,
                           "blk_cap": plane.blk_cap}, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()
