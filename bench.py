#!/usr/bin/env python3
"""Benchmark: Mpps of FlowSentryX verdicts on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch of synthetic packets resident
in HBM, starting from empty maps (fsx_reset is inside the timed step): parse ->
per-source fixed-window rate limit + blacklist -> verdicts + map state
(src/fsx_kern.c:96-347 semantics) -> per-source flow features -> q8 MLP score of
every source with the reference weights (model/model.py:132-137). N=1 workload:
BASELINE config 2 — 64M IPv4/UDP packets from 1M Zipf(1.1) sources over 30 s.

Multi-GPU (torch.distributed.run, one rank per GPU): weak scaling — one stream of
N x 64M packets from one source population at the config's packet rate; rank r holds
the contiguous slice [r*64M, (r+1)*64M) and every source is owned by one rank
(hash of the address): RCCL all-to-all of 32-byte records to the owners, the full
pipeline there, verdicts back by a second all-to-all (flowsentryx_amd/shard.py,
DESIGN.md §7). The result equals the 1-GPU run over the whole stream.

Prints ONE JSON line on rank 0 with the driver's contract plus:
  roofline      the dominant kernel (largest device time per step), its algorithmic
                bytes per launch over its mean launch time measured with HIP events on
                the library's stream inside the timed region;
  pipeline      the whole step against SURVEY §8 d: 77 B/packet + 64 B per source;
  cpu_baseline  the CPU oracle (sharded over host threads) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md

# Algorithmic bytes each kernel's function must move, per element it processes
# (DESIGN.md §3): element = packet (parse) or IP packet (sort / fill).
KERNEL_BYTES = {
    "k_parse": ("packet", 64 + 4 + 8 + 8),      # header record + len + ts in, sort word out
    # one LSD digit pass: sort word + payload word in and out (pass 0 reads ts + len
    # instead of a payload word: 36 B; passes 1-3: 32 B) -> 33 B per launch on average
    "k_tile_scatter": ("ip_packet", 33),
    "k_tile_hist": ("ip_packet", 8),            # sort word in (+ per-tile counts)
    "k_onesweep": ("ip_packet", 16),            # sort word in + out, per digit pass
    "k_flow_features": ("ip_packet", 8 + 4 + 8),  # sort word + len + ts per packet
    "k_walk_fixed": ("ip_packet", 8 + 4 + 8 + 1),  # sort word + len + ts in, mark out
    "k_fill_scatter": ("ip_packet", 1 + 8 + 1),  # mark + sort word in, verdict out
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--packets", type=int, default=None, help="packets per rank (default: config)")
    ap.add_argument("--cpu-sample", type=int, default=64 << 20,
                    help="packets of the CPU baseline sample (default: the whole config-2 stream)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify a prefix against the oracle")
    ap.add_argument("--no-mlp", action="store_true", help="verdicts only (no features/scores)")
    ap.add_argument("--no-reset", action="store_true",
                    help="diagnostics: keep the maps between steps (state carries over)")
    ap.add_argument("--chunks", type=int, default=4,
                    help="N>1: sub-batches per step (the replicated blocklist of one filters "
                         "the next)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="N>1 collectives: nccl (RCCL over xGMI) or gloo (rehearsal on one GPU)")
    ap.add_argument("--limiter", choices=["fixed", "sliding", "token"], default="fixed",
                    help="limiter of the timed main loop (diagnostics; the headline is fixed)")
    ap.add_argument("--rule-steps", type=int, default=5,
                    help="steps of the prefix-blocklist leg (64K rules; 0 skips it)")
    ap.add_argument("--limiter-steps", type=int, default=5,
                    help="timed steps of the sliding-window and token-bucket legs (0: skip)")
    return ap.parse_args()


def main():
    args = parse_args()
    import torch

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    # one rank per GPU; more ranks than GPUs only in a gloo rehearsal on one device
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    from flowsentryx_amd import lib, synth

    p, zipf_s = synth.config_params(args.config, n=args.packets)
    n = int(p.n)
    # weak scaling: ONE stream of world*n packets at the config's packet rate (so
    # world times as long) from one source population; rank r holds the contiguous
    # slice [r*n, (r+1)*n) and the sources are hash-sharded over the ranks (RCCL
    # all-to-all to their owners, flowsentryx_amd/shard.py)
    p.n = n * world
    p.duration_ns = p.duration_ns * world
    d_hdr = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_len = torch.empty(n, dtype=torch.int32, device="cuda")
    d_ts = torch.empty(n, dtype=torch.int64, device="cuda")
    d_v = torch.empty(n, dtype=torch.uint8, device="cuda")
    # N>1: the stream in world*chunks pieces of n/chunks packets, piece j on rank j % world
    # (sub-batch j // world): rank r's slice is its pieces r, r+world, ... in order
    chunks = max(1, args.chunks) if world > 1 else 1
    bounds = [n * i // chunks for i in range(chunks + 1)]
    for i in range(chunks):
        a, b = bounds[i], bounds[i + 1]
        j0 = world * a + rank * (b - a)
        synth.generate_device(p, zipf_s, j0, b - a, d_hdr.data_ptr() + a * 64,
                              d_len.data_ptr() + a * 4, d_ts.data_ptr() + a * 8)
    torch.cuda.synchronize()
    p.n = n
    p.duration_ns = p.duration_ns // world

    max_entries = max(1024, int(p.n_ips) if p.n_ips else n)
    lim_id = {"fixed": lib.LIMIT_FIXED_WINDOW, "sliding": lib.LIMIT_SLIDING_WINDOW,
              "token": lib.LIMIT_TOKEN_BUCKET}[args.limiter]
    ctx = lib.FsxContext(max_batch=n, max_entries=max_entries, device=local, limiter=lim_id)
    from flowsentryx_amd import fsx_load
    ctx.load_q8_model(fsx_load.load_weights(ROOT / "tests" / "golden" / "model_weights.json"))
    fcap = max_entries
    d_keys = torch.empty(fcap * 16, dtype=torch.uint8, device="cuda")
    d_fam = torch.empty(fcap, dtype=torch.uint8, device="cuda")
    d_prob = torch.empty(fcap, dtype=torch.float32, device="cuda")
    d_dec = torch.empty(fcap, dtype=torch.uint8, device="cuda")

    plane = None
    if world > 1:
        from flowsentryx_amd.shard import HipShardEngine, ShardedDataPlane
        eng = HipShardEngine(ctx, n, torch.device("cuda", local))
        if not args.no_mlp:
            eng.enable_flows(fcap)
        plane = ShardedDataPlane(eng)

    def step():
        if not args.no_reset:
            ctx.reset()
        if plane is not None:
            plane.reset()
            plane.verdict_batch(d_hdr, d_len, d_ts, n, d_v, bounds=bounds, chunks=chunks)
        elif args.no_mlp:
            ctx.verdict_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                                     d_v.data_ptr())
        else:
            ctx.process_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                                     d_v.data_ptr(), d_keys.data_ptr(), d_fam.data_ptr(), None,
                                     d_prob.data_ptr(), d_dec.data_ptr(), fcap)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    info = ctx.last_batch_info()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-kernel device times (a HIP event after every kernel) from separate steps, so the
    # timed steps above carry no event records
    ctx.enable_timing(True)
    ctx.last_timings()  # reset accumulators
    for _ in range(max(1, min(args.steps, 5))):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    timings = ctx.last_timings()
    ctx.enable_timing(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    exchange = None
    if plane is not None:
        stats = plane.stats()
        ex = plane.last_exchange or {"sent": [], "received": []}
        exchange = {"records_sent": ex["sent"], "records_received": ex["received"],
                    "dropped_by_replica": ex.get("filtered", 0), "sub_batches": chunks,
                    "record_bytes": sorted(plane.formats) or None, "backend": args.dist_backend}
        malicious = None
        if not args.no_mlp:
            fl = eng.flows
            mal = torch.tensor([int(fl["dec"][:info["sources"]].sum().item())], device="cuda")
            if args.dist_backend == "gloo":
                mal = mal.cpu()
            dist.all_reduce(mal)
            malicious = int(mal.item())
    else:
        stats = ctx.stats()
        malicious = None if args.no_mlp else int(d_dec[:info["sources"]].sum().item())
    ctx.close()

    # BASELINE config 2 also names the sliding-window and token-bucket limiters
    # (build-defined): the same batch through each, verdicts + maps only
    limiters = {}
    if args.limiter_steps > 0 and world == 1:
        for lname, lid in (("sliding_window", lib.LIMIT_SLIDING_WINDOW),
                           ("token_bucket", lib.LIMIT_TOKEN_BUCKET)):
            with lib.FsxContext(max_batch=n, max_entries=max_entries, device=local,
                                limiter=lid) as lc:
                def lstep():
                    lc.reset()
                    lc.verdict_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                                            d_v.data_ptr())
                lstep()
                lc.sync()
                torch.cuda.synchronize()
                if dist:
                    dist.barrier()
                l0 = time.perf_counter()
                for _ in range(args.limiter_steps):
                    lstep()
                lc.sync()
                torch.cuda.synchronize()
                if dist:
                    dist.barrier()
                lt = time.perf_counter() - l0
                if dist:
                    t = torch.tensor([lt], dtype=torch.float64,
                                     device="cuda" if args.dist_backend == "nccl" else "cpu")
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                    lt = float(t.item())
                la, ld = lc.stats()
                limiters[lname] = {"value": round(n * world * args.limiter_steps / lt / 1e6, 2),
                                   "unit": "Mpps", "ms_per_step": round(lt / args.limiter_steps * 1e3, 4),
                                   "steps": args.limiter_steps, "allowed": la, "dropped": ld}

    # prefix blocklists (SURVEY §8 f row 4): the same batch with a 64K-rule
    # table — 61440 random /24 prefixes (mostly missing the stream) and 4096 rules on the
    # stream's own sources (/32 and /28, permanent) — fixed window, verdicts + maps
    rules_leg = None
    if args.rule_steps > 0 and world == 1:
        import numpy as np
        rng = np.random.default_rng(5)
        seen = d_hdr[: min(n, 1 << 16) * 64].view(-1, 64)[:, 26:30].cpu().numpy()
        srcs = np.unique(seen.view(np.uint32).reshape(-1))[:4096]
        r4 = {}
        for a in rng.integers(0, 2**32, 61440, dtype=np.uint64).astype(np.uint32):
            r4[lib.prefix_key((int(a) & 0xFFFFFF).to_bytes(4, "little"), 24)] = 2**64 - 1
        for i, a in enumerate(srcs):
            r4[lib.prefix_key(int(a).to_bytes(4, "little"), 32 if i & 1 else 28)] = 2**64 - 1
        with lib.FsxContext(max_batch=n, max_entries=max_entries, device=local) as rc_:
            rc_.map_update_batch(lib.MAP_IPV4_PREFIX, r4)
            def rstep():
                rc_.reset()
                rc_.verdict_batch_device(d_hdr.data_ptr(), d_len.data_ptr(), d_ts.data_ptr(), n,
                                         d_v.data_ptr())
            rstep()
            rc_.sync()
            torch.cuda.synchronize()
            r0 = time.perf_counter()
            for _ in range(args.rule_steps):
                rstep()
            rc_.sync()
            torch.cuda.synchronize()
            rt = time.perf_counter() - r0
            ri = rc_.last_batch_info()
            ra, rd = rc_.stats()
        rules_leg = {"value": round(n * args.rule_steps / rt / 1e6, 2), "unit": "Mpps",
                     "ms_per_step": round(rt / args.rule_steps * 1e3, 4), "steps": args.rule_steps,
                     "rules": len(r4), "prefix_lengths": [24, 28, 32],
                     "rule_drops": ri["prefix_rule_drops"], "allowed": ra, "dropped": rd}

    check = None
    if args.check and rank == 0:
        from oracle import pyoracle
        m = min(n, 4 << 20)
        hdr, ln, ts = pyoracle.synth(p, zipf_s, 0, m)
        o = pyoracle.Oracle(max_entries=max_entries)
        vo = o.batch(hdr, ln, ts)
        with lib.FsxContext(max_batch=m, max_entries=max_entries, device=local) as c2:
            vg = c2.verdict_batch(hdr, ln, ts)
        check = {"prefix_packets": m, "verdicts_equal": bool((vo == vg).all())}

    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    total = n * world * args.steps
    mpps = total / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3
    ip_packets, sources = info["ip_packets"], info["sources"]

    # dominant kernel: largest device time per step
    dom = max(timings, key=lambda r: r[1]) if timings else None
    roofline = None
    if dom:
        name, ms_per_batch, launches = dom
        unit, per = KERNEL_BYTES.get(name, ("packet", 0))
        units = n if unit == "packet" else ip_packets
        per_launch_ms = ms_per_batch / max(launches, 1e-9)
        bytes_per_launch = per * units
        achieved = bytes_per_launch / (per_launch_ms * 1e-3) / 1e9 if per else None
        traffic = None
        pmc = ROOT / "profiles" / "pmc_traffic.json"
        if pmc.exists():
            doc = json.loads(pmc.read_text())
            wl = doc.get("workload", {})
            if wl.get("packets_per_gpu") == n and wl.get("config") == args.config and world == 1:
                traffic = doc.get("kernels", {}).get(name, {}).get("hbm_bytes_per_launch")
        roofline = {
            "bound": "hbm", "kernel": name, "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic, "bytes_per_launch": bytes_per_launch,
            "launch_ms": round(per_launch_ms, 4), "launches_per_step": launches,
        }
    algo = 77 * n + 64 * sources
    pipe_gbs = algo / (ms_step * 1e-3) / 1e9
    pipeline = {"bound": "hbm", "algorithmic_bytes_per_step": algo,
                "achieved": round(pipe_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(pipe_gbs / HBM_PEAK_GBS, 4)}

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        from oracle import pyoracle
        m = min(n, args.cpu_sample)
        hdr, ln, ts = pyoracle.synth(p, zipf_s, 0, m)
        th = args.cpu_threads
        c0 = time.perf_counter()
        _, _ = pyoracle.batch_sharded(hdr, ln, ts, th, max_entries=max_entries)
        cdt = time.perf_counter() - c0
        cpu = {"value": round(m / cdt / 1e6, 3), "unit": "Mpps", "cores": th, "kind": "port",
               "sample": f"first {m} packets of the config-{args.config} stream, fixed window, "
                         f"oracle/fsx_oracle.c sharded by source over {th} threads "
                         f"({cdt:.2f} s)"}

    out = {
        "metric": "Mpps verdicts (parse+rate-limit+MLP) at 1/2/4/8 GPUs; % of HBM BW peak",
        "value": round(mpps, 2), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (counter-based generator, fsx_synth_common.h)",
        "config": {"workload": f"BASELINE config {args.config}: {n} IPv4/UDP packets per GPU, "
                               f"{p.n_ips} Zipf(1.1) sources, {p.duration_ns / 1e9:g} s; "
                               "fixed-window limiter (src/fsx_kern.c), maps reset each step"
                               + ("; sliding-window and token-bucket legs timed separately "
                                  "(limiters)" if args.limiter_steps > 0 else "")
                               + ("" if args.no_mlp else "; per-source features + q8 MLP score "
                                  "(model_weights.pth)"),
                   "packets_per_gpu": n, "sources": sources,
                   "parallelism": f"dp{world}" + ("" if world == 1 else
                                                  " (sources hash-sharded, all-to-all)")},
        "roofline": roofline, "pipeline": pipeline, "cpu_baseline": cpu,
        "limiters": limiters or None, "prefix_rules": rules_leg, "exchange": exchange,
        "kernels": [{"name": a, "ms_per_step": round(b, 4), "launches": c} for a, b, c in timings],
        "stats": {"allowed": stats[0], "dropped": stats[1], "sources": info["sources"],
                  "light_packets": info["light_packets"], "malicious_sources": malicious},
        "check": check,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
