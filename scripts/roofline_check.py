#!/usr/bin/env python3
"""Recompute the bench line's roofline from a committed profile directory: the dominant
kernel's average duration from rocprofv3 --stats (kernel_stats.csv), the algorithmic bytes
per launch from the bench line recorded under the same profiler run
(bench_under_rocprof.log), and the counter bytes from pmc_traffic.json.
    python3 scripts/roofline_check.py profiles/r02/prof_r02h"""
import csv
import json
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1] if len(sys.argv) > 1 else "profiles/r02/prof_r02h")
    line = json.loads([l for l in (d / "bench_under_rocprof.log").read_text().splitlines() if l.startswith("{")][-1])
    rf = line["roofline"]
    kern = rf["kernel"]
    rows = [r for r in csv.DictReader(open(d / "kernel_stats.csv")) if f"::{kern}<" in r["Name"] or f"::{kern}(" in r["Name"]]
    calls = sum(int(r["Calls"]) for r in rows)
    avg_ns = sum(float(r["TotalDurationNs"]) for r in rows) / calls
    achieved = rf["bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
    out = {"kernel": kern, "rocprof_calls": calls, "rocprof_avg_ms": round(avg_ns / 1e6, 4),
           "bench_launch_ms": rf["launch_ms"], "bytes_per_launch": rf["bytes_per_launch"],
           "achieved_GBps_from_rocprof": round(achieved, 1), "frac_from_rocprof": round(achieved / rf["peak"], 4),
           "frac_bench_line": rf["frac"]}
    pmc = d / "pmc_traffic.json"
    if pmc.exists():
        k = json.loads(pmc.read_text())["kernels"].get(kern, {})
        out["pmc_bytes_per_launch"] = k.get("hbm_bytes_per_launch")
        out["pmc_over_algorithmic"] = round(k["hbm_bytes_per_launch"] / rf["bytes_per_launch"], 3) if k else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
