#!/usr/bin/env python3
"""Recompute a bench line's roofline numbers from a committed profile directory.

The directory holds kernel_stats.csv (rocprofv3 --kernel-trace --stats of the bench command)
and bench_under_rocprof.log (the bench line printed under that same profiler run); the
headline's directory may also hold pmc_traffic.json (counter bytes per launch).

* kernel roofline (`roofline` block): the named kernel's average duration from rocprof and
  the algorithmic bytes per launch from the line -> achieved GB/s and fraction of peak;
* pipeline roofline (`pipeline` block, and the config-4 / config-5 / config-3 legs when
  profiled as the headline with scripts/gpu_legs_profile.sh): algorithmic bytes per step
  over the line's ms per step, next to the device time per batch that rocprof saw (the sum
  of the fsx kernels' durations over the batches: kernels of one batch overlap on three
  streams, so this sum may exceed the step).

    python3 scripts/roofline_check.py profiles/r03/prof_r03_config2 [more dirs]"""
import csv
import json
import sys
from pathlib import Path


def kernel_rows(d):
    return list(csv.DictReader(open(d / "kernel_stats.csv")))


def kernel_avg_ms(rows, kern):
    sel = [r for r in rows if f"::{kern}<" in r["Name"] or f"::{kern}(" in r["Name"]]
    calls = sum(int(r["Calls"]) for r in sel)
    if not calls:
        return None, 0
    return sum(float(r["TotalDurationNs"]) for r in sel) / calls / 1e6, calls


def check(d):
    d = Path(d)
    line = json.loads([l for l in (d / "bench_under_rocprof.log").read_text().splitlines() if l.startswith("{")][-1])
    rows = kernel_rows(d)
    out = {"dir": str(d), "workload": line.get("config", {}).get("workload", "")[:80],
           "ms_per_step_line": line.get("ms_per_step")}
    rf = line.get("roofline") or {}
    if rf.get("kernel") and rf.get("bytes_per_launch"):
        avg, calls = kernel_avg_ms(rows, rf["kernel"])
        if avg:
            achieved = rf["bytes_per_launch"] / (avg * 1e-3) / 1e9
            out["kernel"] = {"name": rf["kernel"], "rocprof_calls": calls, "rocprof_avg_ms": round(avg, 4),
                             "bench_launch_ms": rf.get("launch_ms"), "bytes_per_launch": rf["bytes_per_launch"],
                             "achieved_GBps_from_rocprof": round(achieved, 1),
                             "frac_from_rocprof": round(achieved / rf["peak"], 4), "frac_bench_line": rf.get("frac")}
            pmc = d / "pmc_traffic.json"
            if pmc.exists():
                k = json.loads(pmc.read_text())["kernels"].get(rf["kernel"], {})
                if k.get("hbm_bytes_per_launch"):
                    out["kernel"]["pmc_bytes_per_launch"] = k["hbm_bytes_per_launch"]
                    out["kernel"]["pmc_over_algorithmic"] = round(k["hbm_bytes_per_launch"] / rf["bytes_per_launch"], 3)
    pl = line.get("pipeline") or {}
    if pl.get("algorithmic_bytes_per_step") and line.get("ms_per_step"):
        ach = pl["algorithmic_bytes_per_step"] / (line["ms_per_step"] * 1e-3) / 1e9
        # batches seen by the profiler: the parse runs once per batch
        _, batches = kernel_avg_ms(rows, "k_parse")
        fsx_ns = sum(float(r["TotalDurationNs"]) for r in rows if "fsx::" in r["Name"])
        out["pipeline"] = {"bytes_per_step": pl["algorithmic_bytes_per_step"],
                           "achieved_GBps": round(ach, 1), "frac": round(ach / pl["peak"], 4),
                           "frac_bench_line": pl.get("frac"),
                           "rocprof_batches": batches,
                           "rocprof_device_ms_per_batch": round(fsx_ns / 1e6 / batches, 3) if batches else None}
        top = sorted(((float(r["TotalDurationNs"]) / max(1, batches) / 1e6, r["Name"].split("(")[0].split("::")[-1])
                      for r in rows if "fsx::" in r["Name"]), reverse=True)[:8]
        out["pipeline"]["top_kernels_ms_per_batch"] = [(n, round(t, 4)) for t, n in top]
    # legs measured beside the headline: recompute each pipeline fraction from its own
    # bytes per step and ms per step (as printed under the profiler)
    legs = {}
    for name, leg in (("config3.from_stream", (line.get("config3") or {}).get("from_stream")),
                      ("config4", line.get("config4")), ("config5", line.get("config5"))):
        rf_ = (leg or {}).get("roofline") or {}
        if rf_.get("bytes_per_step") and leg.get("ms_per_step"):
            ach = rf_["bytes_per_step"] / (leg["ms_per_step"] * 1e-3) / 1e9
            legs[name] = {"bytes_per_step": rf_["bytes_per_step"], "ms_per_step": leg["ms_per_step"],
                          "achieved_GBps": round(ach, 1), "frac": round(ach / rf_["peak"], 4),
                          "frac_bench_line": rf_.get("frac")}
    if legs:
        out["legs"] = legs
    return out


def main():
    dirs = sys.argv[1:] or ["profiles/r02/prof_r02h"]
    for d in dirs:
        print(json.dumps(check(d), indent=1))


if __name__ == "__main__":
    main()
