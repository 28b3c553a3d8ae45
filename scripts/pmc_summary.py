#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_<tag>/{fetch,write,sq}) per kernel:
mean per dispatch over the measured bench steps. FETCH_SIZE and WRITE_SIZE are in KiB
(rocprofv3 derived counters); FETCH_SIZE is doubled per the gfx950 correction of
MI355X_MICROARCH.md (HBM section) — both are reported raw and corrected."""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def short_name(k):
    """'void fsx::k_tile_scatter<true>(unsigned long const*, ...)' -> 'k_tile_scatter'."""
    k = k.replace("(anonymous namespace)::", "")
    k = k.split("(")[0].replace("void ", "").strip()
    k = re.sub(r"<.*>", "", k)
    return k.split("::")[-1]


def load(path):
    out = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = short_name(r["Kernel_Name"])
        out[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        out[name]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    d = Path(sys.argv[1])
    res = defaultdict(dict)
    for tag in ("fetch", "write", "sq", "sq2", "tcc"):
        f = d / tag / "run_counter_collection.csv"
        if not f.exists():
            continue
        for k, cs in load(f).items():
            for c, v in cs.items():
                if c == "_dur_ns":
                    continue
                res[k][c] = sum(v) / len(v)
    rows = {}
    for k, cs in sorted(res.items()):
        row = dict(cs)
        if "FETCH_SIZE" in cs:
            row["hbm_read_bytes_raw"] = cs["FETCH_SIZE"] * 1024
            row["hbm_read_bytes"] = cs["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in cs:
            row["hbm_write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in row and "hbm_write_bytes" in row:
            row["hbm_bytes_per_launch"] = row["hbm_read_bytes"] + row["hbm_write_bytes"]
        if cs.get("SQ_WAVE_CYCLES"):
            row["wait_any_frac"] = cs.get("SQ_WAIT_ANY", 0) / cs["SQ_WAVE_CYCLES"]
            row["valu_frac"] = cs.get("SQ_ACTIVE_INST_VALU", 0) / cs["SQ_WAVE_CYCLES"]
            row["lds_frac"] = cs.get("SQ_ACTIVE_INST_LDS", 0) / cs["SQ_WAVE_CYCLES"]
        if cs.get("TCC_HIT_sum") is not None and cs.get("TCC_MISS_sum") is not None:
            tot = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
            row["l2_hit_rate"] = cs["TCC_HIT_sum"] / tot if tot else None
        rows[k] = row
    doc = {"source": f"rocprofv3 --kernel-trace --pmc passes under {d.name} (scripts/gpu_pmc.sh)",
           "workload": {"config": 2, "packets_per_gpu": 67108864, "n_gpus": 1,
                        "command": "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --legs ''", "headline": "stream: consecutive batches, maps carried, pipelined (the first batch inserts every source)"},
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as read",
           "kernels": rows}
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
