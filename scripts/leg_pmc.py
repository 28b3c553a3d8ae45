#!/usr/bin/env python3
"""HBM bytes per batch of a bench leg from two rocprofv3 PMC passes.

    python3 scripts/leg_pmc.py gpurun_out/pmc_r04af_c5

<dir>/FETCH_SIZE/run_counter_collection.csv and <dir>/WRITE_SIZE/... (KiB per dispatch);
FETCH_SIZE doubled per the gfx950 correction of MI355X_MICROARCH.md (HBM section). The leg
is every dispatch after the last synthetic-stream kernel (k_synth), product kernels only
(the library's k_* kernels and its memsets / copies; not the bench's torch-side checks or
map dumps); bytes are summed per kernel and divided by the leg's k_parse launches (one per
batch). A second table is the last batch alone (the steady state: from its prelude — the
memsets, copies and map imports right before its k_parse — to its last kernel), which leaves out the
context's one-time table clear and a first batch into empty maps."""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    k = re.split(r"[<(]", k)[0]
    return k.split("::")[-1]


def leg_rows(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        rows.append((int(r["Start_Timestamp"]), short(r["Kernel_Name"]), float(r["Counter_Value"]) * 1024))
    rows.sort()
    last = max((i for i, r in enumerate(rows) if r[1] == "k_synth"), default=-1)
    keep = lambda k: (k.startswith("k_") and k != "k_map_dump") or k.startswith("__amd_rocclr")
    return [r for r in rows[last + 1:] if keep(r[1])]


def last_batch(rows):
    lp = max((i for i, r in enumerate(rows) if r[1] == "k_parse"), default=0)
    s = lp
    while s > 0 and (rows[s - 1][1].startswith("__amd_rocclr") or rows[s - 1][1] == "k_map_import"):
        s -= 1
    e = max(i for i, r in enumerate(rows) if r[1].startswith("k_"))   # (then the bench's checks)
    return rows[s:e + 1]


def main(d):
    d = Path(d)
    fetch = leg_rows(d / "FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE")
    write = leg_rows(d / "WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE")
    table(fetch, write, "all of the leg's batches")
    table(last_batch(fetch), last_batch(write), "the last batch alone")


def table(fetch, write, what):
    nb = sum(1 for r in fetch if r[1] == "k_parse") or 1
    rd, wr = defaultdict(float), defaultdict(float)
    for _, k, v in fetch:
        rd[k] += 2 * v / nb
    for _, k, v in write:
        wr[k] += v / nb
    tot = 0.0
    print(f"{what}: batches {nb} (FETCH_SIZE x2 + WRITE_SIZE, GB per batch)")
    for k in sorted(set(rd) | set(wr), key=lambda k: -(rd[k] + wr[k])):
        t = rd[k] + wr[k]
        tot += t
        if t >= 5e6:
            print(f"  {k:30s} rd {rd[k] / 1e9:7.3f} wr {wr[k] / 1e9:7.3f}")
    print(f"sum {tot / 1e9:.3f} GB per batch")


if __name__ == "__main__":
    main(sys.argv[1])
