#!/usr/bin/env python3
"""Per-kernel device time of a bench leg from a rocprofv3 kernel trace.

    python3 scripts/leg_trace.py gpurun_out/prof_r04x_c5/run_kernel_trace.csv

The leg is every dispatch after the last synthetic-stream kernel (k_synth: the leg
generates its input first); times are summed per kernel and divided by the leg's
k_parse launches (one per batch), next to the wall span from the first to the last
parse-to-tail dispatch of each batch."""
import csv
import re
import sys
from collections import defaultdict


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    k = re.split(r"[<(]", k)[0]
    return k.split("::")[-1]


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    last_synth = max((i for i, r in enumerate(rows) if r[2] == "k_synth"), default=-1)
    leg = rows[last_synth + 1:]
    nb = sum(1 for r in leg if r[2] == "k_parse") or 1
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, k in leg:
        tot[k] += (e - s) / 1e6
        cnt[k] += 1
    print(f"batches {nb}; wall {(leg[-1][1] - leg[0][0]) / 1e6 / nb:.3f} ms per batch (first to last dispatch)")
    for k in sorted(tot, key=lambda k: -tot[k]):
        if tot[k] / nb >= 0.01:
            print(f"  {k:28s} {tot[k] / nb:9.3f} ms  x{cnt[k] / nb:.1f}")
    # per batch: span from its parse start to the next parse start
    ps = [s for s, e, k in leg if k == "k_parse"]
    for a, b in zip(ps, ps[1:] + [leg[-1][1]]):
        print(f"  batch span {(b - a) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
