"""Print the last bench step of a rocprofv3 kernel-trace CSV as a timeline (us)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))


def name(r):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:30]


# the last TL_STEPS steps (default 1)
import os
start = [i for i, r in enumerate(rows) if name(r) == "k_heavy_sample"][-int(os.environ.get("TL_STEPS", "1"))]
seg = rows[start:]
t0 = min(int(r["Start_Timestamp"]) for r in seg)
for r in seg:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    if name(r).startswith("k_"):
        print(f"{name(r):22s} q{r['Queue_Id']} s{r.get('Stream_Id', '?')} {s:8.1f} {e:8.1f} {e - s:7.1f}")
