#!/usr/bin/env python3
"""Per-launch-group counter medians from rocprofv3 --pmc csv output (recursive under DIR):
consecutive dispatches of the same kernel form one group (a ubench's warm-up + timed reps).
pmc_groups.py DIR [BYTES_PER_DISPATCH] -- with BYTES, prints FETCH_SIZE / WRITE_SIZE (kB,
x1024) as a fraction of it: the calibration of those counters for each access pattern."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
ref = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = defaultdict(dict)  # dispatch id -> {name, counters}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        did = int(r["Dispatch_Id"])
        rows[did]["name"] = r["Kernel_Name"]
        rows[did][r["Counter_Name"]] = rows[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
groups = []
for did in sorted(rows):
    r = rows[did]
    if groups and groups[-1][0] == r["name"]:
        groups[-1][1].append(r)
    else:
        groups.append((r["name"], [r]))
for name, rs in groups:
    cs = sorted({c for r in rs for c in r if c != "name"})
    med = {c: sorted(r.get(c, 0.0) for r in rs)[len(rs) // 2] for c in cs}
    line = f"{name[:70]:70s} n={len(rs):3d} " + " ".join(f"{c}={v:.6g}" for c, v in med.items())
    if ref:
        line += "  " + " ".join(f"{c}/ref={v * 1024 / ref:.3f}" for c, v in med.items() if c.endswith("_SIZE"))
    print(line)
