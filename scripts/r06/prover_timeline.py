#!/usr/bin/env python3
"""Kernel timeline of the last proof in a rocprofv3 kernel trace (after the last idle gap of more
than 0.5 s, scripts/r06/prover_one.py): every dispatch with its start offset, duration and queue,
then per-kernel totals. prover_timeline.py TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cut = 0
for i in range(1, len(rows)):
    if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 500_000_000:
        cut = i
rows = rows[cut:]
t0 = int(rows[0]["Start_Timestamp"])
tot = defaultdict(lambda: [0, 0.0])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    print("%10.1f %9.1f  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Queue_Id", "?"), name[:100]))
    tot[name][0] += 1
    tot[name][1] += (e - s) / 1e3
end = max(int(r["End_Timestamp"]) for r in rows)
print("# span %.1f us, %d dispatches" % ((end - t0) / 1e3, len(rows)))
for name, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print("# %-90s %5d %10.1f us" % (name[:90], c, us))
