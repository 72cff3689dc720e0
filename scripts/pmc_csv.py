#!/usr/bin/env python3
"""Mean per dispatch of every counter per kernel over rocprofv3 --pmc csv outputs under DIR
(recursive): pmc_csv.py DIR [KERNEL_SUBSTRING]."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if key in row["Kernel_Name"]:
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k[:110])
    print("   " + "  ".join(f"{c}={v:.5g}" for c, v in sorted(m.items())))
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        print(f"   WAIT_ANY/WAVE_CYCLES={m.get('SQ_WAIT_ANY', 0) / w:.3f}  "
              f"ACTIVE_VALU/WAVE_CYCLES={m.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f}  "
              f"WAIT_INST/WAVE_CYCLES={m.get('SQ_WAIT_INST_ANY', 0) / w:.3f}")
