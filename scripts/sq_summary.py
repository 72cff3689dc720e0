#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace stats + SQ counter pass per kernel (mean per dispatch)."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
durs = {}
for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        durs[row["Name"]] = float(row["AverageNs"])
        print(f"{float(row['AverageNs'])/1e3:9.1f} us x{row['Calls']:>4}  {row['Name'][:110]}")
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    if "ntt" not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    waves = m.get("SQ_WAVES", 0)
    print(k[:100])
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
    if "GRBM_GUI_ACTIVE" in m and k in durs:
        print(f"   effective clock = GRBM_GUI_ACTIVE/8/duration = {m['GRBM_GUI_ACTIVE']/8/durs[k]/1e3:.3f} GHz")
    if "SQ_INSTS_VALU" in m:
        print(f"   VALU/wave={m['SQ_INSTS_VALU']/max(waves,1):.1f}  LDS/wave={m.get('SQ_INSTS_LDS',0)/max(waves,1):.1f}"
              f"  SALU/wave={m.get('SQ_INSTS_SALU',0)/max(waves,1):.1f}"
              f"  active_valu/wave_cycles={m.get('SQ_ACTIVE_INST_VALU',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.3f}")
