#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 rocpd SQLite output (k_results.db), like
--stats: name, calls, mean / min / max us, total ms. Usage: kstats_db.py DB [SUBSTRING]"""
import sqlite3
import sys

db = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
for name, s, e in rows:
    if key and key not in name:
        continue
    d = (e - s) / 1e3
    a = agg.setdefault(name, [])
    a.append(d)
for name, ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    short = name if len(name) < 90 else name[:87] + "..."
    print(f"{short:90s} {len(ds):5d} mean {sum(ds)/len(ds):9.1f} us  min {min(ds):9.1f}  max {max(ds):9.1f}  total {sum(ds)/1e3:8.3f} ms")
