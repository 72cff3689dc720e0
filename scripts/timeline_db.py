#!/usr/bin/env python3
"""Kernel timeline around the K-th-from-last dispatch whose name contains SUBSTRING in a
rocprofv3 rocpd SQLite output: timeline_db.py DB SUBSTRING [K] [N]. Prints start offset,
duration (us), queue and name of N dispatches from there."""
import sqlite3
import sys

db, key = sys.argv[1], sys.argv[2]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if key in r[0]]
i0 = idx[-k]
t0 = rows[i0][1]
for r in rows[i0:i0 + n]:
    print(f"{(r[1] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:8.1f}  q{r[3]:<3} {r[0][:80]}")
