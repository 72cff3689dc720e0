#!/usr/bin/env python3
"""Per-kernel summary (calls, mean us, total ms) of a rocprofv3 results database.
Usage: kstats.py RESULTS.db [TOP]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
q = ("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels "
     "group by name order by 4 desc limit ?")
print("%-70s %6s %10s %10s" % ("kernel", "calls", "mean_us", "total_ms"))
for r in c.execute(q, (top,)):
    print("%-70s %6d %10.1f %10.2f" % (r[0][:70], r[1], r[2], r[3]))
