#!/usr/bin/env python3
"""Median duration of each pass of a multi-pass Goldilocks NTT from a rocprofv3 results
database (dispatches of ntt_gl_pass_kernel in launch order, P per transform batch).
Usage: pass_split.py RESULTS.db P"""
import sqlite3
import statistics
import sys

db, P = sys.argv[1], int(sys.argv[2])
rows = [r for r in sqlite3.connect(db).execute("select name, start, end from kernels order by start")
        if "ntt_gl_pass" in r[0]]
for i in range(P):
    d = [(r[2] - r[1]) / 1e3 for k, r in enumerate(rows) if k % P == i]
    print(f"pass {i + 1}: median {statistics.median(d):7.1f} us over {len(d)} dispatches  ({rows[i][0][:60]})")
