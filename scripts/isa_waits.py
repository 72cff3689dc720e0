#!/usr/bin/env python3
"""Memory-op / wait / barrier skeleton of one kernel in a gfx950 assembly listing:
isa_waits.py FILE.s KERNEL_SUBSTRING. Prints instruction index, op, and runs of VALU."""
import re
import sys

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
ins = []
for l in lines[start + 1:]:
    if l.startswith(".Lfunc_end"):
        break
    if re.match(r"^\.LBB", l):
        ins.append(l.split()[0])
    elif l.startswith("\t") and not l.strip().startswith((".", ";")):
        ins.append(l.strip())
valu = 0
for k, l in enumerate(ins):
    op = l.split()[0]
    if op.startswith(("s_waitcnt", "s_barrier", "global_load", "global_store", "s_cbranch", "s_branch", ".LBB")):
        if valu:
            print(f"      ... {valu} VALU")
            valu = 0
        print(k, l[:70])
    elif op.startswith("v_"):
        valu += 1
print(f"total {len(ins)} instructions")
