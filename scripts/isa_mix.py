#!/usr/bin/env python3
"""Static instruction mix of one kernel in a gfx950 assembly listing (hipcc -S
--cuda-device-only). Usage: isa_mix.py FILE.s KERNEL_SUBSTRING"""
import collections
import re
import sys

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
body = []
for l in lines[start + 1:]:
    if l.startswith(".Lfunc_end") or re.match(r"^_Z\S*:", l):
        break
    body.append(l)
ins = [l.split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ins)
tot = len(ins)
valu = sum(v for k, v in c.items() if k.startswith("v_"))
print(f"{key}: {tot} instructions, {valu} VALU, {sum(v for k, v in c.items() if k.startswith('s_'))} SALU")
for k, v in c.most_common(40):
    print(f"  {k:28s} {v}")
