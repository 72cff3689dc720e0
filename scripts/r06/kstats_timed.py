#!/usr/bin/env python3
"""Round 6: kernel statistics of the TIMED steps only, from a rocprofv3
--kernel-trace csv of scripts/r06/ntt_steps.py: the warm-up kernels end before a >= 3 ms idle gap,
the timed ones follow it. Prints per-kernel count / mean / total over the timed steps, the sum of
the kernels' busy time per step (their union on the timeline) and the timed window per step."""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2])
rows = [r for r in csv.DictReader(open(path)) if "ntt" in r["Kernel_Name"]]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
cut = 0
for i in range(1, len(ev)):
    if ev[i][0] - max(e for _, e, _ in ev[:i][-64:]) > 3_000_000:  # ns
        cut = i
timed = ev[cut:]
stats = {}
for s, e, n in timed:
    k = n.split("(")[0][:90]
    stats.setdefault(k, []).append((e - s) / 1e3)
span = (max(e for _, e, _ in timed) - timed[0][0]) / 1e3
busy, cur_s, cur_e = 0.0, None, None
for s, e, _ in timed:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += (cur_e - cur_s) / 1e3
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += (cur_e - cur_s) / 1e3
print(f"timed kernels: {len(timed)} over {steps} steps (warm-up kernels before the idle gap: {cut})")
for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:90s} calls {len(v):4d}  mean {sum(v) / len(v):8.1f} us  per step {sum(v) / steps:8.1f} us")
print(f"per step: kernel-union busy {busy / steps:.1f} us, window (first start .. last end) {span / steps:.1f} us")
