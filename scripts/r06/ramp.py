#!/usr/bin/env python3
"""Round 6 diagnostic: per-step time of the headline NTT (2^20 x 32) from a cold start, HIP
events around every step, to see how long the clocks take to settle (bench.py --warmup 5
against 200). Prints one JSON line: step times in ms (and a few summary means)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import pbf  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
idle = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
opts = dict(kv.split("=") for kv in os.environ.get("RAMP_OPTS", "").split(",") if kv)
ctx = pbf.Context(0, options=opts)
sp = torch.cuda.current_stream().cuda_stream
step, _ = bench._single_gpu(ctx, 1 << log_n, B, sp)
torch.cuda.synchronize()
time.sleep(idle)  # let the GPU idle first, as before the driver's timed region
st = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
ev[0].record(st)
for i in range(steps):
    step()
    ev[i + 1].record(st)
torch.cuda.synchronize()
ts = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
def mean(a):
    return sum(a) / len(a)
print(json.dumps({"log_n": log_n, "batch": B, "opts": opts,
                  "first5": [round(x, 4) for x in ts[:5]], "mean_5_25": round(mean(ts[5:25]), 4),
                  "mean_25_50": round(mean(ts[25:50]), 4), "mean_50_100": round(mean(ts[50:100]), 4),
                  "mean_200_300": round(mean(ts[200:300]), 4) if steps >= 300 else None,
                  "per10": [round(mean(ts[i:i + 10]), 4) for i in range(0, steps, 10)]}))
ctx.close()
