#!/usr/bin/env python3
"""Round 6 diagnostic: is the headline's driver window bound by the host's enqueue rate? From a
cold start (2 s idle), per step: the GPU interval between HIP events (as ramp.py) and the host
time spent inside the step call (Python + ctypes + the library's launches), both averaged over
the same windows. Prints one JSON line."""
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
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
opts = dict(kv.split("=") for kv in os.environ.get("RAMP_OPTS", "").split(",") if kv)
ctx = pbf.Context(0, options=opts)
sp = torch.cuda.current_stream().cuda_stream
step, _ = bench._single_gpu(ctx, 1 << log_n, B, sp)
torch.cuda.synchronize()
time.sleep(2.0)
st = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
host = []
ev[0].record(st)
for i in range(steps):
    t0 = time.perf_counter()
    step()
    host.append((time.perf_counter() - t0) * 1e3)
    ev[i + 1].record(st)
torch.cuda.synchronize()
gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]


def mean(a):
    return round(sum(a) / len(a), 4)


out = {"log_n": log_n, "batch": B, "opts": opts}
for name, a, b in (("1_5", 1, 5), ("5_25", 5, 25), ("25_50", 25, 50), ("50_100", 50, 100), ("100_200", 100, 200)):
    out["gpu_" + name] = mean(gpu[a:b])
    out["host_" + name] = mean(host[a:b])
out["host_first5"] = [round(x, 4) for x in host[:5]]
print(json.dumps(out))
ctx.close()
