#!/usr/bin/env python3
"""Round 6: W warm-up steps then K timed steps of the bench workload (batched forward Goldilocks
NTT, HBM-resident, bench.py's buffer rotation), for a kernel trace whose timed steps can be told
apart: a 5 ms idle gap (host sleep after a synchronisation) separates the warm-up kernels from the
timed ones. Prints the event-timed ms per step of the K steps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import pbf  # noqa: E402

log_n, B, W, K = (int(x) for x in sys.argv[1:5])
ctx = pbf.Context(0)
sp = torch.cuda.current_stream().cuda_stream
step, _ = bench._single_gpu(ctx, 1 << log_n, B, sp)
for _ in range(W):
    step()
torch.cuda.synchronize()
time.sleep(0.005)
st = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(K):
    step()
e1.record(st)
torch.cuda.synchronize()
print(f"log_n {log_n} batch {B} warmup {W} steps {K} ms_per_step {e0.elapsed_time(e1) / K:.4f}")
ctx.close()
