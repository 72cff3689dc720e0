"""Pairing-check latency (config 4's KZG check: 2 pairs, prepared G2 lines reused): host round
trip and device time (HIP events on the context's stream), medians of 101 calls."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import pbf  # noqa: E402

G1G = (1, 2)
G2G = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
       (8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531))
negG1 = (1, pbf.BN254_Q - 2)
ctx = pbf.Context(0)
assert ctx.pairing_check_bn254([G1G, negG1], [G2G, G2G])
assert not ctx.pairing_check_bn254([G1G, G1G], [G2G, G2G])
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
dev, wall = [], []
for _ in range(101):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    ok = ctx.pairing_check_bn254([G1G, negG1], [G2G, G2G])
    e1.record()
    torch.cuda.synchronize()
    wall.append((time.perf_counter() - t0) * 1e3)
    dev.append(e0.elapsed_time(e1))
    assert ok
dev.sort()
wall.sort()
print(json.dumps({"device_ms_median": dev[50], "device_ms_min": dev[0], "host_wall_ms_median": wall[50],
                  "env": {k: v for k, v in os.environ.items() if k.startswith("PBF_")}}))
