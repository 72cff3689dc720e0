#!/usr/bin/env python3
"""Round 3: a short 2^20-point MSM workload for PMC passes (two windowed, two fixed-base)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

ctx = pbf.Context(0)
m = 1 << 20
rng = np.random.default_rng(4)
top = np.uint64(pbf.BN254_R >> 192)
sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
sc[:, 3] %= top
s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m, stream=sp)
for _ in range(2):
    ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp)
for _ in range(2):
    ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp)
torch.cuda.synchronize()
print("ok")
