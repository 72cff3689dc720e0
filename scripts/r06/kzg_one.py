#!/usr/bin/env python3
"""Round 6: one fixed-base (KZG) MSM at 2^k points (default 24) after its table build, three
warm-up commits and a 1 s idle (for scripts/r06/prover_timeline.py's last-gap cut)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
m = 1 << log_n
ctx = pbf.Context(0)
rng = np.random.default_rng(6 + log_n)
top = np.uint64(pbf.BN254_R >> 192)
sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
sc[:, 3] %= top
s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m)
for _ in range(4):
    ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)
torch.cuda.synchronize()
time.sleep(1.0)
t0 = time.perf_counter()
ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)
torch.cuda.synchronize()
print("kzg_ms %.2f" % ((time.perf_counter() - t0) * 1e3), flush=True)
