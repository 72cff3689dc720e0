#!/usr/bin/env python3
"""Profiling target: config 3 (fused mul_ntt at 2^23) REPS times with the 29-bit passes (default) or
the 32-bit ones (argv[1] = 32)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
form = sys.argv[1] if len(sys.argv) > 1 else "29"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = pbf.Context(0, options={"ntt256.l29": "0"} if form == "32" else None)
la = 1 << 22
n = 2 * la
w = pow(5, (R - 1) // n, R)
rng = np.random.default_rng(3)
A = torch.zeros(n * 4, dtype=torch.int64, device="cuda")
B = torch.zeros_like(A)
for d in (A, B):
    a = rng.integers(0, 1 << 64, size=(la, 4), dtype=np.uint64)
    a[:, 3] %= np.uint64(R >> 192)
    d[: la * 4] = torch.from_numpy(a.reshape(-1).view(np.int64)).cuda()
C = torch.empty_like(A)
sp = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    ctx.mul_ntt_fr_dev(w, A.data_ptr(), B.data_ptr(), C.data_ptr(), n, 1, stream=sp)
torch.cuda.synchronize()
ctx.close()
