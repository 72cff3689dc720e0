#!/usr/bin/env python3
"""Round 3: config-3 product (2^22 x 2^22 over BN254 Fr, NTT size 2^23) median of 11 with the
library PBF_LIB points at, and a checksum of its output for cross-library agreement."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402
from bench import _median_ms  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
ctx = pbf.Context(0)
sp = torch.cuda.current_stream().cuda_stream
la = 1 << 22
n = 2 * la
w = pow(5, (R - 1) // n, R)
da = torch.zeros(n * 4, dtype=torch.int64, device="cuda")
db = torch.zeros_like(da)
rng = np.random.default_rng(3)
for d in (da, db):
    a = rng.integers(0, 1 << 64, size=(la, 4), dtype=np.uint64)
    a[:, 3] %= np.uint64(R >> 192)
    d[: la * 4] = torch.from_numpy(a.reshape(-1).view(np.int64)).cuda()
dc = torch.empty_like(da)
ctx.mul_ntt_fr_dev(w, da.data_ptr(), db.data_ptr(), dc.data_ptr(), n, 1, stream=sp)
torch.cuda.synchronize()
h = hashlib.sha256(dc.cpu().numpy().tobytes()).hexdigest()[:16]
t = _median_ms(lambda: ctx.mul_ntt_fr_dev(w, da.data_ptr(), db.data_ptr(), dc.data_ptr(), n, 1, stream=sp), reps=11)
lib = os.path.basename(os.environ.get("PBF_LIB", "libpbf.so"))
print(f"{lib:18s} config-3 product {t['ms']:.3f} ms (min {t['ms_min']:.3f})  sha {h}")
