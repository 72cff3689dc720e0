#!/usr/bin/env python3
"""Round 3: 2^20-point windowed and fixed-base MSM medians (HIP events, 11 reps) of the
library PBF_LIB points at, and the results' agreement with the default library's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402
from bench import _median_ms  # noqa: E402

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
torch.cuda.synchronize()
r0 = ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp)
r1 = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp)
w = _median_ms(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp), reps=11)
f = _median_ms(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp), reps=11)
lib = os.path.basename(os.environ.get("PBF_LIB", "libpbf.so"))
print(f"{lib:18s} windowed {w['ms']:.3f} ms  fixed-base {f['ms']:.3f} ms  result {hex(r0[0][0] if isinstance(r0[0], list) else 0)[:6]} same {r0 == r1}")
