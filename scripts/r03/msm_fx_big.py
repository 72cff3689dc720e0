#!/usr/bin/env python3
"""Round 3: fixed-base MSM median (HIP events) at 2^LOG points (argv[1], default 24), with the
fixed-base sort's first pass from 16-bit digit codes (PBF_MSM_FUSED_SORT=1, the default) and
from (key, value) pairs (=0); the two results must agree."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402
from bench import _median_ms  # noqa: E402

log = int(sys.argv[1]) if len(sys.argv) > 1 else 24
m = 1 << log
ctx = pbf.Context(0)
rng = np.random.default_rng(5)
top = np.uint64(pbf.BN254_R >> 192)
sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
sc[:, 3] %= top
s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m, stream=sp)
torch.cuda.synchronize()
res = {}
for rep in range(2):
    for fused in ("1", "0"):
        os.environ["PBF_MSM_FUSED_SORT"] = fused
        res[fused] = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp)
        f = _median_ms(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp),
                       reps=11 if log <= 22 else 5)
        print(f"2^{log} fixed-base PBF_MSM_FUSED_SORT={fused}  {f['ms']:.3f} ms (min {f['ms_min']:.3f})", flush=True)
print("same result", res["0"] == res["1"])
sys.exit(0 if res["0"] == res["1"] else 1)
