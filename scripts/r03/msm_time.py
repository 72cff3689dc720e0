#!/usr/bin/env python3
"""Round 3: 2^20-point MSM timings (windowed with host / device Horner, fixed-base KZG form),
medians of 11 after warm-ups, HIP events on the current stream around each synchronous call."""
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
print("windowed host Horner", _median_ms(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp), reps=11))
for seq in ("2", "4", "16"):
    os.environ["PBF_MSM_CD_SEQ"] = seq
    rs = ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp)
    print(f"windowed cd_seq={seq}", _median_ms(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp),
                                               reps=11), "same result", rs == r0)
del os.environ["PBF_MSM_CD_SEQ"]
os.environ["PBF_MSM_DEVICE_HORNER"] = "1"
r1 = ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp)
print("windowed device Horner", _median_ms(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp), reps=11),
      "same result", r0 == r1)
del os.environ["PBF_MSM_DEVICE_HORNER"]
ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp)
rf = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp)
print("fixed-base", _median_ms(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp), reps=11),
      "same result", rf == r0)
os.environ["PBF_MSM_QUAD"] = "0"
print("windowed single-lane tail", _median_ms(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp), reps=11),
      "same result", ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m, stream=sp) == r0)
print("fixed-base single-lane tail", _median_ms(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp), reps=11),
      "same result", ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m, stream=sp) == r0)
del os.environ["PBF_MSM_QUAD"]
