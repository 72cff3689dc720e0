"""Fixed-base KZG MSM probe: python scripts/probe_msm_fixed.py [log_n] [reps]; prints the mean
wall ms per call and a result hash (compare variants with PBF_LIB). Run under rocprofv3
--kernel-trace for the per-kernel timeline (scripts/msm_timeline.py)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pbf  # noqa: E402


def main(log_n=20, reps=10):
    ctx = pbf.Context(0)
    m = 1 << log_n
    rng = np.random.default_rng(4)
    top = np.uint64(pbf.BN254_R >> 192)
    sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
    sc[:, 3] %= top
    s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
    t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
    pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
    ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m)
    torch.cuda.synchronize()
    r = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)
    r2 = ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m)
    print("fixed == windowed:", r == r2, "hash", hex(hash(r) & 0xFFFFFFFF))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)
        ts.append((time.perf_counter() - t0) * 1e3)
    print("fixed msm 2^%d ms median %.3f min %.3f" % (log_n, sorted(ts)[len(ts) // 2], min(ts)))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
