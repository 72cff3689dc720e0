#!/usr/bin/env python3
"""Round 6: MSM timings of one library build (PBF_LIB selects it): windowed MSM at 2^20, the
fixed-base (KZG) MSM at 2^20 / 2^22 / 2^24 points; medians of host-timed synchronous calls, and
the results (to compare builds bit for bit). Prints one JSON line."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402


def med(fn, reps):
    ts, r = [], None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return r, round(ts[len(ts) // 2], 3)


ctx = pbf.Context(0)
out = {"lib": os.path.basename(os.environ.get("PBF_LIB", "libpbf.so"))}
h = hashlib.sha256()
for log_n in (20, 22, 24):
    m = 1 << log_n
    rng = np.random.default_rng(6 + log_n)
    top = np.uint64(pbf.BN254_R >> 192)
    sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
    sc[:, 3] %= top
    s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
    t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
    pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
    ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m)
    if log_n == 20:
        r, ms = med(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m), 11)
        out["windowed_2p20_ms"] = ms
        h.update(repr(r).encode())
    ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)  # table build
    r, ms = med(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m), 11 if log_n < 24 else 7)
    out[f"fixed_2p{log_n}_ms"] = ms
    h.update(repr(r).encode())
    ctx.release_caches()
    del s, t, pts
    torch.cuda.empty_cache()
out["results_sha"] = h.hexdigest()[:16]
print(json.dumps(out), flush=True)
