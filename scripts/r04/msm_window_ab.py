"""A/B of the fixed-base MSM window width (PBF_MSM_FX_C, csrc/msm.hip FxGeom) and of the sort's
digit widths: python scripts/r04/msm_window_ab.py LOG_N [LOG_N ...]

For every size: random points (P_i = t_i G) and uniformly random scalars, the windowed MSM's
result as the reference, then the fixed-base MSM per window width c (table rebuilt per c; the
first call is the build and is not timed): median / min wall ms of `reps` calls (each call ends
in a D2H sync of the result), and whether the result equals the reference. One JSON line per
(size, variant)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402


def timed(fn, reps):
    ts = []
    r = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return r, ts[len(ts) // 2], ts[0]


def main(log_ns):
    ctx = pbf.Context(0)
    for log_n in log_ns:
        m = 1 << log_n
        reps = 10 if log_n <= 22 else 5
        rng = np.random.default_rng(4 + log_n)
        top = np.uint64(pbf.BN254_R >> 192)
        sc = rng.integers(0, 1 << 64, size=(m, 4), dtype=np.uint64)
        sc[:, 3] %= top
        s = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
        t = torch.from_numpy(rng.integers(1, 1 << 62, size=(m, 4), dtype=np.uint64).reshape(-1).view(np.int64)).cuda()
        pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
        ctx.g1_mul_base_dev(t.data_ptr(), pts.data_ptr(), m)
        torch.cuda.synchronize()
        del t
        for w8 in ("0", "1"):
            if w8 == "1":
                os.environ["PBF_MSM_SORT_W8"] = "1"
            else:
                os.environ.pop("PBF_MSM_SORT_W8", None)
            ref, med, mn = timed(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m), reps)
            print(json.dumps({"log_n": log_n, "variant": "windowed" + (" sort-w8" if w8 == "1" else ""),
                              "ms_median": round(med, 3), "ms_min": round(mn, 3)}), flush=True)
        os.environ.pop("PBF_MSM_SORT_W8", None)
        ctx.release_caches()
        torch.cuda.empty_cache()
        for c, env in ((16, {}), (16, {"PBF_MSM_RAWFLUSH": "0"}), (16, {"PBF_MSM_CHUNK_JOIN": "0"}), (18, {}),
                       (20, {}), (20, {"PBF_MSM_RAWFLUSH": "0"}), (20, {"PBF_MSM_CD_QUAD": "1"}), (22, {})):
            os.environ["PBF_MSM_FX_C"] = str(c)
            for k in ("PBF_MSM_RAWFLUSH", "PBF_MSM_CHUNK_JOIN", "PBF_MSM_CD_QUAD"):
                os.environ.pop(k, None)
            os.environ.update(env)
            t0 = time.perf_counter()
            ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)  # table build
            build = (time.perf_counter() - t0) * 1e3
            r, med, mn = timed(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m), reps)
            print(json.dumps({"log_n": log_n, "variant": "fixed c=%d %s" % (c, env), "ms_median": round(med, 3),
                              "ms_min": round(mn, 3), "first_call_ms": round(build, 1), "equal": r == ref}),
                  flush=True)
            ctx.release_caches()
            torch.cuda.empty_cache()
        for k in ("PBF_MSM_FX_C", "PBF_MSM_RAWFLUSH", "PBF_MSM_CHUNK_JOIN", "PBF_MSM_CD_QUAD"):
            os.environ.pop(k, None)
        del pts, s
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [20])
