"""MSM timings of one library build (PBF_LIB selects it) over a fixed list of cases, for A/B
between builds: python scripts/r04/msm_lib_ab.py [LOG_N ...]. Cases per size: the windowed MSM,
the fixed-base MSM at the size's default window width with the raw-flush accumulation off and on."""
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
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return r, round(ts[len(ts) // 2], 3)


def main(log_ns):
    ctx = pbf.Context(0)
    lib = os.path.basename(os.environ.get("PBF_LIB", "libpbf.so"))
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
        ref, tw = med(lambda: ctx.msm_g1_dev(pts.data_ptr(), s.data_ptr(), m), reps)
        out = {"lib": lib, "log_n": log_n, "windowed_ms": tw}
        for rf in ("0", "1"):
            os.environ["PBF_MSM_RAWFLUSH"] = rf
            ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m)
            r, tf = med(lambda: ctx.msm_g1_fixed_dev(pts.data_ptr(), m, s.data_ptr(), m), reps)
            out["fixed_rawflush%s_ms" % rf] = tf
            out["equal%s" % rf] = r == ref
        os.environ.pop("PBF_MSM_RAWFLUSH", None)
        print(json.dumps(out), flush=True)
        ctx.release_caches()
        del pts, s
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [20])
