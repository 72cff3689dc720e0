"""Fr NTT per-pass twiddle tables against the two-level tables, per PBF_NTT256_TWLOG (the largest
per-pass table, log2 entries): config-3 product (NTT size 2^23) and proofs at 2^20 / 2^24 gates.
python scripts/r04/ntt256_twlog_ab.py TWLOG [TWLOG ...]; every setting must give the same bytes."""
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

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def config3(ctx, reps=20):
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        ctx.mul_ntt_fr_dev(w, da.data_ptr(), db.data_ptr(), dc.data_ptr(), n, 1, stream=sp)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2], ts[0], hashlib.sha256(dc.cpu().numpy().tobytes()).hexdigest()[:16]


def prove(ctx, log_n, reps):
    n = 1 << log_n
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0005, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    srs_m = n + 3
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    ctx.srs_create_dev(0x5EED0005C0FFEE, srs_m - 1, dsrs.data_ptr(), stream=sp)
    chal = [0x1111 * (i + 3) for i in range(5)]
    rnd = [0x2222 * (i + 5) for i in range(9)]
    args = (n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m)
    ctx.plonk_prove_bn254_dev(*args, mode=1, stream=sp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        pts, fs = ctx.plonk_prove_bn254_dev(*args, mode=1, stream=sp)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    h = hashlib.sha256(np.asarray(pts).tobytes() + np.asarray(fs).tobytes()).hexdigest()[:16]
    return ts[len(ts) // 2], ts[0], h


def main(twlogs):
    for tl in twlogs:
        os.environ["PBF_NTT256_TWLOG"] = str(tl)
        ctx = pbf.Context(0)
        out = {"twlog": tl}
        out["config3_ms"], out["config3_min"], out["config3_sha"] = config3(ctx)
        if os.environ.get("AB_CONFIG3_ONLY"):
            print(json.dumps(out), flush=True)
            ctx.close()
            continue
        out["prove20_ms"], out["prove20_min"], out["prove20_sha"] = prove(ctx, 20, 10)
        print(json.dumps(out), flush=True)
        out["prove24_ms"], out["prove24_min"], out["prove24_sha"] = prove(ctx, 24, 3)
        print(json.dumps(out), flush=True)
        ctx.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [20, 24, 26])
