#!/usr/bin/env python3
"""Config 3 workload alone (profiling target): degree-2^22 x 2^22 BN254-Fr product by
mul_ntt (NTT size 2^23), REPS times. Usage: run_polymul.py [REPS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
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
    for _ in range(reps):
        ctx.mul_ntt_fr_dev(w, da.data_ptr(), db.data_ptr(), dc.data_ptr(), n, 1, stream=sp)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
