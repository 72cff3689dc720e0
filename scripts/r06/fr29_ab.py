#!/usr/bin/env python3
"""Round 6: the 29-bit-limb Fr pass kernels (default) against the 32-bit ones (option
ntt256.l29 = 0), alternating on one box: config 3 (degree-2^22 x 2^22 product by the fused
mul_ntt, NTT size 2^23) and a batch of 4 forward transforms of 2^26 points (the 2^24-gate
proof's coset NTTs), event-timed medians; the outputs of both forms compared. One JSON line
per form and round."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def rand(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 1 << 64, size=(n, 4), dtype=np.uint64)
    a[:, 3] %= np.uint64(R >> 192)
    return torch.from_numpy(a.reshape(-1).view(np.int64)).cuda()


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return round(ts[len(ts) // 2], 4)


la = 1 << 22
n3 = 2 * la
w3 = pow(5, (R - 1) // n3, R)
A = torch.zeros(n3 * 4, dtype=torch.int64, device="cuda")
B = torch.zeros_like(A)
A[: la * 4] = rand(la, 3)
B[: la * 4] = rand(la, 4)
n26 = 1 << 26
w26 = pow(5, (R - 1) // n26, R)
X = rand(4 * n26, 5)
Y = torch.empty_like(X)
C = torch.empty_like(A)
digest = {}
for rnd in range(2):
    for form in ("32", "29"):
        ctx = pbf.Context(0, options={"ntt256.l29": "0"} if form == "32" else None)
        sp = torch.cuda.current_stream().cuda_stream
        t3 = timed(lambda: ctx.mul_ntt_fr_dev(w3, A.data_ptr(), B.data_ptr(), C.data_ptr(), n3, 1, stream=sp), 10)
        t26 = timed(lambda: ctx.ntt_fr_batch_dev(w26, X.data_ptr(), Y.data_ptr(), n26, 4, stream=sp), 5)
        ti26 = timed(lambda: ctx.ntt_fr_batch_dev(w26, X.data_ptr(), Y.data_ptr(), n26, 1, inverse=True, stream=sp), 5)
        torch.cuda.synchronize()
        h = hash((C.cpu().numpy().tobytes()[:1 << 20], Y.cpu().numpy().tobytes()[:1 << 20]))
        digest.setdefault(rnd, set()).add(h)
        print(json.dumps({"form": form, "config3_mul_ntt_ms": t3, "fwd_2p26_x4_ms": t26, "inv_2p26_ms": ti26}), flush=True)
        ctx.close()
print(json.dumps({"same_outputs": all(len(v) == 1 for v in digest.values())}))
