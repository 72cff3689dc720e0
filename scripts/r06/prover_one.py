#!/usr/bin/env python3
"""Round 6: one 2^k-gate proof (mode 1, proving key built) after two warm-up proofs and a 1 s idle
gap, for a kernel trace of that proof alone (scripts/r06/prover_timeline.py cuts at the gap)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import torch  # noqa: E402

import pbf  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = 1 << log_n
ctx = pbf.Context(0)
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


def prove():
    return ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                     srs_m, mode=1, stream=sp)


for _ in range(2):
    prove()
    torch.cuda.synchronize()
time.sleep(1.0)
t0 = time.perf_counter()
prove()
torch.cuda.synchronize()
print("proof_ms %.2f" % ((time.perf_counter() - t0) * 1e3), flush=True)
ctx.close()
