"""K proofs of the synthetic 2^LOG_N-gate circuit, nothing else (a profiling target):
python scripts/r04/prove_only.py LOG_N K"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import torch  # noqa: E402

import pbf  # noqa: E402


def main(log_n, k):
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
    for _ in range(k + 1):  # the first builds the proving key and the SRS table
        ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m,
                                  mode=1, stream=sp)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]))
