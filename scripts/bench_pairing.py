"""Pairing latency / throughput probe (run under rocprofv3 for per-kernel times):
python scripts/bench_pairing.py [reps] [batch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import pbf  # noqa: E402

G1G = (1, 2)
G2G = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
       (8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531))


def main(reps=5, batch=4096):
    ctx = pbf.Context(0)
    neg = (1, pbf.BN254_Q - 2)
    assert ctx.pairing_check_bn254([G1G, neg], [G2G, G2G])
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.pairing_check_bn254([G1G, neg], [G2G, G2G])
    print("pairing check ms", (time.perf_counter() - t0) * 1e3 / reps)
    g1 = pbf.ints_to_limbs([c for _ in range(batch) for c in G1G])
    g2 = pbf.ints_to_limbs([c for _ in range(batch) for c in (G2G[0][0], G2G[0][1], G2G[1][0], G2G[1][1])])
    d1, d2 = torch.from_numpy(g1.view(np.int64)).cuda(), torch.from_numpy(g2.view(np.int64)).cuda()
    dout = torch.empty(batch * 48, dtype=torch.int64, device="cuda")
    ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), batch, dout.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), batch, dout.data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("batch", batch, "ms", dt * 1e3, "pairings/s", batch / dt)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
