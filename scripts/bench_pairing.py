#!/usr/bin/env python3
"""BN254 pairing timings: the 2-pair KZG check (first call: prepared G2 lines built;
later calls: reused), and a batch of independent pairings. One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

G1G = (1, 2)
G2G = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
       (8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531))


def main():
    ctx = pbf.Context(0)
    neg = (1, pbf.BN254_Q - 2)
    out = {}
    t0 = time.perf_counter()
    ok = ctx.pairing_check_bn254([G1G, neg], [G2G, G2G])
    out["check_first_ms"] = (time.perf_counter() - t0) * 1e3
    ts = []
    for _ in range(21):
        t0 = time.perf_counter()
        ok = ok and ctx.pairing_check_bn254([G1G, neg], [G2G, G2G])
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    out["check_median_ms"] = ts[len(ts) // 2]
    out["check_min_ms"] = ts[0]
    out["ok"] = bool(ok)
    bad = ctx.pairing_check_bn254([G1G, G1G], [G2G, G2G])
    out["reject_ok"] = not bad
    npair = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    g1 = pbf.ints_to_limbs([c for _ in range(npair) for c in G1G])
    g2 = pbf.ints_to_limbs([c for _ in range(npair) for c in (G2G[0][0], G2G[0][1], G2G[1][0], G2G[1][1])])
    d1, d2 = torch.from_numpy(g1.view(np.int64)).cuda(), torch.from_numpy(g2.view(np.int64)).cuda()
    dout = torch.empty(npair * 48, dtype=torch.int64, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), npair, dout.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), npair, dout.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["batch"] = npair
    out["batch_ms"] = dt * 1e3
    out["pairings_per_s"] = npair / dt
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
