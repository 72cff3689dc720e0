#!/usr/bin/env python3
"""Batched BN254 pairing throughput: the lane-per-pairing engine (default from 64 pairs) at
several batch sizes against the workgroup engine (PBF_PAIR_LANE=0), distinct random P_i and
Q_i (Q_i repeat with period 4096 at the larger batches), HIP-event device time. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

G2G = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
       (8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531))


def main():
    ctx = pbf.Context(0)
    sp = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(7)
    nq = 4096
    qs = ctx.g2_bn254_mul([G2G] * nq, [int(x) for x in rng.integers(1, 1 << 62, size=nq)])
    g2 = pbf.ints_to_limbs([c for q in qs for c in (q[0][0], q[0][1], q[1][0], q[1][1])])
    out = {}
    for npair in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,16384,65536").split(",")]:
        sc = rng.integers(0, 1 << 62, size=(npair, 4), dtype=np.uint64)
        sc[:, 3] = 0
        dsc = torch.from_numpy(sc.reshape(-1).view(np.int64)).cuda()
        d1 = torch.empty(npair * 8, dtype=torch.int64, device="cuda")
        ctx.g1_mul_base_dev(dsc.data_ptr(), d1.data_ptr(), npair, stream=sp)
        reps = (npair + nq - 1) // nq
        d2 = torch.from_numpy(np.tile(g2, reps)[: npair * 16].view(np.int64)).cuda()
        dout = torch.empty(npair * 48, dtype=torch.int64, device="cuda")
        for eng in ("1", "0") if npair <= 4096 else ("1",):
            os.environ["PBF_PAIR_LANE"] = eng
            ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), npair, dout.data_ptr(), stream=sp)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(3):
                e0.record()
                ctx.pairing_bn254_dev(d1.data_ptr(), d2.data_ptr(), npair, dout.data_ptr(), stream=sp)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            key = f"{'lane' if eng == '1' else 'workgroup'}_{npair}"
            out[key] = {"ms": ts[1], "pairings_per_s": npair / (ts[1] / 1e3)}
            if npair <= 4096:
                out[key]["digest"] = int(dout[:4800].sum().item()) & 0xFFFFFFFF
        os.environ.pop("PBF_PAIR_LANE", None)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
