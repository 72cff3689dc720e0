#!/usr/bin/env python3
"""Config-5 prover timing: synthetic 2^k-gate mul circuit generated on the device, SRS on the
device, prove (mode 1 = paper linearisation) timed after a warm-up, then one verify.
Usage: bench_prover.py LOG_N [LOG_N ...]  -> one JSON line per size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402

G2 = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
       11559732032986387107991004021392285783925812861821192530917403151452391805634),
      (8495653923123431417604973247489272438418190587263600148770280649306958101930,
       4082367875863433681332203403145435568316851327593401208105741076214120093531))


def breakdown(ctx, fn) -> dict:
    """Per-round wall times of one proof: context option prover.timing = 1 makes the prover synchronise its
    stream at each round mark and print it on stderr (csrc/prover.hip Prover::mark); fd 2 is
    captured around the call. The marks serialise the proof, so their sum exceeds prove_ms."""
    import tempfile

    ctx.set_option("prover.timing", 1)
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode="w+b") as tf:
        os.dup2(tf.fileno(), 2)
        try:
            fn()
            torch.cuda.synchronize()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
            ctx.set_option("prover.timing", None)
        tf.seek(0)
        text = tf.read().decode(errors="replace")
    out = {}
    for line in text.splitlines():
        if line.startswith("[pbf prover]"):
            body = line[len("[pbf prover]"):].rsplit(None, 2)
            if len(body) == 3 and body[2] == "ms":
                out[body[0].strip()] = float(body[1])
    return out


def run(ctx, log_n: int, reps: int = 2, mode: int = 1, verify: bool = True, no_key: bool = True,
        rounds: bool = True) -> dict:
    n = 1 << log_n
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0005, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    srs_m = (n + 3) if mode == 1 else (2 * n + 2)
    s = 0x5EED0005C0FFEE
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    t0 = time.perf_counter()
    ctx.srs_create_dev(s, srs_m - 1, dsrs.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    t_srs = time.perf_counter() - t0
    chal = [0x1111 * (i + 3) for i in range(5)]
    rnd = [0x2222 * (i + 5) for i in range(9)]
    ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m,
                              mode=mode, stream=sp)  # warm-up (plans, buffers)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):  # each proof returns to the host (its 9 points and 7 fields)
        t0 = time.perf_counter()
        pts, fs = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                            dsrs.data_ptr(), srs_m, mode=mode, stream=sp)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    t_prove = ts[len(ts) // 2]
    out = {"log_n": log_n, "gates": n, "mode": mode,
           "mode_name": "paper linearisation" if mode == 1 else "the reference's r_3 (plonk.rs:414-416)",
           "prove_ms": t_prove * 1e3, "prove_ms_min": ts[0] * 1e3,
           "prove_ms_max": ts[-1] * 1e3, "reps": reps, "proofs_per_s": 1 / t_prove,
           "proving_key": "preprocessed q_*, s_sigma_*, l1 (coefficients + coset evaluations) kept in the "
                          "context per circuit, validated against device copies of q / copies every proof",
           "srs_create_ms": t_srs * 1e3}
    if no_key:
        # the same proof with the circuit's preprocessing (8 INTTs + 9 coset NTTs of the
        # selector / permutation / l1 polynomials) recomputed per proof, as the reference does
        ctx.set_option("prover.pk", 0)
        tc = []
        try:
            for _ in range(max(3, reps // 2)):
                t0 = time.perf_counter()
                pts_c, fs_c = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                                        dsrs.data_ptr(), srs_m, mode=mode, stream=sp)
                torch.cuda.synchronize()
                tc.append(time.perf_counter() - t0)
        finally:
            ctx.set_option("prover.pk", None)
        tc.sort()
        t_cold = tc[len(tc) // 2]
        out.update({"prove_ms_no_key": t_cold * 1e3, "proofs_per_s_no_key": 1 / t_cold, "reps_no_key": len(tc),
                    "same_proof_with_and_without_key": bool(np.array_equal(np.asarray(pts_c), np.asarray(pts))
                                                            and np.array_equal(np.asarray(fs_c), np.asarray(fs)))})
    if rounds:
        out["rounds_ms"] = breakdown(ctx, lambda: ctx.plonk_prove_bn254_dev(
            n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m, mode=mode,
            stream=sp))
        out["rounds_note"] = ("one proof with a stream synchronisation at every round mark "
                              "(option prover.timing): where the time goes, not the overlapped total")
    if verify:
        import ctypes

        g2 = ctx.g2_bn254_mul([G2], [s])[0]
        g2l = pbf._g2_limbs([G2, g2])
        ok = ctypes.c_int(-1)
        tv = []
        for _ in range(6):  # the first call builds the verification key (8 commitments)
            t0 = time.perf_counter()
            pbf._check(ctx.lib.pbf_plonk_verify_bn254_dev(ctx.h, n, dq.data_ptr(), dc.data_ptr(), dsrs.data_ptr(),
                                                          srs_m, pbf._ptr(g2l), pbf._ptr(pts), pbf._ptr(fs),
                                                          pbf._ptr(pbf.ints_to_limbs(chal)),
                                                          pbf._ptr(pbf.ints_to_limbs([12345])),
                                                          pbf._ptr(pbf.ints_to_limbs([2, 3])), mode, ctypes.byref(ok),
                                                          sp))
            tv.append((time.perf_counter() - t0) * 1e3)
            if ok.value != 1:
                break
        out["verify_ms_no_key"] = tv[0]
        out["verify_ms"] = sorted(tv[1:])[len(tv[1:]) // 2] if len(tv) > 1 else tv[0]
        out["verified"] = ok.value == 1
    return out


def throughput(log_n: int, streams: int, proofs: int = 8, mode: int = 1) -> dict:
    """Proofs/s with `streams` proofs in flight: one context, torch stream and host thread each
    (a prover serving many witnesses of one circuit), all reading the same device-resident
    circuit, witness and SRS. Every context warms up first (plans, proving key, SRS window
    table); then each thread runs `proofs` proofs back to back, and the wall time from the
    common start to the last proof's completion gives the rate. The proofs of all threads must
    be identical (same inputs)."""
    import threading

    n = 1 << log_n
    base = pbf.Context(0)
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    base.plonk_synth_circuit_dev(n, 0x5EED0005, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    srs_m = (n + 3) if mode == 1 else (2 * n + 2)
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    base.srs_create_dev(0x5EED0005C0FFEE, srs_m - 1, dsrs.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    base.close()
    chal = [0x1111 * (i + 3) for i in range(5)]
    rnd = [0x2222 * (i + 5) for i in range(9)]
    ctxs = [pbf.Context(0) for _ in range(streams)]
    sts = [torch.cuda.Stream() for _ in range(streams)]
    results = [None] * streams
    go = threading.Barrier(streams + 1)

    def prove(k):
        return ctxs[k].plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                             dsrs.data_ptr(), srs_m, mode=mode, stream=sts[k].cuda_stream)

    def worker(k):
        prove(k)  # warm-up
        sts[k].synchronize()
        go.wait()
        for _ in range(proofs):
            results[k] = prove(k)  # returns after the proof's points and fields reached the host
        sts[k].synchronize()

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(streams)]
    for t in ts:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    same = all(np.array_equal(results[0][0], r[0]) and np.array_equal(results[0][1], r[1]) for r in results)
    for c in ctxs:
        c.close()
    return {"log_n": log_n, "streams": streams, "proofs": streams * proofs, "wall_s": wall,
            "proofs_per_s": streams * proofs / wall, "ms_per_proof": wall / (streams * proofs) * 1e3,
            "identical_proofs": bool(same)}


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--throughput":  # --throughput LOG_N K [K ...]
        for k in sys.argv[3:]:
            print(json.dumps(throughput(int(sys.argv[2]), int(k))), flush=True)
        sys.exit(0)
    ctx = pbf.Context(0)
    for a in sys.argv[1:]:
        print(json.dumps(run(ctx, int(a))), flush=True)
