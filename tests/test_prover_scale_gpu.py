"""Config 5 at BASELINE's proofs/s size: a 2^20-gate proof through the C-ABI
(pbf_plonk_prove_bn254_dev / pbf_plonk_verify_bn254_dev), checked by properties that do
not need an O(n^2) oracle:
* all 7 proof field elements (a_z, b_z, c_z, s_sigma_1_z, s_sigma_2_z, r_z, z_omega_z)
  recomputed in O(n) from the witness by oracle/plonk_bn254.py:commitment_scalars (the
  barycentric form of plonk.rs:393-422; pinned to the literal oracle and its fixtures in
  tests/test_prover_oracle.py), in both modes;
* the quotient's divisibility: the prover fails with PBF_EINVAL unless coefficients
  3n+6.. of t(x) and the remainders of W_z / W_zw are all zero (plonk.rs:370, 438, 442),
  so a successful return certifies them;
* all 9 commitments exactly, in both modes: SRS = [s^i]G with s known, so a_s = [a(s)]G
  etc. with a(s) from the same barycentric form at s (oracle/plonk_bn254.py:
  commitment_scalars); t_lo / t_mid / t_hi through [t(s)]G = t_lo + s^(n+2) t_mid +
  s^(2n+4) t_hi, W_z and W_zw through their division identities at s;
* the verifier: the paper-mode proof verifies, a proof with a changed evaluation or a
  swapped commitment does not. (The reference-mode proof is pinned by its evaluations and
  commitments but is expected NOT to verify: with the reference's r_3(x) an honest proof
  verifies only when k3 = (a_z + beta s1_z + gamma)(b_z + beta s2_z + gamma) alpha = 0, as in the
  reference's n = 4 KAT where (b_z + beta s2_z + gamma) = 170 = 0 mod 17)
"""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bn254_pairing as B  # noqa: E402
import plonk_bn254 as P  # noqa: E402

pytestmark = pytest.mark.gpu


def _points(flat):
    """9 x 8 u64 limbs -> affine int tuples ((0, 0) -> None, the GPU's identity encoding)."""
    import pbf

    v = pbf.limbs_to_ints(np.asarray(flat, dtype=np.uint64).reshape(-1))
    out = []
    for k in range(len(v) // 2):
        x, y = v[2 * k], v[2 * k + 1]
        out.append(None if (x, y) == (0, 0) else (x, y))
    return out


def _ints(t, width):
    import pbf

    a = t.cpu().numpy().view(np.uint64)
    return pbf.limbs_to_ints(a) if width == 4 else a


@pytest.mark.parametrize("log_n", [20])
def test_prove_2p20_gates(ctx, log_n):
    import torch

    import pbf

    n = 1 << log_n
    rng = random.Random(0x5EED0005)
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0005, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    s = rng.randrange(2, P.R)
    srs_m = 2 * n + 2  # long enough for both modes
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    ctx.srs_create_dev(s, srs_m - 1, dsrs.data_ptr(), stream=sp)
    g2s = [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]]
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    u = rng.randrange(P.R)

    pts, fs = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                        srs_m, mode=1, stream=sp)
    chal1 = list(chal)
    pts0, fs0 = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal1, rnd,
                                          dsrs.data_ptr(), srs_m, mode=0, stream=sp)
    torch.cuda.synchronize()

    # commitments: accept, then reject a changed evaluation and a swapped commitment
    verify = lambda p, f, c, md: ctx.plonk_verify_bn254_dev(  # noqa: E731
        n, dq.data_ptr(), dc.data_ptr(), dsrs.data_ptr(), srs_m, g2s, p, f, c, u, mode=md, stream=sp)
    assert verify(pts, fs, chal, 1)
    bad_f = fs.copy()
    bad_f[0] ^= 1  # a_z + / - 1
    assert not verify(pts, bad_f, chal, 1)
    bad_p = pts.copy().reshape(9, 8)
    bad_p[[0, 1]] = bad_p[[1, 0]]  # a_s <-> b_s
    assert not verify(bad_p.reshape(-1), fs, chal, 1)
    assert not verify(pts0, fs0, chal1, 0)  # the reference's r_3: k3 != 0 here

    # field elements and all 9 commitments: O(n) recomputation from the witness and the SRS
    # secret s (oracle/plonk_bn254.py:commitment_scalars, pinned to the literal oracle's
    # proofs in tests/test_prover_oracle.py), in both modes
    qv = _ints(dq, 4)
    q = tuple(qv[i * n:(i + 1) * n] for i in range(5))
    cv = _ints(dc, 2).reshape(3, n, 2)
    copies = tuple([(int(k), int(i)) for k, i in cv[col]] for col in range(3))
    av = _ints(dabc, 4)
    abc = tuple(av[i * n:(i + 1) * n] for i in range(3))
    cs = P.commitment_scalars(n, q, copies, abc, chal, rnd, s)
    assert pbf.limbs_to_ints(fs) == cs["paper"]["fields"]
    assert pbf.limbs_to_ints(fs0) == cs["reference"]["fields"]
    for md, p in (("paper", pts), ("reference", pts0)):
        res = P.commitments_match(n, _points(p), cs[md], s, chal[3])
        assert all(res.values()), (md, res)


def test_synth_circuit_matches_host_restatement(ctx):
    """pbf_plonk_synth_circuit_bn254_dev equals its host restatement (oracle/prover_cpu.cpp
    oracle_synth_circuit), which generates the 2^24-gate fixture's circuit."""
    import torch

    import oracle

    n = 1 << 12
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0024, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr())
    torch.cuda.synchronize()
    q, c, abc = oracle.synth_circuit(n, 0x5EED0024)
    for dev, host in ((dq, q), (dc, c), (dabc, abc)):
        assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)


def test_prove_2p24_gates(ctx):
    """BASELINE config 5 at its own size on one GPU: 2^24 gates, paper mode. The proof is
    pinned exactly: its 7 field elements and all 9 commitments against the scalars the O(n)
    checker computed in the container for the same seeded circuit, SRS secret, challenges and
    blinders (tests/golden/prove_2p24.json, tests/golden/gen_prove_2p24.py:
    oracle_commitment_scalars = oracle/plonk_bn254.py commitment_scalars restated in C++).
    The prover's built-in checks (constraints satisfied, t(x) divisible by Z_H with
    coefficients 3n+6.. zero, zero remainders of W_z / W_zw: plonk.rs:199, 370, 438, 442) pass,
    the proof verifies, and a changed evaluation or two swapped commitments are rejected."""
    import torch

    n = 1 << 24
    rng = random.Random(0x5EED0024)
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0024, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    s = rng.randrange(2, P.R)
    srs_m = n + 3
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    ctx.srs_create_dev(s, srs_m - 1, dsrs.data_ptr(), stream=sp)
    g2s = [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]]
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    u = rng.randrange(P.R)
    pts, fs = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                        srs_m, mode=1, stream=sp)
    torch.cuda.synchronize()
    import json
    import os

    import pbf

    with open(os.path.join(os.path.dirname(__file__), "golden", "prove_2p24.json")) as fh:
        gold = json.load(fh)
    assert (gold["log_n"], gold["seed"], int(gold["s"])) == (24, 0x5EED0024, s)
    assert [int(x) for x in gold["chal"]] == chal and [int(x) for x in gold["rnd"]] == rnd
    assert pbf.limbs_to_ints(fs) == [int(x) for x in gold["paper"]["fields"]]
    cs = {k: int(v) for k, v in gold["paper"].items() if k != "fields"}
    res = P.commitments_match(n, _points(pts), cs, s, chal[3])
    assert all(res.values()), res
    verify = lambda p, f: ctx.plonk_verify_bn254_dev(  # noqa: E731
        n, dq.data_ptr(), dc.data_ptr(), dsrs.data_ptr(), srs_m, g2s, p, f, chal, u, mode=1, stream=sp)
    assert verify(pts, fs)
    bad_f = fs.copy()
    bad_f[5 * 4] ^= 1  # r_z
    assert not verify(pts, bad_f)
    bad_p = pts.copy().reshape(9, 8)
    bad_p[[4, 6]] = bad_p[[6, 4]]  # t_lo <-> t_hi
    assert not verify(bad_p.reshape(-1), fs)
    ctx.release_caches()  # ~24 GB of proving key; later tests start from a clean context


def test_prove_2p24_gates_8_virtual_ranks():
    """Config 5 in its specified form -- 2^24 gates with the work split over 8 ranks -- as 8
    virtual ranks on this one GPU (pbf_plonk_prove_bn254_multi_dev, device-copy exchanges),
    bit-exact against the single-GPU proof of the same inputs. Prints the device bytes in use
    with the 8 ranks' contexts alive (what 8 real GPUs would each hold is about 1/8 of it plus
    the shared inputs)."""
    import torch

    import pbf

    n, G = 1 << 24, 8
    rng = random.Random(0x5EED0024)
    single = pbf.Context(0)
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    single.plonk_synth_circuit_dev(n, 0x5EED0024, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    s = rng.randrange(2, P.R)
    srs_m = n + 3
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    single.srs_create_dev(s, srs_m - 1, dsrs.data_ptr(), stream=sp)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    ref = single.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                       srs_m, mode=1, stream=sp)
    torch.cuda.synchronize()
    single.close()
    free0, total = torch.cuda.mem_get_info()
    ranks = [pbf.Context(0) for _ in range(G)]
    try:
        pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks, n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                                  [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m,
                                                  mode=1)
        free1, _ = torch.cuda.mem_get_info()
        print(f"\n[2^24 x 8 virtual ranks] device bytes in use: {(total - free1) / 2**30:.1f} GiB of "
              f"{total / 2**30:.1f} GiB (inputs + SRS {(total - free0) / 2**30:.1f} GiB); per rank "
              f"{(free0 - free1) / G / 2**30:.1f} GiB")
        assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1])
    finally:
        for c in ranks:
            c.close()
