"""Generalised PLONK prover / verifier over BN254 on the GPU (csrc/prover.hip, BASELINE
config 5) through the C-ABI: bit-exact proofs (9 commitments + 7 evaluations) against
the literal restatement of Plonk::prove (oracle/plonk_bn254.py) via the committed
fixtures (tests/golden/gen_plonk_golden.py), in both modes; prove -> verify at scale
(the paper-mode proofs verify, tampered proofs do not); the reference's asserts as
error codes."""
import json
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bn254_pairing as B  # noqa: E402
import plonk_bn254 as P  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "plonk_bn254.json")))["cases"]
MODES = {"reference": 0, "paper": 1}


@pytest.fixture(scope="module")
def ctx():
    import pbf

    c = pbf.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("case", GOLD, ids=[f"n{c['n']}-{c['mode']}" for c in GOLD])
def test_proof_matches_restatement(ctx, case):
    n = case["n"]
    q, cp, abc = P.mul_gates_circuit(n, case["circuit_seed"])
    srs = ctx.srs_create(case["s"], case["srs_n"])
    pts, fs = ctx.plonk_prove_bn254(q, cp, abc, case["chal"], case["rnd"], srs, mode=MODES[case["mode"]])
    assert fs == case["fields"]
    assert [list(p) if p else None for p in pts] == case["pts"]
    g2s = [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [case["s"]])[0]]
    ok = ctx.plonk_verify_bn254(q, cp, srs, g2s, pts, fs, case["chal"], case["u"], mode=MODES[case["mode"]])
    assert ok == case["verify"]


@pytest.mark.parametrize("log_n", [10, 14])
def test_prove_verify_at_scale(ctx, log_n):
    n = 1 << log_n
    rng = random.Random(log_n)
    s = rng.randrange(1, P.R)
    q, cp, abc = P.mul_gates_circuit(n, 0x5EED0005)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    srs = ctx.srs_create(s, n + 3)
    pts, fs = ctx.plonk_prove_bn254(q, cp, abc, chal, rnd, srs, mode=1)
    g2s = [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]]
    assert ctx.plonk_verify_bn254(q, cp, srs, g2s, pts, fs, chal, 987654321, mode=1)
    bad = list(fs)
    bad[0] = (bad[0] + 1) % P.R
    assert not ctx.plonk_verify_bn254(q, cp, srs, g2s, pts, bad, chal, 987654321, mode=1)
    # rounds 1-4 of the two modes agree (only r_3(x) differs)
    chal1 = [1] + chal[1:]
    srs2 = ctx.srs_create(s, 2 * n + 2)
    pts0, fs0 = ctx.plonk_prove_bn254(q, cp, abc, chal1, rnd, srs2, mode=0)
    pts1, fs1 = ctx.plonk_prove_bn254(q, cp, abc, chal1, rnd, srs2, mode=1)
    assert fs0[:5] == fs1[:5] and pts0[:7] == pts1[:7]  # rounds 1-4 do not depend on the mode


def test_unsatisfied_circuit_rejected(ctx):
    import pbf

    n = 8
    q, cp, abc = P.mul_gates_circuit(n, 1)
    c = list(abc[2])
    c[3] = (c[3] + 1) % P.R
    srs = ctx.srs_create(5, 2 * n + 2)
    with pytest.raises(pbf.PbfError):
        ctx.plonk_prove_bn254(q, cp, (abc[0], abc[1], c), [1, 2, 3, 4, 5], list(range(1, 10)), srs)


def test_short_srs_rejected(ctx):
    import pbf

    n = 8
    q, cp, abc = P.mul_gates_circuit(n, 1)
    srs = ctx.srs_create(5, n)
    with pytest.raises(pbf.PbfError):
        ctx.plonk_prove_bn254(q, cp, abc, [1, 2, 3, 4, 5], list(range(1, 10)), srs, mode=0)


def test_challenge_on_the_evaluation_coset(ctx):
    """The openings divide by (x - z) and (x - z w) on the coefficients (synthetic
    division), so a challenge z on the prover's 4n-point coset g H_4n (or with z w there)
    still gives the reference's proof (its long division, plonk.rs:430-442, has no such
    case); the proof matches the literal oracle."""
    import bn254 as F

    n = 8
    q, cp, abc = P.mul_gates_circuit(n, 3)
    s = 0x1234567
    srs_n = n + 3
    rng = random.Random(8)
    w4n = F.root_of_unity(4 * n)
    for z in (5 * pow(w4n, 3, P.R) % P.R, 5 * pow(w4n, 9, P.R) * pow(F.root_of_unity(n), n - 1, P.R) % P.R):
        chal = [rng.randrange(P.R) for _ in range(3)] + [z, rng.randrange(P.R)]
        rnd = [rng.randrange(P.R) for _ in range(9)]
        st = P.Setup(n, s, srs_n)
        want_pts, want_f, _ = P.prove(st, q, cp, abc, chal, rnd, mode="paper")
        srs = ctx.srs_create(s, srs_n)
        pts, fs = ctx.plonk_prove_bn254(q, cp, abc, chal, rnd, srs, mode=1)
        assert fs == [x % P.R for x in want_f]
        assert [list(p) if p else None for p in pts] == [list(p) if p else None for p in want_pts]


def test_proving_key_cache_matches_cold_proofs():
    """The context keeps the preprocessed polynomials (q_*, s_sigma_*, l1: coefficients and
    coset evaluations) per circuit, checked by fingerprints of the gates and copies on every
    call. Proofs over interleaved circuits and sizes (A A B A C A) on one context equal the
    proofs of the same inputs with every preprocessing step recomputed (option prover.pk = 0)."""
    import pbf

    rng = random.Random(4242)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    circ = {"A": (64, 11), "B": (64, 12), "C": (128, 11)}
    order = ["A", "A", "B", "A", "C", "A"]
    warm = pbf.Context(0)
    try:
        srs = warm.srs_create(77, 2 * 128 + 2)
        got = []
        for name in order:
            n, seed = circ[name]
            got.append(warm.plonk_prove_bn254(*P.mul_gates_circuit(n, seed), chal, rnd, srs, mode=1))
    finally:
        warm.close()
    cold = pbf.Context(0, options={"prover.pk": 0})
    try:
        srs = cold.srs_create(77, 2 * 128 + 2)
        ref = {name: cold.plonk_prove_bn254(*P.mul_gates_circuit(*circ[name]), chal, rnd, srs, mode=1) for name in circ}
    finally:
        cold.close()
    assert got == [ref[name] for name in order]
    assert ref["A"] != ref["B"]


def test_verification_key_cache(ctx):
    """The verifier keeps the 8 preprocessed commitments per (circuit, SRS), fingerprint-
    checked on every call: accept / reject over interleaved inputs (the proof against a
    circuit with one selector changed, with two copy labels swapped, against another SRS)
    equals the answers with the commitments recomputed per call (option verifier.vk = 0)."""
    rng = random.Random(777)
    n = 64
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    s1, s2 = 1234567, 7654321
    srs1, srs2 = ctx.srs_create(s1, n + 3), ctx.srs_create(s2, n + 3)
    g2 = {s: [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]] for s in (s1, s2)}
    q, cp, abc = P.mul_gates_circuit(n, 21)
    q_mod = [list(col) for col in q]
    q_mod[4][0] = (q_mod[4][0] + 1) % P.R
    cp_mod = [list(col) for col in cp]
    cp_mod[0][0], cp_mod[0][1] = cp_mod[0][1], cp_mod[0][0]
    pa = ctx.plonk_prove_bn254(q, cp, abc, chal, rnd, srs1, mode=1)
    pa2 = ctx.plonk_prove_bn254(q, cp, abc, chal, rnd, srs2, mode=1)
    runs = [(q, cp, srs1, s1, pa), (q_mod, cp, srs1, s1, pa), (q, cp_mod, srs1, s1, pa), (q, cp, srs1, s1, pa),
            (q, cp, srs2, s2, pa2), (q, cp, srs2, s2, pa), (q, cp, srs1, s1, pa)]

    def answers():
        return [ctx.plonk_verify_bn254(qq, cc, srs, g2[s], pr[0], pr[1], chal, 99, mode=1)
                for qq, cc, srs, s, pr in runs]

    warm = answers()
    ctx.set_option("verifier.vk", 0)
    try:
        cold = answers()
    finally:
        ctx.set_option("verifier.vk", None)
    assert warm == cold, (warm, cold)
    assert warm == [True, False, False, True, True, False, True], warm


def test_shared_snapshots_across_caches(ctx):
    """The proving key, the verification key and the MSM window table validate against ONE
    device copy per input (q, copies, the SRS points; ADVICE r03: no duplicate copies). A cache
    must still be rebuilt when ANOTHER consumer replaced the shared copy: interleave prove /
    verify over two circuits and two SRSs with stand-alone fixed-base MSMs over other points,
    and every answer equals the cold one."""
    import numpy as np
    import torch

    import bn254

    rng = random.Random(31337)
    n = 64
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    s1, s2 = 1111, 2222
    srs1, srs2 = ctx.srs_create(s1, n + 3), ctx.srs_create(s2, n + 3)
    g2 = {s: [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]] for s in (s1, s2)}
    A, Bc = P.mul_gates_circuit(n, 51), P.mul_gates_circuit(n, 52)
    other = [bn254.g1_mul(bn254.G1_GEN, 5 + i) for i in range(n + 3)]  # same count as the SRS
    sc = [rng.randrange(P.R) for _ in range(n + 3)]
    dp = torch.from_numpy(bn254.ints_to_limbs([v for p in other for v in p]).view(np.int64)).cuda()
    ds = torch.from_numpy(bn254.ints_to_limbs(sc).view(np.int64)).cuda()
    msm_ref = bn254.msm_naive(other, sc)

    def msm():
        assert ctx.msm_g1_fixed_dev(dp.data_ptr(), n + 3, ds.data_ptr(), n + 3) == msm_ref

    pa1 = ctx.plonk_prove_bn254(*A, chal, rnd, srs1, mode=1)
    ver = lambda circ, srs, s, pr: ctx.plonk_verify_bn254(circ[0], circ[1], srs, g2[s], pr[0], pr[1], chal, 5,  # noqa
                                                          mode=1)
    assert ver(A, srs1, s1, pa1)
    msm()                                                       # g1pts <- other points
    assert ctx.plonk_prove_bn254(*A, chal, rnd, srs1, mode=1) == pa1
    pb2 = ctx.plonk_prove_bn254(*Bc, chal, rnd, srs2, mode=1)   # q, copies <- B; g1pts <- srs2
    assert ver(A, srs1, s1, pa1)                                # vk rebuilt for A / srs1
    assert not ver(A, srs1, s1, pb2)
    msm()
    assert ver(Bc, srs2, s2, pb2)
    assert ctx.plonk_prove_bn254(*A, chal, rnd, srs1, mode=1) == pa1
    msm()
    assert ctx.plonk_prove_bn254(*Bc, chal, rnd, srs2, mode=1) == pb2




@pytest.mark.parametrize("n", [1024, 4096])
def test_coset_prefix_transforms_match_32bit_padded(n):
    """The coset transforms read only the written prefix of each 4n slot (29-bit passes, round 6)
    or get the zero padding written first (option ntt256.l29 = 0: the 32-bit passes): the same
    proof either way, with and without the proving-key cache."""
    import pbf

    rng = random.Random(n)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    proofs = []
    for opts in ({}, {"ntt256.l29": "0"}, {"prover.pk": 0}):
        c = pbf.Context(0, options=opts)
        try:
            srs = c.srs_create(91, n + 3)
            proofs.append(c.plonk_prove_bn254(*P.mul_gates_circuit(n, 5), chal, rnd, srs, mode=1))
        finally:
            c.close()
    assert proofs[0] == proofs[1] == proofs[2]
