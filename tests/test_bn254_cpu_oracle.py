"""The C++ BN254 restatements behind the config-3/4 CPU baselines (oracle/bn254_cpu.cpp:
mul_ntt of fft.rs:109-132 with the recursion-faithful CooleyTurkey, the naive fold of
SRS::eval_at_s plonk.rs:51-58, an all-core Pippenger) agree with the Python oracle
(oracle/bn254.py), itself checked against the reference's KATs transcribed for the BN254
instantiation (tests/test_bn254_oracle.py)."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bn254  # noqa: E402
import oracle  # noqa: E402

R = bn254.R


def test_fr_mul_ntt_matches_python_oracle():
    rng = random.Random(7)
    for la, lb in ((64, 64), (100, 28), (1, 1), (3, 5)):
        a = [rng.randrange(R) for _ in range(la)]
        b = [rng.randrange(R) for _ in range(lb)]
        w = bn254.root_of_unity(la + lb)
        got = oracle._ints(oracle.fr_mul_ntt(oracle._limbs(a), oracle._limbs(b), w))
        assert got == bn254.mul_ntt(a, b, w), (la, lb)


def test_msm_naive_and_pippenger_match_python_oracle():
    rng = random.Random(8)
    ks = [rng.randrange(1, R) for _ in range(24)]
    sc = [rng.randrange(R) for _ in range(24)]
    sc[3] = 0
    sc[5] = R - 1
    pts = oracle.g1_mul_gen(oracle._limbs(ks))
    pts[7] = 0  # the identity (0, 0)
    py_pts = [bn254.g1_mul(bn254.G1_GEN, k) for k in ks]
    py_pts[7] = None
    assert [oracle._pts_out(r) for r in pts] == [None if p is None else tuple(p) for p in py_pts]
    want = bn254.msm_naive(py_pts, sc)
    want = None if want is None else tuple(want)
    assert oracle.g1_msm_naive(pts, oracle._limbs(sc)) == want
    for threads in (1, 4, 16):
        assert oracle.g1_msm_pippenger(pts, oracle._limbs(sc), threads) == want


def test_g1_progression():
    pts = oracle.g1_progression(5, 7, 6)
    assert [oracle._pts_out(r) for r in pts] == [tuple(bn254.g1_mul(bn254.G1_GEN, 5 + 7 * i)) for i in range(6)]
