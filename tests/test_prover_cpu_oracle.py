"""The host-side config-5 pieces of oracle/prover_cpu.cpp (test infrastructure; no GPU):

* oracle_plonk_prove_cpu, the generalised prover used as the CPU baseline,
  reproduces the literal restatement's committed proofs (tests/golden/plonk_bn254.json,
  oracle/plonk_bn254.py restating src/plonk.rs:191-466) in both modes, one core and all cores;
* oracle_commitment_scalars, the C++ O(n) checker that pins the 2^24-gate proof
  (tests/golden/prove_2p24.json), equals oracle/plonk_bn254.py commitment_scalars;
* oracle_fr_mul_ntt_par (the all-core config-3 baseline) equals the recursion-faithful
  oracle_fr_mul_ntt (fft.rs:109-132).
"""
import json
import os
import random

import numpy as np
import pytest

import bn254
import oracle
import plonk_bn254 as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = json.load(open(os.path.join(ROOT, "tests", "golden", "plonk_bn254.json")))["cases"]


def _limbs_circuit(q, cp, abc):
    qa = bn254.ints_to_limbs([x for col in q for x in col]).reshape(-1)
    ca = np.array([v for col in cp for (k, i) in col for v in (k, i)], dtype=np.uint64)
    aa = bn254.ints_to_limbs([x for col in abc for x in col]).reshape(-1)
    return qa, ca, aa


def _srs_limbs(s, count):
    return oracle.g1_mul_gen(bn254.ints_to_limbs([pow(s, i, bn254.R) for i in range(count)]))


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("case", CASES, ids=[f"n{c['n']}-{c['mode']}" for c in CASES])
def test_cpu_prover_matches_restatement(case, threads):
    n = case["n"]
    qa, ca, aa = _limbs_circuit(*P.mul_gates_circuit(n, case["circuit_seed"]))
    srs = _srs_limbs(case["s"], case["srs_n"] + 1)
    pts, fs = oracle.plonk_prove_cpu(n, qa, ca, aa, case["chal"], case["rnd"], srs,
                                     mode=0 if case["mode"] == "reference" else 1, threads=threads)
    assert bn254.limbs_to_ints(fs) == case["fields"]
    v = bn254.limbs_to_ints(pts)
    got = [None if (v[2 * i], v[2 * i + 1]) == (0, 0) else [v[2 * i], v[2 * i + 1]] for i in range(9)]
    assert got == case["pts"]


def test_cpu_commitment_scalars_match_python():
    n = 64
    rng = random.Random(64)
    q, cp, abc = P.mul_gates_circuit(n, 77)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    s = rng.randrange(2, P.R)
    want = P.commitment_scalars(n, q, cp, abc, chal, rnd, s)
    got = oracle.commitment_scalars_cpu(n, *_limbs_circuit(q, cp, abc), chal, rnd, s, threads=3)
    for md in ("reference", "paper"):
        for k, v in want[md].items():
            assert got[md][k] == v, (md, k)


def test_synth_circuit_satisfies_its_constraints():
    """The restated synthetic circuit (k_synth_circuit): every gate a*b = c with q_m = 1,
    q_o = -1, and the copy labels point at equal values."""
    n = 256
    q, c, abc = oracle.synth_circuit(n, 0x5EED0005, threads=2)
    qv = bn254.limbs_to_ints(q)
    av = bn254.limbs_to_ints(abc)
    a, b, cc = av[:n], av[n:2 * n], av[2 * n:]
    assert qv[2 * n:3 * n] == [P.R - 1] * n and qv[3 * n:4 * n] == [1] * n and not any(qv[:2 * n] + qv[4 * n:])
    assert all(x * y % P.R == z for x, y, z in zip(a, b, cc))
    cols = c.reshape(3, n, 2)
    for col in range(3):
        for i in range(n):
            kind, idx = int(cols[col, i, 0]), int(cols[col, i, 1])
            assert av[kind * n + idx - 1] == av[col * n + i]


def test_fr_mul_ntt_par_matches_recursion():
    la = lb = 1 << 9
    a = bn254.random_limbs(la, 5).reshape(-1, 4)
    b = bn254.random_limbs(lb, 6).reshape(-1, 4)
    w = bn254.root_of_unity(la + lb)
    assert np.array_equal(oracle.fr_mul_ntt_par(a, b, w, threads=4), oracle.fr_mul_ntt(a, b, w))
