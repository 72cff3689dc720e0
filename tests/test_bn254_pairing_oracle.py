"""The BN254 pairing oracle (oracle/bn254_pairing.py) is a correct reduced pairing:
its tower construction equals an independent flat-Fq12 restatement, it is bilinear and
non-degenerate, and the constants hard-coded in csrc/pairing.hip match their definition
(scripts/gen_pairing_constants.py). The BN254 pairing value itself is not pinned by a
reference test (the reference only pairs its toy curve, src/pbh/pairing.rs:56-75):
"parity unpinned" beyond these properties, SURVEY.md §8c."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import bn254_pairing as B  # noqa: E402


def test_generators_on_curve_and_order_r():
    assert B.g2_on_curve(B.G2_GEN)
    assert B.g2_mul(B.G2_GEN, B.R) is None
    assert (B.G1_GEN[1] ** 2 - B.G1_GEN[0] ** 3 - 3) % B.Q == 0


def test_tower_pairing_equals_flat_restatement():
    p, q = B.g1_mul(B.G1_GEN, 12345), B.g2_mul(B.G2_GEN, 678)
    assert B.tower_to_flat(B.pairing(p, q)) == B.pairing_flat(p, q)


def test_bilinear_nondegenerate_order_r():
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.F12_ONE
    assert B.f12_pow(e, B.R) == B.F12_ONE
    a, b = 0x1234567, 0xABCDEF
    assert B.pairing(B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)) == B.f12_pow(e, a * b)


def test_pairing_check_kzg_identity():
    # e(s P, Q) * e(-P, s Q) == 1; perturbed -> False
    s = 987654321
    p, q = B.g1_mul(B.G1_GEN, 3), B.g2_mul(B.G2_GEN, 5)
    assert B.pairing_check([(B.g1_mul(p, s), q), (B.g1_neg(p), B.g2_mul(q, s))])
    assert not B.pairing_check([(B.g1_mul(p, s + 1), q), (B.g1_neg(p), B.g2_mul(q, s))])


def test_device_constants_match_definition():
    import gen_pairing_constants as G

    c = G.constants()
    src = open(os.path.join(ROOT, "plonk-by-fingers_amd", "csrc", "pairing.hip")).read()

    def arr(name):
        m = re.search(name + r"\[[^=]*=\s*\{(.*?)\};", src, re.S)
        return [int(x, 16) for x in re.findall(r"0x([0-9a-f]+)ull", m.group(1))]

    def limbs(x, n=4):
        return [(x >> (64 * i)) & ((1 << 64) - 1) for i in range(n)]

    frob1 = arr("K_FROB1")
    assert frob1 == sum((limbs(g[0]) + limbs(g[1]) for g in c["FROB1"]), [])
    assert (c["FROB1"][2], c["FROB1"][3]) == (B.GAMMA_X, B.GAMMA_Y)
    frob = arr("K_FROB2")
    assert frob[0] == 1 and frob[1:] == sum((limbs(g[0]) for g in c["FROB2"][1:]), [])
    assert arr("K_R3") == limbs(c["R3"])
    assert c["ATE"] == (1 << 64) + int(re.search(r"K_ATE_LO = 0x([0-9a-f]+)ull", src).group(1), 16)
    assert c["U"] == int(re.search(r"K_BN_U = 0x([0-9a-f]+)ull", src).group(1), 16)
    # the device's hard part uses (q^4 - q^2 + 1)/r = l0 + l1 q + l2 q^2 + l3 q^3 exactly
    lam = c["HARD_LAMBDA"]
    assert sum(l * B.Q ** i for i, l in enumerate(lam)) == c["HARD"]


def _frob1(a, G):
    (a0, a1, a2), (b0, b1, b2) = a
    cj = B.f2_conj
    return ((cj(a0), B.f2_mul(cj(a1), G[2]), B.f2_mul(cj(a2), G[4])),
            (B.f2_mul(cj(b0), G[1]), B.f2_mul(cj(b1), G[3]), B.f2_mul(cj(b2), G[5])))


def test_u_chain_final_exponentiation_is_exact():
    """The device's final exponentiation schedule (csrc/pairing.hip final_exp_w: easy part,
    three exponentiations by u, small powers, Frobenius maps, conjugations) restated on the
    oracle's tower, equal to the literal f^((q^12-1)/r) of oracle/bn254_pairing.py."""
    import random

    import gen_pairing_constants as Gc

    G = Gc.constants()["FROB1"]
    sq, mul, conj = B.f12_sqr, B.f12_mul, B.f12_conj

    def powu(x):
        r = x
        for bit in bin(B.BN_U)[3:]:
            r = sq(r)
            if bit == "1":
                r = mul(r, x)
        return r

    def fe(f):
        f = mul(conj(f), B.f12_inv(f))
        f = mul(_frob1(_frob1(f, G), G), f)
        a = powu(f)
        b = powu(a)
        c = powu(b)
        c4 = sq(sq(c))
        c36 = mul(sq(sq(sq(c4))), c4)
        b2 = sq(b)
        b6 = mul(sq(b2), b2)
        b12 = sq(b6)
        b18, b30 = mul(b12, b6), mul(sq(b12), b6)
        a2 = sq(a)
        a6 = mul(sq(a2), a2)
        a12 = sq(a6)
        a18 = mul(a12, a6)
        t0 = conj(mul(mul(mul(c36, b30), a18), sq(f)))
        t1 = mul(conj(mul(mul(c36, b18), a12)), f)
        t2 = mul(b6, f)
        f3 = _frob1(_frob1(_frob1(f, G), G), G)
        return mul(mul(mul(t0, _frob1(t1, G)), _frob1(_frob1(t2, G), G)), f3)

    rng = random.Random(7)
    f = tuple(tuple((rng.randrange(B.Q), rng.randrange(B.Q)) for _ in range(3)) for _ in range(2))
    assert fe(f) == B.final_exp(f)
