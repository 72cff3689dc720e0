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

    assert arr("K_GX") == limbs(c["GAMMA_X"][0]) + limbs(c["GAMMA_X"][1])
    assert arr("K_GY") == limbs(c["GAMMA_Y"][0]) + limbs(c["GAMMA_Y"][1])
    frob = arr("K_FROB2")
    assert frob[0] == 1 and frob[1:] == sum((limbs(g[0]) for g in c["FROB2"][1:]), [])
    assert arr("K_HARD") == limbs(c["HARD"], 12)
    assert c["ATE"] == (1 << 64) + int(re.search(r"K_ATE_LO = 0x([0-9a-f]+)ull", src).group(1), 16)
    assert (c["GAMMA_X"], c["GAMMA_Y"]) == (B.GAMMA_X, B.GAMMA_Y)
