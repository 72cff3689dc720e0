"""The generic PLONK restatement (oracle/plonk.py) instantiated with the reference's own
PlonkByHandTypes (oracle/pbh_types.py = src/pbh/mod.rs:18-33) reproduces the reference's
end-to-end KAT: the 16-value proof of src/pbh/mod.rs:101-118 and verify == true at
:122-123. The BN254 checker of the GPU prover (oracle/plonk_bn254.py) runs the same
oracle/plonk.py code with BN254 types, so this pins its formulas to the reference."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pbh_types as T  # noqa: E402
import plonk as PL  # noqa: E402


def _setup(k):
    types = T.PlonkByHandTypes
    srs = PL.SRS(types, k["s"], k["srs_n"])  # SRS::create(f101(2), 6)
    return PL.Plonk(types, srs, k["omega_pows"])  # Plonk::new(srs, f17(4))


def _circuit(k):
    g = k["gates_qlqrqoqmqc"]
    q = tuple([row[i] for row in g] for i in range(5))
    copies = tuple([tuple(x) for x in col] for col in k["copies_kind_idx"])
    return q, copies, tuple(k["abc"])


def test_toy_group_kats(kats):
    # g1.rs:233-260, g2.rs:108-119, gt.rs:88-97 through the Python toy types
    g = T.G1_GEN
    two = T.g1_add(g, g)
    four = T.g1_add(two, two)
    eight = T.g1_add(four, four)
    assert two[:2] == (68, 74) and four[:2] == (65, 98) and eight[:2] == (18, 49)
    assert T.g1_add(eight, eight)[:2] == (1, 99) == T.g1_neg(g)[:2]
    assert T.g1_add(two, g)[:2] == (26, 45) and T.g1_add(four, g)[:2] == (12, 32)
    assert T.g1_mul(g, 6) == T.g1_add(T.g1_add(T.g1_add(two, two), g), g)
    assert T.g2_add(T.G2_GEN, T.G2_GEN) == (90, 82)
    assert T.gt_mul((26, 97), (93, 76)) == (97, 89)
    assert T.gt_pow((68, 47), 600) == (97, 89)
    x = (42, 49)
    assert T.gt_pow(x, 101) == T.gt_neg(x)


def test_toy_pairing_bilinear():
    # pairing.rs:56-75
    g, q = T.G1_GEN, T.G2_GEN
    e = T.pairing(g, q)
    assert e != (1, 0)
    assert T.pairing(T.g1_mul(g, 5), q) == T.pairing(g, T.g2_mul(q, 5)) == T.gt_pow(e, 5)
    assert T.pairing(T.g1_add(g, T.g1_mul(g, 4)), q) == T.gt_mul(e, T.pairing(T.g1_mul(g, 4), q))


def test_plonk_by_hand_proof_kat(kats):
    # pbh/mod.rs:44-124: the full proof, value for value, then verify == true
    k = kats["plonk_by_hand"]
    plonk = _setup(k)
    q, copies, abc = _circuit(k)
    pts, fields, _ = plonk.prove(q, copies, abc, k["challenge_alpha_beta_gamma_z_v"], k["rand"])
    assert [list(p[:2]) for p in pts] == k["expected_points"]
    assert all(not p[2] for p in pts)
    assert fields == k["expected_fields"]
    assert plonk.verify(q, copies, pts, fields, k["challenge_alpha_beta_gamma_z_v"], k["verify_u"])


def test_plonk_by_hand_rejects_tampering(kats):
    k = kats["plonk_by_hand"]
    plonk = _setup(k)
    q, copies, abc = _circuit(k)
    chal = k["challenge_alpha_beta_gamma_z_v"]
    pts, fields, _ = plonk.prove(q, copies, abc, chal, k["rand"])
    bad = list(fields)
    bad[5] = (bad[5] + 1) % 17  # r_z
    assert not plonk.verify(q, copies, pts, bad, chal, k["verify_u"])
    bad_pts = list(pts)
    bad_pts[0] = T.g1_add(pts[0], T.G1_GEN)  # a_s moved by G
    assert not plonk.verify(q, copies, bad_pts, fields, chal, k["verify_u"])
    # a witness that breaks a gate fails Constrains::satisfies (plonk.rs:199 assert)
    a2 = [list(x) for x in abc]
    a2[2][0] = (a2[2][0] + 1) % 17
    with pytest.raises(AssertionError):
        plonk.prove(q, copies, a2, chal, k["rand"])


def test_poly_quirks_literal():
    m = 15485863  # the poly.rs tests' field
    P = lambda c: PL.Poly(c, m)  # noqa: E731
    # poly.rs:429-435 schoolbook product
    assert (P([5, 0, 10, 6]) * P([1, 2, 4])).c == [5, 10, 30, 26, 52, 24]
    # SubAssign<&Poly> pushes +rhs where rhs is longer (poly.rs:196)
    assert (P([1]) - P([0, 7])).c == [1, 7]
    # p - f touches coefficient 0 only; zero scalar gives Poly::zero()
    assert (P([3, 4]) - 5).c == [m - 2, 4]
    assert (P([3, 4]) * 0).c == [0]
    # poly.rs:437-449: q * d + r == n
    n, d = P([1, 2, 3, 4, 5]), P([2, 1])
    qq, r = divmod(n, d)
    assert (qq * d + r) == n
    # 0 / 0 never enters the loop (poly.rs:234)
    assert divmod(P([0]), P([0])) == (P([0]), P([0]))
