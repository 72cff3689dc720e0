"""BN254-Fr oracle self-checks (CPU): the fft.rs restatement over Fr agrees with the
iterative checker, inverts, and mul_ntt == schoolbook (the fft.rs:171-183 property)."""
import random

import bn254


def test_root_orders():
    for k in (1, 5, 23, 28):
        w = bn254.root_of_unity(1 << k)
        assert pow(w, 1 << k, bn254.R) == 1 and pow(w, 1 << (k - 1), bn254.R) != 1


def test_ct_fft_matches_iterative_and_inverts():
    rnd = random.Random(1)
    for k in range(1, 8):
        n = 1 << k
        w = bn254.root_of_unity(n)
        a = [rnd.randrange(bn254.R) for _ in range(n)]
        f = bn254.ct_fft(a, w)
        assert f == bn254.ntt(a, w)
        assert bn254.ct_fft_inv(f, w) == a
        assert bn254.ntt(f, w, inverse=True) == a


def test_mul_ntt_equals_schoolbook():
    rnd = random.Random(2)
    for k in (2, 5, 8):
        n = 1 << k
        a = [rnd.randrange(bn254.R) for _ in range(n // 2)]
        b = [rnd.randrange(bn254.R) for _ in range(n // 2)]
        c = bn254.mul_ntt(a, b, bn254.root_of_unity(n))
        assert bn254.normalize(c) == bn254.poly_mul(a, b)


def test_limb_roundtrip():
    a = bn254.random_limbs(100, 3)
    ints = bn254.limbs_to_ints(a)
    assert all(0 <= x < bn254.R for x in ints)
    assert (bn254.ints_to_limbs(ints) == a).all()


def test_g1_oracle_group_law():
    g = bn254.G1_GEN
    assert bn254.g1_on_curve(g)
    assert bn254.g1_mul(g, bn254.R) is None  # G1 has prime order r
    assert bn254.g1_add(bn254.g1_mul(g, 5), bn254.g1_mul(g, 7)) == bn254.g1_mul(g, 12)
    assert bn254.g1_on_curve(bn254.g1_mul(g, 123456789))
