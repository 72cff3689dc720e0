"""The 29-bit-limb Montgomery arithmetic of csrc/msm_l29.hpp (the MSM accumulation, round 3):
its constants against scripts/gen_l29_constants.py, and a Python restatement of its product
(product scanning, one 64-bit accumulator, no carry folds) against a b 2^-261 mod p, with the
64-bit column bound checked on the largest inputs the accumulation feeds it (normalised limbs,
values below 17.3p) and the lazily reduced madd-2008-s bounds of DESIGN.md §3.5 exercised on
random chains. CPU only."""
import os
import random
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import gen_l29_constants as G  # noqa: E402

P = G.P
MASK = (1 << 29) - 1
C = G.constants()


def test_header_constants_match_generator():
    src = open(os.path.join(ROOT, "plonk-by-fingers_amd", "csrc", "msm_l29.hpp")).read()
    for name, vals in C.items():
        m = re.search(r"constexpr uint32_t " + name + r"(?:\[9\])? = \{?([^;}]*)\}?;", src)
        assert m, name
        got = [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]
        assert got == vals, name


def limbs(v):
    return G.limbs(v)


def value(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def mul29(a, b):
    """csrc/msm_l29.hpp l29::mul, step for step."""
    p29, np29 = C["P29"], C["NP29"][0]
    m = [0] * 9
    r = [0] * 9
    acc = 0
    for k in range(17):
        lo, hi = (0, k) if k < 9 else (k - 8, 8)
        for i in range(lo, hi + 1):
            acc += a[i] * b[k - i]
        for i in range(lo, k if k < 9 else 9):
            acc += m[i] * p29[k - i]
        assert acc < 1 << 64, "column overflow"
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * np29) & MASK
            acc += m[k] * p29[0]
            assert acc & MASK == 0
        else:
            r[k - 9] = acc & MASK
        acc >>= 29
    r[8] = acc
    return r


def test_product_matches_montgomery():
    rinv = pow(2, -261, P)
    rng = random.Random(29)
    cases = [(0, 0), (1, 1), (P - 1, P - 1)]
    cases += [(rng.randrange(17 * P), rng.randrange(17 * P)) for _ in range(300)]
    cases += [(int(17.3 * P) - 1, int(17.3 * P) - 1)]
    for x, y in cases:
        r = mul29(limbs(x), limbs(y))
        assert value(r) % P == x * y * rinv % P
        assert all(v <= MASK for v in r[:8])
        assert value(r) < x * y // (1 << 261) + P + 1


def sqr29(a):
    """csrc/msm_l29.hpp l29::sqr, step for step: the doubled symmetric terms taken once."""
    p29, np29 = C["P29"], C["NP29"][0]
    a2 = [2 * v for v in a]
    m = [0] * 9
    r = [0] * 9
    acc = 0
    for k in range(17):
        lo = 0 if k < 9 else k - 8
        i = lo
        while i < k - i:
            acc += a[i] * a2[k - i]
            i += 1
        if k % 2 == 0:
            acc += a[k // 2] * a[k // 2]
        for i in range(lo, k if k < 9 else 9):
            acc += m[i] * p29[k - i]
        assert acc < 1 << 64, "column overflow"
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * np29) & MASK
            acc += m[k] * p29[0]
            assert acc & MASK == 0
        else:
            r[k - 9] = acc & MASK
        acc >>= 29
    r[8] = acc
    return r


def test_square_matches_product():
    """l29::sqr (PP = P^2, RR = R^2 of madd-2008-s) is bit-identical to l29::mul(a, a) up to the
    largest value a square takes (17.02 p) and at the 2^261 limit of the product's inputs."""
    rng = random.Random(261)
    cases = [0, 1, P - 1, int(17.02 * P), (1 << 261) - 1] + [rng.randrange(18 * P) for _ in range(500)]
    for x in cases:
        a = norm(limbs(x)) if x < 1 << 261 else limbs(x)
        assert sqr29(a) == mul29(a, a)


def norm(l):
    l = list(l)
    for i in range(8):
        l[i + 1] += l[i] >> 29
        l[i] &= MASK
    return l


def sub(a, b, M):
    r = [a[i] + M[i] - b[i] for i in range(9)]
    assert all(0 <= v < 1 << 32 for v in r), "limb borrow or overflow"
    return norm(r)


def times32(x):
    """csrc/msm_l29.hpp l29::times32, step for step (a run's first point: x 2^5 mod p)."""
    p29 = C["P29"]
    y = [(x[0] << 5) & MASK] + [((x[i] << 5) | (x[i - 1] >> 24)) & MASK for i in range(1, 9)]
    q = y[8] // (p29[8] + 1)
    r, c = [0] * 9, 0
    for i in range(9):
        v = y[i] - q * p29[i] + c
        r[i] = v & MASK
        c = v >> 29
    assert c == 0
    return r


def test_times32_start_of_run():
    """The run start's x 2^5 by shift and one estimated subtraction: the residue of the product
    by 2^266 it replaces, normalised, below 1.0001 p (inside the product's output bound)."""
    rng = random.Random(32)
    for x in [0, 1, P - 1, P // 2, (P * 31) // 32] + [rng.randrange(P) for _ in range(2000)]:
        r = times32(limbs(x))
        assert value(r) % P == x * 32 % P
        assert all(v <= MASK for v in r)
        assert value(r) < 1.0001 * P
        assert value(r) % P == value(mul29(limbs(x), limbs(pow(2, 266, P)))) % P


def test_lazy_madd_chain_bounds():
    """Random madd-2008-s chains in the kernel's domains and order: every intermediate stays
    within the derived bounds, and the chain's (X, Y, ZZ, ZZZ) agree with plain arithmetic."""
    rng = random.Random(7)
    one = limbs(pow(2, 266, P))
    for _ in range(20):
        X = Y = ZZ = ZZZ = None
        for step in range(40):
            x, y = rng.randrange(P), rng.randrange(P)
            x256, y256 = limbs(x * 2 ** 256 % P), limbs(y * 2 ** 256 % P)
            if X is None:
                X, Y = times32(x256), times32(y256)
                ZZ = ZZZ = one
                continue
            Pv = sub(mul29(x256, ZZ), X, C["M16P"])
            R = sub(mul29(y256, ZZZ), Y, C["M16P"])
            PP = sqr29(Pv)
            ZZ3 = mul29(ZZ, PP)
            PPP = mul29(Pv, PP)
            YP = mul29(Y, PPP)
            ZZZ = mul29(ZZZ, PPP)
            Q = mul29(X, PP)
            RR = sqr29(R)
            X3 = [RR[i] + C["M8P"][i] - PPP[i] - 2 * Q[i] for i in range(9)]
            assert all(0 <= v < 1 << 32 for v in X3)
            X3 = norm(X3)
            Y3 = sub(mul29(R, sub(Q, X3, C["M16P"])), YP, C["M8P"])
            # P = U2 - X with U2 = x ZZ 2^(256+266-261): the domains line up
            u2 = x * 2 ** 256 * value(ZZ) * pow(2, -261, P) % P
            assert value(Pv) % P == (u2 - value(X)) % P
            X, Y, ZZ = X3, Y3, ZZ3
            for v, bound in ((X, 11.3), (Y, 11.3), (ZZ, 1.03), (ZZZ, 1.03), (Pv, 17.02), (R, 17.02)):
                assert value(v) < bound * P


def mulsub29(a, b, c, d):
    """csrc/msm_l29.hpp l29::mulsub, step for step (round 6): a b - c d under ONE Montgomery
    reduction, p 2^261 added at columns 9..17 so the total stays positive; a signed 64-bit
    accumulator with arithmetic carries."""
    p29, np29 = C["P29"], C["NP29"][0]
    m = [0] * 9
    r = [0] * 9
    acc = 0
    for k in range(17):
        lo, hi = (0, k) if k < 9 else (k - 8, 8)
        for i in range(lo, hi + 1):
            acc += a[i] * b[k - i]
        for i in range(lo, hi + 1):
            acc -= c[i] * d[k - i]
        for i in range(lo, k if k < 9 else 9):
            acc += m[i] * p29[k - i]
        assert -(1 << 63) <= acc < 1 << 63, "signed column overflow"
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * np29) & MASK
            acc += m[k] * p29[0]
            assert acc & MASK == 0
        else:
            acc += p29[k - 9]
            r[k - 9] = acc & MASK
        acc >>= 29  # arithmetic, as the kernel's v_ashrrev_i64
    r[8] = acc + p29[8]
    assert r[8] >= 0
    return r


def test_mulsub_matches_montgomery():
    """(a b - c d) 2^-261 + p (mod p), normalised limbs, for the operand ranges madd-2008-s's Y3
    feeds it (R, Q - X3 below 17.3p; Y below 11.3p, PPP below 3.3p) and their extremes."""
    rinv = pow(2, -261, P)
    rng = random.Random(2026)
    cases = [(0, 0, 0, 0), (P - 1, P - 1, 0, 0), (0, 0, int(11.3 * P), int(3.3 * P)),
             (int(17.3 * P), int(17.3 * P), int(11.3 * P), int(3.3 * P))]
    cases += [(rng.randrange(int(17.3 * P)), rng.randrange(int(17.3 * P)), rng.randrange(int(11.3 * P)),
               rng.randrange(int(3.3 * P))) for _ in range(500)]
    for x, y, u, v in cases:
        r = mulsub29(limbs(x), limbs(y), limbs(u), limbs(v))
        assert value(r) % P == (x * y - u * v) * rinv % P
        assert all(0 <= t <= MASK for t in r[:8])
        assert 0 < value(r) < (x * y) // (1 << 261) + 2 * P + 1


def test_lazy_madd_chain_round6_matches_round5():
    """The round-6 madd (Y3 = R (Q - X3) - Y PPP under one reduction, plus p) against the round-5
    form (two products and a lazy difference), step for step over random chains in the kernel's
    domains: equal modulo p at every step, and every intermediate within its bound (Y now below
    4p instead of 11.3p; every product input still below 17.3p)."""
    rng = random.Random(66)
    one = limbs(pow(2, 266, P))
    for _ in range(20):
        X = Y = ZZ = ZZZ = None
        for step in range(40):
            x, y = rng.randrange(P), rng.randrange(P)
            x256, y256 = limbs(x * 2 ** 256 % P), limbs(y * 2 ** 256 % P)
            if X is None:
                X, Y = times32(x256), times32(y256)
                ZZ = ZZZ = one
                continue
            Pv = sub(mul29(x256, ZZ), X, C["M16P"])
            R = sub(mul29(y256, ZZZ), Y, C["M16P"])
            PP = sqr29(Pv)
            ZZ3 = mul29(ZZ, PP)
            PPP = mul29(Pv, PP)
            ZZZ3 = mul29(ZZZ, PPP)
            Q = mul29(X, PP)
            RR = sqr29(R)
            X3 = [RR[i] + C["M8P"][i] - PPP[i] - 2 * Q[i] for i in range(9)]
            assert all(0 <= v < 1 << 32 for v in X3)
            X3 = norm(X3)
            QX = sub(Q, X3, C["M16P"])
            Y3_old = sub(mul29(R, QX), mul29(Y, PPP), C["M8P"])
            Y3 = mulsub29(R, QX, Y, PPP)
            assert value(Y3) % P == value(Y3_old) % P
            for v, bound in ((Pv, 17.3), (R, 17.3), (QX, 17.3), (PP, 3.3), (PPP, 3.3), (Q, 3.3)):
                assert value(v) < bound * P
            X, Y, ZZ, ZZZ = X3, Y3, ZZ3, ZZZ3
            for v, bound in ((X, 11.3), (Y, 4.0), (ZZ, 1.03), (ZZZ, 1.03)):
                assert value(v) < bound * P


def mul_shift_sub29(a, b, E, f):
    """csrc/msm_l29.hpp l29::mul_shift_sub, step for step (round 6): a b 2^-261 + E - f with E and
    f entering at columns 9..17 of one product scan, signed carries from column 9 on."""
    p29, np29 = C["P29"], C["NP29"][0]
    m = [0] * 9
    r = [0] * 9
    acc = 0
    for k in range(17):
        lo, hi = (0, k) if k < 9 else (k - 8, 8)
        for i in range(lo, hi + 1):
            acc += a[i] * b[k - i]
        for i in range(lo, k if k < 9 else 9):
            acc += m[i] * p29[k - i]
        assert -(1 << 63) <= acc < 1 << 63
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * np29) & MASK
            acc += m[k] * p29[0]
            assert acc & MASK == 0 and acc >= 0
        else:
            acc += E[k - 9] - f[k - 9]
            assert -(1 << 63) <= acc < 1 << 63
            r[k - 9] = acc & MASK
        acc >>= 29
    r[8] = acc + E[8] - f[8]
    assert 0 <= r[8] < 1 << 32
    return r


def test_mul_shift_sub_matches_montgomery():
    """P = x ZZ - X + 12p and R = y ZZZ - Y + 4p in one reduction each, over the operand ranges of
    madd-2008-s (x, y canonical points, ZZ, ZZZ below 1.03p, X below 11.3p, Y below 3.8p)."""
    rinv = pow(2, -261, P)
    rng = random.Random(1206)
    for E, fmax, out in ((C["P12"], 11.3, 13.1), (C["P4"], 3.8, 5.1)):
        e = value(E)
        cases = [(0, 0, int(fmax * P) - 1), (P - 1, int(1.03 * P), 0)]
        cases += [(rng.randrange(P), rng.randrange(int(1.03 * P)), rng.randrange(int(fmax * P))) for _ in range(500)]
        for x, zz, f in cases:
            r = mul_shift_sub29(limbs(x), limbs(zz), E, limbs(f))
            assert value(r) % P == (x * zz * rinv + e - f) % P
            assert all(0 <= t <= MASK for t in r[:8])
            assert 0 <= value(r) < out * P


def test_lazy_madd_chain_round6_full():
    """The round-6 madd as the kernel runs it (P, R by mul_shift_sub; Y3 by mulsub) against plain
    modular arithmetic of madd-2008-s over random chains, with every product input below 17.3p."""
    rng = random.Random(67)
    one = limbs(pow(2, 266, P))
    rinv = pow(2, -261, P)
    for _ in range(20):
        X = Y = ZZ = ZZZ = None
        for step in range(40):
            x, y = rng.randrange(P), rng.randrange(P)
            x256, y256 = limbs(x * 2 ** 256 % P), limbs(y * 2 ** 256 % P)
            if X is None:
                X, Y = times32(x256), times32(y256)
                ZZ = ZZZ = one
                continue
            Pv = mul_shift_sub29(x256, ZZ, C["P12"], X)
            R = mul_shift_sub29(y256, ZZZ, C["P4"], Y)
            assert value(Pv) % P == (value(x256) * value(ZZ) * rinv - value(X)) % P
            assert value(R) % P == (value(y256) * value(ZZZ) * rinv - value(Y)) % P
            PP = sqr29(Pv)
            ZZ3 = mul29(ZZ, PP)
            PPP = mul29(Pv, PP)
            ZZZ3 = mul29(ZZZ, PPP)
            Q = mul29(X, PP)
            RR = sqr29(R)
            X3 = [RR[i] + C["M8P"][i] - PPP[i] - 2 * Q[i] for i in range(9)]
            assert all(0 <= v < 1 << 32 for v in X3)
            X3 = norm(X3)
            QX = sub(Q, X3, C["M16P"])
            Y3 = mulsub29(R, QX, Y, PPP)
            assert value(Y3) % P == (value(R) * value(QX) - value(Y) * value(PPP)) * rinv % P
            for v, bound in ((Pv, 13.1), (R, 5.1), (QX, 17.3), (PP, 3.3), (PPP, 3.3), (Q, 3.3)):
                assert value(v) < bound * P
            X, Y, ZZ, ZZZ = X3, Y3, ZZ3, ZZZ3
            for v, bound in ((X, 11.3), (Y, 3.8), (ZZ, 1.03), (ZZZ, 1.03)):
                assert value(v) < bound * P
