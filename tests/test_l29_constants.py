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
                X, Y = mul29(x256, one), mul29(y256, one)
                ZZ = ZZZ = one
                continue
            Pv = sub(mul29(x256, ZZ), X, C["M16P"])
            R = sub(mul29(y256, ZZZ), Y, C["M16P"])
            PP = mul29(Pv, Pv)
            ZZ3 = mul29(ZZ, PP)
            PPP = mul29(Pv, PP)
            YP = mul29(Y, PPP)
            ZZZ = mul29(ZZZ, PPP)
            Q = mul29(X, PP)
            RR = mul29(R, R)
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
