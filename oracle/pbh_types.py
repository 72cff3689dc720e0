"""ORACLE — TEST INFRASTRUCTURE ONLY.

PlonkByHandTypes (src/pbh/mod.rs:18-33) in Python for oracle/plonk.py: HF = F17,
GF = F101, K1 = 2, K2 = 3, OMEGA = 4, gf(x) = F101(x). Literal restatements of
* G1P (src/pbh/g1.rs:18-168): affine y^2 = x^3 + 3 over F101, (x, y, infinite);
  identity (0, 0, True); add with the doubling formula (g1.rs:119-144); LSB-first
  double-and-add returning the identity for a zero scalar (g1.rs:146-168);
* G2P (src/pbh/g2.rs:14-101): a + b u, u^2 = -2, add / double in u units; double-and-add
  (scalar 0 panics in the reference: unwrap on None at g2.rs:99);
* GTP (src/pbh/gt.rs:9-76): F101[u]/(u^2 + 2), pow with the x^101 = conj(x) reduction;
* PBHPairing (src/pbh/pairing.rs:12-47): recursive Miller loop over r = 17, final
  exponent (101^2 - 1) / 17 = 600.
The C++ oracle (oracle/pbh.hpp) restates the same files; both are pinned by the
reference's KATs (tests/golden/reference_kats.json).
"""
from __future__ import annotations

import plonk

P = 101  # GF
R = 17   # HF, the G1 subgroup order (g1.rs:79-81)


def _inv(x: int):
    x %= P
    return pow(x, -1, P) if x else None  # U64Field::inv -> None on zero (u64field.rs:52-63)


def _div(a: int, b: int):
    i = _inv(b)
    if i is None:
        raise ZeroDivisionError("unwrap on a None division (pbh)")
    return a * i % P


# ---------------------------------------------------------------- G1 (g1.rs)
IDENTITY = (0, 0, True)
G1_GEN = (1, 2, False)


def g1_neg(p):  # g1.rs:108-117
    return p if p[2] else (p[0], (-p[1]) % P, False)


def g1_add(p, q):  # g1.rs:119-144
    if p[2]:
        return q
    if q[2]:
        return p
    if p == g1_neg(q):
        return IDENTITY
    if p == q:
        m = _div(3 * p[0] * p[0], 2 * p[1])
        return ((m * m - 2 * p[0]) % P, (m * (3 * p[0] - m * m) - p[1]) % P, False)
    lam = _div(q[1] - p[1], q[0] - p[0])
    x = (lam * lam - p[0] - q[0]) % P
    return (x, (lam * (p[0] - x) - p[1]) % P, False)


def g1_mul(p, s: int):  # g1.rs:146-168 (s an F101 value)
    s %= P
    if s == 0 or p[2]:
        return IDENTITY
    result, base = None, p
    while s > 0:
        if s % 2 == 1:
            result = base if result is None else g1_add(result, base)
        s >>= 1
        base = g1_add(base, base)
    return result


def g1_in_curve(p) -> bool:  # g1.rs:63-65 (also applied to the identity's (0, 0))
    return (p[1] * p[1] - p[0] ** 3 - 3) % P == 0


# ---------------------------------------------------------------- G2 (g2.rs)
G2_GEN = (36, 31)


def g2_add(p, q):  # g2.rs:58-80
    if p == q:
        m_u = _div(3 * p[0] * p[0], 2 * p[1])
        u2inv = _inv(-2)  # 1/u^2 = -1/2
        m2 = m_u * m_u * u2inv % P
        return ((m2 - 2 * p[0]) % P, (u2inv * m_u * (3 * p[0] - m2) - p[1]) % P)
    lam_u = _div(q[1] - p[1], q[0] - p[0])
    lam2 = lam_u * lam_u * (-2) % P
    a = (lam2 - p[0] - q[0]) % P
    return (a, (lam_u * (p[0] - a) - p[1]) % P)


def g2_mul(p, s: int):  # g2.rs:82-101
    s %= P
    result, base = None, p
    while s > 0:
        if s % 2 == 1:
            result = base if result is None else g2_add(result, base)
        s >>= 1
        base = g2_add(base, base)
    if result is None:
        raise ValueError("G2P * 0 panics (g2.rs:99 unwrap)")
    return result


# ---------------------------------------------------------------- GT (gt.rs)
def gt_mul(x, y):  # gt.rs:61-69
    return ((x[0] * y[0] - 2 * x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)


def gt_neg(x):  # gt.rs:21-29 (the conjugate)
    return (x[0], (-x[1]) % P)


def gt_pow(x, n: int):  # gt.rs:31-60
    if n >= 101:
        p, base = gt_neg(gt_pow(x, n // 101)), x
        n %= 101
    else:
        p, base = (1, 0), x
    while n > 0:
        if n % 2 == 1:
            p = gt_mul(p, base)
        n >>= 1
        base = gt_mul(base, base)
    return p


# ---------------------------------------------------------------- pairing (pairing.rs)
def _line(a, b):  # pairing.rs:25-34
    m = (b[0] - a[0]) % P
    n = (b[1] - a[1]) % P
    return n, (-m) % P, (m * a[1] - n * a[0]) % P


def _pairing_f(r: int, p, q):  # pairing.rs:23-47
    if r == 1:
        return (1, 0)
    if r % 2 == 1:
        r -= 1
        x, y, c = _line(g1_mul(p, r), p)
        return gt_mul(_pairing_f(r, p, q), ((q[0] * x + c) % P, q[1] * y % P))
    r //= 2
    x, y, c = _line(g1_mul(p, r), g1_mul(g1_mul(g1_neg(p), r), 2))
    return gt_mul(gt_pow(_pairing_f(r, p, q), 2), ((q[0] * x + c) % P, q[1] * y % P))


def pairing(p, q):  # pairing.rs:12-20
    exp = (P ** 2 - 1) // R
    return gt_pow(_pairing_f(R, p, q), exp)


# ---------------------------------------------------------------- the PlonkTypes instance
class PlonkByHandTypes(plonk.PlonkTypes):
    """pbh/mod.rs:18-33."""

    hf, gf = R, P
    K1, K2, OMEGA = 2, 3, 4
    g1_gen, g1_identity = G1_GEN, IDENTITY
    g2_gen = G2_GEN

    @staticmethod
    def gf_of(x: int) -> int:  # F101::from(sg.as_u64())
        return int(x) % P

    g1_add = staticmethod(g1_add)
    g1_neg = staticmethod(g1_neg)
    g1_mul = staticmethod(g1_mul)
    g1_in_curve = staticmethod(g1_in_curve)
    g2_mul = staticmethod(g2_mul)

    @staticmethod
    def pairing_eq(p1, q1, p2, q2) -> bool:  # plonk.rs:646-650: e_1 == e_2
        return pairing(p1, q1) == pairing(p2, q2)
