"""ORACLE — TEST INFRASTRUCTURE ONLY.

BN254 optimal-ate pairing over Python big integers: the checker of the GPU pairing
(BASELINE config 4, "KZG commit MSM + pairing check"). The
reference's pairing (src/pbh/pairing.rs:12-47) is the reduced Tate pairing of its toy
curve; its BN254 instantiation is the standard optimal ate pairing
e(P, Q) = f_{6u+2,Q}(P) * l_{[6u+2]Q, pi(Q)}(P) * l_{..., -pi^2(Q)}(P), raised to
(q^12 - 1)/r. The value is well defined (no reference test pins it: parity pinned by
bilinearity, non-degeneracy, the KZG check boolean, and an independent flat-Fq12
restatement `pairing_flat`, see tests/test_bn254_pairing_oracle.py).

Tower (the GPU's layout): Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3 - xi), xi = 9+u,
Fq12 = Fq6[w]/(w^2 - v). An Fq12 element is ((c0.a0, c0.a1, c0.a2), (c1.a0, c1.a1, c1.a2))
of Fq2 pairs; flattened to 12 Fq integers in that order.
G2 is the D-type sextic twist y^2 = x^3 + 3/xi over Fq2.
"""
from __future__ import annotations

Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
BN_U = 4965661367192848881
ATE = 6 * BN_U + 2  # 29793968203157093288

G1_GEN = (1, 2)
G2_GEN = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
           11559732032986387107991004021392285783925812861821192530917403151452391805634),
          (8495653923123431417604973247489272438418190587263600148770280649306958101930,
           4082367875863433681332203403145435568316851327593401208105741076214120093531))


# ---------------------------------------------------------------- Fq2
def f2(a0, a1=0):
    return (a0 % Q, a1 % Q)


F2_ZERO, F2_ONE = (0, 0), (1, 0)
XI = (9, 1)


def f2_add(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def f2_sub(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def f2_neg(a):
    return ((-a[0]) % Q, (-a[1]) % Q)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def f2_muls(a, s):
    return (a[0] * s % Q, a[1] * s % Q)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % Q
    ni = pow(n, Q - 2, Q)
    return (a[0] * ni % Q, (-a[1]) * ni % Q)


def f2_conj(a):
    return (a[0], (-a[1]) % Q)


def f2_pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_mul(a, a)
        e >>= 1
    return r


# ---------------------------------------------------------------- Fq6 = Fq2[v]/(v^3 - xi)
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t00, t11, t22 = f2_mul(a0, b0), f2_mul(a1, b1), f2_mul(a2, b2)
    c0 = f2_add(t00, f2_mul(XI, f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul(XI, t22))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t11)
    return (c0, c1, c2)


def f6_mul_v(a):
    """a * v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2."""
    return (f2_mul(XI, a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_mul(a0, a0), f2_mul(XI, f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul(XI, f2_mul(a2, a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_mul(a1, a1), f2_mul(a0, a2))
    n = f2_add(f2_mul(a0, t0), f2_mul(XI, f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    ni = f2_inv(n)
    return (f2_mul(t0, ni), f2_mul(t1, ni), f2_mul(t2, ni))


# ---------------------------------------------------------------- Fq12 = Fq6[w]/(w^2 - v)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0, t1 = f6_mul(a0, b0), f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    """a^(q^6): w -> -w."""
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    n = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ni = f6_inv(n)
    return (f6_mul(a0, ni), f6_neg(f6_mul(a1, ni)))


def f12_pow(a, e):
    r = F12_ONE
    for bit in bin(e)[2:]:
        r = f12_sqr(r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_flat(a):
    """12 Fq integers in tower order c0.a0, c0.a1, c0.a2, c1.a0, c1.a1, c1.a2 (each Fq2 re, im)."""
    out = []
    for c in a:
        for x in c:
            out += [x[0], x[1]]
    return out


def f12_from_flat(v):
    it = iter(v)
    c = [tuple((next(it), next(it)) for _ in range(3)) for _ in range(2)]
    return (c[0], c[1])


# ---------------------------------------------------------------- G2 (twist) affine, None = identity
B2 = f2_mul((3, 0), f2_inv(XI))


def g2_on_curve(p):
    if p is None:
        return True
    x, y = p
    return f2_sub(f2_mul(y, y), f2_add(f2_mul(f2_mul(x, x), x), B2)) == F2_ZERO


def g2_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if f2_add(p[1], q[1]) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_mul(p[0], p[0]), 3), f2_inv(f2_muls(p[1], 2)))
    else:
        lam = f2_mul(f2_sub(q[1], p[1]), f2_inv(f2_sub(q[0], p[0])))
    x3 = f2_sub(f2_sub(f2_mul(lam, lam), p[0]), q[0])
    return (x3, f2_sub(f2_mul(lam, f2_sub(p[0], x3)), p[1]))


def g2_neg(p):
    return None if p is None else (p[0], f2_neg(p[1]))


def g2_mul(p, k):
    r = None
    k %= R
    while k:
        if k & 1:
            r = g2_add(r, p)
        p = g2_add(p, p)
        k >>= 1
    return r


# Frobenius on the twist: pi(x, y) = (conj(x) * xi^((q-1)/3), conj(y) * xi^((q-1)/2))
GAMMA_X = f2_pow(XI, (Q - 1) // 3)
GAMMA_Y = f2_pow(XI, (Q - 1) // 2)


def g2_frob(p):
    return (f2_mul(f2_conj(p[0]), GAMMA_X), f2_mul(f2_conj(p[1]), GAMMA_Y))


# ---------------------------------------------------------------- Miller loop (affine T)
def _line(lam, t, p):
    """Line of slope lam (twisted) through T, at P = (xp, yp) in Fq:
    l = yp - lam*xp*w + (lam*xT - yT)*v*w  (untwist (x, y) -> (x w^2, y w^3), w^3 = v w);
    vertical parts dropped (killed by the final exponentiation)."""
    xp, yp = p
    c0 = ((yp % Q, 0), F2_ZERO, F2_ZERO)
    c1 = (f2_neg(f2_muls(lam, xp)), f2_sub(f2_mul(lam, t[0]), t[1]), F2_ZERO)
    return (c0, c1)


def _dbl_step(t, p):
    lam = f2_mul(f2_muls(f2_mul(t[0], t[0]), 3), f2_inv(f2_muls(t[1], 2)))
    line = _line(lam, t, p)
    x3 = f2_sub(f2_mul(lam, lam), f2_muls(t[0], 2))
    return (x3, f2_sub(f2_mul(lam, f2_sub(t[0], x3)), t[1])), line


def _add_step(t, q, p):
    lam = f2_mul(f2_sub(q[1], t[1]), f2_inv(f2_sub(q[0], t[0])))
    line = _line(lam, t, p)
    x3 = f2_sub(f2_sub(f2_mul(lam, lam), t[0]), q[0])
    return (x3, f2_sub(f2_mul(lam, f2_sub(t[0], x3)), t[1])), line


def miller_loop(p, q):
    """f_{6u+2,Q}(P) * l_{T,pi(Q)}(P) * l_{T',-pi^2(Q)}(P); P affine G1 (Fq), Q affine twist."""
    if p is None or q is None:
        return F12_ONE
    f, t = F12_ONE, q
    for bit in bin(ATE)[3:]:
        t, line = _dbl_step(t, p)
        f = f12_mul(f12_sqr(f), line)
        if bit == "1":
            t, line = _add_step(t, q, p)
            f = f12_mul(f, line)
    q1 = g2_frob(q)
    q2 = g2_neg(g2_frob(q1))
    t, line = _add_step(t, q1, p)
    f = f12_mul(f, line)
    t, line = _add_step(t, q2, p)
    return f12_mul(f, line)


HARD_EXP = (Q ** 4 - Q ** 2 + 1) // R


def final_exp(f):
    """f^((q^12-1)/r) = ((f^(q^6) / f)^(q^2 + 1))^((q^4 - q^2 + 1)/r)."""
    f1 = f12_mul(f12_conj(f), f12_inv(f))
    f2_ = f12_mul(f12_pow(f1, Q * Q), f1)
    return f12_pow(f2_, HARD_EXP)


def pairing(p, q):
    return final_exp(miller_loop(p, q))


def pairing_check(pairs) -> bool:
    """prod_i e(P_i, Q_i) == 1 (one shared final exponentiation)."""
    f = F12_ONE
    for p, q in pairs:
        f = f12_mul(f, miller_loop(p, q))
    return final_exp(f) == F12_ONE


# ---------------------------------------------------------------- G1 helpers
def g1_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % Q == 0:
            return None
        lam = 3 * p[0] * p[0] * pow(2 * p[1], Q - 2, Q) % Q
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], Q - 2, Q) % Q
    x3 = (lam * lam - p[0] - q[0]) % Q
    return (x3, (lam * (p[0] - x3) - p[1]) % Q)


def g1_neg(p):
    return None if p is None else (p[0], (-p[1]) % Q)


def g1_mul(p, k):
    r = None
    k %= R
    while k:
        if k & 1:
            r = g1_add(r, p)
        p = g1_add(p, p)
        k >>= 1
    return r


# ---------------------------------------------------------------- independent flat restatement
# Fq12 as Fq[w]/(w^12 - 18 w^6 + 82) (w^6 = xi = 9 + u); the twist is applied to Q and
# the Miller loop runs on Fq12 points with generic chord/tangent lines (vertical lines
# kept when they occur). A different construction of the same reduced pairing value.
_MOD = [82, 0, 0, 0, 0, 0, -18, 0, 0, 0, 0, 0]  # w^12 = -82 + 18 w^6 -> coefficients of the monic modulus


def _p12_mul(a, b):
    prod = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                prod[i + j] += x * y
    for k in range(22, 11, -1):
        c = prod[k]
        if c:
            prod[k] = 0
            prod[k - 6] += 18 * c
            prod[k - 12] -= 82 * c
    return [x % Q for x in prod[:12]]


def _p12_inv(a):
    # extended Euclid over Fq[w] against the modulus polynomial
    lm, hm = [1] + [0] * 12, [0] * 13
    low, high = list(a) + [0], [82, 0, 0, 0, 0, 0, -18 % Q, 0, 0, 0, 0, 0, 1]

    def deg(p):
        d = len(p) - 1
        while d and p[d] % Q == 0:
            d -= 1
        return d

    while deg(low):
        r = [0] * 13
        dl, dh = deg(low), deg(high)
        temp = list(high)
        inv_lead = pow(low[dl], Q - 2, Q)
        for i in range(dh - dl, -1, -1):
            r[i] = temp[dl + i] * inv_lead % Q
            for j in range(dl + 1):
                temp[i + j] -= low[j] * r[i]
        temp = [x % Q for x in temp]
        nm = list(hm)
        for i in range(13):
            for j in range(13 - i):
                nm[i + j] -= lm[i] * r[j]
        nm = [x % Q for x in nm]
        lm, low, hm, high = nm, temp, lm, low
    inv0 = pow(low[0], Q - 2, Q)
    return [x * inv0 % Q for x in lm[:12]]


def _p12_pow(a, e):
    r = [1] + [0] * 11
    for bit in bin(e)[2:]:
        r = _p12_mul(r, r)
        if bit == "1":
            r = _p12_mul(r, a)
    return r


def _p12_sub(a, b):
    return [(x - y) % Q for x, y in zip(a, b)]


def _fq2_to_p12(a):
    # a0 + a1 u with u = w^6 - 9
    out = [0] * 12
    out[0] = (a[0] - 9 * a[1]) % Q
    out[6] = a[1] % Q
    return out


def _twist(q):
    """(x, y) on the twist -> (x w^2, y w^3) on E(Fq12)."""
    x, y = _fq2_to_p12(q[0]), _fq2_to_p12(q[1])
    w2 = [0, 0, 1] + [0] * 9
    w3 = [0, 0, 0, 1] + [0] * 8
    return (_p12_mul(x, w2), _p12_mul(y, w3))


def _line_flat(p1, p2, t):
    x1, y1 = p1
    x2, y2 = p2
    xt, yt = t
    if x1 != x2:
        m = _p12_mul(_p12_sub(y2, y1), _p12_inv(_p12_sub(x2, x1)))
    elif y1 == y2:
        num = [3 * c % Q for c in _p12_mul(x1, x1)]
        m = _p12_mul(num, _p12_inv([2 * c % Q for c in y1]))
    else:
        return _p12_sub(xt, x1)
    return _p12_sub(_p12_mul(m, _p12_sub(xt, x1)), _p12_sub(yt, y1))


def _add_flat(p1, p2):
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2 and y1 == y2:
        m = _p12_mul([3 * c % Q for c in _p12_mul(x1, x1)], _p12_inv([2 * c % Q for c in y1]))
    else:
        m = _p12_mul(_p12_sub(y2, y1), _p12_inv(_p12_sub(x2, x1)))
    x3 = _p12_sub(_p12_sub(_p12_mul(m, m), x1), x2)
    return (x3, _p12_sub(_p12_mul(m, _p12_sub(x1, x3)), y1))


def pairing_flat(p, q):
    """Independent restatement: Miller loop on twisted Fq12 points, plain final exponent."""
    qt = _twist(q)
    pt = ([p[0] % Q] + [0] * 11, [p[1] % Q] + [0] * 11)
    f = [1] + [0] * 11
    t = qt
    for bit in bin(ATE)[3:]:
        f = _p12_mul(_p12_mul(f, f), _line_flat(t, t, pt))
        t = _add_flat(t, t)
        if bit == "1":
            f = _p12_mul(f, _line_flat(t, qt, pt))
            t = _add_flat(t, qt)
    q1 = (_p12_pow(qt[0], Q), _p12_pow(qt[1], Q))
    nq2 = (_p12_pow(q1[0], Q), [(-c) % Q for c in _p12_pow(q1[1], Q)])
    f = _p12_mul(f, _line_flat(t, q1, pt))
    t = _add_flat(t, q1)
    f = _p12_mul(f, _line_flat(t, nq2, pt))
    return _p12_pow(f, (Q ** 12 - 1) // R)


def tower_to_flat(a):
    """Map a tower Fq12 element to Fq[w]/(w^12 - 18 w^6 + 82): v = w^2, u = w^6 - 9."""
    out = [0] * 12
    for k, c6 in enumerate(a):          # c6 * w^k
        for j, c2 in enumerate(c6):     # c2 * v^j = c2 * w^(2j)
            p = _fq2_to_p12(c2)
            shift = k + 2 * j
            term = _p12_mul(p, [1 if i == shift else 0 for i in range(12)])
            out = [(x + y) % Q for x, y in zip(out, term)]
    return out
