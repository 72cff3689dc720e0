"""ORACLE — TEST INFRASTRUCTURE ONLY.

Literal restatement of Plonk::prove / Plonk::verify (src/plonk.rs:120-650) for a
general number of gates n over BN254 (HF = GF = Fr, G1/G2 of BN254, the optimal-ate
pairing of oracle/bn254_pairing.py): the checker of the GPU prover (BASELINE config 5).

Generalisation of the n = 4 hard-coding: t(x) is split into three
parts of n+2 coefficients (plonk.rs:376-378 uses [0..6], [6..12], [12..18] = n+2 for
n = 4) and t_mid/t_hi are weighted by z^(n+2), z^(2n+4) exactly as plonk.rs:430 and
:617-619 already do. interpolate_at_h (the Vandermonde inverse, plonk.rs:177-179) is
the natural-order inverse DFT, computed here by the oracle NTT.
Everything else follows the reference operation by operation: schoolbook products
(poly.rs:205-218), long division (poly.rs:230-247) with the remainder asserted zero
(plonk.rs:370, :438, :442), Poly normalisation (poly.rs:96-105), and the naive SRS
fold for commitments (plonk.rs:51-58).

mode = "reference" keeps r_3(x) = z(x) * s_sigma_3(x) * (beta z_omega_z) * (...) * alpha
(plonk.rs:414-416, a + sign and a z(x) factor the verifier does not expect: SURVEY.md
§0.7, the n = 4 KAT cannot see it); mode = "paper" uses the linearisation the verifier
checks (plonk.rs:584-611): r_3(x) = -(beta z_omega_z (a_z + beta s1_z + gamma)
(b_z + beta s2_z + gamma) alpha) * s_sigma_3(x), so prove -> verify succeeds for any n.
"""
from __future__ import annotations

import bn254 as F
import bn254_pairing as B

R = B.R


# ---------------------------------------------------------------- Poly (poly.rs)
def norm(c):
    c = [x % R for x in c]
    while c and c[-1] == 0:
        c.pop()
    return c


def padd(a, b):
    n = max(len(a), len(b))
    return norm([(a[i] if i < len(a) else 0) + (b[i] if i < len(b) else 0) for i in range(n)])


def psub(a, b):
    return padd(a, [-x for x in b])


def pmul(a, b):
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] += x * y
    return norm(out)


def pscale(a, s):
    return norm([x * s for x in a])


def pdiv(num, den):
    num, den = norm(num), norm(den)
    q = [0] * max(len(num) - len(den) + 1, 0)
    rem = list(num)
    inv = pow(den[-1], R - 2, R)
    for i in range(len(num) - len(den), -1, -1):
        c = rem[i + len(den) - 1] * inv % R
        q[i] = c
        for j, d in enumerate(den):
            rem[i + j] = (rem[i + j] - c * d) % R
    return norm(q), norm(rem)


def peval(a, x):
    return F.poly_eval(a, x) if a else 0


# ---------------------------------------------------------------- setup
class Setup:
    """Plonk::new (plonk.rs:120-175) + SRS::create (plonk.rs:35-48)."""

    def __init__(self, n: int, s: int, srs_n: int, k1: int = 2, k2: int = 3):
        self.n, self.k1, self.k2 = n, k1, k2
        self.omega = F.root_of_unity(n)
        self.h = [pow(self.omega, i, R) for i in range(n)]
        hs = set(self.h)
        assert k1 not in hs and k2 not in hs
        self.k1_h = [k1 * x % R for x in self.h]
        self.k2_h = [k2 * x % R for x in self.h]
        assert k2 not in set(self.k1_h)
        self.z_h = norm([-1] + [0] * (n - 1) + [1])  # prod (x - h_i) = x^n - 1
        g1s, sp = [B.G1_GEN], s
        for _ in range(srs_n):
            g1s.append(B.g1_mul(B.G1_GEN, sp))
            sp = sp * s % R
        self.g1s = g1s
        self.g2_1 = B.G2_GEN
        self.g2_s = B.g2_mul(B.G2_GEN, s)

    def interpolate(self, v):
        return norm(F.ntt(list(v), self.omega, inverse=True))

    def eval_at_s(self, c):
        acc = None
        for i, x in enumerate(c):
            acc = B.g1_add(acc, B.g1_mul(self.g1s[i], x))
        return acc

    def roots(self, copies):
        """copy_constraints_to_roots (plonk.rs:181-189): (kind 0/1/2, 1-based index)."""
        tab = (self.h, self.k1_h, self.k2_h)
        return [tab[k][i - 1] for k, i in copies]


def prove(st: Setup, q, copies, abc, chal, rnd, mode="reference"):
    """q = (q_l, q_r, q_o, q_m, q_c); copies = (c_a, c_b, c_c) of (kind, idx);
    abc = (a, b, c); chal = (alpha, beta, gamma, z, v); rnd = b1..b9.
    Returns (9 commitments, 7 field elements) like Proof (plonk.rs:61-95) and the
    intermediate polynomials (for tests)."""
    n, omega, k1, k2 = st.n, st.omega, st.k1, st.k2
    q_l, q_r, q_o, q_m, q_c = q
    a, b, c = abc
    alpha, beta, gamma, zc, v = chal
    # satisfies (constraints.rs:198-230, including its q_l * b term)
    for i in range(n):
        assert (q_l[i] * a[i] + q_l[i] * b[i] + q_o[i] * c[i] + q_m[i] * a[i] * b[i] + q_c[i]) % R == 0
    sig = [st.roots(cc) for cc in copies]
    f_a, f_b, f_c = (st.interpolate(x) for x in abc)
    q_o_x, q_m_x, q_l_x, q_r_x, q_c_x = (st.interpolate(x) for x in (q_o, q_m, q_l, q_r, q_c))
    s1, s2, s3 = (st.interpolate(x) for x in sig)
    b1, b2, b3, b4, b5, b6, b7, b8, b9 = rnd
    a_x = padd(pmul(norm([b2, b1]), st.z_h), f_a)
    b_x = padd(pmul(norm([b4, b3]), st.z_h), f_b)
    c_x = padd(pmul(norm([b6, b5]), st.z_h), f_c)
    a_s, b_s, c_s = st.eval_at_s(a_x), st.eval_at_s(b_x), st.eval_at_s(c_x)
    # round 2 (plonk.rs:278-313)
    acc = [1]
    for i in range(1, n):
        ai, bi, ci = a[i - 1], b[i - 1], c[i - 1]
        w = pow(omega, i - 1, R)
        dend = (ai + beta * w + gamma) * (bi + beta * k1 * w + gamma) * (ci + beta * k2 * w + gamma) % R
        dsor = (ai + beta * peval(s1, w) + gamma) * (bi + beta * peval(s2, w) + gamma) \
            * (ci + beta * peval(s3, w) + gamma) % R
        acc.append(acc[-1] * dend * pow(dsor, R - 2, R) % R)
    acc_x = st.interpolate(acc)
    z_x = padd(pmul(norm([b9, b8, b7]), st.z_h), acc_x)
    z_s = st.eval_at_s(z_x)
    # round 3 (plonk.rs:326-382)
    l1 = st.interpolate([1] + [0] * (n - 1))
    t1 = padd(padd(padd(padd(pmul(pmul(a_x, b_x), q_m_x), pmul(a_x, q_l_x)), pmul(b_x, q_r_x)),
                   pmul(c_x, q_o_x)), q_c_x)
    t2 = pmul(pmul(pmul(pscale(padd(a_x, [gamma, beta]), alpha), padd(b_x, [gamma, beta * k1])),
                   padd(c_x, [gamma, beta * k2])), z_x)
    z_omega_x = norm([x * pow(omega, i, R) for i, x in enumerate(z_x)])
    t3 = pmul(pmul(pmul(pscale(padd(padd(a_x, pscale(s1, beta)), [gamma]), alpha),
                        padd(padd(b_x, pscale(s2, beta)), [gamma])),
                   padd(padd(c_x, pscale(s3, beta)), [gamma])), z_omega_x)
    t4 = pmul(pscale(padd(z_x, [-1]), alpha * alpha), l1)
    t_x, rem = pdiv(padd(psub(padd(t1, t2), t3), t4), st.z_h)
    assert rem == []
    m = n + 2
    tc = t_x + [0] * max(0, 3 * m - len(t_x))
    assert len(tc) == 3 * m, "t(x) has more than 3(n+2) coefficients"
    t_lo, t_mid, t_hi = norm(tc[:m]), norm(tc[m:2 * m]), norm(tc[2 * m:3 * m])
    t_hi_s, t_mid_s, t_lo_s = st.eval_at_s(t_hi), st.eval_at_s(t_mid), st.eval_at_s(t_lo)
    # round 4 (plonk.rs:384-422)
    a_z, b_z, c_z = peval(a_x, zc), peval(b_x, zc), peval(c_x, zc)
    s1_z, s2_z = peval(s1, zc), peval(s2, zc)
    t_z = peval(t_x, zc)
    zw_z = peval(z_omega_x, zc)
    r1 = padd(padd(padd(padd(pscale(q_m_x, a_z * b_z), pscale(q_l_x, a_z)), pscale(q_r_x, b_z)),
                   pscale(q_o_x, c_z)), q_c_x)
    r2 = pscale(z_x, (a_z + beta * zc + gamma) * (b_z + beta * k1 * zc + gamma) * (c_z + beta * k2 * zc + gamma) * alpha)
    k3 = (a_z + beta * s1_z + gamma) * (b_z + beta * s2_z + gamma) * alpha
    if mode == "reference":
        r3 = pscale(pmul(z_x, pscale(s3, beta * zw_z)), k3)
    else:
        r3 = pscale(s3, -(beta * zw_z * k3))
    r4 = pscale(z_x, peval(l1, zc) * alpha * alpha)
    r_x = padd(padd(padd(r1, r2), r3), r4)
    r_z = peval(r_x, zc)
    # round 5 (plonk.rs:424-446)
    wz = psub(padd(padd(t_lo, pscale(t_mid, pow(zc, n + 2, R))), pscale(t_hi, pow(zc, 2 * n + 4, R))), [t_z])
    for k, (p, e) in enumerate(((r_x, r_z), (a_x, a_z), (b_x, b_z), (c_x, c_z), (s1, s1_z), (s2, s2_z))):
        wz = padd(wz, pscale(psub(p, [e]), pow(v, k + 1, R)))
    w_z_x, rem = pdiv(wz, [-zc, 1])
    assert rem == []
    w_zw_x, rem = pdiv(psub(z_x, [zw_z]), [-zc * omega, 1])
    assert rem == []
    w_z_s, w_zw_s = st.eval_at_s(w_z_x), st.eval_at_s(w_zw_x)
    pts = [a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_z_s, w_zw_s]
    fields = [a_z, b_z, c_z, s1_z, s2_z, r_z, zw_z]
    polys = {"a": a_x, "b": b_x, "c": c_x, "z": z_x, "t": t_x, "t_lo": t_lo, "t_mid": t_mid, "t_hi": t_hi,
             "r": r_x, "w_z": w_z_x, "w_zw": w_zw_x, "s1": s1, "s2": s2, "s3": s3, "acc": acc}
    return pts, fields, polys


def verify(st: Setup, q, copies, pts, fields, chal, u: int, mode="reference") -> bool:
    """Plonk::verify (plonk.rs:468-650), batched KZG check with one pairing check.
    mode = "reference" keeps step 7's t_z without alpha on the permutation term
    (plonk.rs:575-581; correct only for alpha = 1); "paper" multiplies it
    by alpha, which with the paper linearisation makes every honest proof verify."""
    n, omega, k1, k2 = st.n, st.omega, st.k1, st.k2
    a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_z_s, w_zw_s = pts
    a_z, b_z, c_z, s1_z, s2_z, r_z, zw_z = fields
    alpha, beta, gamma, zc, v = chal
    q_l, q_r, q_o, q_m, q_c = q
    sig = [st.roots(cc) for cc in copies]
    q_m_s, q_l_s, q_r_s, q_o_s, q_c_s = (st.eval_at_s(st.interpolate(x)) for x in (q_m, q_l, q_r, q_o, q_c))
    s1_s, s2_s, s3_s = (st.eval_at_s(st.interpolate(x)) for x in sig)
    for p in pts:
        if p is not None and (p[1] * p[1] - p[0] ** 3 - 3) % B.Q:
            return False
    z_h_z = (pow(zc, n, R) - 1) % R
    l_1_z = peval(st.interpolate([1] + [0] * (n - 1)), zc)
    perm = (a_z + beta * s1_z + gamma) * (b_z + beta * s2_z + gamma) * (c_z + gamma) * zw_z
    if mode != "reference":
        perm *= alpha
    t_z = (r_z - perm - l_1_z * alpha * alpha) * pow(z_h_z, R - 2, R) % R
    mul, add = B.g1_mul, B.g1_add
    d1 = None
    for pt, sc in ((q_m_s, a_z * b_z * v), (q_l_s, a_z * v), (q_r_s, b_z * v), (q_o_s, c_z * v), (q_c_s, v)):
        d1 = add(d1, mul(pt, sc % R))
    d2 = mul(z_s, ((a_z + beta * zc + gamma) * (b_z + beta * k1 * zc + gamma) * (c_z + beta * k2 * zc + gamma)
                   * alpha * v + l_1_z * alpha * alpha * v + u) % R)
    d3 = mul(s3_s, (a_z + beta * s1_z + gamma) * (b_z + beta * s2_z + gamma) * alpha * v * beta * zw_z % R)
    d = add(add(d1, d2), B.g1_neg(d3))
    f = add(add(add(t_lo_s, mul(t_mid_s, pow(zc, n + 2, R))), mul(t_hi_s, pow(zc, 2 * n + 4, R))), d)
    for k, pt in enumerate((a_s, b_s, c_s, s1_s, s2_s)):
        f = add(f, mul(pt, pow(v, k + 2, R)))
    e = mul(st.g1s[0], (t_z + v * r_z + pow(v, 2, R) * a_z + pow(v, 3, R) * b_z + pow(v, 4, R) * c_z
                        + pow(v, 5, R) * s1_z + pow(v, 6, R) * s2_z + u * zw_z) % R)
    e1_q1 = add(w_z_s, mul(w_zw_s, u))
    e2_q1 = add(add(add(mul(w_z_s, zc), mul(w_zw_s, u * zc * omega % R)), f), B.g1_neg(e))
    # e(e1_q1, g2_s) == e(e2_q1, g2_1)  <=>  e(e1_q1, g2_s) * e(-e2_q1, g2_1) == 1
    return B.pairing_check([(e1_q1, st.g2_s), (B.g1_neg(e2_q1), st.g2_1)])


def mul_gates_circuit(n: int, seed: int):
    """BASELINE config 5's synthetic circuit: every gate a * b = c (q_m = 1, q_o = -1),
    a, b uniform; copy constraints a random permutation of the 3n wire labels
    (seed 0x5EED0005) restricted to wires holding equal values: here the
    permutation cycles through the positions of equal witness values (all distinct for
    random a, b, so sigma = identity except for explicitly tied wires)."""
    import random

    rng = random.Random(seed)
    a = [rng.randrange(R) for _ in range(n)]
    b = [rng.randrange(R) for _ in range(n)]
    # tie the wires of gate i+1's a to gate i's c for a few gates (real copy constraints)
    for i in range(0, n - 1, 4):
        a[i + 1] = a[i] * b[i] % R
    c = [x * y % R for x, y in zip(a, b)]
    q = ([0] * n, [0] * n, [R - 1] * n, [1] * n, [0] * n)
    c_a = [(0, i + 1) for i in range(n)]
    c_b = [(1, i + 1) for i in range(n)]
    c_c = [(2, i + 1) for i in range(n)]
    for i in range(0, n - 1, 4):  # swap labels: a_{i+1} <-> c_i
        c_a[i + 1], c_c[i] = (2, i + 1), (0, i + 2)
    return q, (c_a, c_b, c_c), (a, b, c)
