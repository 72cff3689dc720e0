"""ORACLE — TEST INFRASTRUCTURE ONLY.

The BN254 instance of the generic PLONK restatement (oracle/plonk.py, which restates
src/plonk.rs:15-650 operation by operation): HF = GF = Fr, G1 / G2 of BN254 and the
optimal-ate pairing of oracle/bn254_pairing.py. This is the checker of the GPU prover
(BASELINE config 5). The same oracle/plonk.py code instantiated with the reference's
PlonkByHandTypes reproduces the reference's proof KAT (src/pbh/mod.rs:101-123,
tests/test_plonk_oracle_pbh.py), so the formulas checked here are pinned to the
reference; only the types differ.

Type mapping: G1 points are affine tuples (x, y) with None for the identity
(bn254_pairing.py), the GPU's (0, 0) encoding; gf() is the identity (HF = GF);
pairing_eq(e1, s2, e2, g2) is the reference's e(e1, [s]G2) == e(e2, G2)
(plonk.rs:646-650), evaluated as one pairing check e(e1, [s]G2) e(-e2, G2) == 1 (equal
because the pairing is bilinear).

Compatibility API used by the tests / fixture generator: Setup(n, s, srs_n, k1, k2),
prove(st, ...), verify(st, ...), mul_gates_circuit(n, seed), and the list-based Poly
helpers norm / padd / pmul / pdiv.
"""
from __future__ import annotations

import bn254 as F
import bn254_pairing as B
import plonk as PL

R = B.R


class BN254Types(PL.PlonkTypes):
    hf = gf = R
    K1, K2 = 2, 3
    OMEGA = None  # per instance (the n-th root of unity of the circuit size)
    g1_gen, g1_identity = B.G1_GEN, None
    g2_gen = B.G2_GEN

    @staticmethod
    def gf_of(x: int) -> int:
        return int(x) % R

    g1_add = staticmethod(B.g1_add)
    g1_neg = staticmethod(B.g1_neg)

    @staticmethod
    def g1_mul(p, s: int):
        return B.g1_mul(p, int(s) % R)

    @staticmethod
    def g1_in_curve(p) -> bool:  # G1P::in_curve over Fq; the identity is accepted
        return p is None or (p[1] * p[1] - p[0] ** 3 - 3) % B.Q == 0

    @staticmethod
    def g2_mul(p, s: int):
        return B.g2_mul(p, int(s) % R)

    @staticmethod
    def pairing_eq(p1, q1, p2, q2) -> bool:
        return B.pairing_check([(p1, q1), (B.g1_neg(p2), q2)])


def bn254_types(n: int, k1: int = 2, k2: int = 3):
    """PlonkTypes for circuits of n gates: OMEGA = 5^((r-1)/n) (order exactly n)."""
    return type(f"BN254Types_n{n}", (BN254Types,), {"OMEGA": F.root_of_unity(n), "K1": k1, "K2": k2})


class Setup:
    """SRS::create (plonk.rs:35-48) + Plonk::new (plonk.rs:120-175) for n gates."""

    def __init__(self, n: int, s: int, srs_n: int, k1: int = 2, k2: int = 3):
        self.n, self.k1, self.k2 = n, k1, k2
        self.types = bn254_types(n, k1, k2)
        self.omega = self.types.OMEGA
        self.srs = PL.SRS(self.types, s, srs_n)
        self.plonk = PL.Plonk(self.types, self.srs, n)
        self.h = self.plonk.h
        self.g1s, self.g2_1, self.g2_s = self.srs.g1s, self.srs.g2_1, self.srs.g2_s

    def interpolate(self, v):
        return norm(self.plonk.interpolate_at_h(v).c)

    def eval_at_s(self, c):
        return self.srs.eval_at_s(PL.Poly(c, R))


def _lists(polys):
    return {k: (v if k == "acc" else norm(v.c)) for k, v in polys.items()}


def prove(st: Setup, q, copies, abc, chal, rnd, mode="reference"):
    """Plonk::prove through oracle/plonk.py; returns (9 points, 7 fields, polys as lists)."""
    pts, fields, polys = st.plonk.prove(q, copies, abc, chal, rnd, mode=mode)
    return pts, fields, _lists(polys)


def verify(st: Setup, q, copies, pts, fields, chal, u: int, mode="reference") -> bool:
    return st.plonk.verify(q, copies, pts, fields, chal, u, mode=mode)


# ---------------------------------------------------------------- list-based Poly helpers
def norm(c):
    """Normalised coefficients with the zero polynomial as [] (list form)."""
    c = [int(x) % R for x in c]
    while c and c[-1] == 0:
        c.pop()
    return c


def padd(a, b):
    return norm((PL.Poly(a or [0], R) + PL.Poly(b or [0], R)).c)


def pmul(a, b):
    if not a or not b:
        return []
    return norm((PL.Poly(a, R) * PL.Poly(b, R)).c)


def pdiv(num, den):
    q, r = divmod(PL.Poly(num or [0], R), PL.Poly(den, R))
    return norm(q.c), norm(r.c)


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


# ---------------------------------------------------------------- O(n) checks at scale
def _bary_weights(n: int, omega: int, x: int):
    """w_i = omega^i / (x - omega^i) for i < n (one batch inversion), and (x^n - 1) / n."""
    pw, d = [1] * n, [0] * n
    for i in range(n):
        if i:
            pw[i] = pw[i - 1] * omega % R
        d[i] = (x - pw[i]) % R
    assert all(d), "x lies in H"
    pre = [1] * (n + 1)
    for i in range(n):
        pre[i + 1] = pre[i] * d[i] % R
    inv = pow(pre[n], R - 2, R)
    w = [0] * n
    for i in range(n - 1, -1, -1):
        w[i] = inv * pre[i] % R * pw[i] % R
        inv = inv * d[i] % R
    scale = (pow(x, n, R) - 1) * pow(n, R - 2, R) % R
    return w, scale


def _bary(values, w, scale):
    return sum(v * wi for v, wi in zip(values, w)) % R * scale % R


def evaluations_at_z(n, q, copies, abc, chal, rnd, mode="reference", k1=2, k2=3):
    """The 7 field elements of Plonk::prove's Proof (a_z, b_z, c_z, s_sigma_1_z,
    s_sigma_2_z, r_z, z_omega_z; plonk.rs:393-422) in O(n), independently of any
    polynomial arithmetic: every interpolated polynomial f is evaluated from its values
    on H by the barycentric formula f(x) = (x^n - 1)/n sum_i f_i omega^i / (x - omega^i);
    the blinded polynomials add their (b x + b') Z_H(x) terms (plonk.rs:250-252, :315);
    the accumulator values follow plonk.rs:278-299 with s_sigma_k(omega^i) = sigma_k[i];
    r(z) is plonk.rs:401-419 evaluated term by term (r_3 per `mode`; "both" returns a
    dict of the two modes' lists)."""
    omega = F.root_of_unity(n)
    alpha, beta, gamma, z, v = (x % R for x in chal)
    b1, b2, b3, b4, b5, b6, b7, b8, b9 = (x % R for x in rnd)
    h = [1] * n
    for i in range(1, n):
        h[i] = h[i - 1] * omega % R
    tab = (h, [x * k1 % R for x in h], [x * k2 % R for x in h])
    sig = [[tab[k][i - 1] for k, i in col] for col in copies]
    a, b, c = ([x % R for x in col] for col in abc)
    w, scale = _bary_weights(n, omega, z)
    ev = lambda vals: _bary(vals, w, scale)  # noqa: E731
    zh = (pow(z, n, R) - 1) % R
    a_z = ((b1 * z + b2) * zh + ev(a)) % R
    b_z = ((b3 * z + b4) * zh + ev(b)) % R
    c_z = ((b5 * z + b6) * zh + ev(c)) % R
    s1_z, s2_z, s3_z = ev(sig[0]), ev(sig[1]), ev(sig[2])
    q_l_z, q_r_z, q_o_z, q_m_z, q_c_z = (ev([x % R for x in col]) for col in q)
    # acc_i = prod_{j<i} dend_j / dsor_j (plonk.rs:278-299): prefix products, one batch inversion
    nums, dens = [1] * n, [1] * n
    pn = pd = 1
    for i in range(1, n):
        wi = h[i - 1]
        pn = pn * ((a[i - 1] + beta * wi + gamma) * (b[i - 1] + beta * k1 * wi + gamma)
                   * (c[i - 1] + beta * k2 * wi + gamma)) % R
        pd = pd * ((a[i - 1] + beta * sig[0][i - 1] + gamma) * (b[i - 1] + beta * sig[1][i - 1] + gamma)
                   * (c[i - 1] + beta * sig[2][i - 1] + gamma)) % R
        nums[i], dens[i] = pn, pd
    pre = [1] * (n + 1)
    for i in range(n):
        pre[i + 1] = pre[i] * dens[i] % R
    inv = pow(pre[n], R - 2, R)
    acc = [0] * n
    for i in range(n - 1, -1, -1):
        acc[i] = nums[i] * (inv * pre[i] % R) % R
        inv = inv * dens[i] % R
    z_z = ((b7 * z * z + b8 * z + b9) * zh + ev(acc)) % R
    zw = z * omega % R
    w2, scale2 = _bary_weights(n, omega, zw)
    zh2 = (pow(zw, n, R) - 1) % R
    zw_z = ((b7 * zw * zw + b8 * zw + b9) * zh2 + _bary(acc, w2, scale2)) % R
    l1_z = zh * pow(n * (z - 1) % R, R - 2, R) % R  # L_1(z) = (z^n - 1) / (n (z - 1))
    r1 = (q_m_z * a_z * b_z + q_l_z * a_z + q_r_z * b_z + q_o_z * c_z + q_c_z) % R
    r2 = z_z * ((a_z + beta * z + gamma) * (b_z + beta * k1 * z + gamma) * (c_z + beta * k2 * z + gamma)
                * alpha) % R
    k3 = (a_z + beta * s1_z + gamma) * (b_z + beta * s2_z + gamma) * alpha % R
    r4 = z_z * l1_z % R * alpha * alpha % R
    out = {}
    for md in ("reference", "paper"):
        if md == "reference":
            r3 = z_z * s3_z % R * beta * zw_z % R * k3 % R
        else:
            r3 = -(beta * zw_z * k3) * s3_z % R
        out[md] = [a_z, b_z, c_z, s1_z, s2_z, (r1 + r2 + r3 + r4) % R, zw_z]
    return out if mode == "both" else out[mode]


def _accumulator(n, omega, h, sig, a, b, c, beta, gamma, k1, k2):
    """acc_i = prod_{j<i} dend_j / dsor_j (plonk.rs:278-299): prefix products, one batch
    inversion (the same computation as in evaluations_at_z)."""
    nums, dens = [1] * n, [1] * n
    pn = pd = 1
    for i in range(1, n):
        wi = h[i - 1]
        pn = pn * ((a[i - 1] + beta * wi + gamma) * (b[i - 1] + beta * k1 * wi + gamma)
                   * (c[i - 1] + beta * k2 * wi + gamma)) % R
        pd = pd * ((a[i - 1] + beta * sig[0][i - 1] + gamma) * (b[i - 1] + beta * sig[1][i - 1] + gamma)
                   * (c[i - 1] + beta * sig[2][i - 1] + gamma)) % R
        nums[i], dens[i] = pn, pd
    pre = [1] * (n + 1)
    for i in range(n):
        pre[i + 1] = pre[i] * dens[i] % R
    inv = pow(pre[n], R - 2, R)
    acc = [0] * n
    for i in range(n - 1, -1, -1):
        acc[i] = nums[i] * (inv * pre[i] % R) % R
        inv = inv * dens[i] % R
    return acc


def commitment_scalars(n, q, copies, abc, chal, rnd, s, k1=2, k2=3):
    """O(n) pinning of all 9 commitments of Plonk::prove (plonk.rs:245-446) for an SRS
    [s^i]G with known s (SRS::create, plonk.rs:35-48): SRS::eval_at_s(p) = [p(s)]G, and
    every polynomial the prover commits to is evaluated at s from its values on H by the
    barycentric formula (plus its blinding terms), exactly as evaluations_at_z does at z.
    Returns, per mode ("reference", "paper"):
      a, b, c, z:  a(s), b(s), c(s), z(s)                 -> a_s = [a(s)]G, ...
      t:           t(s) = T(s) / Z_H(s) (T = t_1 + t_2 - t_3 + t_4, plonk.rs:339-370)
                                                          -> t_lo + [s^(n+2)] t_mid + [s^(2n+4)] t_hi = [t(s)]G
      wz:          the scalar W with (s - z) W_z(s) = t_lo(s) + z^(n+2) t_mid(s)
                   + z^(2n+4) t_hi(s) + W  (plonk.rs:424-438 with t_z = T(z) / Z_H(z))
                                                          -> [s - z] w_z - t_lo - [z^(n+2)] t_mid - [z^(2n+4)] t_hi = [W]G
      wzw:         (z(s) - z(omega z)) / (s - omega z)    -> w_zw = [wzw]G (plonk.rs:440-442)
      fields:      the proof's 7 field elements (as evaluations_at_z)."""
    omega = F.root_of_unity(n)
    alpha, beta, gamma, z, v = (x % R for x in chal)
    b1, b2, b3, b4, b5, b6, b7, b8, b9 = (x % R for x in rnd)
    s %= R
    h = [1] * n
    for i in range(1, n):
        h[i] = h[i - 1] * omega % R
    tab = (h, [x * k1 % R for x in h], [x * k2 % R for x in h])
    sig = [[tab[k][i - 1] for k, i in col] for col in copies]
    a, b, c = ([x % R for x in col] for col in abc)
    qs = [[x % R for x in col] for col in q]  # q_l q_r q_o q_m q_c
    acc = _accumulator(n, omega, h, sig, a, b, c, beta, gamma, k1, k2)

    def z_at(x):  # z(x) = (b7 x^2 + b8 x + b9) Z_H(x) + acc interpolated (plonk.rs:315)
        w, sc = _bary_weights(n, omega, x)
        return ((b7 * x * x + b8 * x + b9) * (pow(x, n, R) - 1) + _bary(acc, w, sc)) % R

    def at(x):
        w, sc = _bary_weights(n, omega, x)
        ev = lambda vals: _bary(vals, w, sc)  # noqa: E731
        zh = (pow(x, n, R) - 1) % R
        d = {"x": x, "zh": zh}
        d["a"] = ((b1 * x + b2) * zh + ev(a)) % R
        d["b"] = ((b3 * x + b4) * zh + ev(b)) % R
        d["c"] = ((b5 * x + b6) * zh + ev(c)) % R
        d["z"] = ((b7 * x * x + b8 * x + b9) * zh + ev(acc)) % R
        d["s1"], d["s2"], d["s3"] = ev(sig[0]), ev(sig[1]), ev(sig[2])
        d["ql"], d["qr"], d["qo"], d["qm"], d["qc"] = (ev(col) for col in qs)
        d["l1"] = zh * pow(n * (x - 1) % R, R - 2, R) % R
        return d

    def numerator(d, zw):  # T(x) = t_1 + t_2 - t_3 + t_4 (plonk.rs:339-366) from values at x
        x = d["x"]
        t1 = d["a"] * d["b"] * d["qm"] + d["a"] * d["ql"] + d["b"] * d["qr"] + d["c"] * d["qo"] + d["qc"]
        t2 = alpha * (d["a"] + beta * x + gamma) * (d["b"] + beta * k1 * x + gamma) \
            * (d["c"] + beta * k2 * x + gamma) % R * d["z"]
        t3 = alpha * (d["a"] + beta * d["s1"] + gamma) * (d["b"] + beta * d["s2"] + gamma) \
            * (d["c"] + beta * d["s3"] + gamma) % R * zw
        t4 = (d["z"] - 1) * alpha * alpha % R * d["l1"]
        return (t1 + t2 - t3 + t4) % R

    S, Z = at(s), at(z)
    zw_s, zw_z = z_at(omega * s % R), z_at(omega * z % R)
    t_s = numerator(S, zw_s) * pow(S["zh"], R - 2, R) % R
    t_z = numerator(Z, zw_z) * pow(Z["zh"], R - 2, R) % R
    a_z, b_z, c_z, s1_z, s2_z = Z["a"], Z["b"], Z["c"], Z["s1"], Z["s2"]
    k3 = (a_z + beta * s1_z + gamma) * (b_z + beta * s2_z + gamma) * alpha % R
    c2 = (a_z + beta * z + gamma) * (b_z + beta * k1 * z + gamma) * (c_z + beta * k2 * z + gamma) * alpha % R
    out = {}
    for md in ("reference", "paper"):
        def r_at(d, md=md):  # r(x) with the round-4 scalars (plonk.rs:401-419)
            r1 = d["qm"] * a_z * b_z + d["ql"] * a_z + d["qr"] * b_z + d["qo"] * c_z + d["qc"]
            r2 = d["z"] * c2
            if md == "reference":
                r3 = d["z"] * d["s3"] % R * beta * zw_z % R * k3
            else:
                r3 = -(beta * zw_z * k3) * d["s3"]
            r4 = d["z"] * Z["l1"] * alpha * alpha
            return (r1 + r2 + r3 + r4) % R
        r_z = r_at(Z)
        wz = (-t_z + v * (r_at(S) - r_z) + v ** 2 * (S["a"] - a_z) + v ** 3 * (S["b"] - b_z)
              + v ** 4 * (S["c"] - c_z) + v ** 5 * (S["s1"] - s1_z) + v ** 6 * (S["s2"] - s2_z)) % R
        out[md] = {"a": S["a"], "b": S["b"], "c": S["c"], "z": S["z"], "t": t_s, "wz": wz,
                   "wzw": (S["z"] - zw_z) * pow((s - omega * z) % R, R - 2, R) % R,
                   "fields": [a_z, b_z, c_z, s1_z, s2_z, r_z, zw_z]}
    return out


def commitments_match(n, pts, cs, s, z):
    """The five commitment identities of commitment_scalars (one mode's dict `cs`) on the 9
    proof points (affine tuples, None = identity): a_s b_s c_s z_s, the recombined t parts,
    W_z and W_zw. Returns {name: bool}."""
    G, mul, add, neg = B.G1_GEN, B.g1_mul, B.g1_add, B.g1_neg
    a_s, b_s, c_s, z_s, t_lo, t_mid, t_hi, w_z, w_zw = (None if p is None else tuple(p) for p in pts)
    s, z = s % R, z % R
    res = {k: mul(G, cs[k]) == p for k, p in (("a", a_s), ("b", b_s), ("c", c_s), ("z", z_s))}
    t_rec = add(add(t_lo, mul(t_mid, pow(s, n + 2, R))), mul(t_hi, pow(s, 2 * n + 4, R)))
    res["t"] = t_rec == mul(G, cs["t"])
    lhs = add(mul(w_z, (s - z) % R), neg(add(add(t_lo, mul(t_mid, pow(z, n + 2, R))), mul(t_hi, pow(z, 2 * n + 4, R)))))
    res["w_z"] = lhs == mul(G, cs["wz"])
    res["w_zw"] = w_zw == mul(G, cs["wzw"])
    return res
