"""ORACLE — TEST INFRASTRUCTURE ONLY (imported by tests/ and the fixture generators).

Literal restatement of Plonk (src/plonk.rs:15-650) over any `PlonkTypes` instance
(plonk.rs:15-26): the scalar field HF, the group-order field GF, G1 / G2 / pairing and
the constants K1, K2, OMEGA, gf(). Two instances exist:

* oracle/pbh_types.py — the reference's own PlonkByHandTypes (pbh/mod.rs:18-33: F17,
  F101, the toy curve and its reduced Tate pairing). With it this module reproduces the
  reference's end-to-end KAT (pbh/mod.rs:101-123) value for value, which pins every
  formula below to the reference (tests/test_plonk_oracle_pbh.py).
* oracle/plonk_bn254.py — BN254 (HF = GF = Fr), the checker of the GPU prover
  (BASELINE config 5).

Operation-by-operation restatement:
* Poly (poly.rs:11-247): at least one coefficient, normalised by Poly::new / after every
  +=, -=, product (poly.rs:96-105); schoolbook product of length l + r (:205-218);
  scalar product returning Poly::zero() for a zero scalar (:220-228); `p + f` / `p - f`
  touch coefficient 0 only (:179-190); SubAssign<&Poly> keeps the reference's quirk of
  pushing +rhs[i] where rhs is longer (:192-203); long division (:230-247); eval by
  accumulated powers (:71-79).
* interpolate_at_h (plonk.rs:177-179): the Vandermonde inverse times the zero-padded
  value vector is the natural-order inverse DFT over H, computed here by
  the radix-2 inverse NTT of oracle/bn254.py over HF.
* the t(x) split (plonk.rs:376-378, [0..6] [6..12] [12..18] at n = 4) is generalised to
  three slices of n + 2 coefficients; at n = 4 it is the reference's split exactly.

`mode` selects the r_3(x) formula: "reference" = plonk.rs:414-416 literally, "paper" =
the linearisation the verifier checks. The verifier's step 7 keeps
plonk.rs:575-577 (no alpha on the permutation term) in "reference" mode.
"""
from __future__ import annotations

import bn254 as F


# ---------------------------------------------------------------- Poly (poly.rs)
class Poly:
    """Poly<F> (poly.rs:11-125) over Z/m."""

    __slots__ = ("c", "m")

    def __init__(self, coeffs, m: int):
        self.m = m
        self.c = [int(x) % m for x in coeffs] or [0]
        self.normalize()

    @classmethod
    def zero(cls, m):  # poly.rs:34-36
        return cls([0], m)

    def normalize(self):  # poly.rs:96-105
        c = self.c
        while len(c) > 1 and c[-1] == 0:
            c.pop()

    def is_zero(self):  # poly.rs:108-110
        return len(self.c) == 1 and self.c[0] == 0

    def degree(self):  # poly.rs:91-93
        return len(self.c) - 1

    def copy(self):
        p = Poly.__new__(Poly)
        p.m, p.c = self.m, list(self.c)
        return p

    def eval(self, x: int) -> int:  # poly.rs:71-79
        m = self.m
        x_pow, y = 1, self.c[0]
        for ci in self.c[1:]:
            x_pow = x_pow * x % m
            y = (y + x_pow * ci) % m
        return y

    def __add__(self, rhs):
        out = self.copy()
        if isinstance(rhs, Poly):  # AddAssign<&Poly> (poly.rs:165-176)
            for i in range(max(len(out.c), len(rhs.c))):
                if i >= len(out.c):
                    out.c.append(rhs.c[i])
                elif i < len(rhs.c):
                    out.c[i] = (out.c[i] + rhs.c[i]) % out.m
        else:  # AddAssign<&F> (poly.rs:178-183)
            out.c[0] = (out.c[0] + rhs) % out.m
        out.normalize()
        return out

    def __sub__(self, rhs):
        out = self.copy()
        if isinstance(rhs, Poly):  # SubAssign<&Poly> (poly.rs:192-203), quirk at :196 kept
            for i in range(max(len(out.c), len(rhs.c))):
                if i >= len(out.c):
                    out.c.append(rhs.c[i])
                elif i < len(rhs.c):
                    out.c[i] = (out.c[i] - rhs.c[i]) % out.m
        else:  # SubAssign<&F> (poly.rs:185-190)
            out.c[0] = (out.c[0] - rhs) % out.m
        out.normalize()
        return out

    def __mul__(self, rhs):
        m = self.m
        if isinstance(rhs, Poly):  # Mul<&Poly> (poly.rs:205-218)
            out = [0] * (len(self.c) + len(rhs.c))
            for i, x in enumerate(self.c):
                if x:
                    for j, y in enumerate(rhs.c):
                        out[i + j] += x * y
            return Poly(out, m)
        rhs %= m  # MulAssign<&F> (poly.rs:220-228)
        if rhs == 0:
            return Poly.zero(m)
        p = self.copy()
        p.c = [x * rhs % m for x in p.c]
        return p

    def __divmod__(self, rhs):  # Div for Poly (poly.rs:230-247)
        m = self.m
        q, r = Poly.zero(m), self.copy()
        while not r.is_zero() and r.degree() >= rhs.degree():
            lead_r, lead_d = r.c[-1], rhs.c[-1]
            if lead_d % m == 0:
                raise ZeroDivisionError("poly.rs:238 inv().unwrap() on a zero leading coefficient")
            t = Poly.zero(m)
            t.set(len(r.c) - len(rhs.c), lead_r * pow(lead_d, -1, m))
            q = q + t
            r = r - rhs * t
        q.normalize()
        r.normalize()
        return q, r

    def set(self, i, v):  # poly.rs:113-119
        if len(self.c) < i + 1:
            self.c.extend([0] * (i + 1 - len(self.c)))
        self.c[i] = v % self.m
        self.normalize()

    def __eq__(self, other):
        return isinstance(other, Poly) and self.m == other.m and self.c == other.c

    def __repr__(self):
        return f"Poly({self.c})"


def poly_z(points, m):  # Poly::z (poly.rs:64-68)
    acc = Poly([1], m)
    for x in points:
        acc = acc * Poly([-x, 1], m)
    return acc


# ---------------------------------------------------------------- PlonkTypes
class PlonkTypes:
    """plonk.rs:15-26. Subclasses provide the fields, the groups and the constants.

    hf, gf            moduli of HF and GF
    K1, K2, OMEGA     HF constants
    gf_of(x)          P::gf: HF value -> GF value
    g1_gen, g1_identity, g1_add(p, q), g1_neg(p), g1_mul(p, s_gf), g1_in_curve(p)
    g2_gen, g2_mul(p, s_gf)
    pairing_eq(p1, q1, p2, q2)   e(p1, q1) == e(p2, q2)   (plonk.rs:646-650)
    """


# ---------------------------------------------------------------- SRS (plonk.rs:28-59)
class SRS:
    def __init__(self, T: PlonkTypes, s: int, n: int):
        """SRS::create (plonk.rs:35-48): g1s = [G, G s, G s^2, ... G s^n] with the powers
        taken in GF, g2_s = G2 s."""
        self.T = T
        g1s, s_pow = [T.g1_gen], s % T.gf
        for _ in range(n):
            g1s.append(T.g1_mul(T.g1_gen, s_pow))
            s_pow = s_pow * s % T.gf
        self.g1s = g1s
        self.g2_1 = T.g2_gen
        self.g2_s = T.g2_mul(T.g2_gen, s % T.gf)

    def eval_at_s(self, vs: Poly):
        """SRS::eval_at_s (plonk.rs:51-58): left fold from the identity."""
        T = self.T
        acc = T.g1_identity
        for i, v in enumerate(vs.c):
            acc = T.g1_add(acc, T.g1_mul(self.g1s[i], T.gf_of(v)))
        return acc


# ---------------------------------------------------------------- Plonk (plonk.rs:110-650)
class Plonk:
    def __init__(self, T: PlonkTypes, srs: SRS, omega_pows: int):
        """Plonk::new (plonk.rs:120-175)."""
        self.T, self.srs = T, srs
        m = T.hf
        self.h = [pow(T.OMEGA, i, m) for i in range(omega_pows)]
        assert T.K1 not in self.h and T.K2 not in self.h
        self.k1_h = [x * T.K1 % m for x in self.h]
        assert T.K2 not in self.k1_h
        self.k2_h = [x * T.K2 % m for x in self.h]
        self.z_h_x = poly_z(self.h, m)

    def interpolate_at_h(self, vv) -> Poly:
        """plonk.rs:177-179 = natural-order inverse DFT of the zero-padded values
        (matrix.rs:147-155 pads to |H|)."""
        n = len(self.h)
        v = [int(x) % self.T.hf for x in vv] + [0] * (n - len(vv))
        return Poly(F.ntt(v, self.T.OMEGA, inverse=True, p=self.T.hf), self.T.hf)

    def copy_constraints_to_roots(self, cs):
        """plonk.rs:181-189; a copy is (kind 0 = A, 1 = B, 2 = C, 1-based index)."""
        tab = (self.h, self.k1_h, self.k2_h)
        return [tab[k][i - 1] for k, i in cs]

    @staticmethod
    def satisfies(T, q, copies, abc) -> bool:
        """Constrains::satisfies (constraints.rs:198-230), q_l * b quirk at :203 kept."""
        m = T.hf
        q_l, q_r, q_o, q_m, q_c = q
        a, b, c = abc
        for i in range(len(a)):
            r = q_l[i] * a[i] + q_l[i] * b[i] + q_o[i] * c[i] + q_m[i] * a[i] * b[i] + q_c[i]
            if r % m:
                return False
        cols = (a, b, c)
        for i in range(len(a)):
            for col, cs in zip(cols, copies):
                k, j = cs[i]
                if col[i] % m != cols[k][j - 1] % m:
                    return False
        return True

    def prove(self, q, copies, abc, chal, rand, mode="reference"):
        """Plonk::prove (plonk.rs:191-466). q = (q_l, q_r, q_o, q_m, q_c); copies = (c_a, c_b,
        c_c); abc = (a, b, c); chal = (alpha, beta, gamma, z, v); rand = b1..b9.
        Returns (9 G1 points, 7 HF values) in Proof order (plonk.rs:61-95) and the
        intermediate polynomials."""
        T, m = self.T, self.T.hf
        assert Plonk.satisfies(T, q, copies, abc), "constraints.rs:198 (plonk.rs:199 assert)"
        alpha, beta, gamma, z, v = (x % m for x in chal)
        omega, k1, k2 = T.OMEGA, T.K1, T.K2
        n = len(copies[0])
        P = lambda c: Poly(c, m)  # noqa: E731
        ip = self.interpolate_at_h
        sigma_1, sigma_2, sigma_3 = (self.copy_constraints_to_roots(c) for c in copies)
        a_v, b_v, c_v = abc
        q_l, q_r, q_o, q_m, q_c = q
        f_a_x, f_b_x, f_c_x = ip(a_v), ip(b_v), ip(c_v)
        q_o_x, q_m_x, q_l_x, q_r_x, q_c_x = ip(q_o), ip(q_m), ip(q_l), ip(q_r), ip(q_c)
        s_sigma_1, s_sigma_2, s_sigma_3 = ip(sigma_1), ip(sigma_2), ip(sigma_3)
        b1, b2, b3, b4, b5, b6, b7, b8, b9 = (x % m for x in rand)
        # round 1 (plonk.rs:245-257)
        a_x = P([b2, b1]) * self.z_h_x + f_a_x
        b_x = P([b4, b3]) * self.z_h_x + f_b_x
        c_x = P([b6, b5]) * self.z_h_x + f_c_x
        a_s, b_s, c_s = (self.srs.eval_at_s(p) for p in (a_x, b_x, c_x))
        # round 2 (plonk.rs:272-313)
        acc = [1]
        for i in range(1, n):
            a, b, c = a_v[i - 1], b_v[i - 1], c_v[i - 1]
            w = pow(omega, i - 1, m)
            dend = (a + beta * w + gamma) * (b + beta * k1 * w + gamma) * (c + beta * k2 * w + gamma) % m
            dsor = (a + beta * s_sigma_1.eval(w) + gamma) * (b + beta * s_sigma_2.eval(w) + gamma) \
                * (c + beta * s_sigma_3.eval(w) + gamma) % m
            acc.append(acc[i - 1] * (dend * pow(dsor, -1, m)) % m)  # (dend / dsor).unwrap()
        acc_x = ip(acc)
        assert acc_x.eval(pow(omega, n, m)) == 1  # plonk.rs:307
        z_x = P([b9, b8, b7]) * self.z_h_x + acc_x
        z_s = self.srs.eval_at_s(z_x)
        # round 3 (plonk.rs:326-382)
        l_1_x = ip([1] + [0] * (len(self.h) - 1))
        p_i_x = Poly.zero(m)
        a_x_b_x_q_m_x = (a_x * b_x) * q_m_x
        a_x_q_l_x = a_x * q_l_x
        b_x_q_r_x = b_x * q_r_x
        c_x_q_o_x = c_x * q_o_x
        alpha_a_x_beta_x_gamma = (a_x + P([gamma, beta])) * alpha
        b_x_beta_k1_x_gamma = b_x + P([gamma, beta * k1])
        c_x_beta_k2_x_gamma = c_x + P([gamma, beta * k2])
        z_omega_x = P([c * pow(omega, i, m) for i, c in enumerate(z_x.c)])
        alpha_a_x_beta_s_sigma1_x_gamma = (a_x + s_sigma_1 * beta + gamma) * alpha
        b_x_beta_s_sigma2_x_gamma = b_x + s_sigma_2 * beta + gamma
        c_x_beta_s_sigma3_x_gamma = c_x + s_sigma_3 * beta + gamma
        alpha_2_z_x_1_l_1_x = ((z_x + P([m - 1])) * pow(alpha, 2, m)) * l_1_x
        t_1_z_h = a_x_b_x_q_m_x + a_x_q_l_x + b_x_q_r_x + c_x_q_o_x + p_i_x + q_c_x
        t_2_z_h = alpha_a_x_beta_x_gamma * b_x_beta_k1_x_gamma * c_x_beta_k2_x_gamma * z_x
        t_3_z_h = alpha_a_x_beta_s_sigma1_x_gamma * b_x_beta_s_sigma2_x_gamma * c_x_beta_s_sigma3_x_gamma * z_omega_x
        t_4_z_h = alpha_2_z_x_1_l_1_x
        t_x, rem = divmod(t_1_z_h + t_2_z_h - t_3_z_h + t_4_z_h, self.z_h_x)
        assert rem == Poly.zero(m), "plonk.rs:370"
        k = n + 2  # plonk.rs:376-378: [0..6] [6..12] [12..18] at n = 4
        tc = t_x.c + [0] * max(0, 3 * k - len(t_x.c))
        assert len(tc) == 3 * k, "t(x) has more than 3(n+2) coefficients (the slices would panic)"
        t_hi_x, t_mid_x, t_lo_x = P(tc[2 * k:3 * k]), P(tc[k:2 * k]), P(tc[0:k])
        t_hi_s, t_mid_s, t_lo_s = (self.srs.eval_at_s(p) for p in (t_hi_x, t_mid_x, t_lo_x))
        # round 4 (plonk.rs:384-422)
        a_z, b_z, c_z = a_x.eval(z), b_x.eval(z), c_x.eval(z)
        s_sigma_1_z, s_sigma_2_z = s_sigma_1.eval(z), s_sigma_2.eval(z)
        t_z = t_x.eval(z)
        z_omega_z = z_omega_x.eval(z)
        r_1_x = q_m_x * a_z * b_z + q_l_x * a_z + q_r_x * b_z + q_o_x * c_z + q_c_x
        r_2_x = z_x * ((a_z + beta * z + gamma) * (b_z + beta * k1 * z + gamma) * (c_z + beta * k2 * z + gamma)
                       * alpha)
        k3 = (a_z + beta * s_sigma_1_z + gamma) * (b_z + beta * s_sigma_2_z + gamma) * alpha
        if mode == "reference":  # plonk.rs:414-416
            r_3_x = z_x * (s_sigma_3 * beta * z_omega_z) * k3
        else:  # the paper linearisation: -(beta z_omega_z k3) s_sigma_3(x)
            r_3_x = s_sigma_3 * (-(beta * z_omega_z * k3))
        r_4_x = z_x * l_1_x.eval(z) * pow(alpha, 2, m)
        r_x = r_1_x + r_2_x + r_3_x + r_4_x
        r_z = r_x.eval(z)
        # round 5 (plonk.rs:424-446)
        w = (t_lo_x + t_mid_x * pow(z, n + 2, m) + t_hi_x * pow(z, 2 * n + 4, m) - t_z) \
            + (r_x - r_z) * v \
            + (a_x - a_z) * pow(v, 2, m) \
            + (b_x - b_z) * pow(v, 3, m) \
            + (c_x - c_z) * pow(v, 4, m) \
            + (s_sigma_1 - s_sigma_1_z) * pow(v, 5, m) \
            + (s_sigma_2 - s_sigma_2_z) * pow(v, 6, m)
        w_z_x, rem = divmod(w, P([-z, 1]))
        assert rem == Poly.zero(m), "plonk.rs:438"
        w_z_omega_x, rem = divmod(z_x - z_omega_z, P([-z * omega, 1]))
        assert rem == Poly.zero(m), "plonk.rs:442"
        w_z_s, w_z_omega_s = self.srs.eval_at_s(w_z_x), self.srs.eval_at_s(w_z_omega_x)
        pts = [a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_z_s, w_z_omega_s]
        fields = [a_z, b_z, c_z, s_sigma_1_z, s_sigma_2_z, r_z, z_omega_z]
        polys = {"a": a_x, "b": b_x, "c": c_x, "z": z_x, "t": t_x, "t_lo": t_lo_x, "t_mid": t_mid_x,
                 "t_hi": t_hi_x, "r": r_x, "w_z": w_z_x, "w_zw": w_z_omega_x, "s1": s_sigma_1,
                 "s2": s_sigma_2, "s3": s_sigma_3, "acc": acc}
        return pts, fields, polys

    def verify(self, q, copies, pts, fields, chal, u: int, mode="reference") -> bool:
        """Plonk::verify (plonk.rs:468-650); u = rand[0]."""
        T, m, srs = self.T, self.T.hf, self.srs
        a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_z_s, w_z_omega_s = pts
        a_z, b_z, c_z, s_sigma_1_z, s_sigma_2_z, r_z, z_omega_z = (x % m for x in fields)
        alpha, beta, gamma, z, v = (x % m for x in chal)
        omega, k1, k2 = T.OMEGA, T.K1, T.K2
        gf = T.gf_of
        mul, add, neg = T.g1_mul, T.g1_add, T.g1_neg
        ip = self.interpolate_at_h
        q_l, q_r, q_o, q_m, q_c = q
        sigma_1, sigma_2, sigma_3 = (self.copy_constraints_to_roots(c) for c in copies)
        q_m_s, q_l_s, q_r_s, q_o_s, q_c_s = (srs.eval_at_s(ip(x)) for x in (q_m, q_l, q_r, q_o, q_c))
        sigma_1_s, sigma_2_s, sigma_3_s = (srs.eval_at_s(ip(x)) for x in (sigma_1, sigma_2, sigma_3))
        u %= m
        # step 1-2 (plonk.rs:523-547)
        if not all(T.g1_in_curve(p) for p in pts):
            return False
        # step 4-5
        z_h_z = self.z_h_x.eval(z)
        l_1_z = ip([1] + [0] * (len(self.h) - 1)).eval(z)
        p_i_z = 0
        # step 7 (plonk.rs:569-581): no alpha on the permutation term in "reference" mode
        perm = (beta * s_sigma_1_z + gamma + a_z) * (beta * s_sigma_2_z + gamma + b_z) * (c_z + gamma) * z_omega_z
        if mode != "reference":
            perm *= alpha
        if z_h_z % m == 0:
            raise ZeroDivisionError("plonk.rs:581 unwrap(): z is in H")
        t_z = (r_z + p_i_z - perm - l_1_z * pow(alpha, 2, m)) * pow(z_h_z, -1, m) % m
        # step 8
        d_1_s = add(add(add(add(mul(q_m_s, gf(a_z * b_z * v % m)), mul(q_l_s, gf(a_z * v % m))),
                            mul(q_r_s, gf(b_z * v % m))), mul(q_o_s, gf(c_z * v % m))), mul(q_c_s, gf(v)))
        d_2_s = mul(z_s, gf(((a_z + beta * z + gamma) * (b_z + beta * k1 * z + gamma) * (c_z + beta * k2 * z + gamma)
                             * alpha * v + l_1_z * pow(alpha, 2, m) * v + u) % m))
        d_3_s = mul(sigma_3_s, gf((a_z + beta * s_sigma_1_z + gamma) * (b_z + beta * s_sigma_2_z + gamma)
                                  * alpha * v * beta * z_omega_z % m))
        d_s = add(add(d_1_s, d_2_s), neg(d_3_s))
        # step 9
        n = len(copies[0])
        f_s = t_lo_s
        for pt, e in ((t_mid_s, pow(z, n + 2, m)), (t_hi_s, pow(z, 2 * n + 4, m))):
            f_s = add(f_s, mul(pt, gf(e)))
        f_s = add(f_s, d_s)
        for pt, k in ((a_s, 2), (b_s, 3), (c_s, 4), (sigma_1_s, 5), (sigma_2_s, 6)):
            f_s = add(f_s, mul(pt, gf(pow(v, k, m))))
        # step 10
        e_s = mul(srs.eval_at_s(Poly([1], m)), gf((t_z + v * r_z + pow(v, 2, m) * a_z + pow(v, 3, m) * b_z
                                                   + pow(v, 4, m) * c_z + pow(v, 5, m) * s_sigma_1_z
                                                   + pow(v, 6, m) * s_sigma_2_z + u * z_omega_z) % m))
        # step 11 (plonk.rs:636-650)
        e_1_q1 = add(w_z_s, mul(w_z_omega_s, gf(u)))
        e_2_q1 = add(add(add(mul(w_z_s, gf(z)), mul(w_z_omega_s, gf(u * z * omega % m))), f_s), neg(e_s))
        return T.pairing_eq(e_1_q1, srs.g2_s, e_2_q1, srs.g2_1)
