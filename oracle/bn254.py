"""ORACLE — TEST INFRASTRUCTURE ONLY.

BN254 scalar-field restatement of the reference's FFT / Poly algorithms over Python
big integers (the reference itself has no 256-bit field; SURVEY.md §0.5 picks BN254
for BASELINE configs 3-5, so parity there is "the mathematically defined output of
the fft.rs / poly.rs algorithms"). Only tests/ may import this module.

* ct_fft / ct_fft_inv: fft.rs:90-106 / 71-78 (recursive radix-2 DIT, natural order,
  inverse = reversal x n^-1) — small n only (pure Python).
* ntt: iterative radix-2 (checker for larger n; same values).
* mul_ntt: fft.rs:109-132; poly_mul: poly.rs:205-218 (schoolbook, normalised);
  poly_eval: poly.rs:71-79.
"""
from __future__ import annotations

import numpy as np

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
GEN = 5  # quadratic non-residue: 5^((R-1)/2^k) has order exactly 2^k (k <= 28)
TWO_ADICITY = 28


def root_of_unity(n: int) -> int:
    assert n & (n - 1) == 0 and n <= 1 << TWO_ADICITY
    return pow(GEN, (R - 1) // n, R)


def ct_fft(values, omega: int, p: int = R):
    """fft.rs:55-70,90-106 (CooleyTurkey::new + recursion)."""
    n = len(values)
    pows = [1] * n
    for i in range(1, n):
        pows[i] = pows[i - 1] * omega % p

    def rec(vals, dom):
        if len(vals) == 1:
            return [vals[0]]
        half = dom[0::2]
        left = rec(vals[0::2], half)
        right = rec(vals[1::2], half)
        out = [0] * len(vals)
        h = len(vals) // 2
        for i, (x, y) in enumerate(zip(left, right)):
            t = y * dom[i] % p
            out[i] = (x + t) % p
            out[i + h] = (x - t) % p
        return out

    return rec([int(v) for v in values], pows)


def ct_fft_inv(freq, omega: int, p: int = R):
    """fft.rs:71-78: fft then [v0, v_{n-1}, ..., v1] * n^-1."""
    vals = ct_fft(freq, omega, p)
    ninv = pow(len(freq), p - 2, p)
    return [vals[0] * ninv % p] + [v * ninv % p for v in reversed(vals[1:])]


def ntt(values, omega: int, inverse: bool = False, p: int = R):
    """Iterative radix-2 NTT (checker; identical values to ct_fft)."""
    a = [int(v) for v in values]
    n = len(a)
    w = pow(omega, p - 2, p) if inverse else omega
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j ^= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    length = 2
    while length <= n:
        wl = pow(w, n // length, p)
        tw = [1] * (length // 2)
        for k in range(1, length // 2):
            tw[k] = tw[k - 1] * wl % p
        h = length // 2
        for s in range(0, n, length):
            for k in range(h):
                u, v = a[s + k], a[s + k + h] * tw[k] % p
                a[s + k] = (u + v) % p
                a[s + k + h] = (u - v) % p
        length <<= 1
    if inverse:
        ninv = pow(n, p - 2, p)
        a = [x * ninv % p for x in a]
    return a


def mul_ntt(a, b, omega: int, p: int = R):
    """fft.rs:109-132 (un-normalised, length la+lb)."""
    n = len(a) + len(b)
    fa = ntt(list(a) + [0] * (n - len(a)), omega, p=p)
    fb = ntt(list(b) + [0] * (n - len(b)), omega, p=p)
    return ntt([x * y % p for x, y in zip(fa, fb)], omega, inverse=True, p=p)


def poly_mul(a, b, p: int = R):
    """poly.rs:205-218 schoolbook, then Poly::new normalisation."""
    out = [0] * (len(a) + len(b))
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] = (out[i + j] + x * y) % p
    return normalize(out)


def normalize(c):
    c = list(c)
    while len(c) > 1 and c[-1] == 0:
        c.pop()
    return c


def poly_eval(c, x: int, p: int = R) -> int:
    """poly.rs:71-79 (x^i accumulated)."""
    y = int(c[0]) % p
    xp = 1
    for ci in c[1:]:
        xp = xp * x % p
        y = (y + xp * int(ci)) % p
    return y


# ---- random canonical elements as limbs (fast, numpy) ------------------------
_TOP = R >> 192  # top 64-bit limb of R


def random_limbs(n: int, seed: int) -> np.ndarray:
    """n canonical field elements as a flat [n*4] u64 array (top limb < R's top limb)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 1 << 64, size=(n, 4), dtype=np.uint64, endpoint=False)
    a[:, 3] = a[:, 3] % np.uint64(_TOP)
    return a.reshape(-1)


def limbs_to_ints(a: np.ndarray) -> list:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 4).astype(object)
    v = a[:, 0] + (a[:, 1] << 64) + (a[:, 2] << 128) + (a[:, 3] << 192)
    return [int(x) for x in v]


def ints_to_limbs(values) -> np.ndarray:
    v = np.array([int(x) for x in values], dtype=object)
    m = (1 << 64) - 1
    out = np.empty((len(values), 4), dtype=np.uint64)
    for i in range(4):
        out[:, i] = ((v >> (64 * i)) & m).astype(np.uint64)
    return out.reshape(-1)


# ---- BN254 G1 (y^2 = x^3 + 3 over Fq, generator (1, 2)), affine with None = identity.
# Chord/tangent formulas as in the reference's toy G1 (src/pbh/g1.rs:119-144) over Fq.
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
G1_GEN = (1, 2)


def g1_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % Q == 0:
            return None
        m = 3 * p[0] * p[0] * pow(2 * p[1], Q - 2, Q) % Q
    else:
        m = (q[1] - p[1]) * pow(q[0] - p[0], Q - 2, Q) % Q
    x = (m * m - p[0] - q[0]) % Q
    return (x, (m * (p[0] - x) - p[1]) % Q)


def g1_mul(p, k: int):
    """g1.rs:146-168 double-and-add (LSB first)."""
    r, b = None, p
    while k:
        if k & 1:
            r = g1_add(r, b)
        b = g1_add(b, b)
        k >>= 1
    return r


def g1_on_curve(p) -> bool:
    return p is None or (p[1] * p[1] - p[0] ** 3 - 3) % Q == 0


def msm_naive(points, scalars):
    """plonk.rs:51-58 SRS::eval_at_s: left fold of points[i] * scalars[i]."""
    acc = None
    for p, s in zip(points, scalars):
        acc = g1_add(acc, g1_mul(p, s))
    return acc
