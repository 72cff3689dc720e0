"""The 29-bit-limb lazy Fr arithmetic of the NTT passes (csrc/fr29.hpp, ntt256.hip
ntt256l_pass_kernel; round 6): constants against scripts/gen_l29_constants.py, a Python
restatement of every operation step for step (product scanning with its 64-bit columns, the
redundant-limb differences, the quotient-estimate reduction, the final conditional
subtractions), and the bounds the kernel relies on, propagated as intervals through the
radix-4 DIF stage from the largest stage inputs and exercised on
random and extreme elements against exact arithmetic mod r. CPU only."""
import os
import random
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import gen_l29_constants as G  # noqa: E402

R = G.R
MASK = (1 << 29) - 1
C = G.fr_constants()
R29, NR29, QC = C["R29"], C["NR29"][0], C["QC"][0]
B4R, B8R, B2R = C["B4R"], C["B8R"], C["B2R"]
RP = 1 << 261


def test_header_constants_match_generator():
    src = open(os.path.join(ROOT, "plonk-by-fingers_amd", "csrc", "fr29.hpp")).read()
    for name, vals in C.items():
        m = re.search(r"constexpr uint32_t " + name + r"(?:\[9\])? = \{?([^;}]*)\}?;", src)
        assert m, name
        got = [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]
        assert got == vals, name


def val(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def limbs(v):
    return G.limbs(v)


def mul(a, b):
    """fr29::mul: a b 2^-261 mod r, every column below 2^64"""
    m, r, acc = [0] * 9, [0] * 9, 0
    for k in range(17):
        lo, hi = (0, k) if k < 9 else (k - 8, 8)
        for i in range(lo, hi + 1):
            acc += a[i] * b[k - i]
        for i in range(lo, k if k < 9 else 9):
            acc += m[i] * R29[k - i]
        assert acc < 1 << 64, "column overflow"
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * NR29) & MASK
            acc += m[k] * R29[0]
            assert acc < 1 << 64 and acc & MASK == 0
        else:
            r[k - 9] = acc & MASK
        acc >>= 29
    r[8] = acc
    assert r[8] < 1 << 32
    return r


def add(a, b):
    r = [x + y for x, y in zip(a, b)]
    assert all(x < 1 << 32 for x in r)
    return r


def sub(a, b, B):
    assert all(bi <= Bi for bi, Bi in zip(b, B)), "borrow"
    r = [x + (Bi - y) for x, y, Bi in zip(a, b, B)]
    assert all(x < 1 << 32 for x in r)
    return r


def reduce(a):
    t = (a[8] + (a[7] >> 29)) & 0xFFFFFFFF
    q = (t * QC) >> 32
    x = val(a)
    assert q <= x // R, "q overestimates"
    out, acc = [0] * 9, 0
    for i in range(9):
        acc += a[i] - q * R29[i]
        if i < 8:
            out[i] = acc & MASK
            acc >>= 29
    assert acc >= 0
    out[8] = acc
    assert val(out) == x - q * R
    return out


def csub(a):
    d, borrow = [0] * 9, 0
    for i in range(9):
        x = a[i] - R29[i] - borrow
        borrow = 1 if x < 0 else 0
        d[i] = x & MASK if i < 8 else x
    return a if borrow else d


def canon(a):
    v = val(csub(csub(a)))
    assert 0 <= v < R
    return v


# ---- interval bounds: (per-limb maxima, value maximum) of a lazily reduced element
def b_norm(vmax):
    top = vmax >> 232
    return ([MASK] * 8 + [top], vmax)


def b_add(a, b):
    return ([x + y for x, y in zip(a[0], b[0])], a[1] + b[1])


def b_sub(a, b, B):
    assert all(x <= y for x, y in zip(b[0], B)), "bias limb below the subtrahend's"
    return ([x + y for x, y in zip(a[0], B)], a[1] + val(B))


def b_mul(a, w):
    """column maxima of the product scan for limbs up to a's and w's (w: a table twiddle, < r)"""
    for k in range(17):
        lo, hi = (0, k) if k < 9 else (k - 8, 8)
        col = sum(a[0][i] * w[0][k - i] for i in range(lo, hi + 1)) + sum(
            MASK * R29[k - i] for i in range(lo, k if k < 9 else 9))
        assert col + (1 << 35) < 1 << 64, ("column", k)
    return b_norm((a[1] * w[1] + (RP - 1) * R) // RP)


def b_reduce(a):
    """reduce(): t = x's top limb plus limb 7's carry is at least T - 1 (T = x >> 232: the limbs
    below add less than one unit), so q >= floor((T - 1) QC / 2^32); the largest result is at
    the top of a T range just before q steps up, or at the top of the input range"""
    assert all(x < 1 << 32 for x in a[0])
    tmax = a[1] >> 232
    worst = 0
    cands = {tmax}
    for k in range(0, tmax * QC // (1 << 32) + 2):
        t1 = -(-(k + 1) * (1 << 32) // QC)  # smallest T - 1 with q = k + 1
        for T in (t1, t1 - 1, t1 + 1):
            if 0 <= T <= tmax:
                cands.add(T)
    for T in cands:
        x = min(a[1], ((T + 1) << 232) - 1)
        q = max(0, (T - 1) * QC >> 32)
        worst = max(worst, x - q * R)
    return b_norm(worst)


TW = b_norm(R - 1)


def stage_bounds(vin):
    """bounds of the outputs of one radix-4 DIF stage (ntt256.hip dft4_29) from stage inputs
    normalised below vin"""
    v = [b_norm(vin)] * 4
    n0 = b_add(v[0], v[2])
    n2 = b_sub(v[0], v[2], B4R)
    n1 = b_add(v[1], v[3])
    n3 = b_mul(b_sub(v[1], v[3], B4R), TW)
    outs = [b_add(n0, n1), b_sub(n0, n1, B8R), b_add(n2, n3), b_sub(n2, n3, B2R)]
    for o in outs:
        assert all(x < 1 << 32 for x in o[0])
    return outs


def test_stage_bounds_close():
    """From canonical loads (and products of them) the stage outputs, reduced, stay below the
    bound the stage inputs were assumed to have: the invariant holds for every stage of a pass,
    and the radix-2 stage (dft2_29) too."""
    vin = 2 * R + (1 << 234)  # assumed stage-input bound (normalised)
    for _ in range(3):
        outs = stage_bounds(vin)
        # the next stage loads the unreduced outputs: c != 0 rows through the inter-stage
        # twiddle's product (its columns must hold for these limbs), c = 0 rows through reduce()
        assert max(b_reduce(o)[1] for o in outs) < vin
        assert max(b_mul(o, TW)[1] for o in outs) < vin
        # the pass twiddle of a canonical load
        assert b_mul(b_norm(R - 1), TW)[1] < vin
    o2 = [b_add(b_norm(vin), b_norm(vin)), b_sub(b_norm(vin), b_norm(vin), B4R)]
    assert max(b_reduce(o)[1] for o in o2) < vin
    assert max(o[1] for o in stage_bounds(vin)) < RP  # a product may take any of them (not needed)


def dft4(v, w4):
    n0 = add(v[0], v[2])
    n2 = sub(v[0], v[2], B4R)
    n1 = add(v[1], v[3])
    n3 = mul(sub(v[1], v[3], B4R), w4)
    return [add(n0, n1), sub(n0, n1, B8R), add(n2, n3), sub(n2, n3, B2R)]


def test_stage_on_extreme_and_random_elements():
    """Stages of radix-4 DIF with reductions between them on canonical extremes (0, 1, r - 1,
    r - 2) and random values, against exact arithmetic mod r (w4 = a fourth root of unity times
    2^261, as the tables hold it)."""
    w = pow(5, (R - 1) // 4, R)
    w4 = limbs(w * RP % R)
    tw = limbs(pow(5, (R - 1) // 1024, R) * RP % R)
    rng = random.Random(29)
    pools = [[R - 1] * 4, [0, R - 1, 0, R - 1], [R - 1, 0, R - 1, 0], [1, R - 2, R - 1, R - 1]]
    pools += [[rng.randrange(R) for _ in range(4)] for _ in range(200)]
    for xs in pools:
        v = [limbs(x) for x in xs]
        ref = list(xs)
        for _stage in range(3):
            v = dft4(v, w4)
            a, b, c, d = ref
            n0, n2, n1, n3 = (a + c) % R, (a - c) % R, (b + d) % R, (b - d) * w % R
            ref = [(n0 + n1) % R, (n0 - n1) % R, (n2 + n3) % R, (n2 - n3) % R]
            assert [val(x) % R for x in v] == ref
            # the next stage's loads: one row reduced (c = 0), the others through the twiddle
            # product, one of them by w^0 (k = 0)
            f = pow(5, (R - 1) // 1024, R)
            one = limbs(RP % R)
            v = [reduce(v[0]), mul(v[1], tw), mul(v[2], one), mul(v[3], tw)]
            ref = [ref[0], ref[1] * f % R, ref[2], ref[3] * f % R]
        assert [canon(reduce(x)) for x in v] == ref


def test_mul_matches_montgomery():
    rng = random.Random(31)
    for _ in range(300):
        x, y = rng.randrange(R), rng.randrange(R)
        assert val(mul(limbs(x), limbs(y))) % R == x * y * pow(RP, -1, R) % R
    # the largest lazily reduced operand the stage feeds a product: limbs at the interval maxima
    big = [MASK + B4R[i] if i < 8 else (2 * R >> 232) + B4R[8] for i in range(9)]
    assert val(mul(big, limbs(R - 1))) % R == val(big) * (R - 1) * pow(RP, -1, R) % R
