"""GPU parity of the Poly arithmetic of src/poly.rs beyond mul/eval (csrc/poly.hip):
Div for Poly (poly.rs:230-247) against the oracle's literal long division, and
AddAssign / SubAssign<&Poly> (poly.rs:165-176, 192-203, including the :196 quirk) against a
direct restatement here. Both 64-bit NTT primes: Goldilocks and q32 (the reference-literal
prime, where U64Field<M> arithmetic is exactly the reference's)."""
import random

import numpy as np
import pytest

import oracle
import pbf

pytestmark = pytest.mark.gpu
GOLD, Q32 = pbf.GOLDILOCKS, pbf.Q32


def rand_poly(rnd, m, n, lead_nonzero=True):
    p = [rnd.randrange(m) for _ in range(n)]
    if lead_nonzero and n:
        p[-1] = rnd.randrange(1, m)
    return np.array(p, dtype=np.uint64)


def norm(v):
    v = list(int(x) for x in v)
    while len(v) > 1 and v[-1] == 0:
        v.pop()
    return v


@pytest.mark.parametrize("m", [GOLD, Q32])
@pytest.mark.parametrize("nn,nd", [(1, 1), (5, 1), (5, 3), (8, 8), (100, 37), (1000, 999), (2049, 1024),
                                   (3000, 17), (4097, 2)])
def test_poly_div_vs_oracle(ctx, m, nn, nd):
    rnd = random.Random(nn * 7919 + nd + (m & 0xFFFF))
    num, den = rand_poly(rnd, m, nn), rand_poly(rnd, m, nd)
    q, r = ctx.poly_div(m, num, den)
    oq, orr = oracle.poly_div(m, num, den)
    assert norm(q) == norm(oq) and list(q) == list(oq)
    assert list(r) == list(orr)


@pytest.mark.parametrize("m", [GOLD, Q32])
def test_poly_div_edge_cases(ctx, m):
    rnd = random.Random(5)
    den = rand_poly(rnd, m, 40)
    qq = rand_poly(rnd, m, 61)
    exact = oracle.poly_mul(m, den, qq)
    q, r = ctx.poly_div(m, exact, den)  # exact division: r = 0
    assert list(q) == list(qq) and list(r) == [0]
    # trailing zeros of the divisor do not change the result (Poly is normalised)
    den0 = np.concatenate([den, np.zeros(3, dtype=np.uint64)])
    num = rand_poly(rnd, m, 100)
    assert [list(x) for x in ctx.poly_div(m, num, den0)] == [list(x) for x in oracle.poly_div(m, num, den)]
    # deg num < deg den: q = 0, r = num
    small = rand_poly(rnd, m, 10)
    q, r = ctx.poly_div(m, small, den)
    assert list(q) == [0] and list(r) == list(small)
    # zero numerator
    q, r = ctx.poly_div(m, np.zeros(7, dtype=np.uint64), den)
    assert list(q) == [0] and list(r) == [0]
    # zero divisor: the reference panics at poly.rs:238 (inv().unwrap())
    with pytest.raises(pbf.PbfError) as e:
        ctx.poly_div(m, num, np.zeros(4, dtype=np.uint64))
    assert e.value.code == 2
    # 0 / 0: the reference's loop never runs (poly.rs:234), so no panic: (0, 0)
    q, r = ctx.poly_div(m, np.zeros(3, dtype=np.uint64), np.zeros(2, dtype=np.uint64))
    assert list(q) == [0] and list(r) == [0]
    # a non-zero constant divided by 0 does enter the loop and panics there
    with pytest.raises(pbf.PbfError) as e:
        ctx.poly_div(m, np.array([5], dtype=np.uint64), np.zeros(1, dtype=np.uint64))
    assert e.value.code == 2


def test_poly_div_large_identity(ctx):
    """num = q den + r with deg r < deg den at 2^15-ish sizes (oracle schoolbook product)."""
    rnd = random.Random(11)
    num, den = rand_poly(rnd, GOLD, 20000), rand_poly(rnd, GOLD, 7001)
    q, r = ctx.poly_div(GOLD, num, den)
    assert len(q) == 20000 - 7001 + 1 and len(r) <= 7000
    qd = oracle.poly_mul(GOLD, q, den)
    back = [(int(a) + (int(r[i]) if i < len(r) else 0)) % GOLD for i, a in enumerate(qd)]
    assert norm(back) == norm(num)


def ref_addsub(m, a, b, sub):
    """poly.rs:165-176 / 192-203 restated (the :196 quirk: pushed rhs coefficients keep +)."""
    out = [int(x) for x in a]
    for i in range(max(len(a), len(b))):
        if i >= len(out):
            out.append(int(b[i]))
        elif i < len(b):
            out[i] = (out[i] - int(b[i])) % m if sub else (out[i] + int(b[i])) % m
    return norm(out)


@pytest.mark.parametrize("m", [GOLD, Q32])
@pytest.mark.parametrize("la,lb", [(1, 1), (10, 3), (3, 10), (1000, 1000), (5, 5)])
def test_poly_add_sub(ctx, m, la, lb):
    rnd = random.Random(la * 31 + lb)
    a, b = rand_poly(rnd, m, la, False), rand_poly(rnd, m, lb, False)
    assert [int(x) for x in ctx.poly_add(m, a, b)] == ref_addsub(m, a, b, False)
    assert [int(x) for x in ctx.poly_sub(m, a, b)] == ref_addsub(m, a, b, True)
    # cancellation to the zero polynomial normalises to [0]
    assert [int(x) for x in ctx.poly_sub(m, a, a)] == [0]
