"""GPU BN254 pairing (csrc/pairing.hip) through the C-ABI vs the pairing oracle
(oracle/bn254_pairing.py): full Fq12 values, bilinearity, the KZG opening check of
Plonk::verify (src/plonk.rs:646-650) on a GPU MSM commitment, identity inputs, G2
scalar multiplication, input validation."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bn254_pairing as B  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import pbf

    c = pbf.Context(0)
    yield c
    c.close()


def test_pairing_generators_matches_oracle(ctx):
    got = ctx.pairing_bn254([B.G1_GEN], [B.G2_GEN])[0]
    assert got == B.f12_flat(B.pairing(B.G1_GEN, B.G2_GEN))


def test_pairing_batch_random_points(ctx):
    rng = random.Random(4)
    ps = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    qs = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    got = ctx.pairing_bn254(ps, qs)
    for p, q, g in zip(ps, qs, got):
        assert g == B.f12_flat(B.pairing(p, q))


def test_pairing_identity_inputs(ctx):
    one = B.f12_flat(B.F12_ONE)
    got = ctx.pairing_bn254([None, B.G1_GEN], [B.G2_GEN, None])
    assert got == [one, one]


def test_bilinearity_on_device(ctx):
    a, b = 77, 1009
    e1, e2 = ctx.pairing_bn254([B.g1_mul(B.G1_GEN, a), B.G1_GEN], [B.g2_mul(B.G2_GEN, b), B.G2_GEN])
    assert e1 == B.f12_flat(B.f12_pow(B.f12_from_flat(e2), a * b))


@pytest.fixture
def lane_ctx():
    """A context with the lane engine forced (option pair.engine = lane, below its batch
    threshold)."""
    import pbf

    c = pbf.Context(0, options={"pair.engine": "lane"})
    yield c
    c.close()


def test_lane_engine_matches_oracle(lane_ctx):
    """The lane-per-pairing engine (pairing_lane_kernel, option pair.engine = lane forces it
    below its batch threshold) against the oracle: generators, random points, identities,
    bilinearity."""
    ctx = lane_ctx
    rng = random.Random(41)
    ps = [B.G1_GEN, None, B.G1_GEN] + [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(2)]
    qs = [B.G2_GEN, B.G2_GEN, None] + [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(2)]
    got = ctx.pairing_bn254(ps, qs)
    one = B.f12_flat(B.F12_ONE)
    assert got[1] == one and got[2] == one
    for idx in (0, 3, 4):
        assert got[idx] == B.f12_flat(B.pairing(ps[idx], qs[idx])), idx
    a, b = 77, 1009
    e1, e2 = ctx.pairing_bn254([B.g1_mul(B.G1_GEN, a), B.G1_GEN], [B.g2_mul(B.G2_GEN, b), B.G2_GEN])
    assert e1 == B.f12_flat(B.f12_pow(B.f12_from_flat(e2), a * b))


def test_lane_engine_matches_workgroup_engine(ctx):
    """A batch of 131 pairs (two full waves and a ragged one; identities mixed in) through both
    engines, bit for bit (the default for this size is the lane engine)."""
    rng = random.Random(43)
    n = 131
    ks = [rng.randrange(1, B.R) for _ in range(n)]
    ls = [rng.randrange(1, B.R) for _ in range(n)]
    ps = ctx.g1_bn254_mul([B.G1_GEN] * n, ks) if hasattr(ctx, "g1_bn254_mul") else [B.g1_mul(B.G1_GEN, k) for k in ks]
    qs = ctx.g2_bn254_mul([B.G2_GEN] * n, ls)
    ps[5] = None
    qs[77] = None
    try:
        ctx.set_option("pair.engine", "wg")
        wg = ctx.pairing_bn254(ps, qs)
        ctx.set_option("pair.engine", "lane")
        lane = ctx.pairing_bn254(ps, qs)
    finally:
        ctx.set_option("pair.engine", None)
    assert lane == wg


def test_lane_engine_two_wave_build_matches(lane_ctx):
    """The lane kernel built for two waves per SIMD (taken from 2 x 4 x CUs waves, i.e. batches of
    >= 131072 on MI355X) against the unconstrained build, bit for bit, on a ragged batch with
    identities (option pair.lane_wpe forces either build)."""
    ctx = lane_ctx
    rng = random.Random(47)
    n = 150
    ps = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(n)]
    qs = ctx.g2_bn254_mul([B.G2_GEN] * n, [rng.randrange(1, B.R) for _ in range(n)])
    ps[3] = None
    qs[100] = None
    ctx.set_option("pair.lane_wpe", 1)
    one = ctx.pairing_bn254(ps, qs)
    ctx.set_option("pair.lane_wpe", 2)
    two = ctx.pairing_bn254(ps, qs)
    assert one == two
    assert one[7] == B.f12_flat(B.pairing(ps[7], qs[7]))


def test_g2_mul_matches_oracle(ctx):
    rng = random.Random(9)
    ks = [0, 1, 2, B.R - 1, rng.randrange(B.R), rng.randrange(B.R)]
    got = ctx.g2_bn254_mul([B.G2_GEN] * len(ks), ks)
    assert got == [B.g2_mul(B.G2_GEN, k) for k in ks]


def test_kzg_opening_check(ctx):
    """KZG over a GPU MSM commitment: C = [p(s)]_1, W = [(p(s)-y)/(s-z)]_1,
    e(W, [s]G2) * e(-(C - y G + z W), G2) == 1; a wrong y fails."""
    import bn254 as F  # scalar-field oracle (poly eval / division)

    rng = random.Random(5)
    s = rng.randrange(1, B.R)
    n = 16
    srs = ctx.srs_create(s, n)            # [G, sG, ..., s^n G] on the GPU (plonk.rs:35-48)
    coeffs = [rng.randrange(B.R) for _ in range(n)]
    z = rng.randrange(B.R)
    y = F.poly_eval(coeffs, z)
    # quotient (p(x) - y)/(x - z) by synthetic division
    q = [0] * (n - 1)
    acc = 0
    for i in range(n - 1, 0, -1):
        acc = (acc * z + coeffs[i]) % B.R
        q[i - 1] = acc
    c_pt = ctx.msm_g1(srs[:n], coeffs)
    w_pt = ctx.msm_g1(srs[: n - 1], q)
    s2 = ctx.g2_bn254_mul([B.G2_GEN], [s])[0]

    def lhs_point(yv):
        t = B.g1_add(c_pt, B.g1_neg(B.g1_mul(B.G1_GEN, yv)))
        t = B.g1_add(t, B.g1_mul(w_pt, z))
        return B.g1_neg(t)

    assert ctx.pairing_check_bn254([w_pt, lhs_point(y)], [s2, B.G2_GEN])
    assert not ctx.pairing_check_bn254([w_pt, lhs_point((y + 1) % B.R)], [s2, B.G2_GEN])


def test_non_canonical_coordinate_rejected(ctx):
    import pbf

    with pytest.raises(pbf.PbfError):
        ctx.pairing_bn254([(B.Q, 2)], [B.G2_GEN])


def _balanced_pairs(ctx, rng, npairs):
    """npairs (a_i G1, b_i G2) with sum a_i b_i = 0 mod r (product of pairings = 1)."""
    a = [rng.randrange(1, B.R) for _ in range(npairs)]
    b = [rng.randrange(1, B.R) for _ in range(npairs)]
    a[-1] = -sum(x * y for x, y in zip(a[:-1], b[:-1])) * pow(b[-1], B.R - 2, B.R) % B.R
    ps = [B.g1_mul(B.G1_GEN, x) for x in a]
    qs = ctx.g2_bn254_mul([B.G2_GEN] * npairs, b)
    return ps, qs


@pytest.mark.parametrize("npairs", [2, 3, 5])
def test_pairing_check_multi_pair(ctx, npairs):
    """The multi-Miller check (pairs in chunks of two, an odd tail of one, the chunk
    values multiplied before one final exponentiation) against the oracle's check."""
    rng = random.Random(100 + npairs)
    ps, qs = _balanced_pairs(ctx, rng, npairs)
    assert ctx.pairing_check_bn254(ps, qs)
    assert B.pairing_check(list(zip(ps, qs)))
    bad = list(ps)
    bad[npairs // 2] = B.g1_add(bad[npairs // 2], B.G1_GEN)
    assert not ctx.pairing_check_bn254(bad, qs)
    assert not B.pairing_check(list(zip(bad, qs)))


def test_pairing_check_identity_pairs(ctx):
    """Identity pairs contribute 1 anywhere in the product (either side)."""
    rng = random.Random(7)
    ps, qs = _balanced_pairs(ctx, rng, 3)
    assert ctx.pairing_check_bn254([ps[0], None, ps[1], B.G1_GEN, ps[2]], [qs[0], qs[1], qs[1], None, qs[2]])
    assert ctx.pairing_check_bn254([None], [B.G2_GEN])
    assert not ctx.pairing_check_bn254([B.G1_GEN], [B.G2_GEN])


def test_pairing_check_prepared_lines_cache(ctx):
    """The context reuses prepared G2 lines only for the same G2 bytes: alternating G2
    sets and a same-G2 / different-G1 call all give the oracle's answers."""
    rng = random.Random(11)
    p1, q1 = _balanced_pairs(ctx, rng, 2)
    p2, q2 = _balanced_pairs(ctx, rng, 2)
    assert ctx.pairing_check_bn254(p1, q1)
    assert ctx.pairing_check_bn254(p2, q2)
    assert ctx.pairing_check_bn254(p1, q1)
    assert not ctx.pairing_check_bn254(p2, q1)  # same G2 as the cached set, other G1
    assert not ctx.pairing_check_bn254(p1, [q1[0], q2[1]])


def test_pairing_check_empty(ctx):
    assert ctx.pairing_check_bn254([], [])
