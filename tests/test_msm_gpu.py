"""GPU parity of the BN254 G1 MSM (BASELINE config 4) and SRS::create.

Small n: bit-exact vs the oracle's naive fold (plonk.rs:51-58 restated over BN254).
Config-4 size (2^20 points): points P_i = t_i * G from the batch fixed-base kernel
(sampled points re-derived by the oracle, every point on the curve), and the MSM must
equal (sum_i s_i t_i mod r) * G — the discrete-log identity pins the full-size result
exactly, including the canonical affine encoding."""
import random

import numpy as np
import pytest

import bn254
import pbf

pytestmark = pytest.mark.gpu
R, Q = bn254.R, bn254.Q


def enc(p):
    return (0, 0) if p is None else p


def test_srs_create_matches_oracle(ctx):
    s = 123456789
    pts = ctx.srs_create(s, 8)
    assert pts[0] == bn254.G1_GEN
    for i, p in enumerate(pts):
        assert p == enc(bn254.g1_mul(bn254.G1_GEN, pow(s, i, R)))


@pytest.mark.parametrize("n", [1, 2, 5, 64, 300])
def test_msm_small_vs_naive_fold(ctx, n):
    rnd = random.Random(n)
    pts = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(n)]
    sc = [rnd.randrange(R) for _ in range(n)]
    assert ctx.msm_g1(pts, sc) == enc(bn254.msm_naive(pts, sc))


def test_msm_edge_cases(ctx):
    g = bn254.G1_GEN
    g2 = bn254.g1_mul(g, 2)
    neg = (g[0], Q - g[1])
    # P + P in one bucket (doubling branch), P + (-P) (identity), zero scalars, identity points
    cases = [
        ([g, g], [5, 5]),
        ([g, neg], [7, 7]),
        ([g, g2], [0, 0]),
        ([(0, 0), g], [3, 4]),
        ([g] * 40, [1] * 40),
        ([g, g2], [R - 1, 1]),
        ([g], [(1 << 253) + 12345]),
    ]
    for pts, sc in cases:
        ref = bn254.msm_naive([None if p == (0, 0) else p for p in pts], sc)
        assert ctx.msm_g1(pts, sc) == enc(ref), (pts[:2], sc[:2])
    assert ctx.msm_g1([], []) == (0, 0)


def test_msm_config4_discrete_log_identity(ctx):
    import torch

    n = 1 << 20
    t = bn254.random_limbs(n, 401)
    s = bn254.random_limbs(n, 402)
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    ds = torch.from_numpy(s.view(np.int64)).cuda()
    dp = torch.empty(n * 8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ctx.g1_mul_base_dev(dt.data_ptr(), dp.data_ptr(), n, stream=st)
    torch.cuda.synchronize()
    pts_l = dp.cpu().numpy().view(np.uint64)
    ti, si = bn254.limbs_to_ints(t), bn254.limbs_to_ints(s)
    # sampled points re-derived by the oracle
    for i in (0, 1, 777, n - 1):
        x, y = bn254.limbs_to_ints(pts_l[8 * i: 8 * i + 8])
        assert (x, y) == bn254.g1_mul(bn254.G1_GEN, ti[i])
    got = ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n, stream=st)
    z = sum(a * b for a, b in zip(si, ti)) % R
    assert got == enc(bn254.g1_mul(bn254.G1_GEN, z))


def _dlog_msm(ctx, t_ints, s_ints):
    """MSM of P_i = t_i G with scalars s_i, checked against (sum s_i t_i) G."""
    import torch

    n = len(t_ints)
    t = np.array([[(x >> (64 * k)) & ((1 << 64) - 1) for k in range(4)] for x in t_ints], dtype=np.uint64)
    s = np.array([[(x >> (64 * k)) & ((1 << 64) - 1) for k in range(4)] for x in s_ints], dtype=np.uint64)
    dt = torch.from_numpy(t.reshape(-1).view(np.int64)).cuda()
    ds = torch.from_numpy(s.reshape(-1).view(np.int64)).cuda()
    dp = torch.empty(n * 8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ctx.g1_mul_base_dev(dt.data_ptr(), dp.data_ptr(), n, stream=st)
    torch.cuda.synchronize()
    got = ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n, stream=st)
    z = sum(a * b for a, b in zip(s_ints, t_ints)) % R
    return got == enc(bn254.g1_mul(bn254.G1_GEN, z) if z else None)


@pytest.mark.parametrize("kind", ["equal", "digit_edges", "sparse", "chunk_sizes"])
def test_msm_bucket_chunking_and_signed_digits(ctx, kind):
    """Load-balanced accumulation (csrc/msm.hip msm_chunk_acc / msm_chunk_join) and the
    signed-digit recoding: buckets spanning many 32-entry chunks, digits at the recoding
    boundaries (0x7fff, 0x8000, 0x8001, 0xffff carry chains), mostly-zero windows, and sizes
    around the chunk length."""
    rnd = random.Random(hash(kind) & 0xFFFF)
    if kind == "equal":  # one bucket per window holding all n points (spans n/32 chunks)
        n = 5000
        c = rnd.randrange(R)
        sc = [c] * n
    elif kind == "digit_edges":
        n = 3000
        digs = [0x7FFF, 0x8000, 0x8001, 0xFFFF, 0x0001, 0x0000]
        sc = []
        for _ in range(n):
            v = sum(rnd.choice(digs) << (16 * w) for w in range(16))
            sc.append(v % R)
    elif kind == "sparse":  # a few nonzero windows, many equal buckets
        n = 4000
        sc = [(rnd.randrange(1, 4) << (16 * rnd.randrange(16))) % R for _ in range(n)]
    else:
        for n in (31, 32, 33, 63, 64, 65, 97):
            t = [rnd.randrange(1, R) for _ in range(n)]
            s = [rnd.randrange(R) for _ in range(n)]
            assert _dlog_msm(ctx, t, s), n
        return
    t = [rnd.randrange(1, R) for _ in range(n)]
    assert _dlog_msm(ctx, t, sc)


def test_fixed_base_comb_matches_double_and_add(ctx):
    """The byte-window comb of pbf_g1_bn254_mul_base_dev (SRS::create) against the plain
    double-and-add kernel (context option g1.mul_base = daa), including zero bytes, 0xff bytes,
    0 and r - 1."""
    import torch

    n = 4096
    t = bn254.random_limbs(n, 901)
    t[0:4] = 0
    t[4:8] = [0xFFFFFFFFFFFFFFFF, 0xFF00FF00FF00FF00, 0x00FF00FF00FF00FF, 0x0FFFFFFFFFFFFFFF]
    rm1 = R - 1
    t[8:12] = [(rm1 >> (64 * k)) & ((1 << 64) - 1) for k in range(4)]
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    st = torch.cuda.current_stream().cuda_stream
    a = torch.empty(n * 8, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    ctx.g1_mul_base_dev(dt.data_ptr(), a.data_ptr(), n, stream=st)
    ctx.set_option("g1.mul_base", "daa")
    try:
        ctx.g1_mul_base_dev(dt.data_ptr(), b.data_ptr(), n, stream=st)
        torch.cuda.synchronize()
    finally:
        ctx.set_option("g1.mul_base", None)
    assert torch.equal(a, b)
    assert a[:8].tolist() == [0] * 8  # 0 * G = identity
    # parity anchor: the edge scalars and a sample re-derived by the oracle's double-and-add
    al = a.cpu().numpy().view(np.uint64)
    ti = bn254.limbs_to_ints(t)
    for i in [0, 1, 2, 3, 1000, n - 1]:  # 0, the 0xff/0x00 byte patterns, r - 1, samples
        want = bn254.g1_mul(bn254.G1_GEN, ti[i] % R)
        assert tuple(bn254.limbs_to_ints(al[8 * i: 8 * i + 8])) == enc(want), i


def _dev_points(pts):
    import torch

    return torch.from_numpy(pbf._g1_limbs(pts).view(np.int64)).cuda()


def _dev_scalars(sc):
    import torch

    return torch.from_numpy(pbf.ints_to_limbs(sc).view(np.int64)).cuda()


@pytest.mark.parametrize("n_points,n", [(1, 1), (7, 7), (300, 300), (300, 17), (4096, 4000)])
def test_fixed_base_msm_vs_naive_fold(ctx, n_points, n):
    """pbf_msm_g1_bn254_fixed_dev (window table 2^(16w) P_i, one bucket set) == the oracle's
    naive fold of SRS::eval_at_s (plonk.rs:51-58) over the first n base points."""
    rnd = random.Random(n_points * 7 + n)
    pts = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(min(n_points, 64))]
    pts = (pts * (n_points // len(pts) + 1))[:n_points]  # repeats: P + P in one bucket
    sc = [rnd.randrange(R) for _ in range(n)]
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    got = ctx.msm_g1_fixed_dev(dp.data_ptr(), n_points, ds.data_ptr(), n)
    ref = bn254.msm_naive(pts[:n], sc) if n <= 300 else None
    if ref is not None:
        assert got == enc(ref)
    assert got == ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n)  # the windowed Pippenger agrees


def test_fixed_base_msm_edges_and_cache(ctx):
    import torch

    g = bn254.G1_GEN
    neg = (g[0], Q - g[1])
    pts = [g, neg, (0, 0), bn254.g1_mul(g, 2), g]
    sc = [5, 5, 9, 0, R - 1]
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    ref = bn254.msm_naive([None if p == (0, 0) else p for p in pts], sc)
    assert ctx.msm_g1_fixed_dev(dp.data_ptr(), len(pts), ds.data_ptr(), len(pts)) == enc(ref)
    # the cached table is rebuilt when the points at the same address change
    pts2 = [bn254.g1_mul(g, 3 + i) for i in range(len(pts))]
    dp.copy_(_dev_points(pts2))
    torch.cuda.synchronize()
    assert ctx.msm_g1_fixed_dev(dp.data_ptr(), len(pts), ds.data_ptr(), len(pts)) == enc(bn254.msm_naive(pts2, sc))
    # all-zero scalars: the identity
    dz = _dev_scalars([0] * len(pts))
    assert ctx.msm_g1_fixed_dev(dp.data_ptr(), len(pts), dz.data_ptr(), len(pts)) == (0, 0)


@pytest.mark.parametrize("n_points,which", [(3001, 3000), (3001, 0), (70001, 35000)])
def test_fixed_base_cache_sees_one_changed_point(ctx, n_points, which):
    """The table cache's exact-content check (k_snap_compare) notices one point negated in
    place, at the first, the middle or the last position of the set; the answer equals the
    windowed MSM's over the changed points."""
    import torch

    rnd = random.Random(n_points + which)
    base = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(29)]
    pts = (base * (n_points // len(base) + 1))[:n_points]
    sc = [rnd.randrange(R) for _ in range(n_points)]
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    first = ctx.msm_g1_fixed_dev(dp.data_ptr(), n_points, ds.data_ptr(), n_points)
    assert first == ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n_points)
    pts[which] = (pts[which][0], Q - pts[which][1])
    dp.copy_(_dev_points(pts))
    torch.cuda.synchronize()
    got = ctx.msm_g1_fixed_dev(dp.data_ptr(), n_points, ds.data_ptr(), n_points)
    assert got == ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n_points)
    assert got != first


@pytest.mark.parametrize("n_points,n", [(300, 255), (300, 256), (300, 300), (70001, 70001), (70001, 69000)])
def test_fixed_base_digit_sort_matches_windowed(ctx, n_points, n):
    """The MSM sorts' first pass from 16-bit digit codes (msm_sort.hpp RsDigits; fixed-base and
    windowed forms) against the naive fold, including tiles that straddle two windows (n not a
    multiple of the 8192-entry tile). n = 255 is just below the digit-code path's minimum
    (rs_dig_ok: n >= 256: the pair sort there); n = 256 is the smallest digit-code case."""
    rnd = random.Random(n_points + n)
    base = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(32)]
    pts = (base * (n_points // len(base) + 1))[:n_points]
    sc = [rnd.randrange(R) for _ in range(n)]
    sc[::97] = [0] * len(sc[::97])  # zero scalars: every window's code is "no entry"
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    ptr = ds.data_ptr()
    got = ctx.msm_g1_fixed_dev(dp.data_ptr(), n_points, ptr, n)
    assert got == ctx.msm_g1_dev(dp.data_ptr(), ptr, n)  # the windowed form's 3-pass sort
    if n <= 300:
        assert got == enc(bn254.msm_naive(pts[:n], sc))


@pytest.mark.parametrize("n_points,first,n", [(1000, 300, 256), (1000, 1, 999), (70001, 8193, 40000), (600, 599, 1)])
def test_fixed_base_range_first_nonzero(ctx, n_points, first, n):
    """pbf_msm_g1_bn254_fixed_range_dev: scalars against points [first, first + n) of the fixed
    base set -- the value encoding w * n_table + first + i of the digit-code sort with first > 0
    (a sharded commitment's point range) -- equals the windowed MSM and the naive sum."""
    rnd = random.Random(n_points * 7 + first)
    base = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(37)]
    pts = (base * (n_points // len(base) + 1))[:n_points]
    sc = [rnd.randrange(R) for _ in range(n)]
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    res = {"1": ctx.msm_g1_fixed_range_dev(dp.data_ptr(), n_points, first, ds.data_ptr(), n)}
    # the same range as a plain MSM over the sliced points (windowed path, no table)
    dsl = _dev_points(pts[first:first + n])
    assert res["1"] == ctx.msm_g1_dev(dsl.data_ptr(), ds.data_ptr(), n)
    if n <= 1000:
        assert res["1"] == enc(bn254.msm_naive(pts[first:first + n], sc))
    with pytest.raises(pbf.PbfError):
        ctx.msm_g1_fixed_range_dev(dp.data_ptr(), n_points, first, ds.data_ptr(), n_points - first + 1)


def test_fixed_base_msm_2p20_discrete_log(ctx):
    """Config-4 size through the fixed-base path: P_i = t_i G, result (sum s_i t_i) G."""
    import torch

    m = 1 << 20
    rng = np.random.default_rng(44)
    t = bn254.random_limbs(m, 45)
    s = bn254.random_limbs(m, 46)
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    dsc = torch.from_numpy(s.view(np.int64)).cuda()
    pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
    ctx.g1_mul_base_dev(dt.data_ptr(), pts.data_ptr(), m)
    got = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, dsc.data_ptr(), m)
    tv, sv = bn254.limbs_to_ints(t), bn254.limbs_to_ints(s)
    k = sum(a * b for a, b in zip(tv, sv)) % R
    assert got == enc(bn254.g1_mul(bn254.G1_GEN, k))
    del rng


@pytest.mark.parametrize("c", [16, 18, 20, 22])
def test_fixed_base_window_widths(ctx, c):
    """The fixed-base table's window width (option msm.fx_c, round 4: ceil(255 / c) windows of
    2^(c-1) signed-digit buckets, 32-bit digit codes above c = 16, sorts of c key bits in passes
    of balanced digit widths, the generalised quad reduction tail) gives the windowed MSM's
    result: random scalars, digits at the c-bit recoding boundaries with carry chains, zero
    scalars, tiles straddling windows, and a point range."""
    rnd = random.Random(c)
    ctx.set_option("msm.fx_c", c)
    h = 1 << (c - 1)
    edges = [h - 1, h, h + 1, (1 << c) - 1, 1, 0]
    base = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) for _ in range(41)]
    for n_points, n, kind in [(300, 300, "random"), (3000, 3000, "edges"), (70001, 70001, "random"),
                              (5000, 5000, "equal")]:
        pts = (base * (n_points // len(base) + 1))[:n_points]
        if kind == "random":
            sc = [rnd.randrange(R) for _ in range(n)]
            sc[::97] = [0] * len(sc[::97])
        elif kind == "edges":
            sc = [sum(rnd.choice(edges) << (c * w) for w in range(256 // c + 1)) % R for _ in range(n)]
        else:
            sc = [rnd.randrange(R)] * n
        dp, ds = _dev_points(pts), _dev_scalars(sc)
        want = ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n)
        assert ctx.msm_g1_fixed_dev(dp.data_ptr(), n_points, ds.data_ptr(), n) == want, (c, kind)
        if n == 300:
            assert want == enc(bn254.msm_naive(pts, sc))
    first, n = 8193, 40000
    pts = (base * (70001 // len(base) + 1))[:70001]
    sc = [rnd.randrange(R) for _ in range(n)]
    dp, ds = _dev_points(pts), _dev_scalars(sc)
    got = ctx.msm_g1_fixed_range_dev(dp.data_ptr(), len(pts), first, ds.data_ptr(), n)
    assert got == ctx.msm_g1_dev(_dev_points(pts[first:first + n]).data_ptr(), ds.data_ptr(), n)
    ctx.release_caches()
    ctx.set_option("msm.fx_c", None)


@pytest.mark.parametrize("c", [20, 22])
def test_fixed_base_wide_windows_2p20_discrete_log(ctx, c):
    """Config 4's size with the wide-window table: P_i = t_i G, result (sum s_i t_i) G."""
    import torch

    ctx.set_option("msm.fx_c", c)
    m = 1 << 20
    t = bn254.random_limbs(m, 45 + c)
    s = bn254.random_limbs(m, 46 + c)
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    dsc = torch.from_numpy(s.view(np.int64)).cuda()
    pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
    ctx.g1_mul_base_dev(dt.data_ptr(), pts.data_ptr(), m)
    got = ctx.msm_g1_fixed_dev(pts.data_ptr(), m, dsc.data_ptr(), m)
    tv, sv = bn254.limbs_to_ints(t), bn254.limbs_to_ints(s)
    k = sum(a * b for a, b in zip(tv, sv)) % R
    assert got == enc(bn254.g1_mul(bn254.G1_GEN, k))
    ctx.release_caches()
    ctx.set_option("msm.fx_c", None)


@pytest.mark.parametrize("c", [16, 22])
def test_fixed_base_heavy_buckets(ctx, c):
    """Skewed digit distributions through the fixed-base joins: 2^18 equal scalars (every
    window's n entries in ONE bucket: spans of ~6100 chunks, past the per-chunk steps' 4096, so
    msm_join_rest_g finishes them) and 2^18 small scalars (< 2^40: two or three nonzero windows,
    a few thousand heavy buckets). Compared with the windowed MSM; P_i = t_i G random."""
    import torch

    ctx.set_option("msm.fx_c", c)
    m = 1 << 18
    t = bn254.random_limbs(m, 700 + c)
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    pts = torch.empty(m * 8, dtype=torch.int64, device="cuda")
    ctx.g1_mul_base_dev(dt.data_ptr(), pts.data_ptr(), m)
    rng = np.random.default_rng(c)
    eq = np.tile(bn254.random_limbs(1, 800 + c).reshape(1, 4), (m, 1))
    small = np.zeros((m, 4), dtype=np.uint64)
    small[:, 0] = rng.integers(0, 1 << 40, size=m, dtype=np.uint64)
    for sc in (eq, small):
        ds = torch.from_numpy(np.ascontiguousarray(sc).reshape(-1).view(np.int64)).cuda()
        want = ctx.msm_g1_dev(pts.data_ptr(), ds.data_ptr(), m)
        assert ctx.msm_g1_fixed_dev(pts.data_ptr(), m, ds.data_ptr(), m) == want, c
    ctx.release_caches()
    ctx.set_option("msm.fx_c", None)


