"""GPU parity: libpbf.so NTT / mul_ntt / eval vs the oracle and the golden vectors.

Mirrors the reference's fft.rs tests (test_fft_cooley_turkey, test_ntt_poly_mul)
and extends them to every size class the kernels have (small-kernel path,
2-pass and 3-pass Stockham) and to BASELINE's full sizes (2^20, 2^24) through the
golden digests plus size-independent properties (round trip, linearity)."""
import hashlib

import numpy as np
import pytest

import oracle
import pbf

pytestmark = pytest.mark.gpu
GOLD = pbf.GOLDILOCKS
Q32 = 3221225473


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def root(m, n):
    return pow(7 if m == GOLD else 5, (m - 1) // n, m)


def test_fft_cooley_turkey_kat(ctx, kats):
    # fft.rs:154-168 on the GPU, through the FFT trait mirror
    k = kats["fft_337"]
    ct = pbf.CooleyTurkey.new(k["modulus"], pbf.EvaluationDomainGenerator(k["omega"], k["n"]), ctx)
    freq = ct.fft(k["values"])
    assert freq.tolist() == k["freq"]
    assert ct.fft_inv(freq).tolist() == k["values"]


def test_ntt_poly_mul_kat(ctx, kats):
    # fft.rs:170-183
    k = kats["mul_ntt_337"]
    ct = pbf.CooleyTurkey.new(k["modulus"], pbf.EvaluationDomainGenerator(k["omega"], 8), ctx)
    c = pbf.mul_ntt(ct, k["a"], k["b"])
    assert pbf.normalize(c).tolist() == oracle.poly_mul(k["modulus"], k["a"], k["b"]).tolist()


def test_golden_vectors_all_sizes(ctx, vectors):
    for c in vectors["cases"]:
        a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
        fwd = ctx.ntt(c["modulus"], c["omega"], a)
        assert sha(fwd) == c["sha256_fwd"], (c["modulus"], c["n"])
        assert np.array_equal(ctx.ntt(c["modulus"], c["omega"], fwd, inverse=True), a)


@pytest.mark.parametrize("m", [GOLD, Q32])
@pytest.mark.parametrize("logn", [13, 14, 15, 16, 17, 18, 19, 20, 21])
def test_ntt_vs_oracle_multi_pass(ctx, m, logn):
    n = 1 << logn
    w = root(m, n)
    a = oracle.splitmix_field(m, 1000 + logn, n)
    ref = oracle.ntt_iter(m, w, a)
    got = ctx.ntt(m, w, a)
    assert np.array_equal(got, ref)
    inv = ctx.ntt(m, w, got, inverse=True)
    assert np.array_equal(inv, a)
    assert np.array_equal(ctx.ntt(m, w, ref, inverse=True), oracle.ntt_iter(m, w, ref, inverse=True))


EDGE_GL = [0, 1, 2, GOLD - 1, GOLD - 2, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, 1 << 63, (1 << 63) - 1,
           GOLD - (1 << 32), GOLD - (1 << 32) + 1, (1 << 64) - (1 << 33), 0xFFFFFFFE00000001, 0x00000000FFFFFFFF,
           0x7FFFFFFF80000000]


@pytest.mark.parametrize("logn", [10, 14, 16, 20])
def test_ntt_edge_values(ctx, logn):
    """Inputs drawn only from carry/borrow edge values of the Goldilocks add, sub and
    reduction (0, 1, p-1, 2^32 +- 1, 2^63, p - 2^32, ...), so the first butterfly levels see
    every edge pair (e.g. 0 - 1: a borrow with a low word of 2^32 - 1): bit-exact vs the oracle
    both ways."""
    n = 1 << logn
    w = root(GOLD, n)
    rng = np.random.default_rng(logn)
    a = np.array(EDGE_GL, dtype=np.uint64)[rng.integers(0, len(EDGE_GL), n)]
    ref = oracle.ntt_iter(GOLD, w, a)
    got = ctx.ntt(GOLD, w, a)
    assert np.array_equal(got, ref)
    assert np.array_equal(ctx.ntt(GOLD, w, a, inverse=True), oracle.ntt_iter(GOLD, w, a, inverse=True))
    assert np.array_equal(ctx.ntt(GOLD, w, got, inverse=True), a)


def test_ntt_recursion_faithful_2p14(ctx):
    # the exact algorithm of fft.rs:90-106 (allocation-faithful restatement) at 2^14
    n = 1 << 14
    w = root(GOLD, n)
    a = oracle.splitmix_field(GOLD, 77, n)
    assert np.array_equal(ctx.ntt(GOLD, w, a), oracle.ntt_ct(GOLD, w, a))


def test_large_golden_digests(ctx, vectors):
    # BASELINE config 2 (2^20) and the north-star size (2^24)
    for c in vectors["large"]:
        a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
        fwd = ctx.ntt(c["modulus"], c["omega"], a)
        assert sha(fwd) == c["sha256_fwd"], c["n"]
        for k, v in c["samples"].items():
            assert int(fwd[int(k)]) == v
        assert np.array_equal(ctx.ntt(c["modulus"], c["omega"], fwd, inverse=True), a)


def test_linearity_2p24(ctx):
    n = 1 << 24
    w = root(GOLD, n)
    a = oracle.splitmix_field(GOLD, 5, n)
    b = oracle.splitmix_field(GOLD, 6, n)
    s = np.array([oracle.f("add", GOLD, int(x), int(y)) for x, y in zip(a[:8], b[:8])], dtype=np.uint64)
    # full vector add in numpy with exact wraparound correction
    with np.errstate(over="ignore"):
        t = a + b
        wrap = t < a
        t = np.where(wrap, t + np.uint64(0xFFFFFFFF), t)
        t = np.where(t >= np.uint64(GOLD), t - np.uint64(GOLD), t)
    assert np.array_equal(t[:8], s)
    fa, fb, ft = ctx.ntt(GOLD, w, a), ctx.ntt(GOLD, w, b), ctx.ntt(GOLD, w, t)
    with np.errstate(over="ignore"):
        u = fa + fb
        u = np.where(u < fa, u + np.uint64(0xFFFFFFFF), u)
        u = np.where(u >= np.uint64(GOLD), u - np.uint64(GOLD), u)
    assert np.array_equal(ft, u)


@pytest.mark.parametrize("passes", ["12,12", "8,8,8", "6,6,6,6"])
def test_alternative_pass_plans_2p24(passes, vectors):
    # every radix family the planner can pick gives the same (golden) answer (context option
    # ntt.passes, include/pbf.h)
    c2 = pbf.Context(0, options={"ntt.passes": passes})
    c = vectors["large"][2]
    a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
    assert sha(c2.ntt(c["modulus"], c["omega"], a)) == c["sha256_fwd"]
    c2.close()


@pytest.mark.parametrize("inverse", [False, True])
def test_regrouped_2p24_matches_stockham(inverse):
    """The regrouped 2^24 plan (ntt_gl.hpp ntt_gl_rg2_kernel: general twiddles only between
    64-point blocks, the default for 8,8,8; its last pass forming w^(a0 X) as C[r2][X] D[X]^s2)
    against the round-2 passes (option ntt.no_rg=1), batch of 2 (XCD-blocked tiles), forward
    and inverse, bit-exact, and polynomial 0 against the oracle's iterative transform."""
    import torch

    n, batch = 1 << 24, 2
    w = root(GOLD, n)
    host = np.stack([oracle.splitmix_field(GOLD, 900 + i, n) for i in range(batch)])
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for opts in ({}, {"ntt.no_rg": "1"}):
        c = pbf.Context(0, options=opts)
        d_in = torch.from_numpy(host.view(np.int64)).cuda()
        d_out = torch.empty_like(d_in)
        c.ntt_batch_dev(GOLD, w, d_in.data_ptr(), d_out.data_ptr(), n, batch, inverse=inverse, stream=stream)
        torch.cuda.synchronize()
        outs.append(d_out.cpu().numpy().view(np.uint64).copy())
        c.close()
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[0][0], oracle.ntt_gl_par(w, host[0], inverse=inverse))


def test_batch_dev_matches_single(ctx):
    import torch

    n, batch = 1 << 16, 5
    w = root(GOLD, n)
    host = np.stack([oracle.splitmix_field(GOLD, 300 + i, n) for i in range(batch)])
    d_in = torch.from_numpy(host.view(np.int64)).cuda()
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.ntt_batch_dev(GOLD, w, d_in.data_ptr(), d_out.data_ptr(), n, batch, stream=stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint64)
    for i in range(batch):
        assert np.array_equal(got[i], oracle.ntt_iter(GOLD, w, host[i]))
    # in place
    ctx.ntt_batch_dev(GOLD, w, d_in.data_ptr(), d_in.data_ptr(), n, batch, stream=stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_in.cpu().numpy().view(np.uint64), got)


@pytest.mark.parametrize("opts", [{}, {"ntt.group": "2"}, {"ntt.group": "1", "ntt.streams": "3"},
                                  {"ntt.streams": "1"}, {"ntt.group": "0"}, {"ntt.group": "3", "ntt.streams": "4"}])
@pytest.mark.parametrize("logn", [16, 20])
def test_schedule_options_same_result(opts, logn):
    """Every group / stream schedule of the batched Goldilocks NTT (ntt_launch.hip
    run_gl_passes: context options ntt.group, ntt.streams) gives the oracle's answer, forward
    and inverse, on a batch (9: the default 4-polynomial groups on 2 streams, a last group of 1)."""
    import torch

    ctx = pbf.Context(0, options=opts)
    n, batch = 1 << logn, (9 if logn == 16 else 3)
    w = root(GOLD, n)
    host = np.stack([oracle.splitmix_field(GOLD, 700 + i, n) for i in range(batch)])
    d_in = torch.from_numpy(host.view(np.int64)).cuda()
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.ntt_batch_dev(GOLD, w, d_in.data_ptr(), d_out.data_ptr(), n, batch, stream=stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint64)
    for i in range(batch):
        assert np.array_equal(got[i], oracle.ntt_iter(GOLD, w, host[i]))
    ctx.ntt_batch_dev(GOLD, w, d_out.data_ptr(), d_out.data_ptr(), n, batch, inverse=True, stream=stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), host)
    ctx.close()


@pytest.mark.parametrize("opts", [{"ntt.twmax_log": "18"}, {"ntt.twsplit": "1"},
                                  {"ntt.twmax_log": "18", "ntt.twsplit": "0"}])
def test_twiddle_table_paths(vectors, opts):
    """The three sources of the pass twiddle w^(r k): the per-pass [r][k] table (default up to
    2^ntt.twmax_log = 2^24 entries), the last pass's split table B[kb][r] * A[r][w]
    (default beyond; forced by ntt.twsplit=1) and the two-level table (ntt.twsplit=0): the
    paths of transforms above 2^24 points, exercised at test sizes. Must reproduce the 2^16,
    2^20 and 2^24 golden digests and round-trip."""
    c2 = pbf.Context(0, options=opts)
    try:
        for c in vectors["large"]:
            a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
            fwd = c2.ntt(c["modulus"], c["omega"], a)
            assert sha(fwd) == c["sha256_fwd"], c["n"]
            assert np.array_equal(c2.ntt(c["modulus"], c["omega"], fwd, inverse=True), a)
    finally:
        c2.close()


def test_fill_random_matches_host_generator(ctx):
    import torch

    n = 1 << 18
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.fill_random_dev(GOLD, 0x5EED0002, d.data_ptr(), n, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint64), oracle.splitmix_field(GOLD, 0x5EED0002, n))


@pytest.mark.parametrize("m", [GOLD, Q32, 337, 15485863])
def test_mul_ntt_vs_schoolbook(ctx, m):
    # fft.rs:109-132 vs poly.rs:205-218
    if m == 15485863:
        n, w = 2, m - 1  # 15485862 = 2 * 3 * ..., only order-2 roots
    elif m == 337:
        n, w = 16, pow(10, 336 // 16, 337)
    else:
        n, w = 1 << 11, root(m, 1 << 11)
    a = oracle.splitmix_field(m, 11, n // 2)
    b = oracle.splitmix_field(m, 12, n // 2)
    c = ctx.mul_ntt(m, w, a, b)
    assert np.array_equal(c, oracle.mul_ntt(m, w, a, b))
    assert pbf.normalize(c).tolist() == oracle.poly_mul(m, a, b).tolist()


def test_mul_ntt_golden(ctx, vectors):
    for c in vectors["mul_ntt"]:
        a = oracle.splitmix_field(c["modulus"], c["seed_a"], c["la"])
        b = oracle.splitmix_field(c["modulus"], c["seed_b"], c["lb"])
        assert sha(ctx.mul_ntt(c["modulus"], c["omega"], a, b)) == c["sha256"]


def test_mul_ntt_ragged(ctx):
    # la != lb (only la+lb must equal the domain size)
    n = 1 << 12
    w = root(GOLD, n)
    a = oracle.splitmix_field(GOLD, 21, 1000)
    b = oracle.splitmix_field(GOLD, 22, n - 1000)
    assert np.array_equal(ctx.mul_ntt(GOLD, w, a, b), oracle.mul_ntt(GOLD, w, a, b))


@pytest.mark.parametrize("m", [GOLD, 17, 15485863])
def test_poly_eval(ctx, m, kats):
    # poly.rs:71-79 ; KAT poly.rs:478-481 (x^2+2x+1)(2) = 9
    k = kats["poly_15485863"]
    for c, x, y in k["eval"]:
        assert ctx.poly_eval(15485863, c, [x]).tolist() == [y]
    for n in (1, 7, 300, 20000):
        c = oracle.splitmix_field(m, 40 + n, n)
        xs = oracle.splitmix_field(m, 50 + n, 5)
        got = ctx.poly_eval(m, c, xs)
        assert got.tolist() == [oracle.poly_eval(m, c, int(x)) for x in xs]


def test_size_one_and_two(ctx):
    assert ctx.ntt(GOLD, 1, [5]).tolist() == [5]
    assert ctx.ntt(GOLD, 1, [5], inverse=True).tolist() == [5]
    assert ctx.ntt(GOLD, GOLD - 1, [3, 4]).tolist() == [7, GOLD - 1]


def test_error_codes(ctx):
    with pytest.raises(pbf.PbfError) as e:
        ctx.ntt(GOLD, root(GOLD, 8), [1, 2, 3])  # not a power of two
    assert e.value.code == pbf.PBF_EINVAL
    with pytest.raises(pbf.PbfError) as e:
        ctx.ntt(GOLD, root(GOLD, 16), [1] * 8)  # omega has order 16, not 8
    assert e.value.code == pbf.PBF_EINVAL
    with pytest.raises(pbf.PbfError) as e:
        ctx.ntt(GOLD, root(GOLD, 8), [GOLD] * 8)  # non-canonical input
    assert e.value.code == pbf.PBF_EINVAL
    with pytest.raises(pbf.PbfError) as e:
        ctx.ntt((1 << 61) - 1, 1, [1, 2])  # outside the supported moduli
    assert e.value.code == pbf.PBF_EUNSUPPORTED
    # n = 17 has no inverse mod 17 is impossible for powers of two; use M = 3, n = 2 ... n^-1 exists.
    # F_5 with n = 4: ok; the ENOINV branch needs n = 0 mod M, i.e. M = 2 (even, unsupported) — so
    # only check that a valid small-field inverse works (reference test field F17, omega 4).
    assert ctx.ntt(17, 4, [1, 2, 3, 4], inverse=True).tolist() == oracle.ntt_ct(17, 4, [1, 2, 3, 4], True).tolist()


def test_context_options_errors_and_environment(monkeypatch, vectors):
    """pbf_ctx_set_option rejects unknown names (PBF_EINVAL) and null removes an option; the
    retired environment knobs of earlier rounds change nothing: with them set, a fresh context
    still reproduces the golden digests (they are not read at all, test_capi_exports.py)."""
    c = pbf.Context(0)
    try:
        with pytest.raises(pbf.PbfError) as e:
            c.set_option("ntt.no_such_option", "1")
        assert e.value.code == pbf.PBF_EINVAL
        c.set_option("ntt.passes", "12,12")
        c.set_option("ntt.passes", None)
    finally:
        c.close()
    for k, v in {"PBF_NTT_PASSES": "6,6,6,6", "PBF_NTT_GROUP": "1", "PBF_NTT_TILE": "16384", "PBF_NTT_R4K": "1",
                 "PBF_NTT_PAD": "16", "PBF_NTT_EVENTS": "1", "PBF_NTT_IP": "1"}.items():
        monkeypatch.setenv(k, v)
    c = pbf.Context(0)
    try:
        for cv in vectors["large"]:
            a = oracle.splitmix_field(cv["modulus"], cv["seed"], cv["n"])
            assert sha(c.ntt(cv["modulus"], cv["omega"], a)) == cv["sha256_fwd"], cv["n"]
    finally:
        c.close()
