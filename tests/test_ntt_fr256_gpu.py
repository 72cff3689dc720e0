"""GPU parity of the BN254-Fr NTT and mul_ntt (BASELINE config 3) vs the Python
big-integer oracle (oracle/bn254.py): exact at small and medium sizes, and at the
config-3 size (a, b of 2^22 coefficients, NTT size 2^23) exactly too, through the SHA-256
of the whole product that the recursion-faithful C++ oracle computed in the container
(tests/golden/config3_mul_ntt.json, tests/golden/gen_config3_digest.py), plus
size-independent properties (round trip, evaluation identity c(x) = a(x) b(x))."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import bn254
import pbf

pytestmark = pytest.mark.gpu
R = bn254.R


@pytest.mark.parametrize("logn", [0, 1, 2, 3, 5, 8, 11])
def test_small_vs_recursion_faithful(ctx, logn):
    n = 1 << logn
    w = bn254.root_of_unity(n) if n > 1 else 1
    a = bn254.limbs_to_ints(bn254.random_limbs(n, 10 + logn))
    got = ctx.ntt_fr(w, a)
    assert got == (bn254.ct_fft(a, w) if n > 1 else a)
    assert ctx.ntt_fr(w, got, inverse=True) == a


@pytest.mark.parametrize("maxr", [None, "5"])
@pytest.mark.parametrize("logn", [12, 13, 14, 15, 16, 17])
def test_multi_pass_vs_oracle(logn, maxr):
    """Multi-pass Fr NTT both ways vs the oracle; maxr: with passes of at most 2^5 points (context
    option ntt256.maxr: more, lighter passes, the planner's other radix families)."""
    ctx = pbf.Context(0, options={"ntt256.maxr": maxr} if maxr else None)
    n = 1 << logn
    w = bn254.root_of_unity(n)
    a = bn254.limbs_to_ints(bn254.random_limbs(n, 20 + logn))
    got = ctx.ntt_fr(w, a)
    assert got == bn254.ntt(a, w)
    assert ctx.ntt_fr(w, got, inverse=True) == a
    ctx.close()


def test_kat_structure_small_field_values(ctx):
    # DFT of a delta / constant vector has a closed form (any field)
    n = 1 << 13
    w = bn254.root_of_unity(n)
    delta = [0] * n
    delta[1] = 1
    assert ctx.ntt_fr(w, delta)[:4] == [1, w, w * w % R, pow(w, 3, R)]
    assert ctx.ntt_fr(w, [7] * n) == [7 * n % R] + [0] * (n - 1)


@pytest.mark.parametrize("k", [3, 6, 9, 12])
def test_mul_ntt_vs_schoolbook(ctx, k):
    # fft.rs:171-183 property: Poly::new(mul_ntt(a, b)) == a * b
    n = 1 << k
    rnd = random.Random(k)
    a = [rnd.randrange(R) for _ in range(n // 2)]
    b = [rnd.randrange(R) for _ in range(n // 2)]
    c = ctx.mul_ntt_fr(bn254.root_of_unity(n), a, b)
    if k <= 9:
        assert bn254.normalize(c) == bn254.poly_mul(a, b)
    else:
        assert c == bn254.mul_ntt(a, b, bn254.root_of_unity(n))


def test_mul_ntt_config3_size_evaluation_identity(ctx):
    # BASELINE config 3: a, b of 2^22 coefficients -> domain 2^23
    import torch

    la = 1 << 22
    n = 2 * la
    w = bn254.root_of_unity(n)
    a = bn254.random_limbs(la, 301)
    b = bn254.random_limbs(la, 302)
    da = torch.zeros(n * 4, dtype=torch.int64, device="cuda")
    db = torch.zeros_like(da)
    da[: la * 4] = torch.from_numpy(a.view(np.int64)).cuda()
    db[: la * 4] = torch.from_numpy(b.view(np.int64)).cuda()
    dc = torch.empty_like(da)
    ctx.mul_ntt_fr_dev(w, da.data_ptr(), db.data_ptr(), dc.data_ptr(), n, 1,
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = dc.cpu().numpy().view(np.uint64)
    with open(os.path.join(os.path.dirname(__file__), "golden", "config3_mul_ntt.json")) as fh:
        gold = json.load(fh)
    assert (gold["la"], gold["lb"], gold["seeds"]) == (la, la, [301, 302])
    # exact parity of all 2^23 product coefficients with oracle_fr_mul_ntt (fft.rs:109-132)
    assert hashlib.sha256(host.astype("<u8").tobytes()).hexdigest() == gold["sha256_le_u64"]
    c = bn254.limbs_to_ints(host)
    for i, v in gold["samples"].items():
        assert c[int(i)] == int(v)
    ai, bi = bn254.limbs_to_ints(a), bn254.limbs_to_ints(b)
    assert c[-1] == 0  # deg(a*b) = 2^23 - 2
    for x in (3, 123456789123456789):
        assert bn254.poly_eval(c, x) == bn254.poly_eval(ai, x) * bn254.poly_eval(bi, x) % R
    # forward/inverse round trip at 2^23 through the device batch entry point
    dd = torch.empty_like(dc)
    ctx.ntt_fr_batch_dev(w, dc.data_ptr(), dd.data_ptr(), n, 1)
    ctx.ntt_fr_batch_dev(w, dd.data_ptr(), dd.data_ptr(), n, 1, inverse=True)
    torch.cuda.synchronize()
    assert torch.equal(dd, dc)


@pytest.mark.parametrize("logn", [21, 22])
def test_twiddle_table_forms_agree(logn):
    """The last pass's twiddles two ways: a per-pass table filled on the device (default, past
    2^20 entries) and the two-level tables (context option ntt256.twlog = 20, the path of passes
    past 2^26 entries): identical forward and inverse outputs and mul_ntt products, and the round
    trip restores the input."""
    import torch

    n = 1 << logn
    w = bn254.root_of_unity(n)
    x = torch.from_numpy(bn254.random_limbs(n, 40 + logn).view(np.int64)).cuda()
    y = torch.from_numpy(bn254.random_limbs(n, 50 + logn).view(np.int64)).cuda()
    half = torch.zeros_like(x)
    half[: n * 2] = x[: n * 2]  # n/2 coefficients, zero-padded: a mul_ntt operand
    outs = []
    for opts in ({}, {"ntt256.twlog": "20"}):
        c = pbf.Context(0, options=opts)
        try:
            f = torch.empty_like(x)
            c.ntt_fr_batch_dev(w, x.data_ptr(), f.data_ptr(), n, 1)
            i = torch.empty_like(x)
            c.ntt_fr_batch_dev(w, f.data_ptr(), i.data_ptr(), n, 1, inverse=True)
            hy = torch.zeros_like(y)
            hy[: n * 2] = y[: n * 2]
            m = torch.empty_like(x)
            c.mul_ntt_fr_dev(w, half.data_ptr(), hy.data_ptr(), m.data_ptr(), n, 1,
                             stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert torch.equal(i, x)
            outs.append((f, m))
        finally:
            c.close()
    for f, m in outs[1:]:
        assert torch.equal(f, outs[0][0])
        assert torch.equal(m, outs[0][1])


def test_fr_errors(ctx):
    with pytest.raises(pbf.PbfError):
        ctx.ntt_fr(bn254.root_of_unity(16), [1] * 8)  # omega order 16 != 8
    with pytest.raises(pbf.PbfError):
        ctx.ntt_fr(bn254.root_of_unity(8), [R] * 8)  # non-canonical


@pytest.mark.parametrize("logn,maxr", [(12, "4"), (13, "5"), (14, "6"), (15, "7"), (16, "8"), (18, "9"), (21, None),
                                       (23, None)])
def test_l29_passes_match_32bit_passes(logn, maxr):
    """The 29-bit-limb pass kernels (ntt256l_pass_kernel, default; fr29.hpp) against the 32-bit
    ones (context option ntt256.l29 = 0), bit for bit, through every pass radix (4..9) and the
    config-3 size: forward, inverse and the fused mul_ntt, on random inputs and on the worst
    cases of the lazy bounds (every element r - 1; alternating 0 and r - 1)."""
    import torch

    n = 1 << logn
    w = bn254.root_of_unity(n)
    rm1 = np.array([(R - 1) >> (64 * k) & ((1 << 64) - 1) for k in range(4)], dtype=np.uint64)
    inputs = [bn254.random_limbs(n, 70 + logn), np.tile(rm1, n)]
    alt = np.tile(rm1, n).reshape(n, 4)
    alt[::2] = 0
    inputs.append(alt.reshape(-1))
    res = []
    for opts in ({"ntt256.l29": "0"}, {}):
        if maxr:
            opts = dict(opts, **{"ntt256.maxr": maxr})
        c = pbf.Context(0, options=opts)
        try:
            outs = []
            for x_np in inputs:
                x = torch.from_numpy(np.ascontiguousarray(x_np).view(np.int64)).cuda()
                f = torch.empty_like(x)
                c.ntt_fr_batch_dev(w, x.data_ptr(), f.data_ptr(), n, 1)
                i = torch.empty_like(x)
                c.ntt_fr_batch_dev(w, x.data_ptr(), i.data_ptr(), n, 1, inverse=True)
                half = torch.zeros_like(x)
                half[: n * 2] = x[: n * 2]
                hb = torch.zeros_like(x)
                hb[: n * 2] = f[: n * 2]  # canonical values of another shape
                m = torch.empty_like(x)
                c.mul_ntt_fr_dev(w, half.data_ptr(), hb.data_ptr(), m.data_ptr(), n, 1,
                                 stream=torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                outs.append((f.cpu(), i.cpu(), m.cpu()))
            res.append(outs)
        finally:
            c.close()
    for a, b in zip(res[0], res[1]):
        for u, v in zip(a, b):
            assert torch.equal(u, v)
    # every output canonical
    for f, i, m in res[1]:
        for t in (f, i, m):
            top = t.numpy().view(np.uint64).reshape(-1, 4)[:, 3]
            assert int(top.max()) <= (R >> 192)
