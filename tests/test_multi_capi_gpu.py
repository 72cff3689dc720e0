"""The one-process multi-GPU entry points of include/pbf.h (pbf_*_multi, SURVEY.md §8b
pbf_ntt_u64_multi(ctx[], G, ...)): G contexts on this GPU (virtual ranks), the exchange done
inside libpbf.so (device copies ordered by events; RCCL when the contexts are on distinct
devices, which a one-GPU box cannot exercise). Every result is compared bit for bit with the
single-GPU entry point on the same inputs:

* the Goldilocks / q32 / Fr NTT of one vector (fft.rs:66-78 with the top log2 G levels of the
  recursion, fft.rs:94-96, across ranks), both directions;
* mul_ntt (fft.rs:109-132);
* the device form with per-rank streams that are not torch's current stream;
* Plonk::prove (plonk.rs:191-466) with the sharded work split, both modes, G = 2, 4, 8, and at
  config 5's scale: 2^20 gates on 8 ranks, and 2^24 gates on 8 ranks (peak device bytes
  reported).
"""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))

pytestmark = pytest.mark.gpu
GOLD = 0xFFFFFFFF00000001
Q32 = 3221225473
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


@pytest.fixture(scope="module")
def ranks():
    import pbf

    cs = [pbf.Context(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("m,log_n", [(GOLD, 10), (GOLD, 16), (GOLD, 20), (Q32, 14)])
def test_ntt_multi_matches_single(ranks, G, m, log_n):
    import oracle
    import pbf

    n = 1 << log_n
    w = pow(7 if m == GOLD else 5, (m - 1) // n, m)
    a = oracle.splitmix_field(m, 7000 + G + log_n, n)
    ctxs = ranks[:G]
    assert pbf.multi_backend(ctxs) == "device-copies"
    fwd = pbf.ntt_multi(ctxs, m, w, a)
    assert np.array_equal(fwd, ranks[0].ntt(m, w, a)), (G, log_n)
    back = pbf.ntt_multi(ctxs, m, w, fwd, inverse=True)
    assert np.array_equal(back, a)
    if log_n <= 14:
        assert np.array_equal(fwd, oracle.ntt_iter(m, w, a))


def test_ntt_multi_2p20_golden_digest(ranks, vectors):
    """BASELINE config 2's 2^20 golden digest through the 8-rank one-process entry point."""
    import hashlib

    import oracle
    import pbf

    c = vectors["large"][1]
    a = oracle.splitmix_field(GOLD, c["seed"], c["n"])
    out = pbf.ntt_multi(ranks, GOLD, c["omega"], a)
    assert hashlib.sha256(out.astype("<u8").tobytes()).hexdigest() == c["sha256_fwd"]


@pytest.mark.parametrize("G", [2, 8])
def test_ntt_fr_and_mul_ntt_multi(ranks, G):
    import bn254
    import oracle
    import pbf

    ctxs = ranks[:G]
    n = 1 << 12
    w = bn254.root_of_unity(n)
    a = bn254.limbs_to_ints(bn254.random_limbs(n, 90 + G))
    assert pbf.ntt_fr_multi(ctxs, w, a) == ranks[0].ntt_fr(w, a)
    assert pbf.ntt_fr_multi(ctxs, w, ranks[0].ntt_fr(w, a), inverse=True) == a
    la, lb = n // 2 + 3, n // 2 - 3
    assert pbf.mul_ntt_fr_multi(ctxs, w, a[:la], a[la:]) == ranks[0].mul_ntt_fr(w, a[:la], a[la:])
    wg = pow(7, (GOLD - 1) // n, GOLD)
    x = oracle.splitmix_field(GOLD, 95, la)
    y = oracle.splitmix_field(GOLD, 96, lb)
    assert np.array_equal(pbf.mul_ntt_multi(ctxs, GOLD, wg, x, y), ranks[0].mul_ntt(GOLD, wg, x, y))


def test_ntt_multi_dev_on_non_current_streams(ranks):
    """pbf_ntt_u64_multi_dev with per-rank streams delayed behind matmuls while torch's current
    stream is another one: the library orders its copies on the ranks' streams (events), so the
    result equals the single-GPU transform."""
    import torch

    import oracle
    import pbf
    from multigpu import ShardedNtt

    G, nl, batch = 4, 1 << 14, 2
    N = G * nl
    w = pow(7, (GOLD - 1) // N, GOLD)
    glob = np.stack([oracle.splitmix_field(GOLD, 7100 + b, N) for b in range(batch)])
    shards = [torch.from_numpy(np.ascontiguousarray(glob[:, g::G]).reshape(-1).view(np.int64)).cuda()
              for g in range(G)]
    outs = [torch.empty_like(shards[0]) for _ in range(G)]
    streams = [torch.cuda.Stream() for _ in range(G)]
    x = torch.randn(2048, 2048, device="cuda")
    torch.cuda.synchronize()
    for st in streams:
        with torch.cuda.stream(st):
            y = x
            for _ in range(20):
                y = y @ y
                y = y / y.norm()
    cur = torch.cuda.Stream()
    with torch.cuda.stream(cur):
        pbf.ntt_multi_dev(ranks[:G], GOLD, w, [t.data_ptr() for t in shards], [t.data_ptr() for t in outs], nl, batch,
                          streams=[st.cuda_stream for st in streams])
    torch.cuda.synchronize()
    ref = np.stack([ranks[0].ntt(GOLD, w, glob[b]) for b in range(batch)])
    for r in range(G):
        idx = ShardedNtt.output_indices(r, G, nl)
        assert np.array_equal(outs[r].cpu().numpy().view(np.uint64).reshape(batch, nl), ref[:, idx]), r


def test_multi_errors(ranks):
    import pbf

    with pytest.raises(pbf.PbfError):
        pbf.ntt_multi(ranks[:3], GOLD, 7, [1] * 64)  # world 3
    with pytest.raises(pbf.PbfError):
        pbf.ntt_multi([ranks[0], ranks[0]], GOLD, pow(7, (GOLD - 1) // 64, GOLD), [1] * 64)  # one ctx twice
    with pytest.raises(pbf.PbfError):
        pbf.ntt_multi(ranks[:2], GOLD, pow(7, (GOLD - 1) // 64, GOLD), [1] * 48)  # not 2 * power of two
    with pytest.raises(pbf.PbfError):
        pbf.ntt_multi(ranks[:2], GOLD, pow(7, (GOLD - 1) // 64, GOLD), [GOLD] * 64)  # non-canonical


def _device_inputs(ctx, n, seed, mode):
    import torch

    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, seed, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    rng = random.Random(seed)
    srs_m = 2 * n + 2 if mode == 0 else n + 3
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    ctx.srs_create_dev(rng.randrange(2, R), srs_m - 1, dsrs.data_ptr(), stream=sp)
    chal = [rng.randrange(R) for _ in range(5)]
    rnd = [rng.randrange(R) for _ in range(9)]
    torch.cuda.synchronize()
    return dq, dc, dabc, dsrs, srs_m, chal, rnd


@pytest.mark.parametrize("G,log_n,mode", [(2, 10, 1), (4, 10, 0), (8, 10, 1), (8, 12, 0), (2, 6, 1), (8, 6, 0)])
def test_prove_multi_matches_single(ranks, G, log_n, mode):
    import pbf

    n = 1 << log_n
    single = pbf.Context(0)
    try:
        dq, dc, dabc, dsrs, srs_m, chal, rnd = _device_inputs(single, n, 0x5EED5000 + log_n + G, mode)
        ref = single.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                           dsrs.data_ptr(), srs_m, mode=mode)
    finally:
        single.close()
    ctxs = ranks[:G]
    for _ in range(2):  # the second proof takes the ranks' proving keys
        pts, fs = pbf.plonk_prove_bn254_multi_dev(ctxs, n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                                  [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m,
                                                  mode=mode)
        assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1]), (G, log_n, mode)


def test_prove_multi_modes_interleaved_on_one_key(ranks):
    """One circuit proved in mode 1, then mode 0, then mode 1 on the same sharded contexts: the
    ranks' proving keys are laid out on Ls = n (mode 1) or 2n (mode 0) ranges, so a key built in
    one mode must not be taken by the other. Each proof equals the single-GPU one."""
    import pbf

    n, G = 1 << 10, 4
    single = pbf.Context(0)
    try:
        dq, dc, dabc, dsrs, srs_m, chal, rnd = _device_inputs(single, n, 0x5EED7000, 0)  # SRS long enough for mode 0
        ref = {m: single.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                               dsrs.data_ptr(), srs_m, mode=m) for m in (1, 0)}
    finally:
        single.close()
    for m in (1, 0, 1, 0):
        pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                                  [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m,
                                                  mode=m)
        assert np.array_equal(pts, ref[m][0]) and np.array_equal(fs, ref[m][1]), m


def test_prove_multi_host_inputs_match_oracle(ranks):
    """pbf_plonk_prove_bn254_multi (host inputs) against the literal restatement's committed
    proofs (tests/golden/plonk_bn254.json, oracle/plonk_bn254.py) at their largest n."""
    import json

    import pbf
    import plonk_bn254 as P

    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "plonk_bn254.json")))["cases"]
    case = max((c for c in cases if c["mode"] == "paper"), key=lambda c: c["n"])
    n = case["n"]
    G = 2 if n < 16 else 4
    if n < G * G:
        pytest.skip("fixture too small for a sharded prove")
    q, cp, abc = P.mul_gates_circuit(n, case["circuit_seed"])
    srs = ranks[0].srs_create(case["s"], case["srs_n"])
    pts, fs = pbf.plonk_prove_bn254_multi(ranks[:G], q, cp, abc, case["chal"], case["rnd"], srs, mode=1)
    assert fs == case["fields"]
    assert [list(p) if p else None for p in pts] == case["pts"]


def test_prove_multi_2p20_gates_8_ranks(ranks):
    """Config 5's split at 2^20 gates on 8 virtual ranks, bit-exact against the single-GPU proof."""
    import pbf

    n, G = 1 << 20, 8
    single = pbf.Context(0)
    try:
        dq, dc, dabc, dsrs, srs_m, chal, rnd = _device_inputs(single, n, 0x5EED0005, 1)
        ref = single.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                           dsrs.data_ptr(), srs_m, mode=1)
    finally:
        single.close()
    pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                              [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m, mode=1)
    assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1])
    for c in ranks:
        c.release_caches()
