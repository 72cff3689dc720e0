"""The RCCL branch of csrc/group.hip on one GPU (the
all-to-all of the stride-sharded NTT, fft.rs:94-96).

RCCL refuses two ranks on one device, so these tests load a stand-in librccl
(tests/native/fake_rccl.cpp, built by __graft_entry__.build()) through the library's
PBF_RCCL_LIB override and force the RCCL branch for same-device contexts with
PBF_GROUP_FORCE_RCCL=1. The library then runs exactly the code it runs on G distinct GPUs:
ncclCommInitAll, one grouped ncclSend / ncclRecv per peer for every all-to-all at
send[r] + g b -> recv[r] + g b, ncclAllGather for every all-gather, the host barrier before
each collective, ncclCommAbort when a rank fails. The stand-in keeps RCCL's stream semantics
(a receive waits for the sender's stream, a send completes when its receiver has read it), so
every result is compared bit for bit with the single-GPU entry points, as in
tests/test_multi_capi_gpu.py.
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
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
FAKE = os.path.join(ROOT, "tests", "native", "libfake_rccl.so")


@pytest.fixture(scope="module")
def ranks():
    import pbf

    assert os.path.exists(FAKE), "tests/native/libfake_rccl.so missing: run __graft_entry__.build()"
    saved = {k: os.environ.get(k) for k in ("PBF_RCCL_LIB", "PBF_GROUP_FORCE_RCCL")}
    os.environ["PBF_RCCL_LIB"] = FAKE
    os.environ["PBF_GROUP_FORCE_RCCL"] = "1"
    cs = [pbf.Context(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("G", [2, 4, 8])
def test_ntt_through_rccl_branch(ranks, G):
    import oracle
    import pbf

    n = 1 << 16
    w = pow(7, (GOLD - 1) // n, GOLD)
    a = oracle.splitmix_field(GOLD, 9100 + G, n)
    ctxs = ranks[:G]
    assert pbf.multi_backend(ctxs) == "rccl"
    fwd = pbf.ntt_multi(ctxs, GOLD, w, a)
    assert np.array_equal(fwd, ranks[0].ntt(GOLD, w, a))
    assert np.array_equal(pbf.ntt_multi(ctxs, GOLD, w, fwd, inverse=True), a)


def test_ntt_2p20_golden_digest_through_rccl_branch(ranks, vectors):
    import hashlib

    import oracle
    import pbf

    c = vectors["large"][1]
    a = oracle.splitmix_field(GOLD, c["seed"], c["n"])
    out = pbf.ntt_multi(ranks, GOLD, c["omega"], a)
    assert hashlib.sha256(out.astype("<u8").tobytes()).hexdigest() == c["sha256_fwd"]


@pytest.mark.parametrize("G", [2, 8])
def test_fr_ntt_and_mul_ntt_through_rccl_branch(ranks, G):
    import bn254
    import oracle
    import pbf

    ctxs = ranks[:G]
    n = 1 << 12
    w = bn254.root_of_unity(n)
    a = bn254.limbs_to_ints(bn254.random_limbs(n, 190 + G))
    assert pbf.ntt_fr_multi(ctxs, w, a) == ranks[0].ntt_fr(w, a)
    la, lb = n // 2 + 5, n // 2 - 5
    assert pbf.mul_ntt_fr_multi(ctxs, w, a[:la], a[la:]) == ranks[0].mul_ntt_fr(w, a[:la], a[la:])
    wg = pow(7, (GOLD - 1) // n, GOLD)
    x = oracle.splitmix_field(GOLD, 195, la)
    y = oracle.splitmix_field(GOLD, 196, lb)
    assert np.array_equal(pbf.mul_ntt_multi(ctxs, GOLD, wg, x, y), ranks[0].mul_ntt(GOLD, wg, x, y))


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


def _single(n, seed, mode):
    import pbf

    single = pbf.Context(0)
    try:
        inp = _device_inputs(single, n, seed, mode)
        dq, dc, dabc, dsrs, srs_m, chal, rnd = inp
        ref = single.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd,
                                           dsrs.data_ptr(), srs_m, mode=mode)
    finally:
        single.close()
    return inp, ref


@pytest.mark.parametrize("G,log_n,mode", [(4, 10, 0), (8, 12, 1)])
def test_prove_through_rccl_branch(ranks, G, log_n, mode):
    import pbf

    n = 1 << log_n
    (dq, dc, dabc, dsrs, srs_m, chal, rnd), ref = _single(n, 0x5EED9000 + log_n + G, mode)
    for _ in range(2):  # the second proof takes the ranks' proving keys
        pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                                  [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m,
                                                  mode=mode)
        assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1]), (G, log_n, mode)


def test_prove_2p20_gates_8_ranks_through_rccl_branch(ranks):
    """Config 5's split at 2^20 gates, 8 ranks, every exchange through the RCCL calls."""
    import pbf

    n, G = 1 << 20, 8
    (dq, dc, dabc, dsrs, srs_m, chal, rnd), ref = _single(n, 0x5EED0005, 1)
    pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                              [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m, mode=1)
    assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1])
    for c in ranks:
        c.release_caches()


def test_rank_failure_before_a_collective_releases_the_others(ranks):
    """a rank that fails before a collective (here: its SRS point range lies past a
    too-short SRS, checked before the first exchange, on ranks 2 and 3 only) must not leave the
    other ranks' sends without partners. The call returns the failing rank's error; the aborted
    communicators are dropped and the next call on the same contexts builds new ones and
    succeeds."""
    import pbf

    n, G, mode = 1 << 10, 4, 1
    (dq, dc, dabc, dsrs, srs_m, chal, rnd), ref = _single(n, 0x5EEDA000, mode)
    with pytest.raises(pbf.PbfError, match="SRS too short"):
        pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G, [dabc.data_ptr()] * G,
                                        chal, rnd, [dsrs.data_ptr()] * G, n // 2, mode=mode)
    pts, fs = pbf.plonk_prove_bn254_multi_dev(ranks[:G], n, [dq.data_ptr()] * G, [dc.data_ptr()] * G,
                                              [dabc.data_ptr()] * G, chal, rnd, [dsrs.data_ptr()] * G, srs_m,
                                              mode=mode)
    assert np.array_equal(pts, ref[0]) and np.array_equal(fs, ref[1])


def test_release_caches_frees_exchange_buffers(ranks):
    """pbf_ctx_release_caches frees the group's exchange buffers; the next call
    allocates them again."""
    import oracle
    import pbf

    n = 1 << 12
    w = pow(7, (GOLD - 1) // n, GOLD)
    a = oracle.splitmix_field(GOLD, 9300, n)
    ref = ranks[0].ntt(GOLD, w, a)
    assert np.array_equal(pbf.ntt_multi(ranks[:2], GOLD, w, a), ref)
    ranks[1].release_caches()
    assert np.array_equal(pbf.ntt_multi(ranks[:2], GOLD, w, a), ref)


def test_rank_failure_inside_a_later_collective_aborts_safely(ranks, monkeypatch):
    """a rank that fails inside its half of a LATER collective (after every rank
    passed the pre-post barrier; injected in the stand-in: rank 1's 5th ncclSend, i.e. the first
    send of its second all-to-all at G = 4) while the other ranks are inside their own RCCL calls.
    abort_all takes each rank's post lock before aborting its communicator, so no communicator
    is aborted under a thread still using it; the call returns an error naming a rank, and the
    next call on the same contexts builds a new group and is bit-exact."""
    import oracle
    import pbf

    G = 4
    n = 1 << 12
    w = pow(7, (GOLD - 1) // n, GOLD)
    x = oracle.splitmix_field(GOLD, 9400, n // 2)
    y = oracle.splitmix_field(GOLD, 9401, n // 2)
    ref = ranks[0].mul_ntt(GOLD, w, x, y)
    monkeypatch.setenv("FAKE_RCCL_FAIL_SEND", f"1,{G + 1}")
    with pytest.raises(pbf.PbfError, match="rank"):
        pbf.mul_ntt_multi(ranks[:G], GOLD, w, x, y)
    monkeypatch.delenv("FAKE_RCCL_FAIL_SEND")
    assert np.array_equal(pbf.mul_ntt_multi(ranks[:G], GOLD, w, x, y), ref)
