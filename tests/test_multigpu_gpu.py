"""GPU parity of the stride-sharded NTT kernels on one MI355X.

G virtual ranks run the real pbf_ntt_shard_local_dev / pbf_ntt_shard_combine_dev
kernels on their shards; the all-to-all is done by device copies in this
process (the RCCL exchange itself is exercised by bench.py at N > 1 and its
orchestration by tests/test_multigpu_gloo.py). The assembled output must equal
the oracle's whole-vector NTT bit for bit, and the inverse must return the shards."""
import numpy as np
import pytest
import torch

import oracle
import pbf
from multigpu import ShardedNtt

pytestmark = pytest.mark.gpu
GOLD = pbf.GOLDILOCKS
Q32 = 3221225473


def _run(ctx, m, G, nl, batch, seed):
    N = G * nl
    w = pow(7 if m == GOLD else 5, (m - 1) // N, m)
    s = nl // G
    glob = np.stack([oracle.splitmix_field(m, seed + b, N) for b in range(batch)])
    stream = torch.cuda.current_stream().cuda_stream
    shards = [torch.from_numpy(np.ascontiguousarray(glob[:, g::G]).reshape(-1).view(np.int64)).cuda()
              for g in range(G)]
    sends = [torch.empty_like(shards[0]) for _ in range(G)]
    for g in range(G):
        ctx.shard_local_dev(m, w, G, shards[g].data_ptr(), sends[g].data_ptr(), nl, batch, stream=stream)
    # all-to-all: recv_r[g] = send_g[r]
    recvs = [torch.cat([sends[g].view(G, -1)[r] for g in range(G)]) for r in range(G)]
    outs = [torch.empty_like(shards[0]) for _ in range(G)]
    for r in range(G):
        ctx.shard_combine_dev(m, w, G, r, recvs[r].data_ptr(), outs[r].data_ptr(), nl, batch, stream=stream)
    torch.cuda.synchronize()
    X = np.zeros((batch, N), dtype=np.uint64)
    for r in range(G):
        idx = ShardedNtt.output_indices(r, G, nl)
        X[:, idx] = outs[r].cpu().numpy().view(np.uint64).reshape(batch, nl)
    for b in range(batch):
        assert np.array_equal(X[b], oracle.ntt_iter(m, w, glob[b])), (G, nl, b)
    # inverse: combine(inv) -> all-to-all -> local(inv)
    sends2 = [torch.empty_like(shards[0]) for _ in range(G)]
    for r in range(G):
        ctx.shard_combine_dev(m, w, G, r, outs[r].data_ptr(), sends2[r].data_ptr(), nl, batch, inverse=True,
                              stream=stream)
    recvs2 = [torch.cat([sends2[g].view(G, -1)[r] for g in range(G)]) for r in range(G)]
    backs = [torch.empty_like(shards[0]) for _ in range(G)]
    for g in range(G):
        ctx.shard_local_dev(m, w, G, recvs2[g].data_ptr(), backs[g].data_ptr(), nl, batch, inverse=True,
                            stream=stream)
    torch.cuda.synchronize()
    for g in range(G):
        assert torch.equal(backs[g], shards[g]), (G, nl, g)


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("nl", [1 << 6, 1 << 12, 1 << 14, 1 << 17])
def test_sharded_ntt_goldilocks(ctx, G, nl):
    _run(ctx, GOLD, G, nl, 2, 900 + G)


@pytest.mark.parametrize("G", [2, 8])
def test_sharded_ntt_q32(ctx, G):
    _run(ctx, Q32, G, 1 << 13, 3, 950 + G)


def test_sharded_ntt_2p20_global_matches_golden(ctx, vectors):
    # 8 ranks x 2^17 = the 2^20 golden digest of BASELINE config 2
    import hashlib

    c = vectors["large"][1]
    assert c["n"] == 1 << 20
    G, nl = 8, (1 << 20) // 8
    a = oracle.splitmix_field(GOLD, c["seed"], c["n"])
    stream = torch.cuda.current_stream().cuda_stream
    shards = [torch.from_numpy(np.ascontiguousarray(a[g::G]).view(np.int64)).cuda() for g in range(G)]
    sends = [torch.empty_like(shards[0]) for _ in range(G)]
    for g in range(G):
        ctx.shard_local_dev(GOLD, c["omega"], G, shards[g].data_ptr(), sends[g].data_ptr(), nl, 1, stream=stream)
    recvs = [torch.cat([sends[g].view(G, -1)[r] for g in range(G)]) for r in range(G)]
    X = np.zeros(c["n"], dtype=np.uint64)
    for r in range(G):
        out = torch.empty_like(shards[0])
        ctx.shard_combine_dev(GOLD, c["omega"], G, r, recvs[r].data_ptr(), out.data_ptr(), nl, 1, stream=stream)
        torch.cuda.synchronize()
        X[ShardedNtt.output_indices(r, G, nl)] = out.cpu().numpy().view(np.uint64)
    assert hashlib.sha256(X.astype("<u8").tobytes()).hexdigest() == c["sha256_fwd"]


def test_shard_errors(ctx):
    d = torch.empty(64, dtype=torch.int64, device="cuda")
    w = pow(7, (GOLD - 1) // 192, GOLD)
    with pytest.raises(pbf.PbfError):
        ctx.shard_local_dev(GOLD, w, 3, d.data_ptr(), d.data_ptr(), 64, 1)  # G = 3
    w128 = pow(7, (GOLD - 1) // 128, GOLD)
    with pytest.raises(pbf.PbfError):
        ctx.shard_combine_dev(GOLD, w128, 2, 0, d.data_ptr(), d.data_ptr(), 64, 1)  # in == out


@pytest.mark.parametrize("G", [2, 4, 8])
def test_sharded_msm_ranges_gpu(ctx, G):
    """Point-range MSM sharding (multigpu.ShardedMsm) with the real kernels: G virtual ranks
    on one GPU, each a partial MSM of its range, the partial sums combined by GpuMsmOps —
    equal to the MSM of the whole set (the pieces bench.py runs one per GPU)."""
    import bn254
    import torch
    from multigpu import GpuMsmOps, ShardedMsm

    n = 5000
    t = bn254.random_limbs(n, 811)
    s = bn254.random_limbs(n, 812)
    dt = torch.from_numpy(t.view(np.int64)).cuda()
    ds = torch.from_numpy(s.view(np.int64)).cuda()
    dp = torch.empty(n * 8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ctx.g1_mul_base_dev(dt.data_ptr(), dp.data_ptr(), n, stream=st)
    torch.cuda.synchronize()
    ops = GpuMsmOps(ctx, st)
    parts = []
    for r in range(G):
        a, b = ShardedMsm.split(n, G, r)
        parts.append(ops.partial(dp[8 * a:].data_ptr(), ds[4 * a:].data_ptr(), b - a))
    full = ctx.msm_g1_dev(dp.data_ptr(), ds.data_ptr(), n, stream=st)
    got = ops.combine(parts)
    assert got == full
    # parity anchor: P_i = t_i G, so the MSM is (sum_i s_i t_i mod r) G, computed by the oracle
    z = sum(a * b for a, b in zip(bn254.limbs_to_ints(s), bn254.limbs_to_ints(t))) % bn254.R
    assert got == (bn254.g1_mul(bn254.G1_GEN, z) if z else (0, 0))


def _fr_rand(count, seed):
    import bn254

    return bn254.limbs_to_ints(bn254.random_limbs(count, seed))


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("nl", [1 << 4, 1 << 9, 1 << 12])
def test_sharded_ntt_fr256(ctx, G, nl):
    """pbf_ntt_fr256_shard_local_dev / _combine_dev: G virtual ranks, device-copy all-to-all,
    assembled output == the single-GPU Fr NTT of the whole vector; the inverse returns the shards."""
    import bn254

    N, batch = G * nl, 2
    w = bn254.root_of_unity(N)
    glob = [_fr_rand(N, 31 * G + b) for b in range(batch)]
    stream = torch.cuda.current_stream().cuda_stream
    enc = lambda v: torch.from_numpy(bn254.ints_to_limbs(v).view(np.int64)).cuda()  # noqa: E731
    shards = [enc([x for b in range(batch) for x in glob[b][g::G]]) for g in range(G)]
    sends = [torch.empty_like(shards[0]) for _ in range(G)]
    for g in range(G):
        ctx.fr_shard_local_dev(w, G, shards[g].data_ptr(), sends[g].data_ptr(), nl, batch, stream=stream)
    recvs = [torch.cat([sends[g].view(G, -1)[r] for g in range(G)]) for r in range(G)]
    outs = [torch.empty_like(shards[0]) for _ in range(G)]
    for r in range(G):
        ctx.fr_shard_combine_dev(w, G, r, recvs[r].data_ptr(), outs[r].data_ptr(), nl, batch, stream=stream)
    ref = torch.cat([enc(g) for g in glob])
    ctx.ntt_fr_batch_dev(w, ref.data_ptr(), ref.data_ptr(), N, batch, stream=stream)
    torch.cuda.synchronize()
    refv = bn254.limbs_to_ints(ref.cpu().numpy().view(np.uint64))
    for r in range(G):
        got = bn254.limbs_to_ints(outs[r].cpu().numpy().view(np.uint64))
        idx = ShardedNtt.output_indices(r, G, nl)
        for b in range(batch):
            assert got[b * nl:(b + 1) * nl] == [refv[b * N + i] for i in idx], (G, nl, r, b)
    sends2 = [torch.empty_like(shards[0]) for _ in range(G)]
    for r in range(G):
        ctx.fr_shard_combine_dev(w, G, r, outs[r].data_ptr(), sends2[r].data_ptr(), nl, batch, inverse=True,
                                 stream=stream)
    recvs2 = [torch.cat([sends2[g].view(G, -1)[r] for g in range(G)]) for r in range(G)]
    for g in range(G):
        back = torch.empty_like(shards[0])
        ctx.fr_shard_local_dev(w, G, recvs2[g].data_ptr(), back.data_ptr(), nl, batch, inverse=True, stream=stream)
        torch.cuda.synchronize()
        assert torch.equal(back, shards[g]), (G, nl, g)


@pytest.mark.parametrize("field,G,nl", [("gold", 2, 1 << 12), ("gold", 8, 1 << 14), ("fr", 4, 1 << 10),
                                         ("fr", 8, 1 << 8)])
def test_sharded_mul_ntt_virtual_ranks(field, G, nl):
    """multigpu.ShardedMulNtt (mul_ntt, fft.rs:109-132, stride-sharded end to end) with G
    threads on this GPU: each rank's product shard equals the single-GPU mul_ntt's."""
    import threading

    import bn254
    from multigpu import GpuFrShardOps, GpuShardOps, LocalComm, LocalGroup, ShardedMulNtt

    N = G * nl
    la = N // 2 + 5
    lb = N - la
    if field == "gold":
        M, w = GOLD, pow(7, (GOLD - 1) // N, GOLD)
        a = oracle.splitmix_field(GOLD, 61, la)
        b = oracle.splitmix_field(GOLD, 62, lb)
        ref = [int(x) for x in pbf.default_context().mul_ntt(GOLD, w, a, b)]
        pad = lambda v: np.concatenate([np.asarray(v, dtype=np.uint64), np.zeros(N - len(v), dtype=np.uint64)])  # noqa
        A, Bv = pad(a), pad(b)
        enc = lambda v: torch.from_numpy(np.ascontiguousarray(v).view(np.int64)).cuda()  # noqa: E731
        dec = lambda t: [int(x) for x in t.cpu().numpy().view(np.uint64)]  # noqa: E731
        Ops = GpuShardOps
    else:
        M, w = bn254.R, bn254.root_of_unity(N)
        a, b = _fr_rand(la, 63), _fr_rand(lb, 64)
        ref = pbf.default_context().mul_ntt_fr(w, a, b)
        A, Bv = a + [0] * (N - la), b + [0] * (N - lb)
        enc = lambda v: torch.from_numpy(bn254.ints_to_limbs(list(v)).view(np.int64)).cuda()  # noqa: E731
        dec = lambda t: bn254.limbs_to_ints(t.cpu().numpy().view(np.uint64))  # noqa: E731
        Ops = GpuFrShardOps
    group = LocalGroup(G)
    out, errs = [None] * G, []

    def rank_main(r):
        try:
            c = pbf.Context(0)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                sm = ShardedMulNtt(Ops(c, st.cuda_stream), LocalComm(group, r), r, G, nl, modulus=M, omega=w)
                cs = torch.empty(nl * Ops.words, dtype=torch.int64, device="cuda")
                sm.mul(enc(A[r::G]), enc(Bv[r::G]), cs)
                st.synchronize()
                out[r] = dec(cs)
            c.close()
        except Exception as e:
            errs.append(f"rank {r}: {e!r}")
            group.barrier.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not errs, errs
    for r in range(G):
        assert out[r] == list(ref[r::G]), (field, G, r)


@pytest.mark.parametrize("G,field", [(2, "gold"), (4, "gold"), (4, "fr")])
def test_sharded_ntt_on_a_non_current_stream(G, field):
    """multigpu.ShardedNtt / ShardedMulNtt issue their collectives on ops.stream, the stream the
    kernels go to, whatever torch's current stream is. Each virtual rank runs on stream A
    (delayed behind a queue of matmuls) while torch's current stream is B: an exchange ordered
    on B would copy `send` before the local NTT on A wrote it."""
    import threading

    import bn254
    from multigpu import GpuFrShardOps, GpuShardOps, LocalComm, LocalGroup, ShardedMulNtt, ShardedNtt

    nl, batch = 1 << 12, 4
    N = G * nl
    if field == "gold":
        M, w, Ops = GOLD, pow(7, (GOLD - 1) // N, GOLD), GpuShardOps
        glob = np.stack([oracle.splitmix_field(GOLD, 4400 + b, N) for b in range(batch)])
        ref = np.stack([oracle.ntt_iter(GOLD, w, glob[b]) for b in range(batch)])
        enc = lambda v: torch.from_numpy(np.ascontiguousarray(v).reshape(-1).view(np.int64)).cuda()  # noqa: E731
        shard_of = lambda g: enc(glob[:, g::G])  # noqa: E731
    else:
        M, w, Ops = bn254.R, bn254.root_of_unity(N), GpuFrShardOps
        glob = [_fr_rand(N, 4500 + b) for b in range(batch)]
        ctx0 = pbf.default_context()
        ref = [ctx0.ntt_fr(w, g) for g in glob]
        enc = lambda v: torch.from_numpy(bn254.ints_to_limbs(list(v)).view(np.int64)).cuda()  # noqa: E731
        shard_of = lambda g: enc([x for b in range(batch) for x in glob[b][g::G]])  # noqa: E731
    group = LocalGroup(G)
    out, prods, errs = [None] * G, [None] * G, []

    def rank_main(r):
        try:
            c = pbf.Context(0)
            lib_stream, cur_stream = torch.cuda.Stream(), torch.cuda.Stream()
            shard = shard_of(r)
            x = torch.randn(2048, 2048, device="cuda")
            torch.cuda.synchronize()
            with torch.cuda.stream(lib_stream):
                for _ in range(40):  # delays everything enqueued on lib_stream after it
                    x = x @ x
                    x = x / x.norm()
            with torch.cuda.stream(cur_stream):
                ops = Ops(c, lib_stream.cuda_stream)
                nt = ShardedNtt(ops, LocalComm(group, r), r, G, nl, batch, modulus=M, omega=w, chunks=2)
                res = torch.empty_like(shard)
                nt.forward(shard, res)
                sm = ShardedMulNtt(ops, LocalComm(group, r), r, G, nl, modulus=M, omega=w)
                L = nl * Ops.words
                prod = torch.empty(L, dtype=torch.int64, device="cuda")
                sm.mul(shard[:L], shard[L:2 * L], prod)
            lib_stream.synchronize()
            out[r] = res.cpu().numpy().view(np.uint64)
            prods[r] = prod.cpu().numpy().view(np.uint64)
            c.close()
        except Exception as e:  # reported by the main thread
            errs.append(f"rank {r}: {e!r}")
            group.barrier.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "rank hung"
    assert not errs, errs
    for r in range(G):
        idx = ShardedNtt.output_indices(r, G, nl)
        if field == "gold":
            got = out[r].reshape(batch, nl)
            assert np.array_equal(got, ref[:, idx]), (G, r)
        else:
            got = bn254.limbs_to_ints(out[r])
            for b in range(batch):
                assert got[b * nl:(b + 1) * nl] == [ref[b][i] for i in idx], (G, r, b)
    # the product shards: mul_ntt of polynomials 0 and 1 (whole vectors), stride-sharded
    if field == "gold":
        spec = (ref[0].astype(object) * ref[1].astype(object)) % GOLD
        prod_ref = [int(v) for v in oracle.ntt_iter(GOLD, w, np.asarray(spec, dtype=np.uint64), inverse=True)]
        for r in range(G):
            assert [int(v) for v in prods[r]] == prod_ref[r::G], (G, r)
    else:
        R = bn254.R
        spec = [x * y % R for x, y in zip(ref[0], ref[1])]
        prod_ref = pbf.default_context().ntt_fr(w, spec, inverse=True)
        for r in range(G):
            assert bn254.limbs_to_ints(prods[r]) == prod_ref[r::G], (G, r)
