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
    assert ops.combine(parts) == full
