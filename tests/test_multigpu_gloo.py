"""Multi-process (gloo, CPU) test of the stride-sharded NTT orchestration.

ShardedNtt (plonk-by-fingers_amd/multigpu.py) is run by world_size 2 and 4
processes over torch.distributed/gloo. The two device steps are replaced by a
TEST-SIDE emulation built on the oracle (this file only; the product has no CPU
path), so what is checked here is the exchange: buffer layouts, the
all_to_all_single splits and rank ordering, and the decomposition math. The same
class drives the HIP kernels over RCCL in bench.py; the kernels themselves are
checked on the GPU in tests/test_multigpu_gpu.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = 0xFFFFFFFF00000001


class OracleShardOps:
    """Emulates pbf_ntt_shard_local_dev / pbf_ntt_shard_combine_dev with the oracle."""

    def local(self, m, omega, G, src, dst, nl, batch, inverse):
        import oracle

        wl = pow(omega, G, m)
        s = nl // G
        if not inverse:
            x = src.numpy().view(np.uint64).reshape(batch, nl)
            send = dst.numpy().view(np.uint64).reshape(G, batch, s)
            for b in range(batch):
                y = oracle.ntt_iter(m, wl, x[b])
                for g in range(G):
                    send[g, b] = y[g * s:(g + 1) * s]
        else:
            recv = src.numpy().view(np.uint64).reshape(G, batch, s)
            out = dst.numpy().view(np.uint64).reshape(batch, nl)
            for b in range(batch):
                y = np.concatenate([recv[g, b] for g in range(G)])
                out[b] = oracle.ntt_iter(m, wl, y, inverse=True)

    def combine(self, m, omega, G, rank, src, dst, nl, batch, inverse):
        s = nl // G
        w = omega if not inverse else pow(omega, m - 2, m)
        wG = pow(w, nl, m)
        ginv = pow(G, m - 2, m)
        if not inverse:
            recv = src.numpy().view(np.uint64).reshape(G, batch, s)
            out = dst.numpy().view(np.uint64).reshape(batch, nl)
            for b in range(batch):
                for kk in range(s):
                    k = rank * s + kk
                    t = [int(recv[g, b, kk]) * pow(w, g * k, m) % m for g in range(G)]
                    for q in range(G):
                        out[b, q * s + kk] = sum(t[g] * pow(wG, g * q, m) for g in range(G)) % m
        else:
            x = src.numpy().view(np.uint64).reshape(batch, nl)
            send = dst.numpy().view(np.uint64).reshape(G, batch, s)
            for b in range(batch):
                for kk in range(s):
                    k = rank * s + kk
                    for g in range(G):
                        acc = sum(int(x[b, q * s + kk]) * pow(wG, g * q, m) for q in range(G)) % m
                        send[g, b, kk] = acc * pow(w, g * k, m) % m * ginv % m


    def pointwise(self, m, a, b, c, count):
        x, y = a.numpy().view(np.uint64), b.numpy().view(np.uint64)
        c.numpy().view(np.uint64)[:count] = [(int(u) * int(v)) % m for u, v in zip(x[:count], y[:count])]


class OracleFrShardOps:
    """The same emulation over BN254 Fr (4 int64 words per element, oracle/bn254.py)."""

    words = 4

    @staticmethod
    def _ints(t):
        import bn254

        return bn254.limbs_to_ints(t.numpy().view(np.uint64))

    @staticmethod
    def _put(t, vals):
        import bn254

        t.numpy().view(np.uint64)[:] = bn254.ints_to_limbs(vals)

    def local(self, m, omega, G, src, dst, nl, batch, inverse):
        import bn254

        R = bn254.R
        wl = pow(omega, G, R)
        s = nl // G
        x = self._ints(src)
        out = [0] * (nl * batch)
        for b in range(batch):
            if not inverse:
                y = bn254.ntt(x[b * nl:(b + 1) * nl], wl)
                for g in range(G):
                    out[(g * batch + b) * s:(g * batch + b + 1) * s] = y[g * s:(g + 1) * s]
            else:
                yv = [x[(g * batch + b) * s + kk] for g in range(G) for kk in range(s)]
                out[b * nl:(b + 1) * nl] = bn254.ntt(yv, wl, inverse=True)
        self._put(dst, out)

    def combine(self, m, omega, G, rank, src, dst, nl, batch, inverse):
        import bn254

        R = bn254.R
        s = nl // G
        w = omega if not inverse else pow(omega, R - 2, R)
        wG = pow(w, nl, R)
        ginv = pow(G, R - 2, R)
        x = self._ints(src)
        out = [0] * (nl * batch)
        for b in range(batch):
            for kk in range(s):
                k = rank * s + kk
                if not inverse:
                    t = [x[(g * batch + b) * s + kk] * pow(w, g * k, R) % R for g in range(G)]
                    for q in range(G):
                        out[b * nl + q * s + kk] = sum(t[g] * pow(wG, g * q, R) for g in range(G)) % R
                else:
                    for g in range(G):
                        acc = sum(x[b * nl + q * s + kk] * pow(wG, g * q, R) for q in range(G)) % R
                        out[(g * batch + b) * s + kk] = acc * pow(w, g * k, R) % R * ginv % R
        self._put(dst, out)

    def pointwise(self, m, a, b, c, count):
        import bn254

        xa, xb = self._ints(a), self._ints(b)
        self._put(c, [u * v % bn254.R for u, v in zip(xa[:count], xb[:count])])


def _worker(rank, world, port, nl, batch, q, chunks=1):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from multigpu import ShardedNtt

        N = world * nl
        glob = np.stack([oracle.splitmix_field(GOLD, 700 + b, N) for b in range(batch)])
        shard = torch.from_numpy(np.ascontiguousarray(glob[:, rank::world]).view(np.int64).reshape(-1).copy())
        nt = ShardedNtt(OracleShardOps(), dist, rank, world, nl, batch, device="cpu", chunks=chunks)
        assert nt.chunks == chunks
        out = torch.empty_like(shard)
        nt.forward(shard, out)
        w = nt.omega
        idx = ShardedNtt.output_indices(rank, world, nl)
        ok_fwd = True
        for b in range(batch):
            ref = oracle.ntt_iter(GOLD, w, glob[b])
            got = out.numpy().view(np.uint64).reshape(batch, nl)[b]
            ok_fwd &= bool(np.array_equal(got, ref[idx]))
        back = torch.empty_like(shard)
        nt.inverse(out, back)
        ok_inv = bool(np.array_equal(back.numpy(), shard.numpy()))
        q.put((rank, ok_fwd, ok_inv))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,batch,chunks", [(2, 2, 1), (4, 2, 1), (8, 2, 1), (2, 4, 4), (4, 4, 2)])
def test_sharded_ntt_gloo(world, batch, chunks):
    """chunks > 1: the pipelined schedule (async all-to-all per polynomial group)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 64, batch, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert sorted(r for r, _, _ in res) == list(range(world))
    assert all(f for _, f, _ in res), res
    assert all(i for _, _, i in res), res


class OracleMsmOps:
    """Emulates the GPU MSM pieces with the BN254 oracle (test side only): `points` and
    `scalars` are this rank's Python lists."""

    def partial(self, points, scalars, count):
        import bn254

        p = bn254.msm_naive(points[:count], scalars[:count])
        return (0, 0) if p is None else p

    def combine(self, pts):
        import bn254

        acc = None
        for p in pts:
            acc = bn254.g1_add(acc, None if p == (0, 0) else p)
        return (0, 0) if acc is None else acc


def _msm_worker(rank, world, port, n, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import random

        import bn254
        from multigpu import ShardedMsm

        rnd = random.Random(77)
        pts = [bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, bn254.R)) for _ in range(n)]
        sc = [rnd.randrange(bn254.R) for _ in range(n)]
        a, b = ShardedMsm.split(n, world, rank)
        sm = ShardedMsm(OracleMsmOps(), dist, rank, world, device="cpu")
        got = sm.msm(pts[a:b], sc[a:b], b - a)
        ref = bn254.msm_naive(pts, sc)
        q.put((rank, got == ((0, 0) if ref is None else ref)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (4, 9), (4, 3)])
def test_sharded_msm_gloo(world, n):
    """Point-range sharded MSM: partial MSMs, all-gather of the partial sums, combine
    (n < world leaves ranks with no points: their partial is the identity)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_msm_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res


def _mul_worker(rank, world, port, nl, field, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import random

        import bn254
        import oracle
        from multigpu import ShardedMulNtt

        N = world * nl
        la = N // 2 - 3  # ragged: la + lb = N (fft.rs:114-118), trailing zero padding
        lb = N - la
        rnd = random.Random(5)
        if field == "gold":
            M = GOLD
            a = [rnd.randrange(M) for _ in range(la)] + [0] * (N - la)
            b = [rnd.randrange(M) for _ in range(lb)] + [0] * (N - lb)
            ops, w = OracleShardOps(), pow(7, (M - 1) // N, M)
            enc = lambda v: torch.from_numpy(np.array(v, dtype=np.uint64).view(np.int64).copy())  # noqa: E731
            dec = lambda t: [int(x) for x in t.numpy().view(np.uint64)]  # noqa: E731
            ref = [int(x) for x in oracle.mul_ntt(M, w, a[:la], b[:lb])]
        else:
            M = bn254.R
            a = [rnd.randrange(M) for _ in range(la)] + [0] * (N - la)
            b = [rnd.randrange(M) for _ in range(lb)] + [0] * (N - lb)
            ops, w = OracleFrShardOps(), bn254.root_of_unity(N)
            enc = lambda v: torch.from_numpy(bn254.ints_to_limbs(v).view(np.int64).copy())  # noqa: E731
            dec = lambda t: bn254.limbs_to_ints(t.numpy().view(np.uint64))  # noqa: E731
            ref = bn254.mul_ntt(a[:la], b[:lb], w)
        sm = ShardedMulNtt(ops, dist, rank, world, nl, modulus=M, omega=w, device="cpu")
        c = torch.empty(nl * getattr(ops, "words", 1), dtype=torch.int64)
        sm.mul(enc(a[rank::world]), enc(b[rank::world]), c)
        q.put((rank, dec(c) == ref[rank::world]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nl,field", [(2, 16, "gold"), (4, 8, "gold"), (2, 8, "fr"), (4, 4, "fr")])
def test_sharded_mul_ntt_gloo(world, nl, field):
    """mul_ntt (fft.rs:109-132) with a, b and c stride-sharded end to end:
    each rank's shard of the product equals the oracle's mul_ntt at its stride positions."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mul_worker, args=(r, world, port, nl, field, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res


def test_local_comm_threads():
    """multigpu.LocalComm (the virtual-rank communicator of the sharded prover's GPU tests):
    all_to_all_single / all_gather_into_tensor layouts across threads, CPU tensors."""
    import threading

    sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
    from multigpu import LocalComm, LocalGroup

    G, k = 3, 4
    grp = LocalGroup(G)
    res = {}

    def rank_main(r):
        c = LocalComm(grp, r)
        send = torch.arange(G * k, dtype=torch.int64) + 100 * r  # part g -> rank g
        recv = torch.empty(G * k, dtype=torch.int64)
        c.all_to_all_single(recv, send)
        gat = torch.empty(G * k, dtype=torch.int64)
        c.all_gather_into_tensor(gat, send[:k] * 0 + r)
        res[r] = (recv.clone(), gat.clone())

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    for r in range(G):
        recv, gat = res[r]
        for g in range(G):  # recv part g came from rank g's send part r
            assert recv[g * k:(g + 1) * k].tolist() == [100 * g + r * k + j for j in range(k)]
            assert gat[g * k:(g + 1) * k].tolist() == [g] * k


def _distcomm_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from multigpu import DistComm

        k = 3
        c = DistComm(dist, world)
        send = torch.arange(world * k, dtype=torch.int64) + 100 * rank
        recv = torch.empty(world * k, dtype=torch.int64)
        c.all_to_all_single(recv, send)
        gat = torch.empty(world * k, dtype=torch.int64)
        c.all_gather_into_tensor(gat, torch.full((k,), rank, dtype=torch.int64))
        ok = all(recv[g * k:(g + 1) * k].tolist() == [100 * g + rank * k + j for j in range(k)] for g in range(world))
        ok = ok and all(gat[g * k:(g + 1) * k].tolist() == [g] * k for g in range(world))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_dist_comm_gloo():
    """multigpu.DistComm over a real gloo group (world 2): the sharded prover's collectives."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_distcomm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
