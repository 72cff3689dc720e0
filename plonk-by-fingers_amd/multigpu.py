"""Multi-GPU stride-sharded NTT — one process per GPU.

A transform of N = G * nl points is sharded by coefficient stride: rank g holds
a[g + G*m] (the top log2(G) levels of the reference's even/odd recursion,
src/fft.rs:94-96, become the rank index). Forward, on every rank:

    libpbf  pbf_ntt_shard_local_dev   local nl-point NTT (root w^G), stored in the
                                      destination-major send layout [dst][b][kk]
    RCCL    all_to_all_single         nl*batch/G elements to each peer over xGMI
    libpbf  pbf_ntt_shard_combine_dev twiddle w^(g*k) + radix-G butterfly:
                                      out[b][q*S + kk] = X[q*nl + rank*S + kk], S = nl/G

The inverse runs the same three steps backwards. The exchange is the only
collective; there is no other data-path communication.

The batch runs in `chunks` groups of polynomials (independent transforms), software-
pipelined: group c's all-to-all (RCCL's stream, async) overlaps group c+1's local NTT
and group c-1's combine on the compute stream, so a step costs about
max(compute, exchange) instead of their sum.
"""
from __future__ import annotations

import os

import torch

GOLD = 0xFFFFFFFF00000001


class GpuShardOps:
    """The HIP kernels of libpbf.so, enqueued on `stream` (torch's stream)."""

    def __init__(self, ctx, stream: int):
        self.ctx = ctx
        self.stream = stream

    def local(self, modulus, omega, world, src: torch.Tensor, dst: torch.Tensor, nl, batch, inverse):
        self.ctx.shard_local_dev(modulus, omega, world, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                 stream=self.stream)

    def combine(self, modulus, omega, world, rank, src: torch.Tensor, dst: torch.Tensor, nl, batch, inverse):
        self.ctx.shard_combine_dev(modulus, omega, world, rank, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                   stream=self.stream)


class ShardedNtt:
    """Batched forward / inverse NTT of `batch` polynomials of N = world * nl points."""

    def __init__(self, ops, comm, rank: int, world: int, nl: int, batch: int, modulus: int = GOLD,
                 omega: int | None = None, device: str | torch.device = "cuda", chunks: int | None = None):
        if world not in (2, 4, 8):
            raise ValueError("world size must be 2, 4 or 8")
        self.ops, self.comm = ops, comm
        self.rank, self.world, self.nl, self.batch = rank, world, nl, batch
        self.modulus = modulus
        self.n_global = world * nl
        self.omega = omega if omega is not None else pow(7, (modulus - 1) // self.n_global, modulus)
        shape = (batch * nl,)
        self.send = torch.empty(shape, dtype=torch.int64, device=device)
        self.recv = torch.empty(shape, dtype=torch.int64, device=device)
        if chunks is None:
            chunks = int(os.environ.get("PBF_MG_CHUNKS", "4"))
        while chunks > 1 and batch % chunks:
            chunks -= 1
        self.chunks = max(1, chunks)

    def _exchange(self, c: int):
        # equal splits along dim 0 of group c's slice: part r of `send` goes to rank r, part g
        # of `recv` came from rank g (layout [peer][polynomial of the group][kk])
        sl = self._slice(c)
        return self.comm.all_to_all_single(self.recv[sl], self.send[sl], async_op=True)

    def _slice(self, c: int) -> slice:
        L = (self.batch // self.chunks) * self.nl
        return slice(c * L, (c + 1) * L)

    def _pipeline(self, first, second):
        """first(c) produces send[c]; the exchange fills recv[c]; second(c) consumes it."""
        works = []
        for c in range(self.chunks):
            first(c)
            works.append(self._exchange(c))
            if c >= 1:
                works[c - 1].wait()
                second(c - 1)
        works[-1].wait()
        second(self.chunks - 1)

    def forward(self, shard: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """shard[b][m] = a_b[rank + world*m]  ->  out[b][q*S + kk] = X_b[q*nl + rank*S + kk]."""
        bc = self.batch // self.chunks
        self._pipeline(
            lambda c: self.ops.local(self.modulus, self.omega, self.world, shard[self._slice(c)],
                                     self.send[self._slice(c)], self.nl, bc, False),
            lambda c: self.ops.combine(self.modulus, self.omega, self.world, self.rank, self.recv[self._slice(c)],
                                       out[self._slice(c)], self.nl, bc, False))
        return out

    def inverse(self, blocked: torch.Tensor, shard_out: torch.Tensor) -> torch.Tensor:
        """Exact inverse of forward(): blocked outputs -> the stride shard of the coefficients."""
        bc = self.batch // self.chunks
        self._pipeline(
            lambda c: self.ops.combine(self.modulus, self.omega, self.world, self.rank, blocked[self._slice(c)],
                                       self.send[self._slice(c)], self.nl, bc, True),
            lambda c: self.ops.local(self.modulus, self.omega, self.world, self.recv[self._slice(c)],
                                     shard_out[self._slice(c)], self.nl, bc, True))
        return shard_out

    # ---- layout helpers (host side, for tests and the whole-vector entry point)
    @staticmethod
    def output_indices(rank: int, world: int, nl: int):
        """Global output index held at out[q*S + kk] on `rank`."""
        s = nl // world
        return [q * nl + rank * s + kk for q in range(world) for kk in range(s)]


class BenchSharded:
    """bench.py driver: synthetic shards resident in HBM, one forward per step."""

    def __init__(self, ctx, dist, rank: int, world: int, log_n: int, batch: int, stream: int):
        nl = 1 << log_n
        self.nt = ShardedNtt(GpuShardOps(ctx, stream), dist, rank, world, nl, batch)
        self.n_global = self.nt.n_global
        self.shard = torch.empty(batch * nl, dtype=torch.int64, device="cuda")
        self.out = torch.empty_like(self.shard)
        ctx.fill_random_dev(GOLD, 0x5EED0002 + rank, self.shard.data_ptr(), batch * nl, stream=stream)

    def step(self):
        self.nt.forward(self.shard, self.out)


class GpuMsmOps:
    """The MSM of csrc/msm.hip on device-resident ranges, and the sum of G affine points as an
    MSM with unit scalars (the identity encodes as (0, 0))."""

    def __init__(self, ctx, stream: int = 0):
        self.ctx, self.stream = ctx, stream

    def partial(self, d_points: int, d_scalars: int, count: int) -> tuple:
        return self.ctx.msm_g1_dev(d_points, d_scalars, count, stream=self.stream) if count else (0, 0)

    def combine(self, points) -> tuple:
        return self.ctx.msm_g1(points, [1] * len(points))


class ShardedMsm:
    """Multi-GPU G1 MSM (independent point ranges). Rank r owns points and
    scalars [start, end) of split(n, G, r) in HBM and runs its MSM locally; the G partial
    sums (affine, 8 u64 each) are all-gathered and added on every rank. One collective of
    G x 64 B; no other traffic."""

    def __init__(self, ops, comm, rank: int, world: int, device: str | torch.device = "cuda"):
        self.ops, self.comm, self.rank, self.world, self.device = ops, comm, rank, world, device

    @staticmethod
    def split(n: int, world: int, rank: int):
        """[start, end) of rank's point range (the first n % world ranks take one more)."""
        base, extra = divmod(n, world)
        start = rank * base + min(rank, extra)
        return start, start + base + (1 if rank < extra else 0)

    def msm(self, points, scalars, count: int) -> tuple:
        """The MSM of the whole point set, on every rank, from this rank's `count` points."""
        x, y = self.ops.partial(points, scalars, count)
        m = (1 << 64) - 1
        limbs = [(v >> (64 * k)) & m for v in (x, y) for k in range(4)]
        mine = torch.tensor([v - (1 << 64) if v >> 63 else v for v in limbs], dtype=torch.int64, device=self.device)
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        self.comm.all_gather(parts, mine)
        pts = []
        for p in parts:
            u = [int(v) & m for v in p.cpu().tolist()]
            pts.append((sum(u[k] << (64 * k) for k in range(4)), sum(u[4 + k] << (64 * k) for k in range(4))))
        return self.ops.combine(pts)
