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

import contextlib

import os

import torch

GOLD = 0xFFFFFFFF00000001


def _stream_ctx(stream_ptr, like: torch.Tensor):
    """torch.cuda.stream(stream_ptr) for device tensors (0: the device's default stream);
    a no-op for host tensors (the gloo tests' CPU ops)."""
    if not like.is_cuda or stream_ptr is None:
        return contextlib.nullcontext()
    st = (torch.cuda.ExternalStream(stream_ptr, device=like.device) if stream_ptr
          else torch.cuda.default_stream(like.device))
    return torch.cuda.stream(st)


class GpuShardOps:
    """The HIP kernels of libpbf.so, enqueued on `stream` (torch's stream): u64 elements
    (Goldilocks or a 32-bit modulus), one int64 word each."""

    words = 1

    def __init__(self, ctx, stream: int):
        self.ctx = ctx
        self.stream = stream

    def local(self, modulus, omega, world, src: torch.Tensor, dst: torch.Tensor, nl, batch, inverse):
        self.ctx.shard_local_dev(modulus, omega, world, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                 stream=self.stream)

    def combine(self, modulus, omega, world, rank, src: torch.Tensor, dst: torch.Tensor, nl, batch, inverse):
        self.ctx.shard_combine_dev(modulus, omega, world, rank, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                   stream=self.stream)

    def pointwise(self, modulus, a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, count: int):
        self.ctx.pointwise_mul_dev(modulus, a.data_ptr(), b.data_ptr(), c.data_ptr(), count, stream=self.stream)


class GpuFrShardOps(GpuShardOps):
    """The same steps over BN254 Fr (4 int64 words per element; the modulus argument is
    ignored, omega is an int below r)."""

    words = 4

    def local(self, modulus, omega, world, src, dst, nl, batch, inverse):
        self.ctx.fr_shard_local_dev(omega, world, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                    stream=self.stream)

    def combine(self, modulus, omega, world, rank, src, dst, nl, batch, inverse):
        self.ctx.fr_shard_combine_dev(omega, world, rank, src.data_ptr(), dst.data_ptr(), nl, batch, inverse,
                                      stream=self.stream)

    def pointwise(self, modulus, a, b, c, count):
        self.ctx.fr_pointwise_mul_dev(a.data_ptr(), b.data_ptr(), c.data_ptr(), count, stream=self.stream)


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
        self.words = getattr(ops, "words", 1)  # int64 words per element
        shape = (batch * nl * self.words,)
        self.send = torch.empty(shape, dtype=torch.int64, device=device)
        self.recv = torch.empty(shape, dtype=torch.int64, device=device)
        if chunks is None:
            chunks = int(os.environ.get("PBF_MG_CHUNKS", "4"))
        while chunks > 1 and batch % chunks:
            chunks -= 1
        self.chunks = max(1, chunks)

    def _on_ops_stream(self):
        """Issue (and wait for) the exchanges on the stream the kernels are enqueued on
        (ops.stream), not on torch's current stream: torch.distributed (RCCL), LocalComm's
        copies and DistComm's host staging all order against the CURRENT stream, so make
        ops.stream current while they are issued (the ShardedProver callbacks do the same)."""
        return _stream_ctx(getattr(self.ops, "stream", None), self.send)

    def _exchange(self, c: int):
        # equal splits along dim 0 of group c's slice: part r of `send` goes to rank r, part g
        # of `recv` came from rank g (layout [peer][polynomial of the group][kk])
        sl = self._slice(c)
        return self.comm.all_to_all_single(self.recv[sl], self.send[sl], async_op=True)

    def _slice(self, c: int) -> slice:
        L = (self.batch // self.chunks) * self.nl * self.words
        return slice(c * L, (c + 1) * L)

    def _pipeline(self, first, second):
        """first(c) produces send[c]; the exchange fills recv[c]; second(c) consumes it. Every
        collective is issued and waited for on ops.stream (work.wait() orders the stream that
        is current when it is called)."""
        works = []
        with self._on_ops_stream():
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


class ShardedMulNtt:
    """mul_ntt (src/fft.rs:109-132) with every polynomial stride-sharded over the ranks
    ("same stride layout end-to-end, no gather between NTT and
    pointwise"). The product domain has N = la + lb = world * nl points (a power of two,
    fft.rs:114-118); rank g holds a[g + G m] and b[g + G m] (zero-padded), and gets back the
    stride shard c[g + G m] of the un-normalised product INTT(NTT(a) * NTT(b)). Steps: one
    forward sharded NTT of the pair (batch 2), the pointwise product of this rank's blocks
    (pointwise needs no exchange: both spectra have the same blocked layout), one inverse
    sharded NTT. Two all-to-alls in total."""

    def __init__(self, ops, comm, rank: int, world: int, nl: int, modulus: int = GOLD, omega: int | None = None,
                 device: str | torch.device = "cuda"):
        self.fwd = ShardedNtt(ops, comm, rank, world, nl, 2, modulus, omega, device, chunks=1)
        self.inv = ShardedNtt(ops, comm, rank, world, nl, 1, modulus, self.fwd.omega, device, chunks=1)
        self.ops, self.nl, self.modulus, self.words = ops, nl, modulus, self.fwd.words
        self.spec = torch.empty(2 * nl * self.words, dtype=torch.int64, device=device)

    def mul(self, a_shard: torch.Tensor, b_shard: torch.Tensor, c_shard: torch.Tensor) -> torch.Tensor:
        L = self.nl * self.words
        # the concatenation and the allocations are stream-ordered too: ops.stream, like the kernels
        with _stream_ctx(getattr(self.ops, "stream", None), self.spec):
            pair = torch.cat([a_shard.reshape(-1), b_shard.reshape(-1)])
            self.fwd.forward(pair, self.spec)
            prod = torch.empty(L, dtype=torch.int64, device=self.spec.device)
            self.ops.pointwise(self.modulus, self.spec[:L], self.spec[L:], prod, self.nl)
            return self.inv.inverse(prod, c_shard)


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


# ---------------------------------------------------------------- communicators
class _Done:
    def wait(self):
        return True


class LocalGroup:
    """World of `world` virtual ranks in one process, one host thread each (tests and
    single-GPU rehearsals of the multi-GPU paths): collectives meet at a barrier and move
    data with device (or host) copies."""

    def __init__(self, world: int):
        import threading

        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class LocalComm:
    """The torch.distributed calls the sharded paths use, for one virtual rank of a
    LocalGroup (same signatures: all_to_all_single, all_gather, all_gather_into_tensor)."""

    def __init__(self, group: LocalGroup, rank: int):
        self.group, self.rank = group, rank

    def _sync(self, t):
        if t.is_cuda:
            torch.cuda.current_stream().synchronize()

    def _exchange(self, out, inp, pick):
        g = self.group
        self._sync(inp)
        g.slots[self.rank] = inp
        g.barrier.wait()
        parts = out.view(g.world, -1)
        for src in range(g.world):
            parts[src].copy_(pick(g.slots[src]))
        self._sync(out)
        g.barrier.wait()  # every rank has read every slot before any input is reused
        return _Done()

    def all_to_all_single(self, out, inp, async_op=False):
        return self._exchange(out, inp, lambda t: t.view(self.group.world, -1)[self.rank])

    def all_gather_into_tensor(self, out, inp, async_op=False):
        return self._exchange(out, inp, lambda t: t)

    def all_gather(self, outs, inp, async_op=False):
        flat = torch.empty(self.group.world * inp.numel(), dtype=inp.dtype, device=inp.device)
        self._exchange(flat, inp.reshape(-1), lambda t: t.reshape(-1))
        for k, o in enumerate(outs):
            o.copy_(flat.view(self.group.world, -1)[k].view_as(o))
        return _Done()


class DistComm:
    """torch.distributed with equal-split collectives on flat tensors; a gloo group (CPU
    only) gets device tensors staged through the host."""

    def __init__(self, dist, world: int):
        self.dist, self.world = dist, world
        self.staged = dist.get_backend() == "gloo"

    def all_to_all_single(self, out, inp, async_op=False):
        if self.staged and inp.is_cuda:
            o = torch.empty(out.numel(), dtype=out.dtype)
            self.dist.all_to_all_single(o, inp.cpu())
            out.copy_(o.view_as(out))
        else:
            self.dist.all_to_all_single(out, inp)
        return _Done()

    def all_gather_into_tensor(self, out, inp, async_op=False):
        src = inp.cpu() if self.staged and inp.is_cuda else inp
        parts = [torch.empty_like(src) for _ in range(self.world)]
        self.dist.all_gather(parts, src)
        out.view(self.world, -1).copy_(torch.stack([p.reshape(-1) for p in parts]))
        return _Done()

    def all_gather(self, outs, inp, async_op=False):
        return self.dist.all_gather(outs, inp)


# ---------------------------------------------------------------- config 5 across GPUs
class ShardedProver:
    """Plonk::prove (src/plonk.rs:191-466) for BASELINE config 5 with its NTTs sharded across
    the ranks (pbf_plonk_prove_bn254_sharded_dev): every rank calls prove()
    with the same circuit, SRS, challenges and blinders on its own GPU; the library calls back
    here for the all-to-alls of the stride-sharded 4n-point transforms and the all-gathers
    (t / W_z / W_zw coefficients, commitment partial sums). `comm` is torch.distributed
    (RCCL), a DistComm or a LocalComm. Returns the proof (9 points, 7 field elements as
    limb arrays), identical on every rank and to the single-GPU prover's."""

    def __init__(self, ctx, comm, rank: int, world: int, n: int, stream: int = 0, device="cuda"):
        import ctypes

        import pbf

        self.ctx, self.comm, self.rank, self.world, self.n = ctx, comm, rank, world, n
        self.stream = stream
        nl = 4 * n // world
        self.words = 5 * nl * 4  # 5 * nl Fr elements of 4 int64 words (pbf.h: 5 coset NTTs per exchange)
        self.send = torch.empty(self.words, dtype=torch.int64, device=device)
        self.recv = torch.empty(self.words, dtype=torch.int64, device=device)
        cb = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
        on_cuda = torch.device(device).type == "cuda"

        def on_stream(stream_ptr):
            # pbf.h: the exchange is ordered on the stream the library passes. torch.distributed
            # (RCCL), LocalComm's copies and DistComm's host staging all order against torch's
            # CURRENT stream, so make that stream current for the duration of the collective.
            if not on_cuda:
                return contextlib.nullcontext()
            st = (torch.cuda.ExternalStream(stream_ptr) if stream_ptr
                  else torch.cuda.default_stream(torch.device(device)))
            return torch.cuda.stream(st)

        def a2a(_user, nbytes, stream_ptr):
            try:
                k = nbytes // 8
                with on_stream(stream_ptr):
                    self.comm.all_to_all_single(self.recv[:world * k], self.send[:world * k])
                return 0
            except Exception as e:  # surfaces as PBF_ECOMM
                self.error = e
                return 1

        def ag(_user, nbytes, stream_ptr):
            try:
                k = nbytes // 8
                with on_stream(stream_ptr):
                    self.comm.all_gather_into_tensor(self.recv[:world * k], self.send[:k])
                return 0
            except Exception as e:
                self.error = e
                return 1

        self._cbs = (cb(a2a), cb(ag))  # keep the ctypes thunks alive
        self.error = None
        self.c = pbf.Comm(world, rank, self.send.data_ptr(), self.recv.data_ptr(), self.words * 8, *self._cbs)

    def prove(self, d_q, d_copies, d_abc, chal, rnd, d_srs, srs_m, k1k2=(2, 3), mode=1):
        return self.ctx.plonk_prove_bn254_sharded_dev(self.c, self.n, d_q, d_copies, d_abc, chal, rnd, d_srs, srs_m,
                                                      k1k2=k1k2, mode=mode, stream=self.stream)
