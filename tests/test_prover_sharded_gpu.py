"""Config 5 across GPUs: pbf_plonk_prove_bn254_sharded_dev, i.e. Plonk::prove
(src/plonk.rs:191-466) with its 4n-point NTTs stride-sharded over G ranks (one all-to-all each
way), the quotient and opening divisions on each rank's evaluation blocks, and point-range
commitments, checked bit-exact against the single-GPU proof of the same inputs (itself
bit-exact against the literal oracle, tests/test_prover_gpu.py).

* virtual ranks: G = 2, 4, 8 host threads, each with its own context and stream on this GPU,
  exchanging through multigpu.LocalComm (device copies); n >= G^2 (the sharded layouts);
  too small an n is refused;
* two processes over torch.distributed/gloo (host-staged exchanges, multigpu.DistComm),
  both on cuda:0: the same code path the driver's RCCL run takes, with a real process group.
"""
import os
import random
import socket
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))

pytestmark = pytest.mark.gpu
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _inputs(n, seed, mode):
    import torch

    import pbf

    ctx = pbf.Context(0)
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
    ref = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                    srs_m, mode=mode, stream=sp)
    torch.cuda.synchronize()
    return ctx, (dq, dc, dabc, dsrs, srs_m, chal, rnd), ref


@pytest.mark.parametrize("G,log_n,mode", [(2, 10, 1), (4, 10, 1), (8, 10, 1), (2, 12, 0), (4, 11, 0), (8, 6, 1),
                                         (8, 17, 1)])
def test_sharded_prove_virtual_ranks(G, log_n, mode):
    import torch

    import pbf
    from multigpu import LocalComm, LocalGroup, ShardedProver

    n = 1 << log_n
    ctx0, (dq, dc, dabc, dsrs, srs_m, chal, rnd), (pts0, fs0) = _inputs(n, 0x5EED0005 + log_n, mode)
    group = LocalGroup(G)
    out, errs = [None] * G, []

    def rank_main(r):
        try:
            c = pbf.Context(0)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                sp = ShardedProver(c, LocalComm(group, r), r, G, n, stream=st.cuda_stream)
                # twice: the second proof takes the rank's coset blocks from its proving key
                out[r] = [sp.prove(dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m,
                                   mode=mode) for _ in range(2)]
            st.synchronize()
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
        for k, (pts, fs) in enumerate(out[r]):
            assert np.array_equal(pts, pts0) and np.array_equal(fs, fs0), f"rank {r} proof {k} differs from one GPU's"
    ctx0.close()


@pytest.mark.parametrize("G", [2, 4])
def test_sharded_prove_on_a_non_current_stream(G):
    """pbf.h: the comm callbacks are ordered on the stream the library passes, which need not
    be torch's current stream. Each rank proves on stream A while torch's current stream is B,
    and A starts behind a long queue of work, so a collective that ordered itself on B (the
    round-2 bug: ShardedProver ignored the stream argument) would read `send` before the
    library wrote it."""
    import torch

    import pbf
    from multigpu import LocalComm, LocalGroup, ShardedProver

    n = 1 << 10
    ctx0, (dq, dc, dabc, dsrs, srs_m, chal, rnd), (pts0, fs0) = _inputs(n, 0x5EED0777, 1)
    group = LocalGroup(G)
    out, errs = [None] * G, []

    def rank_main(r):
        try:
            c = pbf.Context(0)
            lib_stream, cur_stream = torch.cuda.Stream(), torch.cuda.Stream()
            x = torch.randn(2048, 2048, device="cuda")
            with torch.cuda.stream(lib_stream):
                for _ in range(40):  # delays everything enqueued on lib_stream after it
                    x = x @ x
                    x = x / x.norm()
            with torch.cuda.stream(cur_stream):
                sp = ShardedProver(c, LocalComm(group, r), r, G, n, stream=lib_stream.cuda_stream)
                assert torch.cuda.current_stream().cuda_stream != lib_stream.cuda_stream
                out[r] = sp.prove(dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m,
                                  mode=1)
            lib_stream.synchronize()
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
        pts, fs = out[r]
        assert np.array_equal(pts, pts0) and np.array_equal(fs, fs0), f"rank {r} proof differs from one GPU's"
    ctx0.close()


def test_sharded_prove_rejects_n_below_world_squared():
    import torch

    import pbf
    from multigpu import LocalComm, LocalGroup, ShardedProver

    n, G = 32, 8
    ctx0, (dq, dc, dabc, dsrs, srs_m, chal, rnd), _ = _inputs(n, 5, 1)
    sp = ShardedProver(ctx0, LocalComm(LocalGroup(1), 0), 0, G, n, stream=torch.cuda.current_stream().cuda_stream)
    with pytest.raises(pbf.PbfError):
        sp.prove(dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m, mode=1)
    ctx0.close()


def _gloo_rank(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from multigpu import DistComm, ShardedProver

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx, (dq, dc, dabc, dsrs, srs_m, chal, rnd), (pts0, fs0) = _inputs(n, 77, 1)
        sp = ShardedProver(ctx, DistComm(dist, world), rank, world, n,
                           stream=torch.cuda.current_stream().cuda_stream)
        pts, fs = sp.prove(dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(), srs_m, mode=1)
        torch.cuda.synchronize()
        q.put((rank, bool(np.array_equal(pts, pts0) and np.array_equal(fs, fs0))))
        ctx.close()
    except Exception as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_prove_two_processes_gloo():
    import torch.multiprocessing as mp

    world, n = 2, 1 << 10
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok is True for _, ok in res), res
