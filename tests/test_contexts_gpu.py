"""GPU: distinct contexts are independent (include/pbf.h "Conventions").

Two host threads, each with its own pbf.Context and its own torch stream, run batched
Goldilocks NTTs of 16 polynomials (the batch size at which pbf_ntt_u64_batch_dev forks
half its groups onto the context's private aux stream) concurrently, many times. Every
result must equal the oracle's, and each context's aux streams must be its own
(ntt_launch.hip ForkSet, created and destroyed with the context)."""
import threading

import numpy as np
import pytest

import oracle
import pbf

pytestmark = pytest.mark.gpu
GOLD = pbf.GOLDILOCKS


def test_two_contexts_two_threads():
    import torch

    n, B, reps = 1 << 13, 16, 12
    w = pow(7, (GOLD - 1) // n, GOLD)
    seeds = (11, 22)
    refs = {}
    for s in seeds:
        a = oracle.splitmix_field(GOLD, s, n * B).reshape(B, n)
        refs[s] = np.stack([oracle.ntt_iter(GOLD, w, row) for row in a])
    errors = []

    def worker(seed):
        try:
            ctx = pbf.Context(0)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                din = torch.empty(B * n, dtype=torch.int64, device="cuda")
                dout = torch.empty_like(din)
                ctx.fill_random_dev(GOLD, seed, din.data_ptr(), B * n, stream=st.cuda_stream)
                for _ in range(reps):
                    dout.zero_()
                    ctx.ntt_batch_dev(GOLD, w, din.data_ptr(), dout.data_ptr(), n, B, stream=st.cuda_stream)
                    got = dout.cpu().numpy().view(np.uint64).reshape(B, n)  # syncs st
                    if not np.array_equal(got, refs[seed]):
                        errors.append(f"seed {seed}: mismatch")
                        break
            st.synchronize()
            ctx.close()
        except Exception as e:  # surfaced in the main thread
            errors.append(f"seed {seed}: {e!r}")

    ts = [threading.Thread(target=worker, args=(s,)) for s in seeds]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "worker hung"
    assert not errors, errors


def test_context_on_other_thread_default_device(ctx):
    # a second context created and destroyed while the session context stays usable
    c2 = pbf.Context(0)
    n = 1 << 12
    w = pow(7, (GOLD - 1) // n, GOLD)
    a = oracle.splitmix_field(GOLD, 5, n)
    assert np.array_equal(c2.ntt(GOLD, w, a), oracle.ntt_iter(GOLD, w, a))
    c2.close()
    assert np.array_equal(ctx.ntt(GOLD, w, a), oracle.ntt_iter(GOLD, w, a))


def test_context_churn_pbh_two_threads():
    """Contexts destroyed and recreated in a loop on two threads, running plonk-by-hand
    ops whose device buffers are per-context (pbh.hip dev_for -> pbf_ctx named buffers):
    a context allocated at a freed context's address must not inherit its buffers. Sizes
    change every iteration so the buffers are (re)allocated inside each context."""
    import random

    errors = []

    def worker(seed):
        rng = random.Random(seed)
        try:
            for it in range(25):
                ctx = pbf.Context(0)
                m = rng.randrange(1, 400)
                pts = [list(oracle.g1_mul((1, 2, 0), rng.randrange(1, 17))) for _ in range(m)]
                sc = [rng.randrange(0, 101) for _ in range(m)]
                got = ctx.pbh_g1_mul(pts, sc)
                want = [oracle.g1_mul(tuple(p), s) for p, s in zip(pts, sc)]
                ctx.close()
                if got != want:
                    errors.append(f"seed {seed} iteration {it}: mismatch")
                    return
        except Exception as e:  # surfaced in the main thread
            errors.append(f"seed {seed}: {e!r}")

    ts = [threading.Thread(target=worker, args=(s,)) for s in (5, 6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "worker hung"
    assert not errors, errors
