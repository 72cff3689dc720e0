"""Config 5 at BASELINE's proofs/s size: a 2^20-gate proof through the C-ABI
(pbf_plonk_prove_bn254_dev / pbf_plonk_verify_bn254_dev), checked by properties that do
not need an O(n^2) oracle:
* all 7 proof field elements (a_z, b_z, c_z, s_sigma_1_z, s_sigma_2_z, r_z, z_omega_z)
  recomputed in O(n) from the witness by oracle/plonk_bn254.py:evaluations_at_z (the
  barycentric form of plonk.rs:393-422; pinned to the literal oracle and its fixtures in
  tests/test_prover_oracle.py), in both modes;
* the quotient's divisibility: the prover fails with PBF_EINVAL unless coefficients
  3n+6.. of t(x) and the remainders of W_z / W_zw are all zero (plonk.rs:370, 438, 442),
  so a successful return certifies them;
* the 9 commitments through the verifier: the paper-mode proof verifies, a proof with a
  changed evaluation or a swapped commitment does not. (The reference-mode proof is
  checked by its evaluations only: with the reference's r_3(x) an honest proof verifies
  only when k3 = (a_z + beta s1_z + gamma)(b_z + beta s2_z + gamma) alpha = 0, as in the
  reference's n = 4 KAT where (b_z + beta s2_z + gamma) = 170 = 0 mod 17)
"""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bn254_pairing as B  # noqa: E402
import plonk_bn254 as P  # noqa: E402

pytestmark = pytest.mark.gpu


def _ints(t, width):
    import pbf

    a = t.cpu().numpy().view(np.uint64)
    return pbf.limbs_to_ints(a) if width == 4 else a


@pytest.mark.parametrize("log_n", [20])
def test_prove_2p20_gates(ctx, log_n):
    import torch

    import pbf

    n = 1 << log_n
    rng = random.Random(0x5EED0005)
    sp = torch.cuda.current_stream().cuda_stream
    dq = torch.empty(5 * n * 4, dtype=torch.int64, device="cuda")
    dc = torch.empty(3 * n * 2, dtype=torch.int64, device="cuda")
    dabc = torch.empty(3 * n * 4, dtype=torch.int64, device="cuda")
    ctx.plonk_synth_circuit_dev(n, 0x5EED0005, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), stream=sp)
    s = rng.randrange(2, P.R)
    srs_m = 2 * n + 2  # long enough for both modes
    dsrs = torch.empty(srs_m * 8, dtype=torch.int64, device="cuda")
    ctx.srs_create_dev(s, srs_m - 1, dsrs.data_ptr(), stream=sp)
    g2s = [B.G2_GEN, ctx.g2_bn254_mul([B.G2_GEN], [s])[0]]
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    u = rng.randrange(P.R)

    pts, fs = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal, rnd, dsrs.data_ptr(),
                                        srs_m, mode=1, stream=sp)
    chal1 = list(chal)
    pts0, fs0 = ctx.plonk_prove_bn254_dev(n, dq.data_ptr(), dc.data_ptr(), dabc.data_ptr(), chal1, rnd,
                                          dsrs.data_ptr(), srs_m, mode=0, stream=sp)
    torch.cuda.synchronize()

    # commitments: accept, then reject a changed evaluation and a swapped commitment
    verify = lambda p, f, c, md: ctx.plonk_verify_bn254_dev(  # noqa: E731
        n, dq.data_ptr(), dc.data_ptr(), dsrs.data_ptr(), srs_m, g2s, p, f, c, u, mode=md, stream=sp)
    assert verify(pts, fs, chal, 1)
    bad_f = fs.copy()
    bad_f[0] ^= 1  # a_z + / - 1
    assert not verify(pts, bad_f, chal, 1)
    bad_p = pts.copy().reshape(9, 8)
    bad_p[[0, 1]] = bad_p[[1, 0]]  # a_s <-> b_s
    assert not verify(bad_p.reshape(-1), fs, chal, 1)
    assert not verify(pts0, fs0, chal1, 0)  # the reference's r_3: k3 != 0 here

    # field elements: O(n) recomputation from the witness
    qv = _ints(dq, 4)
    q = tuple(qv[i * n:(i + 1) * n] for i in range(5))
    cv = _ints(dc, 2).reshape(3, n, 2)
    copies = tuple([(int(k), int(i)) for k, i in cv[col]] for col in range(3))
    av = _ints(dabc, 4)
    abc = tuple(av[i * n:(i + 1) * n] for i in range(3))
    ev = P.evaluations_at_z(n, q, copies, abc, chal, rnd, mode="paper")
    assert pbf.limbs_to_ints(fs) == ev
    ev0 = P.evaluations_at_z(n, q, copies, abc, chal1, rnd, mode="reference")
    assert pbf.limbs_to_ints(fs0) == ev0
