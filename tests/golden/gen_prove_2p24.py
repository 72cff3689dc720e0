"""Golden scalars of one seeded 2^24-gate proof (BASELINE config 5 at its size; test
infrastructure, runs in the container): the circuit is the GPU's synthetic circuit
(pbf_plonk_synth_circuit_bn254_dev, seed 0x5EED0024) restated on the host
(oracle/prover_cpu.cpp oracle_synth_circuit), the SRS secret / challenges / blinders come from
random.Random(0x5EED0024) in the order tests/test_prover_scale_gpu.py::test_prove_2p24_gates
draws them, and the O(n) checker (oracle_commitment_scalars = oracle/plonk_bn254.py
commitment_scalars, barycentric evaluations of every polynomial of src/plonk.rs:245-446 at
the SRS secret s and at z) gives, for the paper-mode proof:
  fields  a_z b_z c_z s_sigma_1_z s_sigma_2_z r_z z_omega_z   (the Proof's 7 elements)
  a b c z:  a(s) ... (a_s = [a(s)]G, ...)
  t:        t(s)      (t_lo + [s^(n+2)] t_mid + [s^(2n+4)] t_hi = [t(s)]G)
  wz, wzw:  the W_z / W_zw identities (plonk_bn254.commitments_match)

    python tests/golden/gen_prove_2p24.py        # writes tests/golden/prove_2p24.json (~1-3 min)
"""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import oracle  # noqa: E402

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
LOG_N, SEED = 24, 0x5EED0024


def main():
    n = 1 << LOG_N
    t0 = time.time()
    q, c, abc = oracle.synth_circuit(n, SEED)
    rng = random.Random(SEED)
    s = rng.randrange(2, R)
    chal = [rng.randrange(R) for _ in range(5)]
    rnd = [rng.randrange(R) for _ in range(9)]
    u = rng.randrange(R)
    cs = oracle.commitment_scalars_cpu(n, q, c, abc, chal, rnd, s)
    out = {
        "what": "scalars of the paper-mode Plonk::prove of the seeded 2^24-gate synthetic circuit (O(n) checker)",
        "generator": "tests/golden/gen_prove_2p24.py (oracle/prover_cpu.cpp oracle_synth_circuit + "
                     "oracle_commitment_scalars)",
        "log_n": LOG_N, "seed": SEED, "s": str(s), "chal": [str(x) for x in chal], "rnd": [str(x) for x in rnd],
        "u": str(u),
        "paper": {k: (str(v) if k != "fields" else [str(x) for x in v]) for k, v in cs["paper"].items()},
        "reference_fields": [str(x) for x in cs["reference"]["fields"]],
        "seconds": round(time.time() - t0, 1),
    }
    with open(os.path.join(HERE, "prove_2p24.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
