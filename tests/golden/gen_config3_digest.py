"""Golden digest of BASELINE config 3 at its own size (test infrastructure; runs in the
container, not on the GPU box): mul_ntt (/root/reference/src/fft.rs:109-132) of the seeded
operands of tests/test_ntt_fr256_gpu.py::test_mul_ntt_config3_size_evaluation_identity
(a, b = bn254.random_limbs(2^22, 301 / 302), NTT size 2^23), computed by the oracle's
recursion-faithful C++ restatement (oracle/bn254_cpu.cpp oracle_fr_mul_ntt, one core),
stored as the SHA-256 of the full 2^23 x 4 u64 little-endian output plus sampled values.
Cross-checked at generation time by the evaluation identity c(x) = a(x) b(x) at two points
with Python big integers (independent of the NTT).

    python tests/golden/gen_config3_digest.py     # writes tests/golden/config3_mul_ntt.json
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import bn254  # noqa: E402
import oracle  # noqa: E402

LA = 1 << 22
SEEDS = (301, 302)
SAMPLES = [0, 1, 2, 3, 12345, LA - 1, LA, 2 * LA - 3, 2 * LA - 2, 2 * LA - 1]


def main():
    n = 2 * LA
    w = bn254.root_of_unity(n)
    a = bn254.random_limbs(LA, SEEDS[0])
    b = bn254.random_limbs(LA, SEEDS[1])
    t = time.time()
    c = oracle.fr_mul_ntt(a.reshape(-1, 4), b.reshape(-1, 4), w)
    dt = time.time() - t
    flat = np.ascontiguousarray(c, dtype=np.uint64).reshape(-1)
    digest = hashlib.sha256(flat.astype("<u8").tobytes()).hexdigest()
    ci = bn254.limbs_to_ints(flat)
    ai, bi = bn254.limbs_to_ints(a), bn254.limbs_to_ints(b)
    R = bn254.R
    for x in (3, 123456789123456789):
        assert bn254.poly_eval(ci, x) == bn254.poly_eval(ai, x) * bn254.poly_eval(bi, x) % R
    assert ci[-1] == 0
    out = {
        "what": "mul_ntt (fft.rs:109-132) over BN254 Fr, a, b = bn254.random_limbs(2^22, 301 / 302), NTT size 2^23",
        "generator": "tests/golden/gen_config3_digest.py (oracle/bn254_cpu.cpp oracle_fr_mul_ntt, recursion-faithful)",
        "la": LA, "lb": LA, "seeds": list(SEEDS),
        "sha256_le_u64": digest,
        "samples": {str(i): str(ci[i]) for i in SAMPLES},
        "oracle_seconds": round(dt, 1),
    }
    with open(os.path.join(HERE, "config3_mul_ntt.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
