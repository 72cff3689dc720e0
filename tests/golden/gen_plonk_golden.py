#!/usr/bin/env python3
"""Golden proofs of the generalised prover (config 5) from the literal restatement
oracle/plonk_bn254.py (container-only generator; the fixtures are data):
n = 8 and 16 gates of the synthetic mul circuit, both modes, seeded challenges/blinders.
Writes tests/golden/plonk_bn254.json."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import bn254_pairing as B  # noqa: E402
import plonk_bn254 as P  # noqa: E402

S_SECRET = 0x5EED0005C0FFEE


def case(n, mode, seed):
    st = P.Setup(n, s=S_SECRET, srs_n=2 * n + 2)
    q, cp, abc = P.mul_gates_circuit(n, 0x5EED0005 + n)
    rng = random.Random(seed)
    chal = [rng.randrange(P.R) for _ in range(5)]
    rnd = [rng.randrange(P.R) for _ in range(9)]
    pts, fs, _ = P.prove(st, q, cp, abc, chal, rnd, mode=mode)
    ok = P.verify(st, q, cp, pts, fs, chal, u=0x1234567, mode=mode)
    return {"n": n, "mode": mode, "s": S_SECRET, "srs_n": 2 * n + 2, "circuit_seed": 0x5EED0005 + n,
            "chal": chal, "rnd": rnd, "u": 0x1234567,
            "pts": [list(p) if p else None for p in pts], "fields": fs, "verify": ok}


if __name__ == "__main__":
    cases = [case(8, "reference", 1), case(8, "paper", 2), case(16, "paper", 3), case(16, "reference", 4)]
    with open(os.path.join(HERE, "plonk_bn254.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_plonk_golden.py", "cases": cases}, f)
    print([(c["n"], c["mode"], c["verify"]) for c in cases])
