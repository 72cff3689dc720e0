#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

1. reference_kats.json — the known-answer vectors held by the reference's own
   tests (inputs and expected outputs transcribed as data, each with the
   file:line it comes from). No reference source is copied.
2. ntt_vectors.json — NTT / mul_ntt vectors at sizes 2^1..2^12 (+ a 2^20 and a
   2^24 digest) computed by the oracle's recursion-faithful restatement of
   fft.rs, each cross-checked here against an independent pure-Python
   big-integer DFT (small n) or iterative NTT (large n) before it is written.

Run from the repo root:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

GOLD = oracle.GOLDILOCKS
Q32 = 3221225473  # 3*2^30 + 1, generator 5: U64Field<Q32> arithmetic is the reference's, literally


def root_of_unity(m: int, n: int) -> int:
    g = 7 if m == GOLD else 5
    return pow(g, (m - 1) // n, m)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def py_dft(a, w, m):
    n = len(a)
    return [sum(int(a[j]) * pow(w, j * k, m) for j in range(n)) % m for k in range(n)]


def py_ntt(a, w, m):
    """Independent iterative radix-2 NTT over Python ints."""
    a = [int(x) for x in a]
    n = len(a)
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j ^= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    length = 2
    while length <= n:
        wl = pow(w, n // length, m)
        for s in range(0, n, length):
            wk = 1
            for k in range(length // 2):
                u, v = a[s + k], a[s + k + length // 2] * wk % m
                a[s + k] = (u + v) % m
                a[s + k + length // 2] = (u - v) % m
                wk = wk * wl % m
        length <<= 1
    return a


REFERENCE_KATS = {
    "_source": "adria0/plonk-by-fingers test vectors, transcribed as data (file:line per entry)",
    "u64field_f101": {
        "cite": "src/utils/u64field.rs:239-254",
        "modulus": 101,
        "add": [[100, 100, 99]],
        "sub": [[0, 1, 100]],
        "neg": [[1, 100]],
        "div_by_zero_is_none": [[1, 0]],
        "mul_div_roundtrip": [[12, 4]],
        "neg_div": [[1, 2, 50], [1, 5, 20]],
        "pow": [[100, 0, 1], [100, 2, 1], [100, 3, 100]],
    },
    "fft_337": {
        "cite": "src/fft.rs:140-168",
        "modulus": 337, "omega": 85, "n": 8,
        "values": [3, 1, 4, 1, 5, 9, 2, 6],
        "freq": [31, 70, 109, 74, 334, 181, 232, 4],
    },
    "mul_ntt_337": {
        "cite": "src/fft.rs:171-183",
        "modulus": 337, "omega": 85,
        "a": [24, 12, 28, 8], "b": [4, 26, 29, 23],
    },
    "poly_15485863": {
        "cite": "src/poly.rs:402-487",
        "modulus": 15485863,
        "mul": [[[5, 0, 10, 6], [1, 2, 4], [5, 10, 30, 26, 52, 24]]],
        "add": [[[1, 2, 3], [1, 2, 3], [2, 4, 6]], [[1, 2, 3], [1, 2, 3, 4, 5], [2, 4, 6, 4, 5]],
                [[1, 2, 3, 4, 6], [1, 2, 3], [2, 4, 6, 4, 6]]],
        "sub": [[[1, 2, 3], [1, 2, 3], [0]], [[1, 2, 3], [1, 2], [0, 0, 3]]],
        "div_roundtrip": [[[1], [1, 1]], [[1, 1], [1, 1]], [[1, 2, 1], [1, 1]],
                          [[1, 2, 1, 2, 5, 8, 1, 9], [1, 1, 5, 4]]],
        "z": [[[1, 5], [5, -6, 1]]],
        "eval": [[[1, 2, 1], 2, 9]],
    },
    "g1": {
        "cite": "src/pbh/g1.rs:233-260",
        "generator": [1, 2],
        "neg_g": [1, 99], "2g": [68, 74], "neg_2g": [68, 27], "4g": [65, 98], "neg_4g": [65, 3],
        "8g": [18, 49], "neg_8g": [18, 52], "16g": [1, 99], "3g": [26, 45], "5g": [12, 32], "9g": [18, 52],
    },
    "g2": {"cite": "src/pbh/g2.rs:108-119", "generator": [36, 31], "2g": [90, 82]},
    "gt": {
        "cite": "src/pbh/gt.rs:88-97",
        "mul": [[[26, 97], [93, 76], [97, 89]]],
        "pow": [[[42, 49], 6, [97, 89]], [[68, 47], 600, [97, 89]]],
        "pow101_is_conj": [93, 76],
    },
    "pairing": {"cite": "src/pbh/pairing.rs:56-75", "p_mul": 1, "r_mul": 4, "q_mul": 3, "a": 5},
    "plonk_by_hand": {
        "cite": "src/pbh/mod.rs:44-124",
        "s": 2, "srs_n": 6, "omega_pows": 4,
        "gates_qlqrqoqmqc": [[0, 0, 16, 1, 0], [0, 0, 16, 1, 0], [0, 0, 16, 1, 0], [1, 1, 16, 0, 0]],
        "copies_kind_idx": [[[1, 1], [1, 2], [1, 3], [2, 1]],
                            [[0, 1], [0, 2], [0, 3], [2, 2]],
                            [[0, 4], [1, 4], [2, 4], [2, 3]]],
        "abc": [[3, 4, 5, 9], [3, 4, 5, 16], [9, 16, 25 % 17, 25 % 17]],
        "rand": [7, 4, 11, 12, 16, 2, 14, 11, 7],
        "challenge_alpha_beta_gamma_z_v": [15, 12, 13, 5, 12],
        "verify_u": 4,
        "expected_points": [[91, 66], [26, 45], [91, 35], [32, 59], [12, 32], [26, 45], [91, 66], [91, 35],
                            [65, 98]],
        "expected_fields": [15, 13, 5, 1, 12, 15, 15],
    },
}


def ntt_vectors():
    out = {"_source": "oracle ntt_ct (fft.rs:55-106 restatement), cross-checked vs pure-Python NTT",
           "cases": []}
    fields = [(GOLD, 0x5EED0002), (Q32, 0x5EED0012)]
    for m, seed in fields:
        for logn in range(1, 13):
            n = 1 << logn
            w = root_of_unity(m, n)
            a = oracle.splitmix_field(m, seed + logn, n)
            fwd = oracle.ntt_ct(m, w, a)
            inv = oracle.ntt_ct(m, w, fwd, inverse=True)
            check = py_dft(a, w, m) if n <= 64 else py_ntt(a, w, m)
            assert [int(x) for x in fwd] == check, (m, n)
            assert np.array_equal(inv, a), (m, n)
            case = {"modulus": m, "omega": w, "n": n, "seed": seed + logn, "sha256_fwd": sha(fwd),
                    "head": [int(x) for x in fwd[:4]], "tail": [int(x) for x in fwd[-4:]]}
            if n <= 64:
                case["fwd"] = [int(x) for x in fwd]
            out["cases"].append(case)
    # 337 field: the reference's own KAT field, all sizes dividing 336 = 2^4*21
    for logn in range(1, 5):
        n = 1 << logn
        w = pow(10, 336 // n, 337)  # 10 generates F_337^*
        a = oracle.splitmix_field(337, 0x337 + logn, n)
        fwd = oracle.ntt_ct(337, w, a)
        assert [int(x) for x in fwd] == py_dft(a, w, 337)
        out["cases"].append({"modulus": 337, "omega": w, "n": n, "seed": 0x337 + logn, "sha256_fwd": sha(fwd),
                             "head": [int(x) for x in fwd[:4]], "tail": [int(x) for x in fwd[-4:]],
                             "fwd": [int(x) for x in fwd]})
    # large digests (BASELINE config 2 and the north-star size)
    big = []
    for logn, check_ct in ((16, True), (20, True), (24, False)):
        n = 1 << logn
        w = root_of_unity(GOLD, n)
        a = oracle.splitmix_field(GOLD, 0x5EED0002, n)
        fwd = oracle.ntt_iter(GOLD, w, a)
        if check_ct:
            assert np.array_equal(fwd, oracle.ntt_ct(GOLD, w, a)), logn
        # spot-check 3 outputs by direct evaluation X_k = a(w^k)
        for k in (0, 1, n - 1):
            assert oracle.poly_eval(GOLD, a, pow(w, k, GOLD)) == int(fwd[k]), (logn, k)
        big.append({"modulus": GOLD, "omega": w, "n": n, "seed": 0x5EED0002, "sha256_fwd": sha(fwd),
                    "head": [int(x) for x in fwd[:4]], "tail": [int(x) for x in fwd[-4:]],
                    "samples": {str(k): int(fwd[k]) for k in (0, 1, 12345, n // 2, n - 1)}})
        print("digest", logn, flush=True)
    out["large"] = big
    # mul_ntt vectors (fft.rs:109-132): la = lb = n/2
    muls = []
    for m, seed in fields:
        for logn in (2, 5, 9, 13):
            n = 1 << logn
            w = root_of_unity(m, n)
            a = oracle.splitmix_field(m, seed + 100 + logn, n // 2)
            b = oracle.splitmix_field(m, seed + 200 + logn, n // 2)
            c = oracle.mul_ntt(m, w, a, b)
            assert np.array_equal(oracle.poly_mul(m, a, b), c[: len(oracle.poly_mul(m, a, b))])
            muls.append({"modulus": m, "omega": w, "la": n // 2, "lb": n // 2, "seed_a": seed + 100 + logn,
                         "seed_b": seed + 200 + logn, "sha256": sha(c)})
    out["mul_ntt"] = muls
    return out


def main():
    with open(os.path.join(HERE, "reference_kats.json"), "w") as fh:
        json.dump(REFERENCE_KATS, fh, indent=1)
    v = ntt_vectors()
    with open(os.path.join(HERE, "ntt_vectors.json"), "w") as fh:
        json.dump(v, fh, indent=1)
    print("wrote", len(v["cases"]), "ntt cases,", len(v["large"]), "digests,", len(v["mul_ntt"]), "mul_ntt")


if __name__ == "__main__":
    main()
