"""Oracle vs the committed golden NTT vectors (CPU only, small sizes)."""
import hashlib

import numpy as np

import oracle


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def test_splitmix_inputs_are_canonical_and_stable():
    a = oracle.splitmix_field(oracle.GOLDILOCKS, 0x5EED0002, 1 << 12)
    assert (a < np.uint64(oracle.GOLDILOCKS)).all()
    assert np.array_equal(a[100:200], oracle.splitmix_field(oracle.GOLDILOCKS, 0x5EED0002, 100, offset=100))


def test_ntt_vectors_small(vectors):
    for c in vectors["cases"]:
        if c["n"] > 1024:
            continue
        a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
        fwd = oracle.ntt_ct(c["modulus"], c["omega"], a)
        assert sha(fwd) == c["sha256_fwd"], c["n"]
        if "fwd" in c:
            assert fwd.tolist() == c["fwd"]
        assert np.array_equal(oracle.ntt_ct(c["modulus"], c["omega"], fwd, inverse=True), a)


def test_mul_ntt_vectors(vectors):
    for c in vectors["mul_ntt"]:
        if c["la"] > 512:
            continue
        a = oracle.splitmix_field(c["modulus"], c["seed_a"], c["la"])
        b = oracle.splitmix_field(c["modulus"], c["seed_b"], c["lb"])
        assert sha(oracle.mul_ntt(c["modulus"], c["omega"], a, b)) == c["sha256"]


def test_large_digest_2p16(vectors):
    c = vectors["large"][0]
    assert c["n"] == 1 << 16
    a = oracle.splitmix_field(c["modulus"], c["seed"], c["n"])
    assert sha(oracle.ntt_iter(c["modulus"], c["omega"], a)) == c["sha256_fwd"]


def test_parallel_cpu_ntt_matches_oracle():
    # the all-core CPU baseline (oracle/ntt_par.cpp) computes the same transform as the
    # recursion-faithful restatement of fft.rs:90-106 (and its inverse)
    import numpy as np

    import oracle

    G = 0xFFFFFFFF00000001
    for logn in (1, 3, 11):
        n = 1 << logn
        w = pow(7, (G - 1) // n, G)
        a = oracle.splitmix_field(G, 9 + logn, 3 * n)
        got = oracle.ntt_gl_par(w, a, batch=3, threads=2)
        ref = np.concatenate([oracle.ntt_ct(G, w, a[i * n:(i + 1) * n]) for i in range(3)])
        assert np.array_equal(got, ref)
        assert np.array_equal(oracle.ntt_gl_par(w, got, batch=3, inverse=True, threads=2), a)
