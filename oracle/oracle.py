"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of liboracle.so, the CPU restatement of adria0/plonk-by-fingers
(field.hpp / fft.hpp / pbh.hpp cite the reference file:line they follow).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker; the product path (libpbf.so) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
GOLDILOCKS = 0xFFFFFFFF00000001

_u64 = ctypes.c_uint64
_p64 = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t
_pint = ctypes.POINTER(ctypes.c_int)

_SIG = [
    ("oracle_f_add", _u64, [_u64, _u64, _u64]),
    ("oracle_f_sub", _u64, [_u64, _u64, _u64]),
    ("oracle_f_mul", _u64, [_u64, _u64, _u64]),
    ("oracle_f_neg", _u64, [_u64, _u64]),
    ("oracle_f_pow", _u64, [_u64, _u64, _u64]),
    ("oracle_f_from_i64", _u64, [_u64, ctypes.c_int64]),
    ("oracle_f_inv", ctypes.c_int, [_u64, _u64, _p64]),
    ("oracle_ntt_ct", ctypes.c_int, [_u64, _u64, _p64, _p64, _sz, ctypes.c_int]),
    ("oracle_ntt_gl_par", ctypes.c_int, [_u64, _p64, _p64, _sz, _sz, ctypes.c_int, ctypes.c_int]),
    ("oracle_ntt_vandermonde", ctypes.c_int, [_u64, _u64, _p64, _p64, _sz, ctypes.c_int]),
    ("oracle_ntt_iter", ctypes.c_int, [_u64, _u64, _p64, _p64, _sz, ctypes.c_int]),
    ("oracle_mul_ntt", ctypes.c_int, [_u64, _u64, _p64, _sz, _p64, _sz, _p64]),
    ("oracle_poly_mul", _sz, [_u64, _p64, _sz, _p64, _sz, _p64]),
    ("oracle_poly_eval", _u64, [_u64, _p64, _sz, _u64]),
    ("oracle_poly_div", ctypes.c_int, [_u64, _p64, _sz, _p64, _sz, _p64, ctypes.POINTER(_sz), _p64,
                                       ctypes.POINTER(_sz)]),
    ("oracle_g1_add", ctypes.c_int, [_p64, _p64, _p64]),
    ("oracle_g1_mul", ctypes.c_int, [_p64, _u64, _p64]),
    ("oracle_g1_neg", ctypes.c_int, [_p64, _p64]),
    ("oracle_g1_in_curve", ctypes.c_int, [_p64]),
    ("oracle_g2_add", ctypes.c_int, [_p64, _p64, _p64]),
    ("oracle_g2_mul", ctypes.c_int, [_p64, _u64, _p64]),
    ("oracle_gt_mul", None, [_p64, _p64, _p64]),
    ("oracle_gt_pow", None, [_p64, _u64, _p64]),
    ("oracle_pairing", ctypes.c_int, [_p64, _p64, _p64]),
    ("oracle_fr_mul_ntt", ctypes.c_int, [_p64, _sz, _p64, _sz, _p64, _p64]),
    ("oracle_fr_mul_ntt_par", ctypes.c_int, [_p64, _sz, _p64, _sz, _p64, ctypes.c_int, _p64]),
    ("oracle_synth_circuit", ctypes.c_int, [_sz, ctypes.c_uint64, _p64, _p64, _p64, ctypes.c_int]),
    ("oracle_commitment_scalars", ctypes.c_int, [_sz, _p64, _p64, _p64, _p64, _p64, _p64, _p64, ctypes.c_int, _p64]),
    ("oracle_plonk_prove_cpu", ctypes.c_int, [_sz, _p64, _p64, _p64, _p64, _p64, _p64, _p64, _sz, ctypes.c_int,
                                              ctypes.c_int, _p64, _p64]),
    ("oracle_g1_msm_naive", ctypes.c_int, [_p64, _p64, _sz, _p64]),
    ("oracle_g1_msm_pippenger", ctypes.c_int, [_p64, _p64, _sz, ctypes.c_int, _p64]),
    ("oracle_g1_mul_gen", ctypes.c_int, [_p64, _sz, _p64]),
    ("oracle_g1_progression", ctypes.c_int, [_p64, _p64, _sz, _p64]),
    ("oracle_pbh_prove", ctypes.c_int, [_sz, _p64, _p64, _p64, _p64, _p64, _u64, _u64, _u64, _u64, _p64, _p64,
                                        _pint]),
]

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIG:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _a(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


def _p(a: np.ndarray):
    return a.ctypes.data_as(_p64)


def ntt_ct(m: int, omega: int, values, inverse: bool = False) -> np.ndarray:
    """Recursion-faithful CooleyTurkey::fft / fft_inv (fft.rs:55-106)."""
    a = _a(values)
    out = np.empty_like(a)
    rc = lib().oracle_ntt_ct(m, omega, _p(a), _p(out), a.size, int(inverse))
    if rc:
        raise ValueError(f"oracle_ntt_ct rc={rc}")
    return out


def ntt_vandermonde(m: int, omega: int, values, inverse: bool = False) -> np.ndarray:
    a = _a(values)
    out = np.empty_like(a)
    rc = lib().oracle_ntt_vandermonde(m, omega, _p(a), _p(out), a.size, int(inverse))
    if rc:
        raise ValueError(f"oracle_ntt_vandermonde rc={rc}")
    return out


def ntt_iter(m: int, omega: int, values, inverse: bool = False) -> np.ndarray:
    a = _a(values)
    out = np.empty_like(a)
    rc = lib().oracle_ntt_iter(m, omega, _p(a), _p(out), a.size, int(inverse))
    if rc:
        raise ValueError(f"oracle_ntt_iter rc={rc}")
    return out


def ntt_gl_par(omega: int, values, batch: int = 1, inverse: bool = False, threads: int = 0) -> np.ndarray:
    """Goldilocks NTT of `batch` polynomials, optimised iterative form on `threads` host
    threads (0 = os.cpu_count()): the all-core CPU baseline (ntt_par.cpp)."""
    import os

    a = _a(values)
    out = np.empty_like(a)
    n = a.size // batch
    t = threads or (os.cpu_count() or 1)
    if lib().oracle_ntt_gl_par(omega, _p(a), _p(out), n, batch, int(inverse), t):
        raise ValueError("oracle_ntt_gl_par failed")
    return out


def mul_ntt(m: int, omega: int, a, b) -> np.ndarray:
    a = _a(a)
    b = _a(b)
    out = np.empty(a.size + b.size, dtype=np.uint64)
    rc = lib().oracle_mul_ntt(m, omega, _p(a), a.size, _p(b), b.size, _p(out))
    if rc:
        raise ValueError(f"oracle_mul_ntt rc={rc}")
    return out


def poly_mul(m: int, a, b) -> np.ndarray:
    a = _a(a)
    b = _a(b)
    out = np.empty(a.size + b.size, dtype=np.uint64)
    k = lib().oracle_poly_mul(m, _p(a), a.size, _p(b), b.size, _p(out))
    return out[:k].copy()


def poly_eval(m: int, coeffs, x: int) -> int:
    c = _a(coeffs)
    return int(lib().oracle_poly_eval(m, _p(c), c.size, x))


def poly_div(m: int, num, den):
    n = _a(num)
    d = _a(den)
    q = np.empty(max(n.size, 1) + 1, dtype=np.uint64)
    r = np.empty(max(n.size, 1) + d.size + 1, dtype=np.uint64)
    lq, lr = _sz(), _sz()
    rc = lib().oracle_poly_div(m, _p(n), n.size, _p(d), d.size, _p(q), ctypes.byref(lq), _p(r), ctypes.byref(lr))
    if rc:
        raise ValueError("oracle_poly_div failed")
    return q[: lq.value].copy(), r[: lr.value].copy()


def f(name: str, *args) -> int:
    return int(getattr(lib(), "oracle_f_" + name)(*args))


def f_inv(m: int, a: int):
    out = _u64()
    ok = lib().oracle_f_inv(m, a, ctypes.byref(out))
    return int(out.value) if ok else None


# ---- toy curve (pbh/*.rs); G1 points are (x, y, inf)
def _pt(v):
    return _a(list(v))


def g1_add(p, q):
    o = np.zeros(3, np.uint64)
    if lib().oracle_g1_add(_p(_pt(p)), _p(_pt(q)), _p(o)):
        raise ValueError("g1_add panicked")
    return tuple(int(x) for x in o)


def g1_mul(p, s):
    o = np.zeros(3, np.uint64)
    if lib().oracle_g1_mul(_p(_pt(p)), s, _p(o)):
        raise ValueError("g1_mul panicked")
    return tuple(int(x) for x in o)


def g1_neg(p):
    o = np.zeros(3, np.uint64)
    lib().oracle_g1_neg(_p(_pt(p)), _p(o))
    return tuple(int(x) for x in o)


def g2_add(p, q):
    o = np.zeros(2, np.uint64)
    if lib().oracle_g2_add(_p(_pt(p)), _p(_pt(q)), _p(o)):
        raise ValueError("g2_add panicked")
    return tuple(int(x) for x in o)


def g2_mul(p, s):
    o = np.zeros(2, np.uint64)
    if lib().oracle_g2_mul(_p(_pt(p)), s, _p(o)):
        raise ValueError("g2_mul panicked")
    return tuple(int(x) for x in o)


def gt_mul(a, b):
    o = np.zeros(2, np.uint64)
    lib().oracle_gt_mul(_p(_pt(a)), _p(_pt(b)), _p(o))
    return tuple(int(x) for x in o)


def gt_pow(a, e):
    o = np.zeros(2, np.uint64)
    lib().oracle_gt_pow(_p(_pt(a)), e, _p(o))
    return tuple(int(x) for x in o)


def pairing(p, q):
    o = np.zeros(2, np.uint64)
    if lib().oracle_pairing(_p(_pt(p)), _p(_pt(q)), _p(o)):
        raise ValueError("pairing panicked")
    return tuple(int(x) for x in o)


def pbh_prove(gates, copies, abc, chal, rnd, s=2, srs_n=6, omega_pows=4, verify_u=None):
    """plonk.rs:191-466 over PlonkByHandTypes; returns (points[9], fields[7], verified)."""
    n = len(gates)
    g = _a([x for row in gates for x in row])
    c = _a([x for col in copies for pair in col for x in pair])
    w = _a([x for col in abc for x in col])
    pts = np.zeros(27, np.uint64)
    fs = np.zeros(7, np.uint64)
    ver = ctypes.c_int()
    rc = lib().oracle_pbh_prove(n, _p(g), _p(c), _p(w), _p(_a(chal)), _p(_a(rnd)), s, srs_n, omega_pows,
                                17 if verify_u is None else verify_u, _p(pts), _p(fs), ctypes.byref(ver))
    if rc:
        raise ValueError("oracle_pbh_prove failed (reference would panic)")
    points = [tuple(int(x) for x in pts[3 * i: 3 * i + 3]) for i in range(9)]
    return points, [int(x) for x in fs], (None if verify_u is None else bool(ver.value))


# ---- synthetic inputs (mirrors fill_random_kernel in csrc/ntt_launch.hip)
_G = np.uint64(0x9E3779B97F4A7C15)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_field(modulus: int, seed: int, count: int, offset: int = 0) -> np.ndarray:
    """Element i = mix(seed + (i+1)*golden); Goldilocks re-mixes values >= p,
    other moduli reduce % M."""
    with np.errstate(over="ignore"):
        i = np.arange(offset, offset + count, dtype=np.uint64)
        z = _mix(np.uint64(seed) + (i + np.uint64(1)) * _G)
        if modulus == GOLDILOCKS:
            bad = z >= np.uint64(modulus)
            while bad.any():
                z[bad] = _mix(z[bad] + _G)
                bad = z >= np.uint64(modulus)
        else:
            z = z % np.uint64(modulus)
    return z


# ---------------------------------------------------------------- BN254 CPU baselines (bn254_cpu.cpp)
def _limbs(values, width=4):
    a = np.zeros((len(values), width), dtype=np.uint64)
    for i, v in enumerate(values):
        for j in range(width):
            a[i, j] = (int(v) >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
    return a


def _ints(a, width=4):
    a = np.asarray(a, dtype=np.uint64).reshape(-1, width)
    return [sum(int(r[j]) << (64 * j) for j in range(width)) for r in a]


def fr_mul_ntt(a_limbs: np.ndarray, b_limbs: np.ndarray, omega: int) -> np.ndarray:
    """mul_ntt (fft.rs:109-132) over BN254 Fr, recursion-faithful, 1 core; limb arrays
    (n x 4 u64) in and out."""
    a = np.ascontiguousarray(a_limbs, dtype=np.uint64).reshape(-1, 4)
    b = np.ascontiguousarray(b_limbs, dtype=np.uint64).reshape(-1, 4)
    n = len(a) + len(b)
    out = np.zeros((n, 4), dtype=np.uint64)
    w = _limbs([omega])
    if lib().oracle_fr_mul_ntt(_p(a), len(a), _p(b), len(b), _p(w), _p(out)):
        raise ValueError("la + lb must be a power of two")
    return out


def _pts_out(o):
    x, y = _ints(o.reshape(2, 4))
    return None if (x, y) == (0, 0) else (x, y)


def g1_msm_naive(points: np.ndarray, scalars: np.ndarray):
    """SRS::eval_at_s (plonk.rs:51-58) literally: affine double-and-add per point, left fold."""
    p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 8)
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    o = np.zeros(8, dtype=np.uint64)
    lib().oracle_g1_msm_naive(_p(p), _p(s), len(p), _p(o))
    return _pts_out(o)


def g1_msm_pippenger(points: np.ndarray, scalars: np.ndarray, threads: int = 1):
    p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 8)
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    o = np.zeros(8, dtype=np.uint64)
    lib().oracle_g1_msm_pippenger(_p(p), _p(s), len(p), threads, _p(o))
    return _pts_out(o)


def g1_mul_gen(scalars: np.ndarray) -> np.ndarray:
    """k_i G as affine limb rows (n x 8), the MSM baselines' points."""
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros((len(s), 8), dtype=np.uint64)
    lib().oracle_g1_mul_gen(_p(s), len(s), _p(out))
    return out


def g1_progression(k0: int, d: int, n: int) -> np.ndarray:
    """(k0 + i d) G for i < n, affine limb rows (n x 8)."""
    out = np.zeros((n, 8), dtype=np.uint64)
    lib().oracle_g1_progression(_p(_limbs([k0])), _p(_limbs([d])), n, _p(out))
    return out


# ---------------------------------------------------------------- config 5 on the host (prover_cpu.cpp)
def _threads(t):
    import os

    return t or (os.cpu_count() or 1)


def fr_mul_ntt_par(a_limbs: np.ndarray, b_limbs: np.ndarray, omega: int, threads: int = 0) -> np.ndarray:
    """mul_ntt (fft.rs:109-132) over Fr, iterative NTT on `threads` host threads (0 = all)."""
    a = np.ascontiguousarray(a_limbs, dtype=np.uint64).reshape(-1, 4)
    b = np.ascontiguousarray(b_limbs, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros((len(a) + len(b), 4), dtype=np.uint64)
    if lib().oracle_fr_mul_ntt_par(_p(a), len(a), _p(b), len(b), _p(_limbs([omega])), _threads(threads), _p(out)):
        raise ValueError("la + lb must be a power of two")
    return out


def synth_circuit(n: int, seed: int, threads: int = 0):
    """k_synth_circuit (prover.hip) restated: (q 5n x 4, copies 3n x 2, abc 3n x 4) u64 arrays."""
    q = np.zeros(5 * n * 4, dtype=np.uint64)
    c = np.zeros(3 * n * 2, dtype=np.uint64)
    abc = np.zeros(3 * n * 4, dtype=np.uint64)
    lib().oracle_synth_circuit(n, seed, _p(q), _p(c), _p(abc), _threads(threads))
    return q, c, abc


def commitment_scalars_cpu(n, q, copies, abc, chal, rnd, s, k1k2=(2, 3), threads: int = 0) -> dict:
    """plonk_bn254.commitment_scalars in C++ (limb arrays in): {mode: {a b c z t wz wzw fields}}."""
    out = np.zeros(2 * 14 * 4, dtype=np.uint64)
    rc = lib().oracle_commitment_scalars(n, _p(np.ascontiguousarray(q, dtype=np.uint64)),
                                         _p(np.ascontiguousarray(copies, dtype=np.uint64)),
                                         _p(np.ascontiguousarray(abc, dtype=np.uint64)), _p(_limbs(chal)),
                                         _p(_limbs(rnd)), _p(_limbs([s])), _p(_limbs(k1k2)), _threads(threads), _p(out))
    if rc:
        raise ValueError("s or z lies in H")
    v = _ints(out)
    res = {}
    for md, name in ((0, "reference"), (1, "paper")):
        x = v[14 * md:14 * (md + 1)]
        res[name] = dict(zip(("a", "b", "c", "z", "t", "wz", "wzw"), x[:7]))
        res[name]["fields"] = x[7:]
    return res


def plonk_prove_cpu(n, q, copies, abc, chal, rnd, srs_limbs, k1k2=(2, 3), mode=1, threads: int = 0):
    """The generalised prover on the host (the config-5 CPU baseline): limb arrays in (srs:
    srs_m x 8), returns (9 x 8 point limbs, 7 x 4 field limbs)."""
    srs = np.ascontiguousarray(srs_limbs, dtype=np.uint64).reshape(-1, 8)
    pts = np.zeros(72, dtype=np.uint64)
    fs = np.zeros(28, dtype=np.uint64)
    rc = lib().oracle_plonk_prove_cpu(n, _p(np.ascontiguousarray(q, dtype=np.uint64)),
                                      _p(np.ascontiguousarray(copies, dtype=np.uint64)),
                                      _p(np.ascontiguousarray(abc, dtype=np.uint64)), _p(_limbs(chal)), _p(_limbs(rnd)),
                                      _p(_limbs(k1k2)), _p(srs), len(srs), mode, _threads(threads), _p(pts), _p(fs))
    if rc:
        raise ValueError(f"oracle_plonk_prove_cpu rc={rc}")
    return pts, fs
