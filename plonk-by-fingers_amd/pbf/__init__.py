"""Python host binding of libpbf.so (the MI355X PLONK hot path, gfx950).

Mirrors the reference's FFT trait surface (src/fft.rs:6-21,109-132) and
Poly::eval (src/poly.rs:71-79) over the C-ABI declared in include/pbf.h.
This module is plumbing for tests and bench.py: every call goes through the HIP
library; there is no CPU fallback, and importing it without a built libpbf.so
raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PBF_LIB: an alternative in-tree build (timing experiments, e.g. libpbf_nomath.so)
LIB_PATH = os.environ.get("PBF_LIB") or os.path.join(os.path.dirname(_HERE), "libpbf.so")

GOLDILOCKS = 0xFFFFFFFF00000001

PBF_OK, PBF_EINVAL, PBF_ENOINV, PBF_EDEVICE, PBF_ECOMM, PBF_EUNSUPPORTED = range(6)
_NAMES = {1: "PBF_EINVAL", 2: "PBF_ENOINV", 3: "PBF_EDEVICE", 4: "PBF_ECOMM", 5: "PBF_EUNSUPPORTED"}


class PbfError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_NAMES.get(code, code)}: {msg}")
        self.code = code


_u64 = ctypes.c_uint64
_p64 = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p
_p32 = ctypes.POINTER(ctypes.c_uint32)

# (name, restype, argtypes) for every entry point in include/pbf.h
SIGNATURES = [
    ("pbf_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    ("pbf_ctx_destroy", None, [_vp]),
    ("pbf_last_error", ctypes.c_char_p, []),
    ("pbf_ctx_set_stream", ctypes.c_int, [_vp, _vp]),
    ("pbf_ctx_set_option", ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_char_p]),
    ("pbf_device_sync", ctypes.c_int, [_vp]),
    ("pbf_ctx_release_caches", ctypes.c_int, [_vp]),
    ("pbf_ntt_u64", ctypes.c_int, [_vp, _u64, _u64, _p64, _p64, _sz, ctypes.c_int]),
    ("pbf_ntt_u64_batch_dev", ctypes.c_int, [_vp, _u64, _u64, _vp, _vp, _sz, _sz, ctypes.c_int, _vp]),
    ("pbf_mul_ntt_u64", ctypes.c_int, [_vp, _u64, _u64, _p64, _sz, _p64, _sz, _p64]),
    ("pbf_poly_eval_u64", ctypes.c_int, [_vp, _u64, _p64, _sz, _p64, _sz, _p64]),
    ("pbf_poly_add_u64", ctypes.c_int, [_vp, _u64, _p64, _sz, _p64, _sz, _p64, ctypes.POINTER(_sz)]),
    ("pbf_poly_sub_u64", ctypes.c_int, [_vp, _u64, _p64, _sz, _p64, _sz, _p64, ctypes.POINTER(_sz)]),
    ("pbf_poly_div_u64", ctypes.c_int, [_vp, _u64, _u64, ctypes.c_uint32, _p64, _sz, _p64, _sz, _p64,
                                        ctypes.POINTER(_sz), _p64, ctypes.POINTER(_sz)]),
    ("pbf_fill_random_u64_dev", ctypes.c_int, [_vp, _u64, _u64, _vp, _sz, _vp]),
    ("pbf_pointwise_mul_u64_dev", ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _sz, _vp]),
    ("pbf_ntt_fr256_shard_local_dev", ctypes.c_int, [_vp, _p64, ctypes.c_uint32, _vp, _vp, _sz, _sz, ctypes.c_int,
                                                     _vp]),
    ("pbf_ntt_fr256_shard_combine_dev", ctypes.c_int, [_vp, _p64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _sz,
                                                       _sz, ctypes.c_int, _vp]),
    ("pbf_pointwise_mul_fr256_dev", ctypes.c_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    ("pbf_ntt_fr256", ctypes.c_int, [_vp, _p64, _p64, _p64, _sz, ctypes.c_int]),
    ("pbf_ntt_fr256_batch_dev", ctypes.c_int, [_vp, _p64, _vp, _vp, _sz, _sz, ctypes.c_int, _vp]),
    ("pbf_mul_ntt_fr256", ctypes.c_int, [_vp, _p64, _p64, _sz, _p64, _sz, _p64]),
    ("pbf_mul_ntt_fr256_dev", ctypes.c_int, [_vp, _p64, _vp, _vp, _vp, _sz, _sz, _vp]),
    ("pbf_msm_g1_bn254", ctypes.c_int, [_vp, _p64, _p64, _sz, _p64]),
    ("pbf_msm_g1_bn254_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _p64, _vp]),
    ("pbf_g1_bn254_mul_base_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("pbf_msm_g1_bn254_fixed_dev", ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, _p64, _vp]),
    ("pbf_srs_create_bn254", ctypes.c_int, [_vp, _p64, _sz, _p64]),
    ("pbf_pairing_bn254", ctypes.c_int, [_vp, _p64, _p64, _sz, _p64]),
    ("pbf_pairing_bn254_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("pbf_pairing_check_bn254", ctypes.c_int, [_vp, _p64, _p64, _sz, ctypes.POINTER(ctypes.c_int)]),
    ("pbf_g2_bn254_mul", ctypes.c_int, [_vp, _p64, _p64, _sz, _p64]),
    ("pbf_plonk_prove_bn254", ctypes.c_int, [_vp, _sz, _p64, _p64, _p64, _p64, _p64, _p64, _p64, _sz, ctypes.c_int,
                                             _p64, _p64]),
    ("pbf_plonk_prove_bn254_dev", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _p64, _p64, _p64, _vp, _sz, ctypes.c_int,
                                                 _p64, _p64, _vp]),
    ("pbf_plonk_verify_bn254", ctypes.c_int, [_vp, _sz, _p64, _p64, _p64, _sz, _p64, _p64, _p64, _p64, _p64, _p64,
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("pbf_plonk_verify_bn254_dev", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _sz, _p64, _p64, _p64, _p64, _p64, _p64,
                                                  ctypes.c_int, ctypes.POINTER(ctypes.c_int), _vp]),
    ("pbf_plonk_prove_bn254_sharded_dev", ctypes.c_int, [_vp, _vp, _sz, _vp, _vp, _vp, _p64, _p64, _p64, _vp, _sz,
                                                         ctypes.c_int, _p64, _p64, _vp]),
    ("pbf_plonk_synth_circuit_bn254_dev", ctypes.c_int, [_vp, _sz, _u64, _vp, _vp, _vp, _vp]),
    ("pbf_srs_create_bn254_dev", ctypes.c_int, [_vp, _p64, _sz, _vp, _vp]),
    ("pbf_pbh_g1_mul", ctypes.c_int, [_vp, _p32, _p32, _sz, _p32]),
    ("pbf_pbh_g2_mul", ctypes.c_int, [_vp, _p32, _p32, _sz, _p32]),
    ("pbf_pbh_gt_pow", ctypes.c_int, [_vp, _p32, _p32, _sz, _p32]),
    ("pbf_pbh_pairing", ctypes.c_int, [_vp, _p32, _p32, _sz, _p32]),
    ("pbf_pbh_prove", ctypes.c_int, [_vp, _sz, _p64, _p64, _p64, _p64, _p64, _u64, _u64, _u64, _u64, _p64, _p64,
                                     ctypes.POINTER(ctypes.c_int)]),
    ("pbf_ntt_shard_local_dev", ctypes.c_int, [_vp, _u64, _u64, ctypes.c_uint32, _vp, _vp, _sz, _sz, ctypes.c_int,
                                               _vp]),
    ("pbf_ntt_shard_combine_dev", ctypes.c_int, [_vp, _u64, _u64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _sz,
                                                 _sz, ctypes.c_int, _vp]),
    ("pbf_ntt_u64_multi", ctypes.c_int, [_vp, ctypes.c_uint32, _u64, _u64, _p64, _p64, _sz, ctypes.c_int]),
    ("pbf_ntt_u64_multi_dev", ctypes.c_int, [_vp, ctypes.c_uint32, _u64, _u64, _vp, _vp, _sz, _sz, ctypes.c_int, _vp]),
    ("pbf_ntt_fr256_multi", ctypes.c_int, [_vp, ctypes.c_uint32, _p64, _p64, _p64, _sz, ctypes.c_int]),
    ("pbf_ntt_fr256_multi_dev", ctypes.c_int, [_vp, ctypes.c_uint32, _p64, _vp, _vp, _sz, _sz, ctypes.c_int, _vp]),
    ("pbf_mul_ntt_u64_multi", ctypes.c_int, [_vp, ctypes.c_uint32, _u64, _u64, _p64, _sz, _p64, _sz, _p64]),
    ("pbf_mul_ntt_fr256_multi", ctypes.c_int, [_vp, ctypes.c_uint32, _p64, _p64, _sz, _p64, _sz, _p64]),
    ("pbf_plonk_prove_bn254_multi", ctypes.c_int, [_vp, ctypes.c_uint32, _sz, _p64, _p64, _p64, _p64, _p64, _p64, _p64,
                                                   _sz, ctypes.c_int, _p64, _p64]),
    ("pbf_plonk_prove_bn254_multi_dev", ctypes.c_int, [_vp, ctypes.c_uint32, _sz, _vp, _vp, _vp, _p64, _p64, _p64, _vp,
                                                       _sz, ctypes.c_int, _p64, _p64, _vp]),
    ("pbf_multi_backend", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]),
    ("pbf_msm_g1_bn254_fixed_range_dev", ctypes.c_int, [_vp, _vp, _sz, _sz, _vp, _sz, _p64, _vp]),
]

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libpbf.so (raises if it was not built: no fallback path exists)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so (SONAME
        # libamdhip64.so.7). Loading torch first makes libpbf.so's NEEDED
        # libamdhip64.so.7 bind to that copy instead of mapping /opt/rocm's as a
        # second runtime (two runtimes in one process cannot both own the GPU).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise ImportError(f"libpbf.so not built at {path}; run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _check(rc: int) -> None:
    if rc != PBF_OK:
        msg = load_library().pbf_last_error()
        raise PbfError(rc, msg.decode() if msg else "")


def _as_u64(x: Sequence[int] | np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.uint64))
    return a


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_p64)


class Context:
    """pbf_ctx: one device, one stream, cached twiddle tables and scratch."""

    def __init__(self, device: int = 0, options: dict | None = None):
        lib = load_library()
        h = _vp()
        _check(lib.pbf_ctx_create(device, ctypes.byref(h)))
        self.h = h
        self.lib = lib
        self.device = device
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def close(self) -> None:
        if self.h:
            self.lib.pbf_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def release_caches(self) -> None:
        """pbf_ctx_release_caches: free the proving / verification keys, the fixed-base MSM
        window table, the pairing check's prepared lines and their validating copies."""
        _check(self.lib.pbf_ctx_release_caches(self.h))

    def set_stream(self, stream_ptr: int) -> None:
        _check(self.lib.pbf_ctx_set_stream(self.h, _vp(stream_ptr)))

    def set_option(self, name: str, value) -> None:
        """pbf_ctx_set_option (include/pbf.h): a context option such as "ntt.passes" = "12,12";
        None removes it. Cached plans are rebuilt under the new value."""
        _check(self.lib.pbf_ctx_set_option(self.h, name.encode(), None if value is None else str(value).encode()))

    def sync(self) -> None:
        _check(self.lib.pbf_device_sync(self.h))

    # fft.rs:66-78
    def ntt(self, modulus: int, omega: int, values, inverse: bool = False) -> np.ndarray:
        a = _as_u64(values)
        out = np.empty_like(a)
        _check(self.lib.pbf_ntt_u64(self.h, modulus, omega, _ptr(a), _ptr(out), a.size, int(inverse)))
        return out

    def ntt_batch_dev(self, modulus: int, omega: int, d_in: int, d_out: int, n: int, batch: int,
                      inverse: bool = False, stream: int = 0) -> None:
        _check(self.lib.pbf_ntt_u64_batch_dev(self.h, modulus, omega, _vp(d_in), _vp(d_out), n, batch,
                                              int(inverse), _vp(stream) if stream else None))

    # fft.rs:109-132
    def mul_ntt(self, modulus: int, omega: int, a, b) -> np.ndarray:
        a = _as_u64(a)
        b = _as_u64(b)
        out = np.empty(a.size + b.size, dtype=np.uint64)
        _check(self.lib.pbf_mul_ntt_u64(self.h, modulus, omega, _ptr(a), a.size, _ptr(b), b.size, _ptr(out)))
        return out

    # poly.rs:71-79
    def poly_eval(self, modulus: int, coeffs, xs) -> np.ndarray:
        c = _as_u64(coeffs)
        x = _as_u64(xs)
        y = np.empty_like(x)
        _check(self.lib.pbf_poly_eval_u64(self.h, modulus, _ptr(c), c.size, _ptr(x), x.size, _ptr(y)))
        return y

    # poly.rs:165-203 AddAssign / SubAssign<&Poly> (normalised; sub keeps the :196 quirk)
    def poly_add(self, modulus: int, a, b) -> np.ndarray:
        return self._addsub(self.lib.pbf_poly_add_u64, modulus, a, b)

    def poly_sub(self, modulus: int, a, b) -> np.ndarray:
        return self._addsub(self.lib.pbf_poly_sub_u64, modulus, a, b)

    def _addsub(self, fn, modulus, a, b):
        x, y = _as_u64(a), _as_u64(b)
        out = np.empty(max(x.size, y.size), dtype=np.uint64)
        ln = _sz()
        _check(fn(self.h, modulus, _ptr(x), x.size, _ptr(y), y.size, _ptr(out), ctypes.byref(ln)))
        return out[: ln.value].copy()

    # poly.rs:230-247 Div for Poly -> (q, r); `root` of order 2^root_log bounds the NTT sizes
    def poly_div(self, modulus: int, num, den, root: int | None = None, root_log: int | None = None):
        if root is None:
            root, root_log = default_root(modulus)
        n, d = _as_u64(num), _as_u64(den)
        q = np.empty(max(n.size, 1), dtype=np.uint64)
        r = np.empty(max(n.size, 1), dtype=np.uint64)
        lq, lr = _sz(), _sz()
        _check(self.lib.pbf_poly_div_u64(self.h, modulus, root, root_log, _ptr(n), n.size, _ptr(d), d.size, _ptr(q),
                                         ctypes.byref(lq), _ptr(r), ctypes.byref(lr)))
        return q[: lq.value].copy(), r[: lr.value].copy()

    # multi-GPU stride-sharded NTT pieces (include/pbf.h)
    def shard_local_dev(self, modulus: int, omega: int, world: int, d_in: int, d_out: int, nl: int, batch: int,
                        inverse: bool = False, stream: int = 0) -> None:
        _check(self.lib.pbf_ntt_shard_local_dev(self.h, modulus, omega, world, _vp(d_in), _vp(d_out), nl, batch,
                                                int(inverse), _vp(stream) if stream else None))

    def shard_combine_dev(self, modulus: int, omega: int, world: int, rank: int, d_in: int, d_out: int, nl: int,
                          batch: int, inverse: bool = False, stream: int = 0) -> None:
        _check(self.lib.pbf_ntt_shard_combine_dev(self.h, modulus, omega, world, rank, _vp(d_in), _vp(d_out), nl,
                                                  batch, int(inverse), _vp(stream) if stream else None))

    def pointwise_mul_dev(self, modulus: int, d_a: int, d_b: int, d_c: int, count: int, stream: int = 0) -> None:
        _check(self.lib.pbf_pointwise_mul_u64_dev(self.h, modulus, _vp(d_a), _vp(d_b), _vp(d_c), count,
                                                  _vp(stream) if stream else None))

    def fr_shard_local_dev(self, omega: int, world: int, d_in: int, d_out: int, nl: int, batch: int,
                           inverse: bool = False, stream: int = 0) -> None:
        _check(self.lib.pbf_ntt_fr256_shard_local_dev(self.h, _ptr(ints_to_limbs([omega])), world, _vp(d_in),
                                                      _vp(d_out), nl, batch, int(inverse),
                                                      _vp(stream) if stream else None))

    def fr_shard_combine_dev(self, omega: int, world: int, rank: int, d_in: int, d_out: int, nl: int, batch: int,
                             inverse: bool = False, stream: int = 0) -> None:
        _check(self.lib.pbf_ntt_fr256_shard_combine_dev(self.h, _ptr(ints_to_limbs([omega])), world, rank,
                                                        _vp(d_in), _vp(d_out), nl, batch, int(inverse),
                                                        _vp(stream) if stream else None))

    def fr_pointwise_mul_dev(self, d_a: int, d_b: int, d_c: int, count: int, stream: int = 0) -> None:
        _check(self.lib.pbf_pointwise_mul_fr256_dev(self.h, _vp(d_a), _vp(d_b), _vp(d_c), count,
                                                    _vp(stream) if stream else None))

    # ---- BN254 Fr (elements as Python ints <-> 4 x u64 little-endian)
    def ntt_fr(self, omega: int, values, inverse: bool = False) -> list:
        a = ints_to_limbs(values)
        out = np.empty_like(a)
        w = ints_to_limbs([omega])
        _check(self.lib.pbf_ntt_fr256(self.h, _ptr(w), _ptr(a), _ptr(out), len(values), int(inverse)))
        return limbs_to_ints(out)

    def mul_ntt_fr(self, omega: int, a, b) -> list:
        la, lb = ints_to_limbs(a), ints_to_limbs(b)
        out = np.empty((len(a) + len(b)) * 4, dtype=np.uint64)
        w = ints_to_limbs([omega])
        _check(self.lib.pbf_mul_ntt_fr256(self.h, _ptr(w), _ptr(la), len(a), _ptr(lb), len(b), _ptr(out)))
        return limbs_to_ints(out)

    def ntt_fr_batch_dev(self, omega: int, d_in: int, d_out: int, n: int, batch: int, inverse: bool = False,
                         stream: int = 0) -> None:
        w = ints_to_limbs([omega])
        _check(self.lib.pbf_ntt_fr256_batch_dev(self.h, _ptr(w), _vp(d_in), _vp(d_out), n, batch, int(inverse),
                                                _vp(stream) if stream else None))

    def mul_ntt_fr_dev(self, omega: int, d_a: int, d_b: int, d_out: int, n: int, batch: int, stream: int = 0):
        w = ints_to_limbs([omega])
        _check(self.lib.pbf_mul_ntt_fr256_dev(self.h, _ptr(w), _vp(d_a), _vp(d_b), _vp(d_out), n, batch,
                                              _vp(stream) if stream else None))

    # ---- BN254 G1 (points as (x, y) Python int pairs; identity = (0, 0))
    def msm_g1(self, points, scalars) -> tuple:
        pts = ints_to_limbs([c for pt in points for c in pt])
        sc = ints_to_limbs(scalars)
        out = np.zeros(8, dtype=np.uint64)
        _check(self.lib.pbf_msm_g1_bn254(self.h, _ptr(pts), _ptr(sc), len(scalars), _ptr(out)))
        x, y = limbs_to_ints(out)
        return (x, y)

    def msm_g1_dev(self, d_points: int, d_scalars: int, n: int, stream: int = 0) -> tuple:
        out = np.zeros(8, dtype=np.uint64)
        _check(self.lib.pbf_msm_g1_bn254_dev(self.h, _vp(d_points), _vp(d_scalars), n, _ptr(out),
                                             _vp(stream) if stream else None))
        x, y = limbs_to_ints(out)
        return (x, y)

    def msm_g1_fixed_dev(self, d_points: int, n_points: int, d_scalars: int, n: int, stream: int = 0) -> tuple:
        """sum_{i<n} s_i P_i against the fixed base set of n_points points (KZG commit)."""
        out = np.zeros(8, dtype=np.uint64)
        _check(self.lib.pbf_msm_g1_bn254_fixed_dev(self.h, _vp(d_points), n_points, _vp(d_scalars), n, _ptr(out),
                                                   _vp(stream) if stream else None))
        v = limbs_to_ints(out)
        return v[0], v[1]

    def msm_g1_fixed_range_dev(self, d_points: int, n_points: int, first: int, d_scalars: int, n: int,
                               stream: int = 0) -> tuple:
        """sum_{i<n} s_i P_(first+i) against the fixed base set (one rank's point range)."""
        out = np.zeros(8, dtype=np.uint64)
        _check(self.lib.pbf_msm_g1_bn254_fixed_range_dev(self.h, _vp(d_points), n_points, first, _vp(d_scalars), n,
                                                         _ptr(out), _vp(stream) if stream else None))
        v = limbs_to_ints(out)
        return v[0], v[1]

    def g1_mul_base_dev(self, d_scalars: int, d_out: int, n: int, stream: int = 0) -> None:
        _check(self.lib.pbf_g1_bn254_mul_base_dev(self.h, _vp(d_scalars), _vp(d_out), n,
                                                  _vp(stream) if stream else None))

    def srs_create(self, s: int, n: int) -> list:
        out = np.zeros((n + 1) * 8, dtype=np.uint64)
        _check(self.lib.pbf_srs_create_bn254(self.h, _ptr(ints_to_limbs([s])), n, _ptr(out)))
        v = limbs_to_ints(out)
        return [(v[2 * i], v[2 * i + 1]) for i in range(n + 1)]

    # ---- generalised PLONK over BN254 (config 5; prover.hip)
    def plonk_prove_bn254(self, q, copies, abc, chal, rnd, srs, k1k2=(2, 3), mode=0):
        """q: 5 columns (q_l, q_r, q_o, q_m, q_c) of n ints; copies: 3 columns of (kind, 1-based
        idx); abc: 3 columns; chal: (alpha, beta, gamma, z, v); rnd: b1..b9; srs: affine points.
        Returns (9 points, 7 field ints) as Proof (plonk.rs:61-95)."""
        n = len(abc[0])
        qa = ints_to_limbs([x for col in q for x in col])
        ca = np.array([v for col in copies for (k, i) in col for v in (k, i)], dtype=np.uint64)
        aa = ints_to_limbs([x for col in abc for x in col])
        sa = _g1_limbs(srs)
        pts = np.zeros(72, dtype=np.uint64)
        fs = np.zeros(28, dtype=np.uint64)
        _check(self.lib.pbf_plonk_prove_bn254(self.h, n, _ptr(qa), _ptr(ca), _ptr(aa), _ptr(ints_to_limbs(chal)),
                                              _ptr(ints_to_limbs(rnd)), _ptr(ints_to_limbs(k1k2)), _ptr(sa), len(srs),
                                              mode, _ptr(pts), _ptr(fs)))
        pv = limbs_to_ints(pts)
        return [None if pv[2 * i] == 0 and pv[2 * i + 1] == 0 else (pv[2 * i], pv[2 * i + 1]) for i in range(9)], \
            limbs_to_ints(fs)

    def plonk_verify_bn254(self, q, copies, srs, g2s, pts, fields, chal, u, k1k2=(2, 3), mode=0) -> bool:
        n = len(q[0])
        qa = ints_to_limbs([x for col in q for x in col])
        ca = np.array([v for col in copies for (k, i) in col for v in (k, i)], dtype=np.uint64)
        sa = _g1_limbs(srs)
        ok = ctypes.c_int(-1)
        _check(self.lib.pbf_plonk_verify_bn254(self.h, n, _ptr(qa), _ptr(ca), _ptr(sa), len(srs), _ptr(_g2_limbs(g2s)),
                                               _ptr(_g1_limbs(pts)), _ptr(ints_to_limbs(fields)),
                                               _ptr(ints_to_limbs(chal)), _ptr(ints_to_limbs([u])),
                                               _ptr(ints_to_limbs(k1k2)), mode, ctypes.byref(ok)))
        return ok.value == 1

    def plonk_synth_circuit_dev(self, n, seed, d_q, d_copies, d_abc, stream: int = 0) -> None:
        _check(self.lib.pbf_plonk_synth_circuit_bn254_dev(self.h, n, seed, d_q, d_copies, d_abc, stream))

    def srs_create_dev(self, s: int, n: int, d_out: int, stream: int = 0) -> None:
        _check(self.lib.pbf_srs_create_bn254_dev(self.h, _ptr(ints_to_limbs([s])), n, d_out, stream))

    def plonk_prove_bn254_dev(self, n, d_q, d_copies, d_abc, chal, rnd, d_srs, srs_m, k1k2=(2, 3), mode=0,
                              stream: int = 0):
        pts = np.zeros(72, dtype=np.uint64)
        fs = np.zeros(28, dtype=np.uint64)
        _check(self.lib.pbf_plonk_prove_bn254_dev(self.h, n, d_q, d_copies, d_abc, _ptr(ints_to_limbs(chal)),
                                                  _ptr(ints_to_limbs(rnd)), _ptr(ints_to_limbs(k1k2)), d_srs, srs_m,
                                                  mode, _ptr(pts), _ptr(fs), stream))
        return pts, fs

    def plonk_verify_bn254_dev(self, n, d_q, d_copies, d_srs, srs_m, g2s, pts, fields, chal, u, k1k2=(2, 3),
                               mode=0, stream: int = 0) -> bool:
        """Plonk::verify (plonk.rs:468-650) with the circuit and SRS on the device; pts / fields
        as plonk_prove_bn254_dev returns them (limb arrays) or as ints / points."""
        pa = pts if isinstance(pts, np.ndarray) else _g1_limbs(pts)
        fa = fields if isinstance(fields, np.ndarray) else ints_to_limbs(fields)
        ok = ctypes.c_int(-1)
        _check(self.lib.pbf_plonk_verify_bn254_dev(self.h, n, d_q, d_copies, d_srs, srs_m, _ptr(_g2_limbs(g2s)),
                                                   _ptr(np.ascontiguousarray(pa, dtype=np.uint64)),
                                                   _ptr(np.ascontiguousarray(fa, dtype=np.uint64)),
                                                   _ptr(ints_to_limbs(chal)), _ptr(ints_to_limbs([u])),
                                                   _ptr(ints_to_limbs(k1k2)), mode, ctypes.byref(ok), stream))
        return ok.value == 1

    def plonk_prove_bn254_sharded_dev(self, comm: "Comm", n, d_q, d_copies, d_abc, chal, rnd, d_srs, srs_m,
                                      k1k2=(2, 3), mode=0, stream: int = 0):
        """This rank's part of the multi-GPU prove (include/pbf.h); comm: a Comm struct."""
        pts = np.zeros(72, dtype=np.uint64)
        fs = np.zeros(28, dtype=np.uint64)
        _check(self.lib.pbf_plonk_prove_bn254_sharded_dev(self.h, ctypes.addressof(comm), n, d_q, d_copies, d_abc,
                                                          _ptr(ints_to_limbs(chal)), _ptr(ints_to_limbs(rnd)),
                                                          _ptr(ints_to_limbs(k1k2)), d_srs, srs_m, mode, _ptr(pts),
                                                          _ptr(fs), stream))
        return pts, fs

    # ---- plonk-by-hand types (src/pbh/*.rs), batched on the GPU
    def _u32call(self, fn, a, b, width_out, n):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))
        b = np.ascontiguousarray(np.asarray(b, dtype=np.uint32).reshape(-1))
        out = np.zeros(n * width_out, dtype=np.uint32)
        _check(fn(self.h, a.ctypes.data_as(_p32), b.ctypes.data_as(_p32), n, out.ctypes.data_as(_p32)))
        return [tuple(int(x) for x in out[i * width_out:(i + 1) * width_out]) for i in range(n)]

    # ---- BN254 pairing (config 4 pairing check; pairing.hip)
    def pairing_bn254(self, g1s, g2s) -> np.ndarray:
        """[(x, y)] G1 affine and [((x0, x1), (y0, y1))] G2 affine (None = identity) ->
        n x 12 Fq ints (tower order c0.a0.re, c0.a0.im, ..., c1.a2.im)."""
        n = len(g1s)
        a = _g1_limbs(g1s)
        b = _g2_limbs(g2s)
        out = np.zeros(n * 48, dtype=np.uint64)
        _check(self.lib.pbf_pairing_bn254(self.h, _ptr(a), _ptr(b), n, _ptr(out)))
        return [limbs_to_ints(out[48 * i: 48 * (i + 1)]) for i in range(n)]

    def pairing_bn254_dev(self, d_g1: int, d_g2: int, n: int, d_out: int, stream: int = 0) -> None:
        _check(self.lib.pbf_pairing_bn254_dev(self.h, d_g1, d_g2, n, d_out, stream))

    def pairing_check_bn254(self, g1s, g2s) -> bool:
        a = _g1_limbs(g1s)
        b = _g2_limbs(g2s)
        ok = ctypes.c_int(-1)
        _check(self.lib.pbf_pairing_check_bn254(self.h, _ptr(a), _ptr(b), len(g1s), ctypes.byref(ok)))
        return ok.value == 1

    def g2_bn254_mul(self, pts, scalars) -> list:
        n = len(pts)
        a = _g2_limbs(pts)
        s = ints_to_limbs([int(x) for x in scalars])
        out = np.zeros(n * 16, dtype=np.uint64)
        _check(self.lib.pbf_g2_bn254_mul(self.h, _ptr(a), _ptr(s), n, _ptr(out)))
        res = []
        for i in range(n):
            v = limbs_to_ints(out[16 * i: 16 * (i + 1)])
            res.append(None if not any(v) else ((v[0], v[1]), (v[2], v[3])))
        return res

    def pbh_g1_mul(self, pts, scalars):
        return self._u32call(self.lib.pbf_pbh_g1_mul, pts, scalars, 3, len(scalars))

    def pbh_g2_mul(self, pts, scalars):
        return self._u32call(self.lib.pbf_pbh_g2_mul, pts, scalars, 2, len(scalars))

    def pbh_gt_pow(self, xs, es):
        return self._u32call(self.lib.pbf_pbh_gt_pow, xs, es, 2, len(es))

    def pbh_pairing(self, g1s, g2s):
        return self._u32call(self.lib.pbf_pbh_pairing, g1s, g2s, 2, len(g2s))

    def pbh_prove(self, gates, copies, abc, chal, rnd, s=2, srs_n=6, omega_pows=4, verify_u=None):
        """Plonk::prove (+verify) over PlonkByHandTypes; same layout as oracle.pbh_prove."""
        n = len(gates)
        a = lambda v: np.ascontiguousarray(np.asarray(v, dtype=np.uint64).reshape(-1))  # noqa: E731
        g, c, w = a(gates), a(copies), a(abc)
        ch, rd = a(chal), a(rnd)
        pts = np.zeros(27, np.uint64)
        fs = np.zeros(7, np.uint64)
        ver = ctypes.c_int()
        _check(self.lib.pbf_pbh_prove(self.h, n, _ptr(g), _ptr(c), _ptr(w), _ptr(ch), _ptr(rd), s, srs_n,
                                      omega_pows, 17 if verify_u is None else verify_u, _ptr(pts), _ptr(fs),
                                      ctypes.byref(ver)))
        points = [tuple(int(x) for x in pts[3 * i: 3 * i + 3]) for i in range(9)]
        return points, [int(x) for x in fs], (None if verify_u is None else bool(ver.value))

    def fill_random_dev(self, modulus: int, seed: int, d_out: int, count: int, stream: int = 0) -> None:
        _check(self.lib.pbf_fill_random_u64_dev(self.h, modulus, seed, _vp(d_out), count,
                                                _vp(stream) if stream else None))


Q32 = 3221225473  # 3 * 2^30 + 1 (the reference-literal cross-check prime)


class Comm(ctypes.Structure):
    """struct pbf_comm (include/pbf.h): world, rank, user, send, recv, capacity and the
    all_to_all / all_gather callbacks (CFUNCTYPE(c_int, c_void_p, c_size_t, c_void_p))."""

    _fields_ = [("world", ctypes.c_uint32), ("rank", ctypes.c_uint32), ("user", ctypes.c_void_p),
                ("send", ctypes.c_void_p), ("recv", ctypes.c_void_p), ("capacity", ctypes.c_size_t),
                ("all_to_all", ctypes.c_void_p), ("all_gather", ctypes.c_void_p)]

    def __init__(self, world, rank, send, recv, capacity, a2a, ag):
        super().__init__(world, rank, None, send, recv, capacity, ctypes.cast(a2a, ctypes.c_void_p),
                         ctypes.cast(ag, ctypes.c_void_p))


def default_root(modulus: int):
    """(root, log2 of its order) of a maximal 2-power root of unity for the supported NTT
    primes: Goldilocks (generator 7, 2-adicity 32) and q32 (generator 5, 2-adicity 30)."""
    if modulus == GOLDILOCKS:
        return pow(7, (modulus - 1) >> 32, modulus), 32
    if modulus == Q32:
        return pow(5, (modulus - 1) >> 30, modulus), 30
    raise ValueError("pass root and root_log for this modulus")


BN254_R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
BN254_Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583


def _g1_limbs(pts) -> np.ndarray:
    return ints_to_limbs([c for p in pts for c in ((0, 0) if p is None else p)])


def _g2_limbs(pts) -> np.ndarray:
    return ints_to_limbs([c for p in pts for c in ((0, 0, 0, 0) if p is None else (p[0][0], p[0][1], p[1][0], p[1][1]))])


def ints_to_limbs(values) -> np.ndarray:
    """Python ints -> flat array of 4 x u64 little-endian limbs per element."""
    out = np.empty(len(values) * 4, dtype=np.uint64)
    m = (1 << 64) - 1
    for i, v in enumerate(values):
        v = int(v)
        out[4 * i: 4 * i + 4] = [v & m, (v >> 64) & m, (v >> 128) & m, (v >> 192) & m]
    return out


def limbs_to_ints(a: np.ndarray) -> list:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 4)
    return [int(r[0]) | (int(r[1]) << 64) | (int(r[2]) << 128) | (int(r[3]) << 192) for r in a]


# ---- multi-GPU from one process (pbf_*_multi): a list of Contexts, rank g = ctxs[g] -----------
def _ctx_array(ctxs):
    arr = (_vp * len(ctxs))(*[c.h for c in ctxs])
    return arr, len(ctxs)


def _ptr_array(ptrs):
    return (_vp * len(ptrs))(*[_vp(p) if p else None for p in ptrs])


def multi_backend(ctxs) -> str:
    arr, w = _ctx_array(ctxs)
    b = ctypes.c_int(-1)
    _check(load_library().pbf_multi_backend(arr, w, ctypes.byref(b)))
    return {0: "device-copies", 1: "rccl"}[b.value]


def ntt_multi(ctxs, modulus: int, omega: int, values, inverse: bool = False) -> np.ndarray:
    """pbf_ntt_u64_multi: fft.rs:66-78 of one vector with its top log2(G) levels across the ranks."""
    arr, w = _ctx_array(ctxs)
    a = _as_u64(values)
    out = np.empty_like(a)
    _check(load_library().pbf_ntt_u64_multi(arr, w, modulus, omega, _ptr(a), _ptr(out), a.size, int(inverse)))
    return out


def ntt_multi_dev(ctxs, modulus: int, omega: int, d_in, d_out, nl: int, batch: int, inverse: bool = False,
                  streams=None) -> None:
    arr, w = _ctx_array(ctxs)
    _check(load_library().pbf_ntt_u64_multi_dev(arr, w, modulus, omega, _ptr_array(d_in), _ptr_array(d_out), nl, batch,
                                                int(inverse), _ptr_array(streams) if streams else None))


def ntt_fr_multi(ctxs, omega: int, values, inverse: bool = False) -> list:
    arr, w = _ctx_array(ctxs)
    a = ints_to_limbs(values)
    out = np.empty_like(a)
    _check(load_library().pbf_ntt_fr256_multi(arr, w, _ptr(ints_to_limbs([omega])), _ptr(a), _ptr(out), len(values),
                                              int(inverse)))
    return limbs_to_ints(out)


def mul_ntt_multi(ctxs, modulus: int, omega: int, a, b) -> np.ndarray:
    arr, w = _ctx_array(ctxs)
    a = _as_u64(a)
    b = _as_u64(b)
    out = np.empty(a.size + b.size, dtype=np.uint64)
    _check(load_library().pbf_mul_ntt_u64_multi(arr, w, modulus, omega, _ptr(a), a.size, _ptr(b), b.size, _ptr(out)))
    return out


def mul_ntt_fr_multi(ctxs, omega: int, a, b) -> list:
    arr, w = _ctx_array(ctxs)
    al, bl = ints_to_limbs(a), ints_to_limbs(b)
    out = np.empty((len(a) + len(b)) * 4, dtype=np.uint64)
    _check(load_library().pbf_mul_ntt_fr256_multi(arr, w, _ptr(ints_to_limbs([omega])), _ptr(al), len(a), _ptr(bl),
                                                  len(b), _ptr(out)))
    return limbs_to_ints(out)


def plonk_prove_bn254_multi(ctxs, q, copies, abc, chal, rnd, srs, k1k2=(2, 3), mode=1):
    """pbf_plonk_prove_bn254_multi (host inputs; same conventions as Context.plonk_prove_bn254)."""
    arr, w = _ctx_array(ctxs)
    n = len(abc[0])
    qa = ints_to_limbs([x for col in q for x in col])
    ca = np.array([v for col in copies for (k, i) in col for v in (k, i)], dtype=np.uint64)
    aa = ints_to_limbs([x for col in abc for x in col])
    sa = _g1_limbs(srs)
    pts = np.zeros(72, dtype=np.uint64)
    fs = np.zeros(28, dtype=np.uint64)
    _check(load_library().pbf_plonk_prove_bn254_multi(arr, w, n, _ptr(qa), _ptr(ca), _ptr(aa), _ptr(ints_to_limbs(chal)),
                                                      _ptr(ints_to_limbs(rnd)), _ptr(ints_to_limbs(k1k2)), _ptr(sa),
                                                      len(srs), mode, _ptr(pts), _ptr(fs)))
    pv = limbs_to_ints(pts)
    return [None if pv[2 * i] == 0 and pv[2 * i + 1] == 0 else (pv[2 * i], pv[2 * i + 1]) for i in range(9)], \
        limbs_to_ints(fs)


def plonk_prove_bn254_multi_dev(ctxs, n, d_q, d_copies, d_abc, chal, rnd, d_srs, srs_m, k1k2=(2, 3), mode=1,
                                streams=None):
    """pbf_plonk_prove_bn254_multi_dev: per-rank device inputs (lists of pointers); returns the
    proof as limb arrays (9 x 8 u64 points, 7 x 4 u64 fields)."""
    arr, w = _ctx_array(ctxs)
    pts = np.zeros(72, dtype=np.uint64)
    fs = np.zeros(28, dtype=np.uint64)
    _check(load_library().pbf_plonk_prove_bn254_multi_dev(
        arr, w, n, _ptr_array(d_q), _ptr_array(d_copies), _ptr_array(d_abc), _ptr(ints_to_limbs(chal)),
        _ptr(ints_to_limbs(rnd)), _ptr(ints_to_limbs(k1k2)), _ptr_array(d_srs), srs_m, mode, _ptr(pts), _ptr(fs),
        _ptr_array(streams) if streams else None))
    return pts, fs


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# ---- the reference's FFT trait surface (fft.rs:6-21) ------------------------
class EvaluationDomainGenerator:
    """fft.rs:6-15"""

    def __init__(self, omega: int, size: int):
        self.omega = int(omega)
        self.size = int(size)


class CooleyTurkey:
    """FFT<F> for U64Field<modulus> on the GPU (fft.rs:51-79). `fft` and
    `fft_inv` take and return canonical residues, natural order."""

    def __init__(self, modulus: int, domain: EvaluationDomainGenerator, ctx: Context | None = None):
        self.modulus = int(modulus)
        self.domain = domain
        self.ctx = ctx or default_context()

    @classmethod
    def new(cls, modulus: int, domain: EvaluationDomainGenerator, ctx: Context | None = None) -> "CooleyTurkey":
        return cls(modulus, domain, ctx)

    def fft(self, values) -> np.ndarray:
        return self.ctx.ntt(self.modulus, self.domain.omega, values, inverse=False)

    def fft_inv(self, freq) -> np.ndarray:
        return self.ctx.ntt(self.modulus, self.domain.omega, freq, inverse=True)


def mul_ntt(fft: CooleyTurkey, a_vals, b_vals) -> np.ndarray:
    """fft.rs:109-132: length la+lb, not normalised."""
    return fft.ctx.mul_ntt(fft.modulus, fft.domain.omega, a_vals, b_vals)


def normalize(coeffs: np.ndarray) -> np.ndarray:
    """poly.rs:96-105 Poly::new normalisation (strip trailing zeros, keep one)."""
    c = np.asarray(coeffs, dtype=np.uint64)
    nz = np.nonzero(c)[0]
    return c[: (nz[-1] + 1 if nz.size else 1)].copy()
