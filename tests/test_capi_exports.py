"""The C-ABI library builds, loads and exports every symbol include/pbf.h declares
(CPU only: no compute calls are made without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pbf.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pbf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("pbf_ctx_create", "pbf_ntt_u64", "pbf_ntt_u64_batch_dev", "pbf_mul_ntt_u64", "pbf_poly_eval_u64"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    import pbf

    lib = pbf.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # the Python binding describes every declared entry point
    assert sorted(n for n, _, _ in pbf.SIGNATURES) == declared_symbols()


def test_exported_symbols_have_c_linkage():
    import pbf

    out = subprocess.run(["nm", "-D", "--defined-only", pbf.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (pbf_[a-z0-9_]+)", out.stdout))
    assert set(declared_symbols()) <= exported


def test_library_does_not_link_the_oracle():
    import pbf

    out = subprocess.run(["nm", "-D", pbf.LIB_PATH], capture_output=True, text=True, check=True)
    assert "oracle_" not in out.stdout
    ldd = subprocess.run(["ldd", pbf.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in ldd


def test_missing_library_fails_loudly(tmp_path):
    import pbf

    saved = pbf._lib
    pbf._lib = None
    try:
        with pytest.raises(ImportError):
            pbf.load_library(str(tmp_path / "nope.so"))
    finally:
        pbf._lib = saved


def test_last_error_callable_without_gpu():
    import pbf

    lib = pbf.load_library()
    assert isinstance(lib.pbf_last_error(), (bytes, type(None)))
    h = ctypes.c_void_p()
    rc = lib.pbf_ctx_create(-1, ctypes.byref(h))
    assert rc != 0  # invalid device index (or no device here) is an error code, not a crash


def test_single_hip_runtime_in_process():
    import pbf

    pbf.load_library()
    maps = open("/proc/self/maps").read()
    paths = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(paths) == 1, paths
