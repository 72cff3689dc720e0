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


def test_product_library_reads_no_tuning_environment():
    """the product build never takes a schedule or a code path from the
    environment -- tuning goes through pbf_ctx_set_option (include/pbf.h) and the A/B switches
    of measured-negative variants are compiled in only with -DPBF_AB (make ab). The only
    variable names left in libpbf.so are the RCCL library path and the single-device test hook
    of the RCCL branch (csrc/group.hip)."""
    import pbf

    data = open(pbf.LIB_PATH, "rb").read()
    names = set(re.findall(rb"PBF_[A-Z0-9_]{3,}", data))
    assert names <= {b"PBF_RCCL_LIB", b"PBF_GROUP_FORCE_RCCL"}, sorted(names)
    src = os.path.join(ROOT, "plonk-by-fingers_amd", "csrc")
    calls = []
    for fn in os.listdir(src):
        if fn.endswith((".hip", ".hpp")):
            calls += [(fn, m) for m in re.findall(r"getenv\((\"?[A-Za-z_]+\"?)\)", open(os.path.join(src, fn)).read())]
    # group.hip's two names and internal.hpp's ab_env (PBF_AB builds only)
    assert sorted(calls) == [("group.hip", '"PBF_GROUP_FORCE_RCCL"'), ("group.hip", '"PBF_RCCL_LIB"'),
                             ("internal.hpp", "name")], calls


def test_set_option_is_declared_with_its_names():
    src = open(HEADER).read()
    assert "pbf_ctx_set_option" in src
    capi = open(os.path.join(ROOT, "plonk-by-fingers_amd", "csrc", "capi.hip")).read()
    known = re.search(r"known\[\] = \{(.*?)\};", capi, flags=re.S).group(1)
    for name in re.findall(r"\"([a-z0-9_.]+)\"", known):
        assert name in src, name  # every accepted option is documented in pbf.h
