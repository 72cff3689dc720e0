"""CPU test: the device Goldilocks arithmetic of csrc/field.hpp, compiled for the host,
against 128-bit integer arithmetic (edge values, random operands, every shift twiddle)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_goldilocks_field_host(tmp_path):
    exe = str(tmp_path / "field_host_check")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-w",
                    os.path.join(HERE, "native", "field_host_check.hip"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout
    shutil.rmtree(tmp_path, ignore_errors=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fp256_host_mul(tmp_path):
    """The host 4 x 64-bit CIOS product (MSM Horner, csrc/fp256.hpp) equals the 8 x 32-bit
    CIOS product for Fr and Fq on edge and random canonical operands."""
    exe = str(tmp_path / "fp256_host_check")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-w",
                    os.path.join(HERE, "native", "fp256_host_check.hip"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout
    shutil.rmtree(tmp_path, ignore_errors=True)
