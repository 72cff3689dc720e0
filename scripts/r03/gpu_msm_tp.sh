#!/bin/bash
# Round 3: single-chain Montgomery product in the MSM accumulation -- MSM parity on the
# default build, then timing of the default (3 waves/SIMD), the 4-wave build (spills 20 B)
# and the two-chain product (libpbf_m2c.so, round-2 form).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/msmtp; mkdir -p $O
L=plonk-by-fingers_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for lib in libpbf.so libpbf_m4.so libpbf_m2c.so; do
  PBF_LIB=$L/$lib timeout -k 10 180 python scripts/r03/msm_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
done
