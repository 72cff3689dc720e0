#!/bin/bash
# Round 3: throughput-form additions in the windowed MSM's sequential bucket sums -- MSM
# parity, then windowed / fixed-base timing against the previous build (libpbf_prev.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/addtp; mkdir -p $O
L=plonk-by-fingers_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for lib in libpbf.so libpbf_prev.so; do
  PBF_LIB=$L/$lib timeout -k 10 180 python scripts/r03/msm_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
done
