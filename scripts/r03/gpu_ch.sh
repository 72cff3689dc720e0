#!/bin/bash
# Round 3: MSM accumulation chunk size (entries per thread: 43 default, 64, 86) -- timing of
# the windowed and fixed-base 2^20 MSM, results compared across builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
L=plonk-by-fingers_amd
for rep in 1 2; do
for lib in libpbf.so libpbf_ch64.so libpbf_ch86.so; do
  PBF_LIB=$L/$lib timeout -k 10 180 python scripts/r03/msm_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
done
