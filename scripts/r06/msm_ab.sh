#!/bin/bash
# Round 6: madd with Y3 under one reduction (libpbf.so) against the round-5 madd (libpbf_base.so):
# MSM tests on the new build, then alternating timings, equal results
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py \
  > gpurun_out/r06/pytest_msm.log 2>&1; rc=$?
tail -2 gpurun_out/r06/pytest_msm.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/pytest_msm.log | head; exit 1; }
for i in 1 2; do
  for L in libpbf_base.so libpbf.so; do
    PBF_LIB=$PWD/plonk-by-fingers_amd/$L timeout -k 10 300 python scripts/r06/msm_ab.py || exit 1
  done
done | tee gpurun_out/r06/msm_ab_${TAG:-x}.log
