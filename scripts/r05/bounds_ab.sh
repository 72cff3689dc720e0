#!/bin/bash
# bucket bounds four keys per thread (default) vs the grid-stride form (PBF_MSM_BOUNDS1=1), with
# the max-span kernel's fewer atomics in both; MSM tests first, then the 2^24 timeline
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05/bounds_tests.log 2>&1 || { tail -30 gpurun_out/r05/bounds_tests.log; exit 1; }
tail -1 gpurun_out/r05/bounds_tests.log
for i in 1 2; do
  for LOG in 24 20; do
    for V in 0 1; do
      echo "n=2^$LOG bounds1=$V $(PBF_MSM_BOUNDS1=$V timeout -k 10 200 python scripts/probe_msm_fixed.py $LOG 9 2>/dev/null | tr '\n' ' ')"
    done
  done
done
N=44 bash scripts/r05/msm24_prof.sh 2>&1 | grep -v amdgpu.ids
