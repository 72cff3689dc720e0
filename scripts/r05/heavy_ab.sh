#!/bin/bash
# wide-window join: heavy buckets listed and joined by lane groups (default) vs the tree steps
# (PBF_MSM_HEAVY_JOIN=0); MSM tests first, then the 2^24 timeline
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05/heavy_tests.log 2>&1 || { tail -30 gpurun_out/r05/heavy_tests.log; exit 1; }
tail -1 gpurun_out/r05/heavy_tests.log
for i in 1 2; do
  for LOG in 24 20; do
    for V in 1 0; do
      echo "n=2^$LOG heavy=$V $(PBF_MSM_HEAVY_JOIN=$V timeout -k 10 200 python scripts/probe_msm_fixed.py $LOG 9 2>/dev/null | tr '\n' ' ')"
    done
  done
done
N=36 bash scripts/r05/msm24_prof.sh 2>&1 | grep -v amdgpu.ids
