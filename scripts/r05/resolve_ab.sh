#!/bin/bash
# wide-window tail: spanning buckets resolved once before the C / D sums (default) vs each sum
# adding the parts (PBF_MSM_CD_RESOLVE=0); MSM tests first
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05/resolve_tests.log 2>&1 || { tail -30 gpurun_out/r05/resolve_tests.log; exit 1; }
tail -2 gpurun_out/r05/resolve_tests.log
for i in 1 2; do
  for LOG in 24 22; do
    for V in 1 0; do
      echo "n=2^$LOG resolve=$V $(PBF_MSM_CD_RESOLVE=$V timeout -k 10 200 python scripts/probe_msm_fixed.py $LOG 7 | tr '\n' ' ')"
    done
  done
done
