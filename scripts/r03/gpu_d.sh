#!/bin/bash
# Round 3, GPU call D: MSM with the hand-written radix sort (parity + timing), the prover
# tests incl. the 2^20 commitment pinning and the 2^24-gate prove, and the NTT PMC A/B.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_prover_gpu.py \
  > gpurun_out/r03/pytest_d1.log 2>&1 || { tail -40 gpurun_out/r03/pytest_d1.log; exit 1; }
tail -1 gpurun_out/r03/pytest_d1.log
timeout -k 10 240 python -u scripts/r03/msm_time.py 2>&1 | grep -v amdgpu.ids || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r03/msm_prof -o k -- python scripts/r03/msm_time.py > /dev/null 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_prover_scale_gpu.py \
  > gpurun_out/r03/pytest_d2.log 2>&1 || { tail -40 gpurun_out/r03/pytest_d2.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03/pytest_d2.log | tail -4
