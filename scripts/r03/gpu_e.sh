#!/bin/bash
# Round 3, GPU call E: MSM sort v2 (parity + timing + kernel profile), then the NTT PMC A/B.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py \
  > gpurun_out/r03/pytest_e.log 2>&1 || { tail -40 gpurun_out/r03/pytest_e.log; exit 1; }
tail -1 gpurun_out/r03/pytest_e.log
timeout -k 10 240 python -u scripts/r03/msm_time.py 2>&1 | grep -v amdgpu.ids || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/r03/msm_prof2
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r03/msm_prof2 -o k -- python scripts/r03/msm_time.py > /dev/null 2>&1 || exit 1
scripts/r03/pmc_ab.sh && scripts/r03/fetch_cal.sh
