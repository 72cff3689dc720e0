#!/bin/bash
# Round 3: 29-bit-limb accumulation (msm_chunk_acc_l29) and the first-pass pre-twiddle as
# defaults -- MSM and NTT parity, MSM timing against PBF_MSM_L29=0, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/l29; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_ntt_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for env in "PBF_X=0" "PBF_MSM_L29=0"; do
  env $env timeout -k 10 180 python scripts/r03/msm_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$env /" || exit 1
done
done
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof -o k -- python scripts/r03/msm_ab.py > /dev/null 2>&1 || exit 1
echo done
