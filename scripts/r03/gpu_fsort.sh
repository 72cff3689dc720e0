#!/bin/bash
# Round 3: fixed-base MSM sort with its first pass from 16-bit digit codes -- MSM / prover
# GPU tests, then 2^20 and 2^24 timing against the (key, value) pair sort, and the 8192-entry
# tile A/B of the sort itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/fsort
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_msm_gpu.py \
  tests/test_prover_sharded_gpu.py tests/test_prover_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for f in 1 0 1 0; do PBF_MSM_FUSED_SORT=$f timeout -k 10 120 python scripts/r03/msm_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/fused=$f /" | tee -a $O/msm_ab.log || exit 1; done
timeout -k 10 120 python scripts/r03/msm_fx_big.py 20 2>&1 | grep -v amdgpu.ids | tee $O/fx20.log || exit 1
timeout -k 10 240 python scripts/r03/msm_fx_big.py 24 2>&1 | grep -v amdgpu.ids | tee $O/fx24.log || exit 1
cd scripts/ubench && timeout -k 10 120 ./sort_bench 28 5 2>&1 | tee ../../$O/sort28.log
