#!/bin/bash
# Round 3, GPU call A: tests touched by the context / cache / stream-contract changes, then the
# data-movement floor experiment of the 2^24 plan.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_contexts_gpu.py tests/test_prover_sharded_gpu.py tests/test_prover_gpu.py tests/test_msm_gpu.py \
  tests/test_pairing_gpu.py > gpurun_out/r03/pytest_a.log 2>&1 || { tail -30 gpurun_out/r03/pytest_a.log; exit 1; }
tail -3 gpurun_out/r03/pytest_a.log
scripts/r03/mall_floor.sh
