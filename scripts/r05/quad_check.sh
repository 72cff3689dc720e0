#!/bin/bash
# branch-free quad select: latency, MSM / prover parity, KZG and windowed MSM call times
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 60 scripts/ubench/quad_lat > gpurun_out/r05/quad_lat.log 2>&1 || exit 1
cat gpurun_out/r05/quad_lat.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_prover_gpu.py > gpurun_out/r05/pytest_quad.log 2>&1; rc=$?
tail -2 gpurun_out/r05/pytest_quad.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/probe_msm_fixed.py 20 40
timeout -k 10 120 python scripts/bench_msm.py 20 10
