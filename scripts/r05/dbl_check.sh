#!/bin/bash
# G1Quad::dbl in three product rounds: latency, MSM + prover parity, KZG call time
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 120 scripts/ubench/pairing_lat > gpurun_out/r05/pairing_lat4.log 2>&1 || exit 1
grep "G1" gpurun_out/r05/pairing_lat4.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_prover_gpu.py > gpurun_out/r05/pytest_dbl.log 2>&1; rc=$?
tail -3 gpurun_out/r05/pytest_dbl.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/probe_msm_fixed.py 20 40
