#!/bin/bash
# workgroup pairing engine: latency ubench, parity tests, check latency
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 120 scripts/ubench/pairing_lat > gpurun_out/r05/pairing_lat.log 2>&1; rc=$?
cat gpurun_out/r05/pairing_lat.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pairing_gpu.py > gpurun_out/r05/pytest_pair_wg.log 2>&1; rc=$?
tail -5 gpurun_out/r05/pytest_pair_wg.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/r05/pair_check_time.py | tee gpurun_out/r05/pair_check_time.json
