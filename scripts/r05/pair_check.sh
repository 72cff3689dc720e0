#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pairing_gpu.py > gpurun_out/r05/pytest_pair.log 2>&1; rc=$?
tail -25 gpurun_out/r05/pytest_pair.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/r05/pair_tp.py 4096,16384,65536 | tee gpurun_out/r05/pair_tp.json
