#!/bin/bash
# pairing tests + batch throughput (two lane builds), NTT data floors at steady clocks
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pairing_gpu.py > gpurun_out/r05/pytest_pair_w2.log 2>&1; rc=$?
tail -4 gpurun_out/r05/pytest_pair_w2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/r05/pair_tp.py 65536,262144 | tee gpurun_out/r05/pair_tp_w2.json || exit 1
timeout -k 10 300 scripts/ubench/ntt_floor > gpurun_out/r05/ntt_floor_steady.log 2>&1; rc=$?
cat gpurun_out/r05/ntt_floor_steady.log; exit $rc
