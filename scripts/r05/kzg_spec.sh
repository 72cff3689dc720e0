#!/bin/bash
# fixed-base MSM with the table check deferred to the result: MSM parity (incl. points changed in
# place), the KZG call time, and the timeline
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_prover_gpu.py > gpurun_out/r05/pytest_kzgspec.log 2>&1; rc=$?
tail -2 gpurun_out/r05/pytest_kzgspec.log; [ $rc -eq 0 ] || exit 1
bash scripts/r05/kzg_prof.sh | head -8
