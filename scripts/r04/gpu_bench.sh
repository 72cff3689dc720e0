#!/bin/bash
# Round-4 evidence: batch-affine microbenchmark, then the default bench line (N = 1).
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 scripts/ubench/batch_affine > gpurun_out/r04/batch_affine.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err || exit $?
