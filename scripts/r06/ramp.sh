#!/bin/bash
# Round 6: cold-start per-step times of the headline (memop joins and events), twice each
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python scripts/r06/ramp.py 20 32 300 2 || exit 1
  PBF_NTT_EVENTS=1 timeout -k 10 120 python scripts/r06/ramp.py 20 32 300 2 || exit 1
done > gpurun_out/r06/ramp.log
timeout -k 10 120 python scripts/r06/ramp.py 24 2 300 2 >> gpurun_out/r06/ramp.log || exit 1
cat gpurun_out/r06/ramp.log
