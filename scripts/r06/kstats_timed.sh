#!/bin/bash
# Round 6: kernel statistics of the timed steps only (2^20 x 32 and 2^24 x 2)
set -o pipefail
mkdir -p gpurun_out/r06/kt
export TMPDIR=/tmp
for cfg in "20 32 200 20" "24 2 50 20"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06/kt/$1 -o kt -- \
    python3 scripts/r06/ntt_steps.py $1 $2 $3 $4 > gpurun_out/r06/kt/steps_$1.log 2>&1 || exit 1
  f=$(find gpurun_out/r06/kt/$1 -name "*kernel_trace.csv" | head -1)
  grep ms_per_step gpurun_out/r06/kt/steps_$1.log
  python3 scripts/r06/kstats_timed.py "$f" $4 || exit 1
done > gpurun_out/r06/kstats_timed.txt
cat gpurun_out/r06/kstats_timed.txt
