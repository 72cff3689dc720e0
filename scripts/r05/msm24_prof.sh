#!/bin/bash
# fixed-base MSM of 2^24 points: wall time and the kernel timeline of the last call
set -o pipefail
mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python scripts/probe_msm_fixed.py 24 4 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05/kzgprof24 -o kzg -- python scripts/probe_msm_fixed.py 24 3 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/r05/kzgprof24 -name "*kernel_trace.csv" | head -1)
python scripts/msm_timeline.py "$f" ${N:-40} | tee gpurun_out/r05/kzg24_timeline.txt
