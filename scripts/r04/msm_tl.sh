#!/bin/bash
# Kernel timeline of the last standalone fixed-base MSM calls at 2^20 points
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04tl
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r04tl/t
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r04tl/t -o t -- python3 $R/scripts/probe_msm_fixed.py 20 3 > $R/gpurun_out/r04tl/probe.log 2>&1 || exit 1
cd $R
python3 scripts/msm_timeline.py $(find gpurun_out/r04tl/t -name "*kernel_trace.csv") 40
