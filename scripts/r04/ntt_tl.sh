#!/bin/bash
# Kernel timeline of the headline NTT steps (2^20 x 32): gaps between dependent launches
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04ntl
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r04ntl/t
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04ntl/t -o t -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu --no-extra --no-traffic > $R/gpurun_out/r04ntl/b.log 2>&1 || exit 1
cd $R
python3 scripts/msm_timeline.py $(find gpurun_out/r04ntl/t -name "*kernel_trace.csv") 40
