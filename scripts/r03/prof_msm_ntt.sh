#!/bin/bash
# Round 3: kernel statistics of the 2^20 MSMs (windowed, fixed-base) and of the default
# 2^24 x 2 NTT step (per-pass durations).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/r03/msm_time.py > $O/msm_time.log 2>&1 || { tail $O/msm_time.log; exit 1; }
grep -v amdgpu.ids $O/msm_time.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/msm -o k -- python scripts/r03/msm_time.py > /dev/null 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ntt24 -o k -- python bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
find $O -name "*kernel_stats.csv" | head
