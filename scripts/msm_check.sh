#!/bin/bash
# MSM parity tests, then the fixed-base probe under a kernel trace (timeline of the last call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_msm.log 2>&1; rc=$?
tail -3 gpurun_out/t_msm.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_msm.log | head -20; exit 1; }
timeout -k 10 120 python scripts/probe_msm_fixed.py 20 20 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/msmprof
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/msmprof -o msm -- python3 $GRAFT_REPO_ROOT/scripts/probe_msm_fixed.py 20 3 > $GRAFT_REPO_ROOT/gpurun_out/msmprobe.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/msm_timeline.py $(find gpurun_out/msmprof -name "*kernel_trace.csv") ${1:-30}
