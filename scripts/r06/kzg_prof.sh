#!/bin/bash
# kernel timeline of one 2^k-point KZG commit (default 24)
set -o pipefail
R=$GRAFT_REPO_ROOT
L=${1:-24}
mkdir -p $R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r06/kprof$L
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06/kprof$L -o k -- python3 $R/scripts/r06/kzg_one.py $L > $R/gpurun_out/r06/kprof$L.log 2>&1 || exit 1
grep kzg_ms $R/gpurun_out/r06/kprof$L.log
f=$(find $R/gpurun_out/r06/kprof$L -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/r06/prover_timeline.py "$f" > $R/gpurun_out/r06/kzg_timeline_2p$L.txt
rm -rf $R/gpurun_out/r06/kprof$L
cat $R/gpurun_out/r06/kzg_timeline_2p$L.txt
