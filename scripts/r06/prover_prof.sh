#!/bin/bash
# kernel timeline of one 2^k-gate proof (default 24) after two warm-up proofs
set -o pipefail
R=$GRAFT_REPO_ROOT
L=${1:-24}
mkdir -p $R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r06/pprof$L
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06/pprof$L -o p -- python3 $R/scripts/r06/prover_one.py $L > $R/gpurun_out/r06/pprof$L.log 2>&1 || exit 1
grep proof_ms $R/gpurun_out/r06/pprof$L.log
f=$(find $R/gpurun_out/r06/pprof$L -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/r06/prover_timeline.py "$f" > $R/gpurun_out/r06/prover_timeline_2p$L.txt
rm -rf $R/gpurun_out/r06/pprof$L
grep "^#" $R/gpurun_out/r06/prover_timeline_2p$L.txt | head -40
