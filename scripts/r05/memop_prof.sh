#!/bin/bash
# does the stream-memop fork/join survive rocprofv3 kernel tracing and PMC passes?
set -o pipefail
mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "kernel-trace"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05/memop_kt -o k --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > $R/gpurun_out/r05/memop_kt.log 2>&1; echo "rc=$?"
echo "pmc events"
PBF_NTT_EVENTS=1 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05/memop_pmc_ev -o p -- python3 $R/bench.py --steps 6 --warmup 0 --no-cpu --no-extra --no-traffic > $R/gpurun_out/r05/memop_pmc_ev.log 2>&1; echo "rc=$?"
echo "pmc memop"
timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05/memop_pmc -o p -- python3 $R/bench.py --steps 6 --warmup 0 --no-cpu --no-extra --no-traffic > $R/gpurun_out/r05/memop_pmc.log 2>&1; echo "rc=$?"
