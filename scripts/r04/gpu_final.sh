#!/bin/bash
# Round-4 final evidence: the default bench line (N = 1), then the kernel stats of the same
# workload under rocprofv3 (no PMC children: --no-traffic; no CPU legs: --no-cpu).
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04y}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/kprof -o b -- python3 $R/bench.py --no-traffic --no-cpu > $R/gpurun_out/$T/bench_prof.json 2> $R/gpurun_out/$T/bench_prof.err || exit $?
