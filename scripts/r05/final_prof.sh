#!/bin/bash
# rocprofv3 kernel statistics of the default bench (no PMC children under the profiler)
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
TAG=${1:-r05z}
start=$(date +%s)
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/bprof_$TAG -o b -- python bench.py --no-traffic > gpurun_out/r05/bench_prof_$TAG.json 2> gpurun_out/r05/bench_prof_$TAG.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 50; echo "profiled bench running $(( $(date +%s) - start )) s"; done
wait $pid || { tail -20 gpurun_out/r05/bench_prof_$TAG.err; exit 1; }
f=$(find gpurun_out/r05/bprof_$TAG -name "*.db" | head -1)
python scripts/kstats.py "$f" 60 > gpurun_out/r05/bench_kstats_$TAG.txt
head -30 gpurun_out/r05/bench_kstats_$TAG.txt
