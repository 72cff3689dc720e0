#!/bin/bash
# rocprofv3 kernel statistics of the default bench (no PMC children under the profiler)
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
TAG=${1:-r06g}
start=$(date +%s)
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/bprof_$TAG -o b -- python bench.py --no-traffic > gpurun_out/r06/bench_prof_$TAG.json 2> gpurun_out/r06/bench_prof_$TAG.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 50; echo "profiled bench running $(( $(date +%s) - start )) s"; done
wait $pid || { tail -20 gpurun_out/r06/bench_prof_$TAG.err; exit 1; }
f=$(find gpurun_out/r06/bprof_$TAG -name "*.db" | head -1)
python scripts/kstats.py "$f" 60 > gpurun_out/r06/bench_kstats_$TAG.txt
s=$(find gpurun_out/r06/bprof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$s" ] && cp "$s" gpurun_out/r06/bench_kernel_stats_$TAG.csv
rm -rf gpurun_out/r06/bprof_$TAG
head -30 gpurun_out/r06/bench_kstats_$TAG.txt
