#!/bin/bash
# GPU box check: parity tests, smoke, bench lines, rocprof kernel summary.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit 1; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench-2p20
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step bench-2p24
for P in default; do
  if [ $P = default ]; then unset PBF_NTT_PASSES; else export PBF_NTT_PASSES=$P; fi
  timeout -k 10 300 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench24_$P.json 2>> gpurun_out/bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench24_$P.json'));print('$P', d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
done
unset PBF_NTT_PASSES
step rocprof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o ntt2p20 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/rocprof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/prof -name "*stats*" | head
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do head -8 $f; done
