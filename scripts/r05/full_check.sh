#!/bin/bash
# Round 5: the whole GPU suite (unless SKIP_TESTS=1), smoke(), then the driver's default bench
# line (a heartbeat line per minute while the bench runs: its CPU baselines print nothing)
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_gpu_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05/pytest_gpu_$TAG.log | head -20; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke_$TAG.log 2>&1 || { cat gpurun_out/r05/smoke_$TAG.log; exit 1; }
fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/r05/bench_$TAG.json 2> gpurun_out/r05/bench_$TAG.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 50; echo "bench running $(( $(date +%s) - start )) s"; done
wait $pid; rc=$?
echo "bench rc=$rc after $(( $(date +%s) - start )) s"
[ $rc -eq 0 ] || { tail -20 gpurun_out/r05/bench_$TAG.err; exit 1; }
tail -c 2500 gpurun_out/r05/bench_$TAG.json
