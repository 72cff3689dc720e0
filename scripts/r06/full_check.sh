#!/bin/bash
# Round 6: the whole GPU suite (unless SKIP_TESTS=1), smoke(), then bench lines (SKIP_BENCH=1: none;
# QUICK=1: the headline at the driver's settings without side configs; else the full default line)
set -o pipefail
TAG=${1:-r06a}
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1500 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/pytest_gpu_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/r06/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06/pytest_gpu_$TAG.log | head -20; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke_$TAG.log 2>&1 || { cat gpurun_out/r06/smoke_$TAG.log; exit 1; }
fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
if [ "${QUICK:-0}" = 1 ]; then
  for i in 1 2 3; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r06/q.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r06/q.json'));print('2^20x32 driver settings', d['ms_per_step'], round(d['roofline']['frac'],4))"
    timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 50 --no-cpu --no-extra --no-traffic > gpurun_out/r06/q.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r06/q.json'));print('2^24x2 (50 warm-up)', d['ms_per_step'], round(d['roofline']['frac'],4))"
  done | tee gpurun_out/r06/quick_$TAG.log
  exit 0
fi
start=$(date +%s)
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r06/bench_$TAG.json 2> gpurun_out/r06/bench_$TAG.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 50; echo "bench running $(( $(date +%s) - start )) s"; done
wait $pid; rc=$?
echo "bench rc=$rc after $(( $(date +%s) - start )) s"
[ $rc -eq 0 ] || { tail -20 gpurun_out/r06/bench_$TAG.err; exit 1; }
tail -c 2500 gpurun_out/r06/bench_$TAG.json
