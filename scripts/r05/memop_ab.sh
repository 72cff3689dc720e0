#!/bin/bash
# Round 5: fork/join of the two-stream NTT schedule by stream memory operations
# (PBF_NTT_MEMOP=1: hipStreamWriteValue64 / hipStreamWaitValue64) against events, 2^20 x 32
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
PBF_NTT_MEMOP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ntt_gpu.py -k "schedule_knobs or batch_dev or golden or dual" > gpurun_out/r05/pytest_memop.log 2>&1; rc=$?
tail -3 gpurun_out/r05/pytest_memop.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for V in 0 1; do
    if [ $V = 1 ]; then export PBF_NTT_MEMOP=1; else unset PBF_NTT_MEMOP; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/bm_$V.json 2>>gpurun_out/r05/memop_ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/bm_$V.json'));print('memop=$V', d['ms_per_step'], d['roofline']['frac'])"
  done
done | tee gpurun_out/r05/memop_ab.log
