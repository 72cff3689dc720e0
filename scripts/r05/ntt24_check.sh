#!/bin/bash
# Round 5: NTT parity suite, then 2 x 2^24 (one polynomial per stream, default) time and
# calibrated HBM traffic against the single-stream group (PBF_NTT_GROUP=2)
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py tests/test_multigpu_gpu.py > gpurun_out/r05/pytest_ntt24.log 2>&1; rc=$?
tail -3 gpurun_out/r05/pytest_ntt24.log; [ $rc -eq 0 ] || exit 1
for V in default 2; do
  if [ $V = 2 ]; then export PBF_NTT_GROUP=2; else unset PBF_NTT_GROUP; fi
  timeout -k 10 400 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/r05/n24_$V.json 2>>gpurun_out/r05/n24.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r05/n24_$V.json'));t=d['roofline'].get('traffic_detail') or {}
f=t.get('fetch_counter_bytes_per_step',0)*2; w=t.get('write_bytes_per_step',0)
print('$V ms', d['ms_per_step'], 'calibrated GB', (f+w)/1e9)" | tee -a gpurun_out/r05/ntt24_check.log
done
