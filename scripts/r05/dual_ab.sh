#!/bin/bash
# Round 5: the dual-group single-stream schedule (default) against the two-stream schedule
# (PBF_NTT_NO_DUAL=1) at 2^20 x 32: parity, alternating bench lines, kernel trace of both.
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_ntt_gpu.py -k "dual or schedule_knobs or batch_dev or golden" > gpurun_out/r05/pytest_dual.log 2>&1; rc=$?
tail -5 gpurun_out/r05/pytest_dual.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for V in 0 1; do
    if [ $V = 1 ]; then export PBF_NTT_NO_DUAL=1; else unset PBF_NTT_NO_DUAL; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/b20_$V.json 2>>gpurun_out/r05/dual_ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/b20_$V.json'));print('no_dual=$V', d['ms_per_step'], d['roofline']['frac'])"
  done
done | tee gpurun_out/r05/dual_ab.log
unset PBF_NTT_NO_DUAL
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05/prof_dual -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
head -6 gpurun_out/r05/prof_dual/k_kernel_stats.csv | cut -c1-200
