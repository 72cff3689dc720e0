#!/bin/bash
# Round 5: the two-pass 4096 x 4096 plan (PBF_NTT_R4K=1) against the default three-pass plan at
# 2 x 2^24: parity first, then alternating bench lines, then kernel stats of both.
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_ntt_gpu.py -k "r4k" > gpurun_out/r05/pytest_r4k.log 2>&1; rc=$?
tail -12 gpurun_out/r05/pytest_r4k.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for V in 0 1 2; do
    if [ $V != 0 ]; then export PBF_NTT_R4K=$V; else unset PBF_NTT_R4K; fi
    timeout -k 10 200 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/b24_$V.json 2>>gpurun_out/r05/r4k_ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/b24_$V.json'));print('r4k=$V', d['ms_per_step'], d['roofline']['frac'])"
  done
done | tee gpurun_out/r05/r4k_ab.log
unset PBF_NTT_R4K
cd /tmp
for V in 0 1 2; do
  if [ $V != 0 ]; then export PBF_NTT_R4K=$V; else unset PBF_NTT_R4K; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05/prof_r4k$V -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for f in $(find gpurun_out/r05/prof_r4k* -name "*kernel_stats.csv"); do echo $f; head -6 $f | cut -c1-220; done
