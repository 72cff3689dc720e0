#!/bin/bash
# Round 6: work-queue schedule of the two-pass NTT (one launch) against the two-stream schedule
# (PBF_NTT_NO_QUEUE=1), 2^20 x 32: parity first, then bench lines at the driver's settings
# (--steps 20 --warmup 5) and at steady clocks (--steps 100 --warmup 200)
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ntt_gpu.py \
  -k "schedule_knobs or batch_dev or golden or dual or twiddle_table" > gpurun_out/r06/pytest_queue.log 2>&1; rc=$?
tail -3 gpurun_out/r06/pytest_queue.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/pytest_queue.log | head -20; exit 1; }
run() {  # label env...
  local label=$1; shift
  for WU in "20 5" "100 200"; do
    set -- $WU
    env $ENVS timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu --no-extra --no-traffic > gpurun_out/r06/q.json 2>>gpurun_out/r06/queue_ab.err || return 1
    python -c "import json;d=json.load(open('gpurun_out/r06/q.json'));print('$label', 'steps $1 warmup $2', d['ms_per_step'], round(d['roofline']['frac'],4))"
  done
}
for i in 1 2; do
  ENVS="PBF_NTT_NO_QUEUE=1" run base || exit 1
  ENVS="PBF_NTT_QPUB=0" run pub0 || exit 1
  ENVS="PBF_NTT_QPUB=1" run pub1 || exit 1
  ENVS="PBF_NTT_QPUB=2" run pub2 || exit 1
done | tee gpurun_out/r06/queue_ab.log
for v in "PBF_NTT_QLAG=2" "PBF_NTT_QG=2" "PBF_NTT_QG=8" "PBF_NTT_QG=2 PBF_NTT_QLAG=2"; do
  ENVS="$v" run "$v" || exit 1
done | tee -a gpurun_out/r06/queue_ab.log
