#!/bin/bash
# NTT parity tests, then the 2^24 x 2 step with the new default order against PBF_NTT_ORDER=1
set -o pipefail
mkdir -p gpurun_out/r04oc
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04oc/pytest.log 2>&1 || exit 1
out=gpurun_out/r04oc/check.log
: > $out
for i in 1 2 3; do
  for o in default 1; do
    if [ "$o" = "default" ]; then unset PBF_NTT_ORDER; else export PBF_NTT_ORDER=$o; fi
    timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04oc/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04oc/b.json')); print('2^24 order $o ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
  done
done
unset PBF_NTT_ORDER
cat $out
