#!/bin/bash
# NTT parity tests, then 2^20 x 32 with the new default (k-major first pass) against the
# round-3 orders (PBF_NTT_ORDERS=01), alternated three times
set -o pipefail
mkdir -p gpurun_out/r04fk
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_multigpu_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04fk/pytest.log 2>&1 || exit 1
out=gpurun_out/r04fk/check.log
: > $out
for i in 1 2 3; do
  for o in default 01; do
    if [ "$o" = "default" ]; then unset PBF_NTT_ORDERS; else export PBF_NTT_ORDERS=$o; fi
    timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04fk/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04fk/b.json')); print('2^20 orders $o ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
  done
done
unset PBF_NTT_ORDERS
cat $out
