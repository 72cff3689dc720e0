#!/bin/bash
# Per-pass tile orders (PBF_NTT_ORDERS, one digit per pass: 0 linear, 1 XCD k-major, 2 XCD-blocked)
set -o pipefail
mkdir -p gpurun_out/r04os
out=gpurun_out/r04os/sweep.log
: > $out
for rep in 1 2; do
  for o in 01 02 11 12 21 22 20 10; do
    PBF_NTT_ORDERS=$o timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04os/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04os/b.json')); print('2^20 orders $o ms/step %.4f' % d['ms_per_step'])
" >> $out
  done
  for o in 222 122 212 221 022 220 111; do
    PBF_NTT_ORDERS=$o timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04os/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04os/b.json')); print('2^24 orders $o ms/step %.4f' % d['ms_per_step'])
" >> $out
  done
done
sort $out
