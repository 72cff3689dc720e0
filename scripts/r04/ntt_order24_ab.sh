#!/bin/bash
# Tile order A/B at 2^24 x 2 (the regrouped 3-pass plan): orders 0 / 1 / 2 alternated five times
set -o pipefail
mkdir -p gpurun_out/r04o24
out=gpurun_out/r04o24/ab.log
: > $out
for rep in 1 2 3 4 5; do
  for o in 1 2 0; do
    PBF_NTT_ORDER=$o timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04o24/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04o24/b.json')); print('order $o log_n 24 ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
  done
done
cat $out
