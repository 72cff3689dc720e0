#!/bin/bash
# Tile order A/B on the final tree: PBF_NTT_ORDER=1 (default: XCD k-major) against 2 (XCD-blocked,
# polynomial-major), alternated four times, 2^20 x 32 and 2^24 x 2
set -o pipefail
mkdir -p gpurun_out/r04or
out=gpurun_out/r04or/ab.log
: > $out
for rep in 1 2 3 4; do
  for o in 1 2; do
    for cfg in "20 32" "24 2"; do
      set -- $cfg
      PBF_NTT_ORDER=$o timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04or/b.json || exit 1
      python -c "
import json
d=json.load(open('gpurun_out/r04or/b.json')); print('order $o log_n $1 ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
    done
  done
done
cat $out
