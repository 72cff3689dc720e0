#!/bin/bash
# Polynomial groups per stream (PBF_NTT_GROUP) with the k-major first pass, 2^20 x 32
set -o pipefail
mkdir -p gpurun_out/r04gs
out=gpurun_out/r04gs/sweep.log
: > $out
for rep in 1 2; do
  for g in 4 8 16 2; do
    PBF_NTT_GROUP=$g timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04gs/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04gs/b.json')); print('2^20 group $g ms/step %.4f' % d['ms_per_step'])
" >> $out
  done
done
sort $out
