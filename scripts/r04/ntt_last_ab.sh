#!/bin/bash
# NTT group order A/B: the last group on the caller's stream (default) against the round-3
# order (PBF_NTT_LAST_AUX=1), alternated three times, 2^20 x 32 and 2^24 x 2
set -o pipefail
mkdir -p gpurun_out/r04la
out=gpurun_out/r04la/ab.log
: > $out
for rep in 1 2 3; do
  for v in 0 1; do
    for cfg in "20 32" "24 2"; do
      set -- $cfg
      PBF_NTT_LAST_AUX=$v timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04la/b.json || exit 1
      python -c "
import json
d=json.load(open('gpurun_out/r04la/b.json')); print('last_aux $v log_n $1 ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
    done
  done
done
cat $out
