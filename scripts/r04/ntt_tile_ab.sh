#!/bin/bash
# 128-B (and wider) runs on both sides (verdict r03 item 6): the default tiles against
# PBF_NTT_TILE=16384 at 2^20 (W = 16: 128-B runs, one workgroup per CU) and PBF_NTT_TILE=8192
# at 2^24 (W = 32: 256-B runs, two workgroups per CU), alternated three times.
set -o pipefail
mkdir -p gpurun_out/r04t
out=gpurun_out/r04t/ntt_tile_ab.log
: > $out
for rep in 1 2 3; do
  for cfg in "20 32 0" "20 32 16384" "24 2 0" "24 2 8192"; do
    set -- $cfg
    if [ "$3" = "0" ]; then unset PBF_NTT_TILE; else export PBF_NTT_TILE=$3; fi
    timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04t/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04t/b.json')); print('log_n $1 batch $2 tile $3 ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
  done
done
unset PBF_NTT_TILE
cat $out
