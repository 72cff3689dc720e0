#!/bin/bash
# Schedule knobs of the 2^20 x 32 step on the final tree: streams (2 / 3) and tile order
# (PBF_NTT_ORDER 0 / 1 / 2), alternated twice
set -o pipefail
mkdir -p gpurun_out/r04kn
out=gpurun_out/r04kn/ab.log
: > $out
for rep in 1 2; do
  for cfg in "default" "PBF_NTT_STREAMS=3" "PBF_NTT_ORDER=0" "PBF_NTT_ORDER=2" "PBF_NTT_GROUP=8" ; do
    if [ "$cfg" = "default" ]; then envs=""; else envs="$cfg"; fi
    env $envs timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r04kn/b.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/r04kn/b.json')); print('$cfg ms/step %.4f frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))
" >> $out
  done
done
cat $out
