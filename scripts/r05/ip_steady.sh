#!/bin/bash
# the in-place digit-slot schedule (PBF_NTT_IP=1) against the default at steady clocks
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2; do
  for V in 0 1; do
    for cfg in "24 2" "20 32"; do
      set -- $cfg
      if [ $V = 1 ]; then export PBF_NTT_IP=1; else unset PBF_NTT_IP; fi
      timeout -k 10 200 python bench.py --log-n $1 --batch $2 --no-cpu --no-extra --no-traffic > gpurun_out/r05/ip.json 2>>gpurun_out/r05/ip.err || exit 1
      python -c "import json;d=json.load(open('gpurun_out/r05/ip.json'));print('ip=$V 2^$1 x $2', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
    done
  done
done | tee gpurun_out/r05/ip_steady.log
