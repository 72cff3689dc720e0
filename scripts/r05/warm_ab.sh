#!/bin/bash
# headline sensitivity to warmup / steps (NTT 2^20 x 32 only)
set -o pipefail
mkdir -p gpurun_out/r05
for cfg in "20 3" "100 50" "20 3" "100 50" "20 200" "200 200"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-extra --no-cpu --no-traffic --steps $1 --warmup $2 > gpurun_out/r05/warm.json 2>gpurun_out/r05/warm.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r05/warm.json'));print('steps',$1,'warmup',$2,'ms',round(d['ms_per_step'],4),'frac',round(d['roofline']['frac'],4))"
done
