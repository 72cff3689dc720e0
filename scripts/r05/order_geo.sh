#!/bin/bash
# 2^24 tile orders with the geometric last pass (the k-major last pass was chosen for T3 reuse)
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2; do
  for O in 221 222 220 211; do
    PBF_NTT_ORDERS=$O timeout -k 10 200 python bench.py --log-n 24 --batch 2 --no-cpu --no-extra --no-traffic > gpurun_out/r05/og.json 2>>gpurun_out/r05/og.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/og.json'));print('orders=$O', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done | tee gpurun_out/r05/order_geo.log
