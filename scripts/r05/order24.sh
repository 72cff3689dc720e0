#!/bin/bash
# Round 5: per-pass tile orders of the regrouped 2^24 plan (PBF_NTT_ORDERS: one digit per pass,
# 0 linear, 1 XCD k-major, 2 XCD-blocked) -- time and calibrated HBM traffic per order
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  for O in 222 221 220 122 121 211 111; do
    export PBF_NTT_ORDERS=$O
    timeout -k 10 200 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/o24_$O.json 2>>gpurun_out/r05/order24.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/o24_$O.json'));print('orders=$O', d['ms_per_step'], d['roofline']['frac'])"
  done
done | tee gpurun_out/r05/order24.log
for O in 222 221 121; do
  export PBF_NTT_ORDERS=$O
  timeout -k 10 400 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/r05/o24t_$O.json 2>>gpurun_out/r05/order24.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r05/o24t_$O.json'));t=d['roofline'].get('traffic_detail') or {}
f=t.get('fetch_counter_bytes_per_step',0)*2; w=t.get('write_bytes_per_step',0)
print('orders=$O ms', d['ms_per_step'], 'calibrated GB', (f+w)/1e9, 'fetch', f/1e9, 'write', w/1e9)" | tee -a gpurun_out/r05/order24.log
done
