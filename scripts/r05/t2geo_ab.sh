#!/bin/bash
# geometric last-pass twiddles of the 2^24 plan (PBF_NTT_T2GEO=1): NTT parity under the knob,
# then time and traffic against the 128 MiB table
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
PBF_NTT_T2GEO=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py > gpurun_out/r05/pytest_t2geo.log 2>&1; rc=$?
tail -3 gpurun_out/r05/pytest_t2geo.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for V in 0 1; do
    if [ $V = 1 ]; then export PBF_NTT_T2GEO=1; else unset PBF_NTT_T2GEO; fi
    timeout -k 10 200 python bench.py --log-n 24 --batch 2 --no-cpu --no-extra --no-traffic > gpurun_out/r05/t2.json 2>>gpurun_out/r05/t2.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/t2.json'));print('t2geo=$V', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done | tee gpurun_out/r05/t2geo_ab.log
for V in 0 1; do
  if [ $V = 1 ]; then export PBF_NTT_T2GEO=1; else unset PBF_NTT_T2GEO; fi
  timeout -k 10 300 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 50 --no-cpu --no-extra > gpurun_out/r05/t2tr.json 2>>gpurun_out/r05/t2.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r05/t2tr.json'));t=d['roofline']['traffic_detail'];print('t2geo=$V traffic GB', round(t['hbm_bytes_per_step']/1e9,4) if t.get('hbm_bytes_per_step') else t)" | tee -a gpurun_out/r05/t2geo_ab.log
done
