#!/bin/bash
# geometric last pass + XCD-blocked last-pass order: NTT parity, time, traffic
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py tests/test_multigpu_gpu.py > gpurun_out/r05/pytest_geo222.log 2>&1; rc=$?
tail -2 gpurun_out/r05/pytest_geo222.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --log-n 24 --batch 2 --no-cpu --no-extra --no-traffic > gpurun_out/r05/gf.json 2>>gpurun_out/r05/gf.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r05/gf.json'));print('2^24 default', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
done | tee gpurun_out/r05/geo_final.log
timeout -k 10 300 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 50 --no-cpu --no-extra > gpurun_out/r05/gft.json 2>>gpurun_out/r05/gf.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r05/gft.json'));print('traffic', json.dumps(d['roofline']['traffic_detail']))" | tee -a gpurun_out/r05/geo_final.log
