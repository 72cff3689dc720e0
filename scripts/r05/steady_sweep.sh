#!/bin/bash
# Round 5: the NTT schedule knobs re-measured at steady clocks (200 warm-up steps)
set -o pipefail
mkdir -p gpurun_out/r05
run() {  # label, log_n, batch, env...
  local label=$1 ln=$2 b=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --log-n $ln --batch $b --steps 100 --warmup 200 --no-cpu --no-extra --no-traffic > gpurun_out/r05/ss.json 2>>gpurun_out/r05/ss.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r05/ss.json'));print('$label', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
}
for i in 1 2; do
  run "2^20 default" 20 32 PBF_X=0
  run "2^20 events" 20 32 PBF_NTT_EVENTS=1
  run "2^20 G=2" 20 32 PBF_NTT_GROUP=2
  run "2^20 G=8" 20 32 PBF_NTT_GROUP=8
  run "2^20 one-group" 20 32 PBF_NTT_GROUP=32
  run "2^20 dual" 20 32 PBF_NTT_DUAL=1
  run "2^24 default" 24 2 PBF_X=0
  run "2^24 G=1" 24 2 PBF_NTT_GROUP=1
  run "2^24 orders 222" 24 2 PBF_NTT_ORDERS=222
  run "2^24 orders 111" 24 2 PBF_NTT_ORDERS=111
done | tee gpurun_out/r05/steady_sweep.log
