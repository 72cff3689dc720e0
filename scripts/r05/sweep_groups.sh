#!/bin/bash
# Round 5: polynomial groups x streams with the memop fork/join (2^20 x 32), and 2^24 x 2 split
# over two streams
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2; do
  for cfg in "4 2" "2 2" "8 2" "4 3" "2 4" "4 4" "8 4"; do
    set -- $cfg
    PBF_NTT_GROUP=$1 PBF_NTT_STREAMS=$2 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/sg.json 2>>gpurun_out/r05/sg.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/sg.json'));print('2^20 G=$1 S=$2', d['ms_per_step'])"
  done
  for cfg in "2 1" "1 2"; do
    set -- $cfg
    PBF_NTT_GROUP=$1 PBF_NTT_STREAMS=$2 timeout -k 10 200 python bench.py --log-n 24 --batch 2 --steps 50 --warmup 5 --no-cpu --no-extra --no-traffic > gpurun_out/r05/sg.json 2>>gpurun_out/r05/sg.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/sg.json'));print('2^24 G=$1 S=$2', d['ms_per_step'])"
  done
done | tee gpurun_out/r05/sweep_groups.log
