#!/bin/bash
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 120 scripts/ubench/ntt_floor > gpurun_out/r03/ntt_floor.log 2>&1 || { cat gpurun_out/r03/ntt_floor.log; exit 1; }
cat gpurun_out/r03/ntt_floor.log
scripts/r03/mall_floor.sh
