#!/bin/bash
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 180 scripts/ubench/ntt_floor > gpurun_out/r03/ntt_floor_c.log 2>&1 || { cat gpurun_out/r03/ntt_floor_c.log; exit 1; }
cat gpurun_out/r03/ntt_floor_c.log
