#!/bin/bash
# batch pairing engine held at 1 / 2 / 3 waves per SIMD (libpbf_lanew*.so): throughput at 65536
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2; do
  for V in "" lanew2 lanew3; do
    if [ -n "$V" ]; then export PBF_LIB=$PWD/plonk-by-fingers_amd/libpbf_$V.so; else unset PBF_LIB; fi
    timeout -k 10 300 python scripts/r05/pair_tp.py 65536,262144 > gpurun_out/r05/lanew.json 2>>gpurun_out/r05/lanew.err || exit 1
    echo "${V:-default} $(cat gpurun_out/r05/lanew.json)"
  done
done | tee gpurun_out/r05/lanew_ab.log
