#!/bin/bash
# entries per accumulation thread: 43 (libpbf.so) vs 64 vs 86 (make ch64 ch86), fixed-base MSM
set -o pipefail
for i in 1 2; do
  for LOG in 24 22 20; do
    for L in libpbf libpbf_ch64 libpbf_ch86; do
      echo "n=2^$LOG $L $(PBF_LIB=plonk-by-fingers_amd/$L.so timeout -k 10 200 python scripts/probe_msm_fixed.py $LOG 7 2>/dev/null | tr '\n' ' ')"
    done
  done
done
