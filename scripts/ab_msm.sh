#!/bin/bash
# A/B of MSM variant builds: ab_msm.sh libpbf_va.so libpbf_vb.so ... (default build first)
set -o pipefail
for lib in libpbf.so "$@"; do
  echo "== $lib"
  PBF_LIB=plonk-by-fingers_amd/$lib timeout -k 10 120 python scripts/bench_msm.py 20 10 || exit 1
done
