#!/bin/bash
# A/B of variant builds on the bench's config 3/4/5 side measurements: ab_extra.sh libpbf_vX.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in libpbf.so "$@"; do
  PBF_LIB=plonk-by-fingers_amd/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_$lib.json || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/ab_$lib.json'))['extra']
print('%-18s polymul %.3f ms  msm %.3f ms  pairing_chk %.3f ms  prove2^20 %.2f ms verified=%s' % ('$lib', d['config3_bn254_polymul_2p22']['ms'], d['config4_bn254_msm_2p20']['ms'], d['config4_pairing_check']['ms'], d['config5_prove_2p20']['prove_ms'], d['config5_prove_2p20']['verified']))"
done
