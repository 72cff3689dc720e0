#!/bin/bash
# Fr NTT plans with a lower radix cap (PBF_NTT256_MAXR): the 2^24-gate proof (its 2^26-point
# coset transforms: 9,9,8 by default) and the Fr NTT parity tests under the knob
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2; do
  for R in 9 8 7; do
    PBF_NTT256_MAXR=$R timeout -k 10 300 python scripts/bench_prover.py 24 > gpurun_out/r05/maxr.json 2>>gpurun_out/r05/maxr.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r05/maxr.json'));r=d['rounds_ms'];print('maxr=$R prove_ms', round(d['prove_ms'],1), 'min', round(d['prove_ms_min'],1), 'coset', r['round 3 coset NTTs (4, key)'], 'quot', r['round 3 quotient + INTT'])"
  done
done | tee gpurun_out/r05/maxr_ab.log
