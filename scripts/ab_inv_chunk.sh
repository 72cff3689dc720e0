#!/bin/bash
# prover A/B over batch-inversion chunk builds (libpbf_ic*.so)
set -o pipefail
for cfg in X=0 PBF_LIB=plonk-by-fingers_amd/libpbf_ic16.so PBF_LIB=plonk-by-fingers_amd/libpbf_ic8.so X=0 PBF_LIB=plonk-by-fingers_amd/libpbf_ic16.so PBF_LIB=plonk-by-fingers_amd/libpbf_ic8.so; do
  env $cfg timeout -k 10 240 python scripts/bench_prover.py 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%-50s prove %.2f ms (no key %.2f)' % ('$cfg', d['prove_ms'], d['prove_ms_no_key']))" || exit 1
done
