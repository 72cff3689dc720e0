#!/bin/bash
# Round 3: single-chain product in the Fr NTT pass kernels -- Fr NTT / prover parity on the
# default build, config-3 product timing against the two-chain build (libpbf_n2c.so), and the
# 2^20-gate proof on both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/frtp; mkdir -p $O
L=plonk-by-fingers_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_fr256_gpu.py tests/test_prover_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for lib in libpbf.so libpbf_n2c.so; do
  PBF_LIB=$L/$lib timeout -k 10 180 python scripts/r03/fr_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  PBF_LIB=$L/$lib timeout -k 10 300 python scripts/bench_prover.py 20 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', 'prove 2^20', d.get('prove_ms'), 'ms')" || exit 1
done
done
