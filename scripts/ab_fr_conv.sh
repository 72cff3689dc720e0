#!/bin/bash
# Fr NTT parity (with and without the Montgomery conversions) + config 3 / config 5 timing A/B
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_ntt_fr256_gpu.py tests/test_prover_gpu.py tests/test_multigpu_gpu.py tests/test_prover_sharded_gpu.py tests/test_prover_scale_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_fr.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/t_fr.log; [ $rc -eq 0 ] || exit 1
for c in X=0 PBF_NTT256_CONV=1 X=0; do
  env $c timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-traffic 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin)['extra']; print('$c', 'polymul %.3f ms' % d['config3_bn254_polymul_2p22']['ms'], 'prove %.2f ms' % d['config5_prove_2p20']['prove_ms'])" || exit 1
done
