set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_prover_gpu.py tests/test_prover_scale_gpu.py tests/test_prover_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pv2.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/t_pv2.log
for c in 32 16 8 32 16; do
  PBF_QUOT_CHUNK=$c timeout -k 10 240 python scripts/bench_prover.py 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('quot chunk $c: prove %.2f ms (no key %.2f)'%(d['prove_ms'], d['prove_ms_no_key']))"
done
