#!/bin/bash
# sharded prover (virtual ranks, proving key hit on the second proof) + single-GPU prover tests,
# then the N=2 bench rehearsal over gloo
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_prover_sharded_gpu.py tests/test_prover_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/t_sh.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/t_sh.log; grep -E "^E " gpurun_out/t_sh.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29540 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --prove-log-n 16 2>/dev/null | tail -c 400
