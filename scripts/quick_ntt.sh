#!/bin/bash
# Quick GPU loop for NTT kernel work: parity tests of the u64 NTT, then 2^20 x 32 and 2^24 x 2 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_multigpu_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/quick_pytest.log | head -20; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/q20.json || exit 1
timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/q24.json || exit 1
python -c "
import json
for f in ['gpurun_out/q20.json','gpurun_out/q24.json']:
    d=json.load(open(f)); print(f, 'ms/step %.4f'%d['ms_per_step'], 'GB/s %.1f'%d['roofline']['achieved'], 'frac %.4f'%d['roofline']['frac'])
"
