#!/bin/bash
# Prover with and without the MSM prep stream (PBF_MSM_PREP), 2^20 and 2^24 gates
set -o pipefail
mkdir -p gpurun_out/r04i
for v in 1 0 1; do
  PBF_MSM_PREP=$v timeout -k 10 300 python -u -c "
import sys, json, os
sys.path.insert(0, 'scripts')
import bench_prover, pbf
ctx = pbf.Context(0)
for ln in (20, 24):
    r = bench_prover.run(ctx, ln, reps=10 if ln == 20 else 3, no_key=False, rounds=False)
    print(json.dumps({'prep': os.environ['PBF_MSM_PREP'], 'log_n': ln, 'prove_ms': r['prove_ms'], 'min': r['prove_ms_min'], 'verified': r.get('verified')}), flush=True)
    ctx.release_caches()
" >> gpurun_out/r04i/prep_ab.log 2>&1 || exit 1
done
