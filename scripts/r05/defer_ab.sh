#!/bin/bash
# wide-window tail: partials of buckets spanning <= 1024 chunks converted as the heavy join and the
# resolve read them (default) vs all converted by msm_l29_finish (PBF_MSM_DEFER_CONV=0); MSM tests first
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05/defer_tests.log 2>&1 || { tail -30 gpurun_out/r05/defer_tests.log; exit 1; }
tail -1 gpurun_out/r05/defer_tests.log
for i in 1 2; do
  for LOG in 24 22; do
    for V in 1 0; do
      echo "n=2^$LOG defer=$V $(PBF_MSM_DEFER_CONV=$V timeout -k 10 200 python scripts/probe_msm_fixed.py $LOG 9 2>/dev/null | tr '\n' ' ')"
    done
  done
done
for V in 1 0; do
  PBF_MSM_DEFER_CONV=$V timeout -k 10 300 python - <<'PY' 2>/dev/null || exit 1
import os, sys
sys.path.insert(0, "scripts")
import bench_prover as bp
import pbf
ctx = pbf.Context(0)
r = bp.run(ctx, 24, reps=5, verify=False, no_key=False, rounds=False)
print("defer=%s 2^24 gates prove ms median %.2f min %.2f" % (os.environ["PBF_MSM_DEFER_CONV"], r["prove_ms"], r["prove_ms_min"]), flush=True)
PY
done
N=36 bash scripts/r05/msm24_prof.sh 2>&1 | grep -v amdgpu.ids
