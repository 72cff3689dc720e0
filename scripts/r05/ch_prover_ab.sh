#!/bin/bash
# entries per accumulation thread 43 vs 86: windowed MSM (2^20) and the 2^20 / 2^24-gate proofs
set -o pipefail
for L in libpbf libpbf_ch86 libpbf libpbf_ch86; do
  echo "$L windowed: $(PBF_LIB=plonk-by-fingers_amd/$L.so timeout -k 10 200 python scripts/bench_msm.py 20 20 2>/dev/null | tr '\n' ' ')"
done
for L in libpbf libpbf_ch86; do
  PBF_LIB=plonk-by-fingers_amd/$L.so timeout -k 10 300 python - <<'PY' 2>/dev/null || exit 1
import os, sys, json
sys.path.insert(0, "scripts")
import bench_prover as bp
import pbf
ctx = pbf.Context(0)
for ln, reps in ((20, 9), (24, 5)):
    r = bp.run(ctx, ln, reps=reps, verify=False, no_key=False, rounds=False)
    print(os.environ["PBF_LIB"].split("/")[-1], "2^%d gates prove ms median %.2f min %.2f max %.2f" % (ln, r["prove_ms"], r["prove_ms_min"], r["prove_ms_max"]), flush=True)
PY
done
