#!/bin/bash
# Round 6: the headline's schedule options in the driver's window (steps 5-25 after an idle GPU)
# and at steady clocks: cold-start per-step times, twice each
set -o pipefail
mkdir -p gpurun_out/r06
for i in 1 2; do
  for o in "" "ntt.group=8" "ntt.streams=1" "ntt.group=0" "ntt.group=2" "ntt.streams=3" "ntt.group=8,ntt.streams=4"; do
    RAMP_OPTS="$o" timeout -k 10 120 python scripts/r06/ramp.py 20 32 300 2 || exit 1
  done
done > gpurun_out/r06/ramp_sched.log
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r06/ramp_sched.log") if l.startswith("{")]
for r in rows:
    print(f"{str(r['opts']):40s} steps5-25 {r['mean_5_25']:.4f}  25-50 {r['mean_25_50']:.4f}  200-300 {r['mean_200_300']:.4f}")
PY
