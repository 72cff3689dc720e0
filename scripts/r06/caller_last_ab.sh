#!/bin/bash
# Round 6: the last group of a batched NTT on the caller's stream (option ntt.caller_last) against
# the default (group 0 on the caller's stream), cold start: driver window and steady clocks
set -o pipefail
mkdir -p gpurun_out/r06
for i in 1 2 3; do
  for o in "" "ntt.caller_last=1"; do
    RAMP_OPTS="$o" timeout -k 10 120 python scripts/r06/ramp.py 20 32 300 2 || exit 1
  done
done > gpurun_out/r06/caller_last_ab.log
python3 - <<'PY'
import json
for l in open("gpurun_out/r06/caller_last_ab.log"):
    if l.startswith("{"):
        r = json.loads(l)
        print(f"{str(r['opts']):30s} steps5-25 {r['mean_5_25']:.4f}  25-50 {r['mean_25_50']:.4f}  200-300 {r['mean_200_300']:.4f}")
PY
