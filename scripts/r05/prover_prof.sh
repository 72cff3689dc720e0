#!/bin/bash
# 2^24-gate proof: wall time (steady clocks after the warm-up proof) and per-kernel stats
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_prover.py 24 | tee gpurun_out/r05/prover24.json || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof24 -o p24 -- python scripts/bench_prover.py 24 > gpurun_out/r05/prof24.log 2>&1 || exit 1
f=$(find gpurun_out/r05/prof24 -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY' | tee gpurun_out/r05/prover24_kstats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print("%-80s %6s %10.1f %9.2f" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
