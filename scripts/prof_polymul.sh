#!/bin/bash
# Config 3 (BN254-Fr mul_ntt 2^22 x 2^22): kernel trace + one SQ counter pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pm; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 scripts/run_polymul.py 5 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 scripts/kstats.py $OUT/trace/run_results.db 12
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT -o sq -- python3 scripts/run_polymul.py 3 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/pm/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    print(k[:70], " ".join(f"{c}={v:.3g}" for c, v in sorted(m.items())))
    print("   VALU/wave=%.0f  active_valu/wave_cycles=%.3f  busy=%.3g" % (m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_ACTIVE_INST_VALU", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1), m.get("SQ_BUSY_CYCLES", 0)))
PY
