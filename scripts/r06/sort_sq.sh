#!/bin/bash
# SQ counters of the three-kernel sort passes (scripts/ubench/sort_os_bench: both sorts of 3 cases)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/ssq
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p -o p -- $R/scripts/ubench/sort_os_bench 1 > $O/pm.log 2>&1 || exit 1
cd $R
python3 - <<'PY' | tee gpurun_out/r06/sort_sq_counters.txt
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/r06/ssq/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rs_" not in r["Kernel_Name"]:
            continue
        acc[(r["Kernel_Name"][:60], r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = defaultdict(lambda: defaultdict(list))
for (k, d), cs in acc.items():
    for c, v in cs.items():
        per[k][c].append(sum(v))
print("# per dispatch averages over both sorts' dispatches of the benchmark's 3 cases")
for k, cs in sorted(per.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print("%-60s VALU/wave %.0f LDS/wave %.0f bank_conflict/LDS_active %.3f wait_any/wave_cycles %.3f" % (
        k, m["SQ_INSTS_VALU"] / m["SQ_WAVES"], m["SQ_INSTS_LDS"] / m["SQ_WAVES"],
        m["SQ_LDS_BANK_CONFLICT"] / max(1, m["SQ_ACTIVE_INST_LDS"]), m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]))
PY
