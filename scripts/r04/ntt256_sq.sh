#!/bin/bash
# SQ counters of the BN254-Fr NTT pass kernels in the config-3 product (NTT size 2^23: passes of
# radix 2^8, 2^8, 2^7): VALU / LDS / VMEM instructions per element and the VALU issue share.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rm -rf $O/p $O/t
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $O/p -o p -- python3 $R/scripts/run_polymul.py 5 > $O/pm.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o t -- python3 $R/scripts/run_polymul.py 5 > $O/tm.log 2>&1 || exit 1
cd $R
python3 - <<'PY' | tee gpurun_out/r04n/summary.txt
import csv, glob
from collections import defaultdict
O = "gpurun_out/r04n"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{O}/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ntt256" not in r["Kernel_Name"] and "pointwise" not in r["Kernel_Name"]:
            continue
        acc[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in glob.glob(f"{O}/t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        gs = int(r.get("Grid_Size", 0) or 0) or int(r.get("Grid_Size_X", 0) or 0)
        dur[(r["Kernel_Name"], gs)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (k, gs), cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    ds = sorted(dur.get((k, gs), [0]))
    d = ds[len(ds) // 2]
    elems = gs * 4 if "ntt256" in k else gs  # 4 elements per pass-kernel thread
    valu = m["SQ_INSTS_VALU"]
    util = valu * 4 / (d * 1e-9 * 2.4e9 * 1024) if d else 0
    print(k[:70], "grid", gs)
    print("   waves %.0f  median %.1f us (%d calls)  per element: VALU %.1f  SALU %.1f  LDS %.2f  VMEM rd %.2f  wr %.2f"
          "  (elements %d)  VALU issue share of the 4-cycle ceiling %.2f" % (
              m["SQ_WAVES"], d / 1e3, len(ds), valu / elems, m["SQ_INSTS_SALU"] / elems, m["SQ_INSTS_LDS"] / elems,
              m["SQ_INSTS_VMEM_RD"] / elems, m["SQ_INSTS_VMEM_WR"] / elems, elems, util))
PY
