#!/bin/bash
# SQ counters and kernel durations of the Fr pass kernels, 29-bit and 32-bit forms (config 3)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/frsq
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for f in 29 32; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/p$f -o p -- python3 $R/scripts/r06/fr29_probe.py $f 3 > $O/pm$f.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$f -o t -- python3 $R/scripts/r06/fr29_probe.py $f 5 > $O/tm$f.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY' | tee gpurun_out/r06/fr29_sq_counters.txt
import csv, glob
from collections import defaultdict
print("# scripts/r06/fr29_sq.sh: Fr pass kernels of config 3 (fused mul_ntt, 2^23 points: 3 passes of")
print("# radix 2^8, 2^8, 2^7 per transform), 29-bit (ntt256l_pass_kernel) and 32-bit forms. Per element and")
print("# pass: VALU = SQ_INSTS_VALU x 64 / elements; issue share = VALU x 4 cycles / (duration x 2.4 GHz x 1024).")
for f in ("29", "32"):
    acc = defaultdict(lambda: defaultdict(list))
    for fn in glob.glob(f"gpurun_out/r06/frsq/p{f}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "ntt256" not in r["Kernel_Name"]:
                continue
            acc[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = defaultdict(lambda: defaultdict(list))
    for (k, d), cs in acc.items():
        for c, v in cs.items():
            per[k][c].append(sum(v))
    dur = {}
    for fn in glob.glob(f"gpurun_out/r06/frsq/t{f}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            dur[r["Name"]] = float(r["AverageNs"])
    for k, cs in sorted(per.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = next((v for nm, v in dur.items() if nm.startswith(k[:50])), 0.0)
        elems = (1 << 23) * 2 if "9ELi4" not in k else 0
        valu = m["SQ_INSTS_VALU"]
        print(f"{f}-bit {k[:64]}")
        print("   VALU %.3g  LDS %.3g  SALU %.3g  VMEM %.3g per dispatch; waves %.0f; VALU/wave %.0f; wait_any/busy %.2f; avg %.1f us; issue share %.2f" % (
            valu, m["SQ_INSTS_LDS"], m["SQ_INSTS_SALU"], m["SQ_INSTS_VMEM"], m["SQ_WAVES"], valu / m["SQ_WAVES"],
            m["SQ_WAIT_INST_ANY"] / max(1.0, m["SQ_WAVE_CYCLES"]), d / 1e3, valu * 4 / (d * 1e-9 * 2.4e9 * 1024) if d else 0))
PY
