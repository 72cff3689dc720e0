#!/bin/bash
# SQ counters of the fixed-base MSM kernels at 2^20 (c = 16) and 2^24 (c = 22) points
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04q
cd /tmp && export TMPDIR=/tmp
for ln in 20 24; do
  rm -rf $R/gpurun_out/r04q/p$ln $R/gpurun_out/r04q/t$ln
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r04q/p$ln -o p -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $R/gpurun_out/r04q/pm$ln.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04q/t$ln -o t -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $R/gpurun_out/r04q/tm$ln.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for ln in ("20", "24"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/r04q/p{ln}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "chunk_acc" not in r["Kernel_Name"]:
                continue
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    for f in glob.glob(f"gpurun_out/r04q/t{ln}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Name"]] = float(r["AverageNs"])
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = next((v for n, v in dur.items() if n.startswith(k[:60])), 0.0)
        valu = m["SQ_INSTS_VALU"]
        # VALU issue ceiling: one 4-cycle wave-instruction per SIMD, 1024 SIMDs, 2.4 GHz
        util = valu * 4 / (d * 1e-9 * 2.4e9 * 1024) if d else 0
        print(f"2^{ln} {k[:70]}")
        print("   waves %.0f  VALU/wave %.0f  SALU/wave %.0f  avg duration %.1f us  VALU issue share of 4-cycle ceiling %.2f" % (
            m["SQ_WAVES"], valu / m["SQ_WAVES"], m.get("SQ_INSTS_SALU", 0) / m["SQ_WAVES"], d / 1e3, util))
PY
