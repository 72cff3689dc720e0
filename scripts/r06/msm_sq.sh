#!/bin/bash
# Round 6: SQ counters of the fixed-base MSM accumulation (msm_chunk_acc_l29r) at 2^20 and 2^24
# points on the final kernel: VALU per mixed addition = SQ_INSTS_VALU x 64
# lanes / (entries); one counter pass plus a kernel-trace pass for the durations
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06/msq
cd /tmp && export TMPDIR=/tmp
for ln in 20 24; do
  rm -rf $R/gpurun_out/r06/msq/p$ln $R/gpurun_out/r06/msq/t$ln
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r06/msq/p$ln -o p -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $R/gpurun_out/r06/msq/pm$ln.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06/msq/t$ln -o t -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $R/gpurun_out/r06/msq/tm$ln.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY' | tee gpurun_out/r06/msm_acc_sq_counters.txt
import csv, glob
from collections import defaultdict
print("# scripts/r06/msm_sq.sh: SQ counters of the fixed-base MSM accumulation, round-6 kernel (Y3 under one")
print("# reduction, P / R differences inside their products' reductions). Per addition = per sorted entry:")
print("# MSM_CH = 43 entries per lane, so VALU per addition = SQ_INSTS_VALU / SQ_WAVES / 43 (wave-instructions of")
print("# 64 lanes each, one entry per lane). 'issue share' = VALU x 4 cycles / (duration x 2.4 GHz x 1024 SIMDs).")
for ln in ("20", "24"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/r06/msq/p{ln}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "chunk_acc" not in r["Kernel_Name"]:
                continue
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    for f in glob.glob(f"gpurun_out/r06/msq/t{ln}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Name"]] = float(r["AverageNs"])
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = next((v for n, v in dur.items() if n.startswith(k[:60])), 0.0)
        valu = m["SQ_INSTS_VALU"]
        util = valu * 4 / (d * 1e-9 * 2.4e9 * 1024) if d else 0
        print(f"2^{ln} {k[:70]}")
        print("   waves %.0f  VALU/wave %.0f (%.0f per addition)  SALU/wave %.0f  avg duration %.1f us  VALU issue share %.2f" % (
            m["SQ_WAVES"], valu / m["SQ_WAVES"], valu / m["SQ_WAVES"] / 43, m.get("SQ_INSTS_SALU", 0) / m["SQ_WAVES"], d / 1e3, util))
PY
