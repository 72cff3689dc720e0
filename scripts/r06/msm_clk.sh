#!/bin/bash
# Round 6: is the 2^24-point accumulation's lower issue share (0.75 against 0.83 at 2^20) the clock
# or stalls? GRBM_GUI_ACTIVE (GPU clock cycles while busy) over the kernel's duration gives the
# clock; SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES the share of wave time waiting on a dependency
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/mclk
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ln in 20 24; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p$ln -o p -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $O/pm$ln.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$ln -o t -- python3 $R/scripts/probe_msm_fixed.py $ln 3 > $O/tm$ln.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY' | tee gpurun_out/r06/msm_acc_clock.txt
import csv, glob
from collections import defaultdict
print("# scripts/r06/msm_clk.sh: the fixed-base accumulation (msm_chunk_acc_l29r) at 2^20 and 2^24 points")
for ln in ("20", "24"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/r06/mclk/p{ln}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "chunk_acc_l29r" not in r["Kernel_Name"]:
                continue
            acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = 0.0
    for f in glob.glob(f"gpurun_out/r06/mclk/t{ln}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "chunk_acc_l29r" in r["Name"]:
                dur = float(r["AverageNs"])
    ds = list(acc.values())
    m = {c: sum(sum(d[c]) for d in ds) / len(ds) for c in ds[0]}
    print(f"2^{ln}: dispatches {len(ds)}, avg duration {dur/1e3:.1f} us (kernel trace run)")
    print("   GRBM_GUI_ACTIVE %.4g  GRBM_COUNT %.4g  -> clock %.2f GHz over the traced duration" % (
        m["GRBM_GUI_ACTIVE"], m["GRBM_COUNT"], m["GRBM_GUI_ACTIVE"] / dur if dur else 0))
    print("   VALU/wave %.0f  wait_any/wave_cycles %.3f  active_valu/wave_cycles %.3f  busy %.4g" % (
        m["SQ_INSTS_VALU"] / m["SQ_WAVES"], m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"],
        m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"], m["SQ_BUSY_CYCLES"]))
PY
