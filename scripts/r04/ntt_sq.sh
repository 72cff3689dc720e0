#!/bin/bash
# SQ counters of the NTT pass kernels (2^20 x 32 and 2^24 x 2): VALU instructions per element
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04s
cd /tmp && export TMPDIR=/tmp
for cfg in "20 32" "24 2"; do
  set -- $cfg
  rm -rf $R/gpurun_out/r04s/p$1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r04s/p$1 -o p -- python3 $R/bench.py --log-n $1 --batch $2 --steps 5 --warmup 2 --no-cpu --no-extra --no-traffic > $R/gpurun_out/r04s/b$1.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for ln in ("20", "24"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/r04s/p{ln}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gl_" not in r["Kernel_Name"]:
                continue
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        w = m.get("SQ_WAVES", 1)
        print(f"2^{ln}", k[:90])
        print("   dispatches %d  waves %.0f  VALU/wave %.0f  VALU per element %.1f  SALU per element %.1f  LDS per element %.2f" % (
            len(cs.get("SQ_WAVES", [])), w, m["SQ_INSTS_VALU"] / w, m["SQ_INSTS_VALU"] / w / 16,
            m.get("SQ_INSTS_SALU", 0) / w / 16, m.get("SQ_INSTS_LDS", 0) / w / 16))
PY
