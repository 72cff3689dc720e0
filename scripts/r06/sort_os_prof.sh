#!/bin/bash
# kernel statistics of the one-sweep sort benchmark (scripts/ubench/sort_os_bench.hip)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r06/sortprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06/sortprof -o s -- $R/scripts/ubench/sort_os_bench ${1:-3} > $R/gpurun_out/r06/sort_os_prof.log 2>&1 || exit 1
cd $R
grep -v "^E2\|^W2" gpurun_out/r06/sort_os_prof.log | grep -v rocprofv3 | tail -4
f=$(find gpurun_out/r06/sortprof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print("%-70s calls %5s  avg %10.1f us  total %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
