#!/bin/bash
# Per-kernel stats of the fixed-base MSM per window width: msm_window_prof.sh LOG_N C [C ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
ln=$1; shift
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  rm -rf $R/gpurun_out/r04w/prof_c$c
  PBF_MSM_FX_C=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04w/prof_c$c -o p -- python3 $R/scripts/probe_msm_fixed.py $ln 5 > $R/gpurun_out/r04w/probe_c$c.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/r04w/prof_c$c -name "*kernel_stats.csv" | head -1)
  echo "== c=$c $(grep -v amdgpu.ids $R/gpurun_out/r04w/probe_c$c.log | tr '\n' ' ')"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:22]: print('%-60s %5s %10.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
