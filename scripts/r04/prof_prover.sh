#!/bin/bash
# Kernel stats of K proofs at 2^LOG_N gates: prof_prover.sh LOG_N K
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04p
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r04p/p$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04p/p$1 -o p -- python3 $R/scripts/r04/prove_only.py $1 $2 > $R/gpurun_out/r04p/prove$1.log 2>&1 || exit 1
f=$(find $R/gpurun_out/r04p/p$1 -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms', tot/1e6)
for r in rows[:40]: print('%-80s %6s %10.1f %9.2f %6.2f' % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6, float(r['Percentage'])))
"
