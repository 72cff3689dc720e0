#!/bin/bash
# Round 3: SQ counters of the MSM kernels (accumulation occupancy / VALU share / waits) and
# FETCH_SIZE of the accumulation, separate passes over a short MSM run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/pmcmsm; mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"
i=0
for ctr in "$SQ" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/p$i -o c -- python scripts/r03/msm_pmc.py > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail $O/p$i.log; exit 1; }
done
echo pmc done
