#!/bin/bash
# Round 3: PMC A/B of the 2^24 x 2 NTT passes, round-2 kernels (PBF_NTT_V2=1) against the
# in-place schedule: SQ counters (one pass), FETCH_SIZE, WRITE_SIZE (separate passes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03/pmc
B="python bench.py --log-n ${LOGN:-24} --batch ${BATCH:-2} --steps 6 --warmup 1 --no-cpu --no-extra --no-traffic"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in "v2 PBF_NTT_V2=1" "ip PBF_NTT_IP=1"; do
  set -- $v; name=$1; shift
  i=0
  for ctr in "$SQ" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    env "$@" timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/r03/pmc/${name}_$i -o c -- $B > /dev/null 2>&1 || { echo "pmc pass $name $i failed"; exit 1; }
  done
done
echo pmc done
