#!/bin/bash
# rocprofv3 kernel trace + one SQ counter pass of the 2^20 x 32 NTT bench (args: tag [log_n batch])
set -o pipefail
TAG=${1:-x}; LOGN=${2:-20}; B=${3:-32}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-extra --log-n $LOGN --batch $B"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $CMD > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d $OUT -o sq -- $CMD > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
cd $R
python3 scripts/sq_summary.py $OUT
