#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel-trace summary + PMC traffic passes
# (FETCH_SIZE and WRITE_SIZE each in their own run, per MI355X_MICROARCH.md), written
# under gpurun_out/prof_rXX and summarised into profiles/rXX/. Usage: scripts/profile_round.sh r01
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $CMD > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch -- $CMD > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write -- $CMD > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o sq -- $CMD > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
# calibration: tile_copy moves a known 256 MiB per kernel in the NTT's access patterns
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o calib_fetch -- $R/scripts/ubench/tile_copy > $OUT/calib_fetch.log 2>&1 || { tail -5 $OUT/calib_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o calib_write -- $R/scripts/ubench/tile_copy > $OUT/calib_write.log 2>&1 || { tail -5 $OUT/calib_write.log; exit 1; }
echo profiled
