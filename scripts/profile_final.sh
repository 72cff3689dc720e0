#!/bin/bash
# End-of-round evidence: the driver's default bench line (JSON), a rocprofv3 kernel-trace
# summary of the bench workload and an SQ counter pass (VALU / LDS instructions per wave),
# each GPU step under its own time limit. Usage: scripts/profile_final.sh TAG
set -o pipefail
TAG=${1:-r02b}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
echo bench done
CMD="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $CMD > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
echo trace done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o sq -- $CMD > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
echo sq done
CMD24="python3 $R/bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o sq24 -- $CMD24 > $OUT/sq24.log 2>&1 || { tail -5 $OUT/sq24.log; exit 1; }
echo profiled
