#!/bin/bash
# SQ counters of the two-pass 2^24 kernels (PBF_NTT_R4K=1) and the default three-pass plan
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05/sq
cd /tmp && export TMPDIR=/tmp
for V in 0 1; do
  if [ $V != 0 ]; then export PBF_NTT_R4K=$V; else unset PBF_NTT_R4K; fi
  rm -rf $R/gpurun_out/r05/sq/a$V $R/gpurun_out/r05/sq/b$V
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/r05/sq/a$V -o p -- python3 $R/bench.py --log-n 24 --batch 2 --steps 5 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r05/sq/b$V -o p -- python3 $R/bench.py --log-n 24 --batch 2 --steps 5 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
done
cd $R
for V in 0 1; do for P in a b; do echo "== $V $P"; python3 scripts/sq_summary.py gpurun_out/r05/sq/$P$V 2>&1 | grep -v fill_random | grep -v rocclr; done; done
