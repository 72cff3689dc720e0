#!/bin/bash
# Round 3: PMC of the default NTT plans (2^24 x 2 regrouped, 2^20 x 32): SQ counters, then
# FETCH_SIZE and WRITE_SIZE, each in a pass of its own; and the FETCH/WRITE calibration on
# tile_copy (known bytes) for the 64-B and 128-B run lengths of those plans.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/pmc2; mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
for sz in "24 2" "20 32"; do
  set -- $sz
  B="python bench.py --log-n $1 --batch $2 --steps 6 --warmup 1 --no-cpu --no-extra --no-traffic"
  i=0
  for ctr in "$SQ" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/n$1_$i -o c -- $B > /dev/null 2>&1 || { echo "pmc pass $1 $i failed"; exit 1; }
  done
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/cal_$ctr -o c -- scripts/ubench/tile_copy > $O/cal_$ctr.log 2>&1 || { echo "cal pass $ctr failed"; exit 1; }
done
python3 scripts/pmc_groups.py $O/cal_FETCH_SIZE $((256*1024*1024)) > $O/cal_fetch.txt
python3 scripts/pmc_groups.py $O/cal_WRITE_SIZE $((256*1024*1024)) > $O/cal_write.txt
head -40 $O/cal_FETCH_SIZE.log
echo pmc done
