#!/bin/bash
# Round 3: FETCH_SIZE / WRITE_SIZE calibration on the tile-copy microbenchmark (known bytes:
# every launch reads and writes 256 MiB; the last 2^20 launches 128 MiB), one counter per
# pass. Covers 64-B runs (W=8) and 128-B runs (W=16), the two run lengths of the NTT plans.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03/cal
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/r03/cal/$ctr -o c -- scripts/ubench/tile_copy > gpurun_out/r03/cal/$ctr.log 2>&1 || { echo "cal pass $ctr failed"; exit 1; }
done
python3 scripts/pmc_groups.py gpurun_out/r03/cal $((256*1024*1024)) > gpurun_out/r03/cal/summary.txt
echo cal done
