#!/bin/bash
# host enqueue time against the GPU interval per step, cold start, default schedule and one stream
set -o pipefail
mkdir -p gpurun_out/r06
L=gpurun_out/r06/host_enqueue.log
: > $L
for o in "" "ntt.streams=1" ""; do
  RAMP_OPTS="$o" timeout -k 10 120 python3 scripts/r06/host_enqueue.py 20 32 200 >> $L || exit 1
done
RAMP_OPTS="" timeout -k 10 120 python3 scripts/r06/host_enqueue.py 24 2 200 >> $L || exit 1
cat $L
