#!/bin/bash
# Round 3: data-movement floor of the 2^24 x 2 plan with and without one-polynomial groups
# (intermediates Infinity-Cache resident), per pass (rocprof kernel trace).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
L=plonk-by-fingers_amd
run() {  # label lib env...
  local label=$1 lib=$2; shift 2
  out=$(env PBF_LIB=$L/$lib "$@" timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-34s 2^24 x 2: %.4f ms  frac %.4f'%('$label',d['ms_per_step'],d['roofline']['frac']))"
}
for lib in libpbf.so libpbf_nomath.so libpbf_nomem.so; do
  run "$lib default" $lib || exit 1
  run "$lib GROUP=1" $lib PBF_NTT_GROUP=1 || exit 1
  run "$lib GROUP=1 STREAMS=1" $lib PBF_NTT_GROUP=1 PBF_NTT_STREAMS=1 || exit 1
done
export TMPDIR=/tmp
for g in 2 1; do
  PBF_LIB=$L/libpbf_nomath.so PBF_NTT_GROUP=$g PBF_NTT_STREAMS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/nomath_g$g -o k -- python bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null || exit 1
done
