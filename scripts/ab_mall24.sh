#!/bin/bash
# 2^24 x 2 (and 2^20 x 32) with the full / data-only / compute-only builds, default schedule vs
# one polynomial per group (its 128 MiB intermediate can stay in the Infinity Cache).
set -o pipefail
L=plonk-by-fingers_amd
run() {  # label lib log_n batch env...
  local label=$1 lib=$2 ln=$3 b=$4; shift 4
  out=$(env PBF_LIB=$L/$lib "$@" timeout -k 10 120 python bench.py --log-n $ln --batch $b --steps 20 --warmup 3 --no-cpu --no-extra) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-34s 2^$ln x $b: %.4f ms  frac %.4f'%('$label',d['ms_per_step'],d['roofline']['frac']))"
}
for lib in libpbf.so libpbf_nomath.so libpbf_nomem.so; do
  run "$lib default" $lib 24 2 || exit 1
  run "$lib GROUP=1" $lib 24 2 PBF_NTT_GROUP=1 || exit 1
  run "$lib GROUP=1 STREAMS=1" $lib 24 2 PBF_NTT_GROUP=1 PBF_NTT_STREAMS=1 || exit 1
  run "$lib default" $lib 20 32 || exit 1
done
