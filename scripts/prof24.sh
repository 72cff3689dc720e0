#!/bin/bash
# 2^24 x 2 NTT: per-pass kernel durations (rocprofv3 kernel trace) of the full and the
# no-math (data movement only) builds, plus env-knob timings. Output under gpurun_out/p24.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p24
B="python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic"
for cfg in "X=0" "PBF_NTT_TILE=8192"; do
  out=$(env $cfg timeout -k 10 120 $B 2>/dev/null) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-60s %.4f ms'%('$cfg',d['ms_per_step']))"
done
for v in full; do
  lib=plonk-by-fingers_amd/libpbf.so; [ $v = nomath ] && lib=plonk-by-fingers_amd/libpbf_nomath.so
  PBF_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/p24/$v -o run -- python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic > gpurun_out/p24/$v.log 2>&1 || exit 1
  f=gpurun_out/p24/$v/run_results.db
  echo "== $v"; python scripts/pass_split.py "$f" 3
done
