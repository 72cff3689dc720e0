#!/bin/bash
# per-pass kernel durations at steady clocks (200 warm-up steps), 2^24 x 2 and 2^20 x 32
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for cfg in "24 2" "20 32"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/ks$1 -o ks -- python bench.py --log-n $1 --batch $2 --no-extra --no-cpu --no-traffic > gpurun_out/r05/ks$1.json 2> gpurun_out/r05/ks$1.err || exit 1
  f=$(find gpurun_out/r05/ks$1 -name "*.db" | head -1)
  echo "== 2^$1 x $2: $(python -c "import json;print(json.load(open('gpurun_out/r05/ks$1.json'))['ms_per_step'])") ms per step"
  python scripts/kstats.py "$f" 8
done | tee gpurun_out/r05/ntt_kstats_steady.txt
