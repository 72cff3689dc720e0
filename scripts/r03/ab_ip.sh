#!/bin/bash
# Round 3: timing A/B of the default 2^24 / 2^20 NTT schedule against the in-place
# (digit-slot) schedule and its variants.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
b() {  # label log_n batch env...
  local label=$1 ln=$2 bt=$3; shift 3
  out=$(env "$@" timeout -k 10 120 python bench.py --log-n $ln --batch $bt --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-28s 2^$ln x $bt: %.4f ms  frac %.4f'%('$label',d['ms_per_step'],d['roofline']['frac']))"
}
for sz in "24 2" "20 32"; do
  b "default" $sz PBF_X=0 || exit 1
  b "ip" $sz PBF_NTT_IP=1 || exit 1
  b "ip one tile/WG" $sz PBF_NTT_IP=1 PBF_NTT_IP_GRID=0 || exit 1
  b "ip 8,8,8" $sz PBF_NTT_IP=1 PBF_NTT_IP_PASSES=8,8,8 || exit 1
done
