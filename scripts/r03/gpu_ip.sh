#!/bin/bash
# Round 3: the in-place / persistent NTT schedule (ntt_ip.hpp): parity, then A/B timing.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ntt_gpu.py \
  > gpurun_out/r03/pytest_ip.log 2>&1 || { tail -40 gpurun_out/r03/pytest_ip.log; exit 1; }
tail -3 gpurun_out/r03/pytest_ip.log
b() {  # label log_n batch env...
  local label=$1 ln=$2 bt=$3; shift 3
  out=$(env "$@" timeout -k 10 120 python bench.py --log-n $ln --batch $bt --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-28s 2^$ln x $bt: %.4f ms  frac %.4f'%('$label',d['ms_per_step'],d['roofline']['frac']))"
}
b "r03 ip" 24 2 PBF_X=0 || exit 1
b "r02 (PBF_NTT_V2)" 24 2 PBF_NTT_V2=1 || exit 1
b "r03 ip" 20 32 PBF_X=0 || exit 1
b "r02 (PBF_NTT_V2)" 20 32 PBF_NTT_V2=1 || exit 1
b "r03 ip no XCD" 24 2 PBF_NTT_NO_XCD=1 || exit 1
b "r03 ip no XCD" 20 32 PBF_NTT_NO_XCD=1 || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ip24 -o k -- python bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ip20 -o k -- python bench.py --log-n 20 --batch 32 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null || exit 1
find gpurun_out/r03/ip24 gpurun_out/r03/ip20 -name "*kernel_stats.csv" | head
