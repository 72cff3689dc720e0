#!/bin/bash
# Round 3: A/B of the in-place NTT schedule variants (persistent + prefetch with the entry
# stores, without them, one tile per workgroup) against the round-2 kernels, with per-pass
# kernel times.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ntt_gpu.py \
  > gpurun_out/r03/pytest_ip2.log 2>&1 || { tail -40 gpurun_out/r03/pytest_ip2.log; exit 1; }
tail -1 gpurun_out/r03/pytest_ip2.log
b() {  # label log_n batch env...
  local label=$1 ln=$2 bt=$3; shift 3
  out=$(env "$@" timeout -k 10 120 python bench.py --log-n $ln --batch $bt --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-28s 2^$ln x $bt: %.4f ms  frac %.4f'%('$label',d['ms_per_step'],d['roofline']['frac']))"
}
for sz in "24 2" "20 32"; do
  b "ip persistent+prime" $sz PBF_X=0 || exit 1
  b "ip persistent noprime" $sz PBF_NTT_IP_NOPRIME=1 || exit 1
  b "ip one tile/WG" $sz PBF_NTT_IP_GRID=0 || exit 1
  b "r02 (PBF_NTT_V2)" $sz PBF_NTT_V2=1 || exit 1
done
export TMPDIR=/tmp
for v in "def PBF_X=0" "grid0 PBF_NTT_IP_GRID=0"; do
  set -- $v
  for sz in "24 2" "20 32"; do
    set -- $v
    name=$1; shift
    s1=${sz% *}; s2=${sz#* }
    env "$@" timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r03/p_${name}_$s1 -o k -- python bench.py --log-n $s1 --batch $s2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
  done
done
echo done
