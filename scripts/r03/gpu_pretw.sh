#!/bin/bash
# Round 3: two-pass plans with the second pass's twiddle applied at the first pass's stores
# (PBF_NTT_PRETW=1) -- NTT parity under the option, then 2^20 x 32 timing A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/pretw; mkdir -p $O
PBF_NTT_PRETW=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for env in "PBF_X=0" "PBF_NTT_PRETW=1"; do
  for sz in "20 32" "22 8"; do
    set -- $sz
    out=$(env $env timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
    echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-16s 2^$1 x $2: %.4f ms  frac %.4f'%('$env',d['ms_per_step'],d['roofline']['frac']))"
  done
done
done
