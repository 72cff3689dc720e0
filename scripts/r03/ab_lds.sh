#!/bin/bash
# Round 3: 2^24 / 2^20 NTT with the XOR-swizzled Y layout (32 KiB tiles, five workgroups per
# CU) against the padded layout (libpbf_pady.so) and the regrouped middle pass at four waves
# (libpbf_rg2w4.so); NTT parity on the default build first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/lds; mkdir -p $O
L=plonk-by-fingers_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for lib in libpbf.so libpbf_pady.so libpbf_rg2w4.so; do
  for sz in "24 2" "20 32"; do
    set -- $sz
    out=$(PBF_LIB=$L/$lib timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
    echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-18s 2^$1 x $2: %.4f ms  frac %.4f'%('$lib',d['ms_per_step'],d['roofline']['frac']))"
  done
done
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof -o k -- python bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
echo done
