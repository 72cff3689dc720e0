#!/bin/bash
# Round 3: regrouped 2^24 NTT plan -- parity (NTT GPU tests incl. the RG-vs-round-2 test),
# timing A/B against PBF_NTT_NO_RG=1, per-pass kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/rg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ntt_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for env in "PBF_X=0" "PBF_NTT_NO_RG=1"; do
  out=$(env $env timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-18s 2^24 x 2: %.4f ms  frac %.4f'%('$env',d['ms_per_step'],d['roofline']['frac']))"
done
done
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof -o k -- python bench.py --log-n 24 --batch 2 --steps 10 --warmup 2 --no-cpu --no-extra --no-traffic > /dev/null 2>&1 || exit 1
echo done
