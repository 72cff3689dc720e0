#!/bin/bash
# Round 3: MSM quad-lane tail + two-ahead index prefetch -- parity (MSM tests), timing A/B
# against the single-lane tail, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03/msmq; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python -u scripts/r03/msm_time.py > $O/msm_time.log 2>&1 || { tail $O/msm_time.log; exit 1; }
grep -v amdgpu.ids $O/msm_time.log
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof -o k -- python scripts/r03/msm_time.py > /dev/null 2>&1 || exit 1
echo done
# NTT: wavefront-shuffle stage-C twiddle broadcast (libpbf_shfltw.so) against the default
L=plonk-by-fingers_amd
PBF_LIB=$L/libpbf_shfltw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ntt_gpu.py -k "golden or kat or oracle" > $O/pytest_shfl.log 2>&1 || { tail -30 $O/pytest_shfl.log; exit 1; }
tail -1 $O/pytest_shfl.log
for rep in 1 2; do
for lib in libpbf.so libpbf_shfltw.so; do
  for sz in "24 2" "20 32"; do
    set -- $sz
    out=$(PBF_LIB=$L/$lib timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
    echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-18s 2^$1 x $2: %.4f ms  frac %.4f'%('$lib',d['ms_per_step'],d['roofline']['frac']))"
  done
done
done
