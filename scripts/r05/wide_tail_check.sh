set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -k "wide_tail_forms or heavy_buckets" -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/wide_tail_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/r05/wide_tail_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
for i in 1 2; do for V in 0 1; do echo "seq32=$V $(PBF_MSM_CD_SEQ32=$V timeout -k 10 200 python scripts/probe_msm_fixed.py 24 9 2>/dev/null | tr '\n' ' ')"; done; done
