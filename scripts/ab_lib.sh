set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py tests/test_poly_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ntt.log 2>&1; rc=$?; tail -3 gpurun_out/t_ntt.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
bash scripts/quick_ab.sh "PBF_LIB=plonk-by-fingers_amd/libpbf_base.so" "X=1" || exit 1
done
