set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv/prof -o run -- python scripts/bench_prover.py 20 > gpurun_out/pv/bp.log 2>&1 || exit 1
python scripts/kstats.py gpurun_out/pv/prof/run_results.db 30 > gpurun_out/pv/kstats.txt
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
