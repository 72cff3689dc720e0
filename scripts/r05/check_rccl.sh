#!/bin/bash
# Round 5: the RCCL branch through the stand-in librccl, the interleaved-mode sharded key test,
# then a quick bench line in the compacted form.
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_rccl_branch_gpu.py "tests/test_multi_capi_gpu.py::test_prove_multi_modes_interleaved_on_one_key" \
  tests/test_multi_capi_gpu.py::test_multi_errors > gpurun_out/r05/pytest_rccl.log 2>&1; rc=$?
tail -25 gpurun_out/r05/pytest_rccl.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-traffic --no-extra > gpurun_out/r05/bench_quick.json 2> gpurun_out/r05/bench_quick.err || { tail -20 gpurun_out/r05/bench_quick.err; exit 1; }
cat gpurun_out/r05/bench_quick.json
