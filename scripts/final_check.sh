#!/bin/bash
# End-of-round check of the committed tree: the whole GPU suite, smoke(), and the driver's
# default bench line with its kernel-trace + SQ counter profile (scripts/profile_final.sh)
set -o pipefail
TAG=${1:-r02d}
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash scripts/profile_final.sh $TAG
