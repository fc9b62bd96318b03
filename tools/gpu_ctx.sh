#!/bin/bash
# GPU session: context-ABI tests first (new code), then the rest of the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ctx}
timeout -k 10 300 python -u -m pytest tests/test_gpu_context.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_ctx.log 2>&1
rc=$?; echo "ctx pytest rc=$rc"; tail -25 gpurun_out/${TAG}_ctx.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_all.log 2>&1
rc=$?; echo "all pytest rc=$rc"; tail -5 gpurun_out/${TAG}_all.log
exit $rc
