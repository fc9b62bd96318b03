#!/bin/bash
# Context ABI (callback / in-process / plain-C host) and one-process
# multi-device GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ctx}
timeout -k 10 600 python -u -m pytest tests/test_gpu_context.py tests/test_gpu_multi.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -6 gpurun_out/${TAG}_tests.log; exit $rc
