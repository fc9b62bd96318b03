#!/bin/bash
# SoA inputs: the GPU tests, then HBM planes read in place / gathered vs rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_soa.py tests/test_gpu_multirank.py -x -v --timeout 250 --timeout-method thread > gpurun_out/soa2_tests.log 2>&1
rc=$?; tail -4 gpurun_out/soa2_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_device_soa.py > gpurun_out/device_soa2.txt 2>&1
rc=$?; cat gpurun_out/device_soa2.txt; exit $rc
