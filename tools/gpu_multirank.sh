cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 180 --timeout-method thread > gpurun_out/mr_tests.log 2>&1
rc=$?; tail -15 gpurun_out/mr_tests.log; exit $rc
