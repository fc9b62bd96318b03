cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_xtc.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r2p_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2p_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 ./tools/stride_probe > gpurun_out/r2p_stride.txt 2>&1; rc=$?; cat gpurun_out/r2p_stride.txt; exit $rc
