#!/bin/bash
# Round 6: gather A/B, sparse probe, and the tests touched since the last suite run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6c}
mkdir -p $O
timeout -k 10 300 python -u tools/ab_compact.py plain > $O/ab_gather.txt 2>&1 || { tail -20 $O/ab_gather.txt; exit 1; }
grep -v amdgpu $O/ab_gather.txt
timeout -k 10 300 python -u tools/probe_sparse.py 3 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu $O/probe.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact_aligned.py tests/test_reduce_order.py tests/test_gpu_bench.py \
    tests/test_gpu_kernels.py tests/test_gpu_context.py tests/test_gpu_multi.py tests/test_framelist.py \
    -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
exit $rc
