#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6sp}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact_aligned.py -k "compacted" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 \
    || { grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probe_sparse.py 3 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu $O/probe.txt
