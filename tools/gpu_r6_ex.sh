#!/bin/bash
# Round 6: exact aligned tests, then the exact-aligned cost probe with this build and tools/_ab/librmsf_$1.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${2:-r6ex}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_aligned.py tests/test_gpu_exact.py tests/test_reduce_order.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 \
    || { grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/probe_exact_aligned.py 2 > $O/cur.txt 2>&1 || { tail -5 $O/cur.txt; exit 1; }
grep -v amdgpu $O/cur.txt
if [ -n "$1" ] && [ "$1" != "-" ]; then
  RMSF_AB_LIB=tools/_ab/librmsf_$1.so timeout -k 10 600 python -u tools/probe_exact_aligned.py 1 > $O/$1.txt 2>&1 || { tail -5 $O/$1.txt; exit 1; }
  grep -v amdgpu $O/$1.txt
fi
