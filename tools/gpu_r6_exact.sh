#!/bin/bash
# Round 6, first GPU pass: the exact aligned path (tests/test_gpu_exact_aligned.py),
# the existing exact / reference-vector suites, smoke(), then the few-frame sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_aligned.py tests/test_gpu_exact.py tests/test_reference_vectors.py \
    tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -E "literal shape|100k x 256" $O/tests.log || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u tools/fuzz_fewframes.py ${1:-50} > $O/fuzz_fewframes.txt 2>&1 || { tail -20 $O/fuzz_fewframes.txt; exit 1; }
cat $O/fuzz_fewframes.txt
