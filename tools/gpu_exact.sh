#!/bin/bash
# exact=True (RMSF.py:120-146 bit for bit): kernel timing tool, the exact
# tests and the full-size unaligned tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/exact
mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u tools/seq_welford.py > $O/seq.txt 2>&1 || { tail -20 $O/seq.txt; exit 1; }
grep -v amdgpu.ids $O/seq.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py "tests/test_gpu_fullsize.py::test_full_size_unaligned" -v -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.txt | cut -c1-140 | tail -30
