#!/bin/bash
# Round 6: selected GPU tests (-k expression $1), log under gpurun_out/$2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${2:-r6t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "$1" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
grep -E "FAILED|ERROR|Error" $O/tests.log | head -20
exit $rc
