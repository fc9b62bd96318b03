#!/bin/bash
# Round 6: the whole GPU suite (driver's form) and smoke(); the log under gpurun_out/$1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
grep -E "FAILED|ERROR" $O/tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
exit $rc
