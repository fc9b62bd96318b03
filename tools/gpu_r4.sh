#!/bin/bash
# Round-4 GPU session: the given test files, then optional tools.  Each GPU
# step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r4}
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 280 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$TOOL" ]; then
  timeout -k 10 ${TOOL_LIMIT:-300} $TOOL > gpurun_out/${TAG}_tool.log 2>&1
  rc=$?; echo "tool rc=$rc"; tail -20 gpurun_out/${TAG}_tool.log
  exit $rc
fi
