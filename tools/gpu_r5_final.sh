#!/bin/bash
# Round-5 last-tree pass (one gpurun call): the whole GPU suite, smoke(),
# then the rocprof kernel trace of the driver's bench command with its own
# JSON line and the roofline recomputed from the trace (tools/gpu_r5_prof.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_r5_prof.sh ${1:-r05final}
