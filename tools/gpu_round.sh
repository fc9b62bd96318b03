#!/bin/bash
# Round-end rehearsal on one MI355X: every -m gpu test, smoke(), the default
# bench line, and the rocprofv3 kernel summary of a short bench run.
mkdir -p gpurun_out
tag=${1:-r03}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
    || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -c 600 gpurun_out/${tag}_bench.json
