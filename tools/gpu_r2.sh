#!/bin/bash
# Round-2 GPU session: parity tests (all, -x), then the driver's default bench.
# usage: tools/gpu_r2.sh TAG [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r2}; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -s > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
exit $rc
