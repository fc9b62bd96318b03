#!/bin/bash
# GPU session: parity tests, then bench under rocprofv3 kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-prof}
shift
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_bench.err; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_rocprof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/${TAG}_rocprof.log
find gpurun_out/${TAG}_rocprof -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-220
exit $rc
