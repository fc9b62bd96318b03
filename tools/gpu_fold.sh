#!/bin/bash
# Fold kernel check: all GPU tests, the C2 step at the 2,500-frame N=8 share
# and the full size, and a rocprofv3 kernel trace of the 2,500-frame step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fold}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for F in 2500 20000 2500 20000; do
  timeout -k 10 200 python -u bench.py --frames $F --steps 40 --warmup 5 --no-modes --no-cpu-baseline > gpurun_out/${TAG}_b.json 2>/dev/null
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc"; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))" gpurun_out/${TAG}_b.json $F | tee -a gpurun_out/${TAG}_b.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_rocprof -o run -- python3 bench.py --frames 2500 --steps 20 --warmup 5 --no-modes --no-cpu-baseline > gpurun_out/${TAG}_rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
