#!/bin/bash
# GPU session for the XTC paths: decoder tests, C5 bench with GPU and host
# decode, and a kernel-trace profile of the GPU-decode bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-xg}
timeout -k 10 300 python -u -m pytest tests/test_xtc_gpu.py tests/test_gpu_xtc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for D in gpu host; do
  timeout -k 10 200 python -u bench.py --workload c5xtc --xtc-decode $D --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_bench_$D.json 2> gpurun_out/${TAG}_bench_$D.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$D.json'));print('$D', d['value'], d['ms_per_step'], d['stager'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_rocprof -o run -- python3 bench.py --workload c5xtc --xtc-decode gpu --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/${TAG}_rocprof -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-200
exit $rc
