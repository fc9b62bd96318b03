#!/bin/bash
# Round-2 first GPU session: host probe, parity tests, smoke, the driver's default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > gpurun_out/r2_host.txt
nproc >> gpurun_out/r2_host.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r2_host.txt 2>/dev/null; free -g >> gpurun_out/r2_host.txt
cat gpurun_out/r2_host.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r2_first_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_first_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_first_bench.json 2> gpurun_out/r2_first_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2_first_bench.json; tail -3 gpurun_out/r2_first_bench.err
exit $rc
