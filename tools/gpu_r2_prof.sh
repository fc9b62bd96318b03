#!/bin/bash
# GPU session: parity tests; the driver's default bench; the same command under
# rocprofv3 --kernel-trace --stats; FETCH_SIZE / WRITE_SIZE passes (one each) of
# the C3 workload (superposition sums + aligned accumulate) and of C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2prof}
bash tools/gpu_r2.sh ${TAG} || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_rocprof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}_rocprof.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
for W in c3 c2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_pmc_${W}_${C} -o run -- python3 bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline --no-modes > gpurun_out/${TAG}_pmc_${W}_${C}.log 2>&1
    rc=$?; echo "pmc $W $C rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_pmc_${W}_${C}.log; exit $rc; fi
  done
done
exit 0
