#!/bin/bash
# HBM traffic of the bench kernels: one rocprofv3 --pmc pass per TCC counter
# group (FETCH_SIZE uses 3 of the 4 TCC slots, WRITE_SIZE 2: never together).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmc}
shift
ARGS="--steps 2 --warmup 0 --no-cpu-baseline $*"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_${C} -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_${C}.log 2>&1
  rc=$?; echo "$C rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_${C}.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE
