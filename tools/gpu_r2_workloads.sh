#!/bin/bash
# GPU session: every bench workload, then the same command under rocprofv3
# --kernel-trace --stats (the kernel averages must agree with the bench's
# per-launch HIP-event roofline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2w}
run() {  # name, bench args...
  local N=$1; shift
  timeout -k 10 240 python3 -u bench.py "$@" > gpurun_out/${TAG}_${N}.json 2> gpurun_out/${TAG}_${N}.err
  local rc=$?; echo "$N bench rc=$rc"; cut -c1-200 gpurun_out/${TAG}_${N}.json
  [ $rc -ne 0 ] && { tail -3 gpurun_out/${TAG}_${N}.err; return $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${N}_rocprof -o run -- python3 bench.py "$@" > gpurun_out/${TAG}_${N}_rocprof.log 2>&1
  rc=$?; echo "$N rocprof rc=$rc"; return $rc
}
run c3 --workload c3 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
run average --workload average --steps 5 --warmup 2 --no-cpu-baseline || exit $?
run c4 --workload c4 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
run c5 --workload c5 --steps 5 --warmup 2 || exit $?
run c5_avg --workload c5 --align average --host-cache --steps 5 --warmup 2 || exit $?
run c5xtc --workload c5xtc --steps 3 --warmup 1 || exit $?
run c5xtc_avg --workload c5xtc --align average --xtc-cache --steps 3 --warmup 1 || exit $?
exit 0
