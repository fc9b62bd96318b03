#!/bin/bash
# Refresh the per-config bench lines (C3, RMSF.py average mode, C4 share,
# C5 XTC two-sweep with HBM cache).  Each step has its own time limit; the
# first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-rf}
run() {
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-modes "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "$name failed rc=$?"; tail -5 gpurun_out/${TAG}_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', '%.3e' % d['value'], round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
}
run c3 --workload c3
run average --workload average
run c4 --workload c4
run c5xtc_avg --workload c5xtc --align average --xtc-cache
