#!/bin/bash
# rocprof kernel-trace stats of the aligned workloads' bench lines (C3 and
# RMSF.py's two sweeps), each with its own JSON line from the same run.
set -e
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$repo"
mkdir -p gpurun_out
for w in c3 average; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$w -o bench \
      -- python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$w.log 2>&1
  find gpurun_out/prof_$w -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$w.csv \;
  echo "$w done"
done
