#!/bin/bash
# Round 6: per-kernel times of the exact aligned path (rocprofv3 --kernel-trace --stats over tools/probe_exact_aligned.py, one shape).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-exprof}
mkdir -p $O
PROBE_SHAPE=${2:-1,3} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/probe_exact_aligned.py 2 > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
grep -E "k_seq|k_ref_seq|k_accum_seq|Name" $O/kernel_stats.csv | cut -d, -f1-8
