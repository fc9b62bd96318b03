#!/bin/bash
# Round 6: gathered-read cache-policy micro-benchmark (tools/ubench_gather_policy.hip), times and L2 fetch sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${1:-r6ugp}
mkdir -p $O
for s in 10 220; do
  timeout -k 10 120 tools/_ab/ugp $s 4000 > $O/time_s$s.txt 2>&1 || { cat $O/time_s$s.txt; exit 1; }
  cat $O/time_s$s.txt
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $O/pmc_s$s -o run -- tools/_ab/ugp $s 4000 > $O/pmc_s$s.log 2>&1 || { tail -5 $O/pmc_s$s.log; exit 1; }
done
python3 tools/pmc_r6_summary.py $O > $O/summary.txt && cat $O/summary.txt
