#!/bin/bash
# Round 6, verdict item 4: C4's 1M x 2,500 share vs 100k x 25,000 (same bytes), plain and
# under separate rocprofv3 --pmc passes (translation / TA / L2 counters when they exist).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${1:-r6c4}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o -E "\b(TCP_UTCL1[A-Z_]*|UTCL2[A-Z_]*|TCP_TCP_TA_DATA_STALL_CYCLES[a-z_]*|TA_TA_BUSY[a-z_]*|TA_BUSY[a-z_]*|TCP_PENDING_STALL[A-Z_a-z]*|TCC_HIT[a-z_]*|TCC_MISS[a-z_]*|TCP_TOTAL_CACHE_ACCESSES[a-z_]*|TCC_EA0_RDREQ[A-Z_0-9a-z]*)\b" $O/counters.txt | sort -u > $O/counters_of_interest.txt
cat $O/counters_of_interest.txt | tr '\n' ' '; echo
timeout -k 10 200 python3 tools/c4_once.py 5 > $O/plain.txt 2>&1 || { tail -5 $O/plain.txt; exit 1; }
grep -v amdgpu $O/plain.txt
