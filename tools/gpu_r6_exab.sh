#!/bin/bash
# Round 6: the exact aligned probe A/B/A on one box -- this build, tools/_ab/librmsf_$1.so, this build (shapes $3, default 1,3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${2:-exab}
mkdir -p $O
export PROBE_SHAPE=${3:-1,3}
timeout -k 10 300 python -u tools/probe_exact_aligned.py 3 > $O/a1.txt 2>&1 || { tail -5 $O/a1.txt; exit 1; }
RMSF_AB_LIB=tools/_ab/librmsf_$1.so timeout -k 10 300 python -u tools/probe_exact_aligned.py 3 > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
timeout -k 10 300 python -u tools/probe_exact_aligned.py 3 > $O/a2.txt 2>&1 || { tail -5 $O/a2.txt; exit 1; }
for f in a1 b a2; do echo "== $f"; grep "exact=True" $O/$f.txt; done
