#!/bin/bash
# Round 6: A/B of the current build against tools/_ab/librmsf_$1.so on one box
# (sparse probe, alternating), then the gathered/aligned GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${2:-r6ab}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 240 python -u tools/probe_sparse.py 3 > $O/cur_$r.txt 2>&1 || { tail -20 $O/cur_$r.txt; exit 1; }
  RMSF_AB_LIB=tools/_ab/librmsf_$1.so timeout -k 10 240 python -u tools/probe_sparse.py 3 > $O/$1_$r.txt 2>&1 || { tail -20 $O/$1_$r.txt; exit 1; }
done
for f in $O/cur_1.txt $O/$1_1.txt $O/cur_2.txt $O/$1_2.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
