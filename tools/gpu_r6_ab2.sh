#!/bin/bash
# Round 6: the sparse probe's C3 1-in-10 case with the current build and each
# tools/_ab/librmsf_<v>.so named on the command line, alternating, on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp RMSF_PROBE_ONLY=${RMSF_PROBE_ONLY:-10:frame0}
O=gpurun_out/${AB_OUT:-r6ab2}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 180 python -u tools/probe_sparse.py 3 > $O/cur_$r.txt 2>&1 || { tail -20 $O/cur_$r.txt; exit 1; }
  for v in "$@"; do
    RMSF_AB_LIB=tools/_ab/librmsf_$v.so timeout -k 10 180 python -u tools/probe_sparse.py 3 > $O/${v}_$r.txt 2>&1 || { tail -20 $O/${v}_$r.txt; exit 1; }
  done
done
for f in $O/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
