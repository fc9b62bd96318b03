#!/bin/bash
# Round 6: exact-aligned cost probe (PROBE_SHAPE) with this build and each tools/_ab/librmsf_<v>.so, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PROBE_SHAPE=${PROBE_SHAPE:-1,3}
O=gpurun_out/${AB_OUT:-r6abx}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 240 python -u tools/probe_exact_aligned.py 2 > $O/cur_$r.txt 2>&1 || { tail -20 $O/cur_$r.txt; exit 1; }
  for v in "$@"; do
    RMSF_AB_LIB=tools/_ab/librmsf_$v.so timeout -k 10 240 python -u tools/probe_exact_aligned.py 2 > $O/${v}_$r.txt 2>&1 || { tail -20 $O/${v}_$r.txt; exit 1; }
  done
done
for f in $O/*.txt; do echo "== $f"; grep -v amdgpu $f | grep "exact=True"; done
