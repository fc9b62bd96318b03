#!/bin/bash
# Round 6: segments-per-chunk cap of the balanced plan (RMSF_SK_MAX_SEGS) on the sparse modes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6segs}
mkdir -p $O
for m in 1000000 256 64 16; do
  echo "== RMSF_SK_MAX_SEGS=$m" | tee -a $O/segs.txt
  RMSF_SK_MAX_SEGS=$m timeout -k 10 300 python -u tools/probe_sparse.py 3 >> $O/segs.txt 2>&1 || { tail -20 $O/segs.txt; exit 1; }
done
grep -v amdgpu.ids $O/segs.txt
