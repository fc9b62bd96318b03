#!/bin/bash
# The sequential Welford (RMSF.py:137-138 as written): exactness and time,
# per lane-width / frames-in-flight variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/seq
mkdir -p $O
set -o pipefail
for V in ${@:-0}; do
  echo "== variant $V"
  RMSF_SEQ_VARIANT=$V timeout -k 10 400 python -u tools/seq_welford.py > $O/seq_v$V.txt 2>&1 || { tail -20 $O/seq_v$V.txt; exit 1; }
  grep -v amdgpu.ids $O/seq_v$V.txt
done
