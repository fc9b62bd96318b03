#!/bin/bash
# Round-4 fold A/B: the per-lane k_fold_sk (tools/_ab/librmsf_old.so, the
# tree's kernel) against itself and against the per-coordinate variant
# (tools/_ab/librmsf_percoord.so), per buffer bit for bit, and timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fold_r4
mkdir -p $O
set -o pipefail


timeout -k 10 300 python -u tools/ab_fold.py --new tools/_ab/librmsf_percoord.so --dump $O/diff_segments.json > $O/ab_percoord.txt 2>&1 || { tail -20 $O/ab_percoord.txt; exit 1; }
cat $O/ab_percoord.txt
