#!/bin/bash
# Round 6: the few-frame parity sweep (tools/fuzz_fewframes.py $1 seeds) over FUZZ_SHAPES=$2, into gpurun_out/$3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${3:-fuzz}
mkdir -p $O
FUZZ_SHAPES=$2 timeout -k 10 1000 python -u tools/fuzz_fewframes.py $1 > $O/fuzz_$2.txt 2>&1 || { tail -20 $O/fuzz_$2.txt; exit 1; }
grep -v amdgpu $O/fuzz_$2.txt
