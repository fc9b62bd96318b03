#!/bin/bash
# Round 6: the parity sweep above the exact threshold (FUZZ_FRAMES=256,384,512, $1 seeds) into gpurun_out/$2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${2:-fuzz512}
mkdir -p $O
FUZZ_FRAMES=256,384,512 timeout -k 10 1000 python -u tools/fuzz_fewframes.py $1 > $O/fuzz.txt 2>&1 || { tail -20 $O/fuzz.txt; exit 1; }
grep -v amdgpu $O/fuzz.txt
