#!/bin/bash
# A/B of config C1's RMSF.py computation (hipGraph replay and eager) between
# tools/_ab/librmsf_old.so and the current library, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c1_ab.txt
: > $out
for lib in tools/_ab/librmsf_old.so mdanalysis-mpi_amd/lib/librmsf_hip.so tools/_ab/librmsf_old.so mdanalysis-mpi_amd/lib/librmsf_hip.so tools/_ab/librmsf_old.so mdanalysis-mpi_amd/lib/librmsf_hip.so; do
  timeout -k 10 120 python3 -u tools/c1_kernels.py 3000 --lib $lib >> $out 2>&1 || exit $?
done
grep C1 $out
