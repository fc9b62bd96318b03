#!/bin/bash
# Build an A/B variant of librmsf_hip.so into tools/_ab/librmsf_$1.so with extra -D flags ($2...).
set -e
cd "$(dirname "$0")/../mdanalysis-mpi_amd/csrc"
name=$1; shift
mkdir -p ../../tools/_ab/$name
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -I../../include $*"
/opt/rocm/bin/hipcc $F -c rmsf_kernels.hip -o ../../tools/_ab/$name/k.o
for f in stager xtc context; do /opt/rocm/bin/hipcc $F -x hip -c $f.cpp -o ../../tools/_ab/$name/$f.o; done
/opt/rocm/bin/hipcc $F -c xtc_gpu.hip -o ../../tools/_ab/$name/xg.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/_ab/librmsf_$name.so ../../tools/_ab/$name/*.o -lpthread -ldl
rm -rf ../../tools/_ab/$name
