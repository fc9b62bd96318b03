#!/bin/bash
# GPU session: superposition-sums ablation (tools/ubench_stats2), parity tests, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r2s}
timeout -k 10 200 ./tools/ubench_stats2 > gpurun_out/${TAG}_ubstats2.txt 2>&1
rc=$?; echo "ubench rc=$rc"; cat gpurun_out/${TAG}_ubstats2.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r2.sh ${TAG}
