#!/bin/bash
# A/B of two library builds on the C5 XTC bench (same box, alternating):
# tools/altlib/librmsf_hip_{oldread,new}.so are copied over the in-tree
# library in turn.  Not product code.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=mdanalysis-mpi_amd/lib/librmsf_hip.so
for V in ${AB_VARIANTS:-new oldread new oldread}; do
  cp tools/altlib/librmsf_hip_$V.so $L
  timeout -k 10 200 python -u bench.py --workload c5xtc --xtc-decode gpu --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/abc5_$V.json 2> gpurun_out/abc5_$V.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/abc5_$V.json'));print('$V', round(d['ms_per_step'],2), 'ms', round(d['stager']['xtc_frames_per_s']), 'frames/s', round(d['stager']['xtc_gb_per_s_compressed'],1), 'GB/s')"
done
cp tools/altlib/librmsf_hip_new.so $L
