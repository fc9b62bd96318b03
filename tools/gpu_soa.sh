#!/bin/bash
# SoA (coordinate-plane) host input: its GPU tests, then C5 host streaming
# with the [F, n_atoms, 3] and the [F, 3, n_atoms] layouts (A/B/A).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_soa.py -x -v --timeout 200 --timeout-method thread > gpurun_out/soa_tests.log 2>&1
rc=$?; tail -4 gpurun_out/soa_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for L in fac soa; do
  timeout -k 10 300 python -u bench.py --workload c5 --host-layout $L --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/c5_$L.json 2> gpurun_out/c5_$L.err
  rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/c5_$L.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5_$L.json').read().strip().splitlines()[-1]); print('$L', round(d['stager']['h2d_gbs'],1), 'GB/s H2D', d['stager']['host_layout'], d['rmsf_checksum'])"
done
