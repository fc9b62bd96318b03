#!/bin/bash
# Round 5 evidence runs (one gpurun call):
#  1. bench.py --gpus 8 --rehearse (one process, 8 contexts on device 0, host
#     fold): the one-process line with merge_timing per device (VERDICT r4
#     item 3), at the C2 workload;
#  2. PMC traffic of every kernel of the default N=1 line, modes included:
#     one rocprofv3 --pmc pass per TCC counter group, never combined.
set -e
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$repo"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --gpus 8 --rehearse --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r05_rehearse8.json 2> gpurun_out/r05_rehearse8.err
tail -c 400 gpurun_out/r05_rehearse8.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r05_pmc_$C -o run \
      -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --mode-steps 1 > gpurun_out/r05_pmc_$C.log 2>&1
  echo "$C done"
done
python3 tools/pmc_summary.py gpurun_out/r05_pmc_FETCH_SIZE gpurun_out/r05_pmc_WRITE_SIZE \
    gpurun_out/r05_pmc_all.json "k_welford_flat_sk<4>" 100000 20000 > gpurun_out/r05_pmc_summary.txt
head -60 gpurun_out/r05_pmc_summary.txt
