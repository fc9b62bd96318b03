#!/bin/bash
# Round 6 rocprof evidence of the driver's bench command (as tools/gpu_r5_prof.sh): kernel-trace
# stats of `bench.py --gpus 1 --steps 20 --warmup 5` (CPU baseline off), its JSON line from the same
# run, the roofline recomputed from the trace; then the C2 launch's HBM bytes from separate --pmc
# passes (L2->memory read requests by size, WRITE_SIZE).
set -e
tag=${1:-r06}
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$repo"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o bench \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1
tail -c 300 gpurun_out/prof_${tag}.log
python3 tools/roofline_vs_rocprof.py gpurun_out/prof_${tag} gpurun_out/prof_${tag}.log \
    --out gpurun_out/roofline_${tag}.json || echo "roofline check failed (see gpurun_out/roofline_${tag}.json)"
find gpurun_out/prof_${tag} -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_${tag}.csv \;
for p in "rd:TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "wr:WRITE_SIZE"; do
  n=${p%%:*}; c=${p#*:}
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${tag}_$n -o run \
      -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-modes > gpurun_out/pmc_${tag}_$n.log 2>&1
  echo "pmc $n rc=$?"
done
