#!/bin/bash
# rocprofv3 evidence for one round, from the driver's own bench command:
#  1. kernel-trace stats of `bench.py --gpus 1 --steps 20 --warmup 5` (no CPU
#     baseline: it forks worker processes, and the profile is of the GPU
#     kernels), its JSON line kept from the same run, and the roofline
#     recomputed from the profile (tools/roofline_vs_rocprof.py);
#  2. one --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) on a short C2
#     bench -- each pass its own run, never combined with other tracing.
set -e
tag=${1:-r04}
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$repo"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o bench \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1
tail -c 300 gpurun_out/prof_${tag}.log
python3 tools/roofline_vs_rocprof.py gpurun_out/prof_${tag} gpurun_out/prof_${tag}.log \
    --out gpurun_out/roofline_${tag}.json || echo "roofline check failed (see gpurun_out/roofline_${tag}.json)"
if [ "${2:-}" = "pmc" ]; then
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${tag}_fetch -o c2 \
      -- python3 bench.py --no-cpu-baseline --no-modes --steps 3 --warmup 1 > gpurun_out/pmc_${tag}_fetch.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${tag}_write -o c2 \
      -- python3 bench.py --no-cpu-baseline --no-modes --steps 3 --warmup 1 > gpurun_out/pmc_${tag}_write.log 2>&1
fi
find gpurun_out/prof_${tag} -name "*.csv" | head
