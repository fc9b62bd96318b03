#!/bin/bash
# Round 5 rocprof evidence of the driver's bench command (see gpu_prof.sh):
# kernel-trace stats of `bench.py --gpus 1 --steps 20 --warmup 5` (CPU
# baseline off: it forks workers, and the profile is of the GPU kernels),
# its JSON line from the same run, the roofline recomputed from the trace.
set -e
tag=${1:-r05}
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$repo"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o bench \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1
tail -c 300 gpurun_out/prof_${tag}.log
python3 tools/roofline_vs_rocprof.py gpurun_out/prof_${tag} gpurun_out/prof_${tag}.log \
    --out gpurun_out/roofline_${tag}.json || echo "roofline check failed (see gpurun_out/roofline_${tag}.json)"
find gpurun_out/prof_${tag} -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_${tag}.csv \;
