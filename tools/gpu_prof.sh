#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the default bench
# command, then one --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) on a short
# C2 bench -- each pass its own run, never combined with other tracing.
set -e
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o bench \
    -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1
tail -c 200 gpurun_out/prof_${tag}.log
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${tag}_fetch -o c2 \
    -- python3 bench.py --no-cpu-baseline --no-modes --steps 3 --warmup 1 > gpurun_out/pmc_${tag}_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${tag}_write -o c2 \
    -- python3 bench.py --no-cpu-baseline --no-modes --steps 3 --warmup 1 > gpurun_out/pmc_${tag}_write.log 2>&1
find gpurun_out/prof_${tag} gpurun_out/pmc_${tag}_fetch gpurun_out/pmc_${tag}_write -name "*.csv" | head
