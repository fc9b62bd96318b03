#!/bin/bash
# Does the GPU's idle period during the CPU baseline (or a short warm-up)
# slow the timed C2 kernel?  Alternating runs on one box: with the CPU
# baseline and 5 or 200 warm-up steps, and without the baseline.
# (Round 4: no -- 3.648-3.657 ms kernel in all six runs,
# profiles/r04_workloads/warmup_cpu_baseline_ab.txt.)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/warm_ab
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-modes > gpurun_out/warm_ab/cpu_w5_$i.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 200 --no-modes > gpurun_out/warm_ab/cpu_w200_$i.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-modes --no-cpu-baseline > gpurun_out/warm_ab/nocpu_w5_$i.json 2>/dev/null || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/warm_ab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), round(d["roofline"]["avg_launch_ms"], 4))
PY
