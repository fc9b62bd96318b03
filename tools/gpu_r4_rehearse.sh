#!/bin/bash
# One-process --gpus N rehearsals (device 0 listed N times) against the
# 1-GPU run and the torchrun gloo rehearsal, C2 at 100k x 20k: checksums and
# step times; then the multi-context host-cost timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4_rehearse
O=gpurun_out/r4_rehearse
set -o pipefail
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-modes > $O/one_gpu.json 2> $O/one_gpu.err || exit $?
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --gpus $n --rehearse --steps 10 --warmup 3 --no-cpu-baseline > $O/single_process_fold_$n.json 2> $O/single_process_fold_$n.err || exit $?
  timeout -k 10 200 python -u bench.py --gpus $n --rehearse --rehearse-transport noop --steps 10 --warmup 3 --no-cpu-baseline > $O/single_process_noop_$n.json 2> $O/single_process_noop_$n.err || exit $?
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/torchrun_gloo_8.json 2> $O/torchrun_gloo_8.err || exit $?
timeout -k 10 300 python -u tools/time_multi_step.py > $O/time_multi_step.txt 2>&1 || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4_rehearse/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["n_gpus"], round(d["ms_per_step"], 4), d.get("host_enqueue_ms_per_step"), repr(d["rmsf_checksum"]))
PY
tail -3 $O/time_multi_step.txt
