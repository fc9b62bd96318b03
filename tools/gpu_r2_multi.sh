#!/bin/bash
# GPU session: all parity tests, then the multi-GPU bench forms rehearsed on one GPU:
# one process with 2 device contexts on device 0 (--rehearse), and 2 torch.distributed
# ranks sharing device 0 over gloo.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r2m}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 2 --rehearse --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_single2.json 2> gpurun_out/${TAG}_single2.err
rc=$?; echo "single-process rc=$rc"; cat gpurun_out/${TAG}_single2.json; tail -3 gpurun_out/${TAG}_single2.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err
rc=$?; echo "gloo rc=$rc"; cat gpurun_out/${TAG}_gloo2.json; tail -3 gpurun_out/${TAG}_gloo2.err
exit $rc
