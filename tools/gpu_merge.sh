#!/bin/bash
# All GPU tests, then a 2-rank torch.distributed rehearsal of bench.py (gloo
# ranks sharing the device: the N>1 code path, not an RCCL measurement).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-merge}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for W in c2 c3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo --workload $W > gpurun_out/${TAG}_gloo2_$W.json 2> gpurun_out/${TAG}_gloo2_$W.err
  rc=$?; echo "gloo2 $W rc=$rc"; cut -c1-700 gpurun_out/${TAG}_gloo2_$W.json
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_gloo2_$W.err; exit $rc; fi
done
exit 0
