#!/bin/bash
# The reduce-to-root merge (RMSF.py:143's shape): its GPU tests (gloo ranks
# sharing the GPU) and the torchrun bench form with --merge-root at N = 2, 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v -k "merge_to_root or merge_slabs or sharded" --timeout 250 --timeout-method thread > gpurun_out/root_tests.log 2>&1
rc=$?; tail -4 gpurun_out/root_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
export MASTER_ADDR=127.0.0.1
port() { python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])"; }
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $(port) bench.py --gpus $n --backend gloo --steps 3 --warmup 1 --merge-root \
      > gpurun_out/rehearse${n}_root.json 2> gpurun_out/rehearse${n}_root.err
  rc=$?; echo "N=$n rc=$rc"; if [ $rc -ne 0 ]; then tail -20 gpurun_out/rehearse${n}_root.err; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/rehearse${n}_root.json').read().strip().splitlines()[-1]); print($n, d['rmsf_checksum'], d['config'].get('merge'))"
done
