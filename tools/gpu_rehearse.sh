#!/bin/bash
# Randomised parity sweep on the current kernels, then the driver's torchrun
# form rehearsed with 4 gloo ranks sharing the one GPU (C2 strong scaling;
# C4 weak scaling with the final sweep in atom slabs).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fuzz_parity.py 150 > gpurun_out/fuzz_r03.txt 2>&1
tail -3 gpurun_out/fuzz_r03.txt
export MASTER_ADDR=127.0.0.1
port() { python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])"; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $(port) bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 \
    > gpurun_out/rehearse4_c2.json 2> gpurun_out/rehearse4_c2.err
tail -c 400 gpurun_out/rehearse4_c2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $(port) bench.py --gpus 4 --backend gloo --workload c4 --frames 400 --steps 2 --warmup 1 \
    > gpurun_out/rehearse4_c4.json 2> gpurun_out/rehearse4_c4.err
tail -c 400 gpurun_out/rehearse4_c4.json
