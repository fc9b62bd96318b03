#!/bin/bash
# chain micro-benchmark (tools/ubench_chain2.hip, prebuilt into tools/_ab/uch2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/_ab/uch2 > gpurun_out/chain2.txt 2>&1
