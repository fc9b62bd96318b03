#!/bin/bash
# A/B of the fused single-read sweep against the two-pass path (tools/fused_sweep/ab_fused)
set -e
mkdir -p gpurun_out
PRESET=1 timeout -k 10 120 tools/fused_sweep/ab_fused 100000 2000 2 0 > gpurun_out/fused_mid.txt 2>&1
PRESET=1 timeout -k 10 300 tools/fused_sweep/ab_fused 100000 20000 2 0 > gpurun_out/fused_c3.txt 2>&1
cat gpurun_out/fused_mid.txt gpurun_out/fused_c3.txt
