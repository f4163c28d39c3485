#!/bin/bash
# r02k: fixed vs per-block cost of the trunk kernel, device-staged vs pinned-host planes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kernel_breakdown.py --precision fp32 --variants 21,11 --batches 1024 --blocks 0,1,2,6 > gpurun_out/r02k_fp32_staged.txt 2>&1 &&
timeout -k 10 300 python -u tools/kernel_breakdown.py --precision fp32 --variants 21 --batches 1024 --blocks 0,1,2,6 --pinned > gpurun_out/r02k_fp32_pinned.txt 2>&1 &&
timeout -k 10 300 python -u tools/kernel_breakdown.py --precision bf16 --variants 21 --batches 1024 --blocks 0,1,2,6 --pinned > gpurun_out/r02k_bf16_pinned.txt 2>&1
