#!/bin/bash
# per-phase workgroup cycles of the trunk kernel (GZ_KERNEL_STAMPS) at 1,024 rows, fp32 and bf16
set -o pipefail
T=gpurun_out/${1:-stamps}
mkdir -p $T
timeout -k 10 200 python -u tools/kernel_breakdown.py --precision fp32 --variants 21 --batches 1024 --blocks 0,6 > $T/fp32.txt 2>&1 || { echo "fp32 failed"; exit 1; }
timeout -k 10 200 python -u tools/kernel_breakdown.py --precision bf16 --variants 21 --batches 1024 --blocks 0,6 > $T/bf16.txt 2>&1 || { echo "bf16 failed"; exit 1; }
cat $T/fp32.txt $T/bf16.txt
echo ALL OK
