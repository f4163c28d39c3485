#!/bin/bash
# r02o: fused dense heads in the two-image trunk kernels: every GPU test, forward timings by launch
# size (bf16 / fp32), fixed vs per-block cost
set -o pipefail
T=gpurun_out/${1:-r02o}
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 256,512,1024,2048 --reps 20 --precision bf16 > $T/variants_bf16.txt 2>&1 || { echo "bf16 timing failed"; exit 1; }
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 256,512,1024,2048 --reps 20 --precision fp32 --variants default,11,21 > $T/variants_fp32.txt 2>&1 || { echo "fp32 timing failed"; exit 1; }
timeout -k 10 300 python -u tools/kernel_breakdown.py --precision fp32 --variants 21 --batches 1024 --blocks 0,1,2,6 --pinned > $T/breakdown_fp32_pinned.txt 2>&1 || { echo "breakdown failed"; exit 1; }
grep -E 'N= 1024' $T/variants_bf16.txt $T/variants_fp32.txt
cat $T/breakdown_fp32_pinned.txt
echo ALL OK
