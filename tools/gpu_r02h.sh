#!/bin/bash
# r02h: wrapped 256-byte LDS rows (F = 128) + split-precision two-board kernel: NN GPU tests and
# kernel timings by launch size (bf16 / fp32, variants)
set -o pipefail
T=gpurun_out/r02h
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py -v -s --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 256,512,1024,2048 --reps 20 --precision bf16 > $T/variants_bf16.txt 2>&1 || { echo "bf16 timing failed"; exit 1; }
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 256,512,1024,2048 --reps 20 --precision fp32 --variants default,11,21 > $T/variants_fp32.txt 2>&1 || { echo "fp32 timing failed"; exit 1; }
cat $T/variants_bf16.txt $T/variants_fp32.txt
echo ALL OK
