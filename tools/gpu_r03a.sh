#!/bin/bash
# r03a: epilogue changes (max-form activation, scratch row) + the split 12 variant: NN GPU tests,
# fp32 variant timings (cfg2, cfg3), per-block breakdown of variants 12 and 21
set -o pipefail
T=gpurun_out/${1:-r03a}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py -x -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3 --batches 256,512,768,1024,2048 --reps 20 --precision fp32 --variants default,11,12,21 > $T/variants_fp32.txt 2>&1 || { echo "fp32 timing failed"; tail -5 $T/variants_fp32.txt; exit 1; }
cat $T/variants_fp32.txt
for v in 12 21; do
timeout -k 10 300 python -u tools/kernel_breakdown.py --precision fp32 --variants $v --batches 1024 --blocks 0,1,2,6 --pinned > $T/breakdown_fp32_$v.txt 2>&1 || { echo "breakdown failed"; tail -5 $T/breakdown_fp32_$v.txt; exit 1; }
cat $T/breakdown_fp32_$v.txt
done
echo ALL OK
