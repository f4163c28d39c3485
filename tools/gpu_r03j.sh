#!/bin/bash
# r03j: the 8-wave split kernel (variant 22): identity tests, then timing against 21 (isolated forward)
set -o pipefail
T=gpurun_out/${1:-r03j}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -v -s --timeout 120 --timeout-method thread -k "variants_identical_fp32 or wave_group" > $T/wg_tests.log 2>&1 || { echo "wg tests failed"; grep -E "FAILED|Error|assert" $T/wg_tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/wg_tests.log | tail -1
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3 --batches 512,1024,2048 --reps 20 --precision fp32 --variants 21,22 > $T/variants_fp32.txt 2>&1 || { echo "variants failed"; tail -5 $T/variants_fp32.txt; exit 1; }
cat $T/variants_fp32.txt
echo ALL OK
