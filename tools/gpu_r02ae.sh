#!/bin/bash
# r02ae: k-step scheduling barrier in the single-image kernels: NN GPU tests, cfg4/5 forward timings
set -o pipefail
T=gpurun_out/${1:-r02ae}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_v2_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u tools/kernel_variants.py --configs 4,5 --batches 256,1024 --reps 10 --precision bf16 --variants default > $T/variants_cfg45.txt 2>&1 || { echo "timing failed"; tail -5 $T/variants_cfg45.txt; exit 1; }
cat $T/variants_cfg45.txt
echo ALL OK
