#!/bin/bash
# r03h: padded-row LDS layout + single-buffered B (looped conv): NN parity tests, same-box timing vs
# the previous looped kernel (tools/kexp lib_base), stamps
set -o pipefail
T=gpurun_out/${1:-r03h}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -v -s --timeout 300 --timeout-method thread > $T/nn_tests.log 2>&1 || { echo "nn tests failed"; grep -E "FAILED|Error|assert" $T/nn_tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/nn_tests.log | tail -1
bash tools/gpu_kexp.sh $1/kexp base pad || exit 1
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3,5 --batches 512,1024,2048 --reps 10 --precision fp32 --variants default > $T/variants_fp32.txt 2>&1 || { echo "variants failed"; tail -5 $T/variants_fp32.txt; exit 1; }
cat $T/variants_fp32.txt
echo ALL OK
