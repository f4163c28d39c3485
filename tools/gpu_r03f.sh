#!/bin/bash
# r03f: looped conv kernel: NN parity tests (incl. bench shape / deep configs), same-box timing of the
# looped vs the unrolled kernel (tools/kexp), per-phase stamps
set -o pipefail
T=gpurun_out/${1:-r03f}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -v -s --timeout 300 --timeout-method thread > $T/nn_tests.log 2>&1 || { echo "nn tests failed"; grep -E "FAILED|Error|assert" $T/nn_tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/nn_tests.log | tail -1
bash tools/gpu_kexp.sh $1/kexp base unrolled || exit 1
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3 --batches 256,512,1024,2048 --reps 20 --precision fp32 --variants default,11,21 > $T/variants_fp32.txt 2>&1 || { echo "variants failed"; tail -5 $T/variants_fp32.txt; exit 1; }
grep "N= 1024\|N= 2048" $T/variants_fp32.txt
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3,4,5 --batches 256,1024 --reps 10 --precision bf16 --variants default > $T/variants_bf16.txt 2>&1 || { echo "variants bf16 failed"; tail -5 $T/variants_bf16.txt; exit 1; }
grep "N= 1024" $T/variants_bf16.txt
echo ALL OK
