#!/bin/bash
# r04t: the 8-wave co-split kernel (variant 24) against variant 21: identity tests, timing
# (kernel_variants, cfg2 split) and stamps, then the NN GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04t
mkdir -p $T
cd $R
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 512,1024,2048 --reps 20 --precision fp32 --variants 21,24 > $T/v21_v24.txt 2>&1 || { echo "variants failed"; tail -5 $T/v21_v24.txt; exit 1; }
cat $T/v21_v24.txt
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2 --batches 512,1024,2048 --reps 20 --precision fp32 --variants 21,24 > $T/v21_v24_b.txt 2>&1 || exit 1
cat $T/v21_v24_b.txt
for v in 21 24; do
  timeout -k 10 120 python -u tools/kernel_breakdown.py --precision fp32 --variants $v --batches 1024 --blocks 0,6 > $T/stamps_$v.txt 2>&1 || { echo "stamps failed"; exit 1; }
  echo "$v: $(grep -E 'stamps|fixed' $T/stamps_$v.txt | tr '\n' ' ')"
done
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -x -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
