#!/bin/bash
# r05t: kernels built with -ffp-contract=on -- variant 23 vs 21 differences, the NN GPU suite, the
# MFMA probe's 2 x 2 split loops and the variant-23 forward A/B
set -o pipefail
TAG=${1:-r05t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 200 python -u tools/variant_diff.py 21 23 > $T/diff.txt 2>&1 || { tail -5 $T/diff.txt; exit 1; }
cat $T/diff.txt
timeout -k 10 700 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_v2_gpu.py tests/test_nn_19x19_gpu.py tests/test_weight_roll_gpu.py tests/test_bench_shape_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $T/nn_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $T/nn_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/probes/mfma_shape.exe 2016 1024 30 > $T/mfma_shape5.txt 2>&1 || exit 1
cat $T/mfma_shape5.txt
for round in 1 2; do
  for v in 21 23; do
    echo "== round $round variant $v"
    GZ_KERNEL_VARIANT=$v timeout -k 10 120 python -u tools/time_forward.py --config 2 --rows 1024 --reps 15 --precision fp32 || exit 1
  done
done 2>&1 | tee $T/ab_v23.txt
