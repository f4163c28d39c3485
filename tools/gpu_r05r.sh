#!/bin/bash
# r05r: variant 23 (trunk_kernel_h2: two groups of two waves, a board each) -- identity tests, the
# MFMA probe's 2 x 2 split loops (s25 / s26), and the forward A/B against variant 21 at 1,024 rows
set -o pipefail
TAG=${1:-r05r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -k "variants_identical or wave_group" -x -q --timeout 120 --timeout-method thread > $T/variant_tests.log 2>&1
rc=$?; tail -2 $T/variant_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/probes/mfma_shape.exe 2016 1024 30 > $T/mfma_shape5.txt 2>&1 || exit 1
cat $T/mfma_shape5.txt
for round in 1 2; do
  for v in 21 23; do
    for rows in 1024 2048; do
      echo "== round $round variant $v rows $rows"
      GZ_KERNEL_VARIANT=$v timeout -k 10 120 python -u tools/time_forward.py --config 2 --rows $rows --reps 15 --precision fp32 || exit 1
    done
  done
done 2>&1 | tee $T/ab_v23.txt
