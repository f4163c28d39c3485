#!/bin/bash
# r04u: PMC passes of the default large kernel (now trunk_kernel_w8), then the long runner GPU tests
set -o pipefail
TAG=${1:-r04u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
bash tools/gpu_pmc_r04.sh $TAG/pmc > $T/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $T/pmc.log; exit 1; }
grep -A14 "trunk_kernel" $T/pmc/summary.txt
timeout -k 10 600 python -u -m pytest tests/test_runner_verify_gpu.py tests/test_runner_roll_gpu.py tests/test_runner_deep_gpu.py -v -s --timeout 500 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
grep -E "window_nn_free|verified" $T/tests.log | tail -2 | cut -c1-400
echo ALL OK
