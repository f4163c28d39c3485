#!/bin/bash
# r04s (final tree): the long runner GPU tests (aged verify window, roll timeout / recreate, deep
# runner, concat), the PMC passes of the split trunk, then the driver's bench command
set -o pipefail
TAG=${1:-r04s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 600 python -u -m pytest tests/test_runner_verify_gpu.py tests/test_runner_roll_gpu.py tests/test_runner_deep_gpu.py -v -s --timeout 500 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
bash tools/gpu_pmc_r04.sh $TAG/pmc > $T/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $T/pmc.log; exit 1; }
grep -A14 "trunk_kernel<128, 4, 2" $T/pmc/summary.txt
timeout -k 10 900 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-400
echo ALL OK
