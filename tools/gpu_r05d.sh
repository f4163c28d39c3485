#!/bin/bash
# r05d: the forward suites after the large-board / split-geometry changes
set -o pipefail
TAG=${1:-r05d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_nn_gpu.py tests/test_nn_v2_gpu.py tests/test_nn_19x19_gpu.py tests/test_runner_roll_gpu.py > $T/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $T/tests.log | tail -15
exit $rc
