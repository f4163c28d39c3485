#!/bin/bash
# r05b: boards beyond 64 positions in split precision and 19 x 19: errors vs the oracle, then the
# existing forward parity suites (regression of the kernels the new geometry touches)
set -o pipefail
TAG=${1:-r05b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 400 python -u tools/large_board_errors.py > $T/errors.log 2>&1 || { echo "errors script failed"; tail -20 $T/errors.log; exit 1; }
cat $T/errors.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_gpu.py tests/test_nn_v2_gpu.py > $T/nn_tests.log 2>&1 || { echo "nn tests failed"; tail -30 $T/nn_tests.log; exit 1; }
tail -3 $T/nn_tests.log
