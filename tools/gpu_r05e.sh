#!/bin/bash
# r05e: device-resident weight roll (byte-identical images, timing), live-runner rolls, bench ranks
set -o pipefail
TAG=${1:-r05e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_weight_roll_gpu.py tests/test_runner_roll_gpu.py tests/test_bench_gpu.py > $T/tests.log 2>&1
rc=$?
grep -E "identical|weight roll|roll|PASSED|FAILED|ERROR|passed|failed" $T/tests.log | tail -40
exit $rc
