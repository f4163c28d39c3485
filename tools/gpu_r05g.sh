#!/bin/bash
# r05g: deep configs' parity in probability space (damped, launch shape) + the deep amazons replay
set -o pipefail
TAG=${1:-r05g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 500 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_bench_shape_gpu.py > $T/shape.log 2>&1
rc1=$?
grep -E "damped|out[0-9]:|PASSED|FAILED|passed|failed" $T/shape.log | cut -c1-220 | tail -40
[ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
timeout -k 10 640 python -u -m pytest -v -s --timeout 600 --timeout-method thread "tests/test_runner_deep_gpu.py::test_deep_config_runner_matches_oracle[amazons_cfg5_deep]" > $T/deep.log 2>&1
rc2=$?
grep -E "oracle pool|samples of|runner stats|PASSED|FAILED|passed|failed|Error" $T/deep.log | cut -c1-300 | tail -30
exit $((rc1 + rc2))
