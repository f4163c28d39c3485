#!/bin/bash
# r06g: a complete-game oracle replay at 200 evals/move (GZ_LONG_TESTS cases of
# tests/test_runner_deep_gpu.py::test_deep_config_runner_matches_oracle_200)
set -o pipefail
TAG=${1:-r06g}; CASE=${2:-amazons_cfg5_200}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
GZ_LONG_TESTS=1 timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 1080 --timeout-method thread tests/test_runner_deep_gpu.py -k "$CASE" > $T/replay_$CASE.log 2>&1 || { echo "replay failed"; tail -30 $T/replay_$CASE.log; exit 1; }
grep -E "PASSED|FAILED|identical|runner \{" $T/replay_$CASE.log | cut -c1-600
