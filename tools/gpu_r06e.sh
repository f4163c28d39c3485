#!/bin/bash
# r06e/f: runner verification of a config and / or the 200-evals complete-game oracle replays
set -o pipefail
TAG=${1:-r06e}; VSEL=${2:-}; RSEL=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$VSEL" ]; then
  timeout -k 10 500 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_runner_verify_gpu.py -k "$VSEL" > $T/verify.log 2>&1 || { echo "verify failed"; tail -40 $T/verify.log; exit 1; }
  grep -E "PASSED|FAILED|^\{" $T/verify.log | cut -c1-700
fi
if [ -n "$RSEL" ]; then
  timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 1080 --timeout-method thread tests/test_runner_deep_gpu.py -k "$RSEL" > $T/replay.log 2>&1 || { echo "replay failed"; tail -40 $T/replay.log; exit 1; }
  grep -E "PASSED|FAILED|identical|runner \{" $T/replay.log | cut -c1-700
fi
