#!/bin/bash
# r06b/c: the aged bench regimes verified live (tests/test_runner_verify_gpu.py), two configs per call
set -o pipefail
TAG=${1:-r06b}; SEL=${2:-"cfg2 or cfg3"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_runner_verify_gpu.py -k "$SEL" > $T/verify.log 2>&1 || { echo "verify failed"; tail -40 $T/verify.log; exit 1; }
grep -E "PASSED|FAILED|\{\"config" $T/verify.log | cut -c1-700
