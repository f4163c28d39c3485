#!/bin/bash
# r06a: the driver's command on the round-6 engine (root-latch spin fast path, bounded stop), then
# the bounded-stop GPU test
set -o pipefail
TAG=${1:-r06a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -5 $T/bench.log; exit 1; }
grep "^{" $T/bench.log | tail -1 | cut -c1-600
timeout -k 10 320 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_runner_stop_gpu.py > $T/stop_test.log 2>&1 || { echo "stop test failed"; tail -30 $T/stop_test.log; exit 1; }
tail -5 $T/stop_test.log
