#!/bin/bash
# r06h: a config's bench line on the current engine (no CPU leg), then optional pytest selections
set -o pipefail
TAG=${1:-r06h}; CFG=${2:-3}; AGE=${3:-300}; SEL=${4:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 800 python -u bench.py --config $CFG --age-seconds $AGE --no-cpu-baseline > $T/bench_cfg$CFG.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_cfg$CFG.log; exit 1; }
grep "^{" $T/bench_cfg$CFG.log | tail -1 | cut -c1-300
if [ -n "$SEL" ]; then
  timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread $SEL > $T/tests.log 2>&1 || { echo "tests failed"; tail -40 $T/tests.log; exit 1; }
  grep -E "PASSED|FAILED|^\{|identical" $T/tests.log | cut -c1-600
fi
