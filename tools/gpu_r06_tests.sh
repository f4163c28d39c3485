#!/bin/bash
# Round-6 final tree: the GPU suite in two halves (each under its own limit) and the smoke.
#   fast: everything but the long runner tests;  long1: the aged-window verification per config;
#   long2: the deep-config runner replays, the roll / recreate / stop runner tests
set -o pipefail
TAG=${1:-r06t}; PART=${2:-fast}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
# heartbeat under gpurun_out (long tests -- the oracle replays -- print nothing for minutes)
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
LONG1="tests/test_runner_verify_gpu.py"; LONG2="tests/test_runner_deep_gpu.py tests/test_runner_roll_gpu.py tests/test_runner_stop_gpu.py"; LONG="$LONG1 $LONG2"; [ "$PART" = long1 ] && LONG=$LONG1; [ "$PART" = long2 ] && LONG=$LONG2
if [ "$PART" = fast ]; then
  DESEL=""; for f in $LONG; do DESEL="$DESEL --ignore=$f"; done
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread $DESEL > $T/gpu_fast.log 2>&1
  rc=$?
  grep -E "passed|failed|FAILED|ERROR" $T/gpu_fast.log | tail -8
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $T/smoke.log; exit 1; }
  cat $T/smoke.log
else
  timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s --timeout 900 --timeout-method thread > $T/gpu_$PART.log 2>&1
  rc=$?
  grep -E "passed|failed|FAILED|ERROR|identical|verified" $T/gpu_$PART.log | tail -12
  exit $rc
fi
