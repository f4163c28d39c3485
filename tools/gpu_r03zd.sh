#!/bin/bash
# r03zd: "tests" = every GPU test and the smoke on the final tree; "bench" = the driver's bench command
set -o pipefail
TAG=${1:-r03zd}
MODE=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
if [ "$MODE" = tests ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
else
timeout -k 10 580 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-300
fi
echo ALL OK
