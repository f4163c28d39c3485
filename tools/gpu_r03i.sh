#!/bin/bash
# r03i: state of the tree at session start: every GPU test, the smoke, the driver's bench command
set -o pipefail
TAG=${1:-r03i}
T=gpurun_out/$TAG
mkdir -p $T
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head; exit 1; }
tail -1 $T/tests.log
timeout -k 10 200 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
timeout -k 10 420 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-600
echo ALL OK
