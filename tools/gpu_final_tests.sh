#!/bin/bash
# every GPU test and the smoke on the final tree
set -o pipefail
T=gpurun_out/${1:-final_tests}
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
echo ALL OK
