#!/bin/bash
# r04f: every GPU test except the long runner ones (verify / roll / deep: tools/gpu_r04b.sh) + smoke
set -o pipefail
T=gpurun_out/${1:-r04f}
mkdir -p $T
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
    --ignore=tests/test_runner_verify_gpu.py --ignore=tests/test_runner_roll_gpu.py --ignore=tests/test_runner_deep_gpu.py \
    > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
timeout -k 10 240 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
echo ALL OK
