#!/bin/bash
# r03z: the two-pass split kernel (F = 256 on 13 x 13): parity tests, then kernel time per precision
set -o pipefail
T=gpurun_out/${1:-r03z}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
    -k "cfg4 or 13x13 or cfg2 or cfg5" > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $T/tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/tests.log | tail -1
timeout -k 10 200 python -u tools/time_forward.py --config 4 --rows 1024 > $T/time_cfg4.log 2>&1 || { echo "timing failed"; tail -5 $T/time_cfg4.log; exit 1; }
cat $T/time_cfg4.log
echo ALL OK
