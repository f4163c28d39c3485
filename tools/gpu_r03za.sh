#!/bin/bash
# r03za: cfg4 split (two-pass kernel, pass 1 hi-only weight loads): parity, kernel time, then the
# aged cfg4 bench under rocprofv3
set -o pipefail
T=gpurun_out/${1:-r03za}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
    -k "fp32 and (cfg4 or 13x13)" > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $T/tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/tests.log | tail -1
timeout -k 10 200 python -u tools/time_forward.py --config 4 --rows 1024 --precision fp32 > $T/time_cfg4.log 2>&1 || { echo "timing failed"; tail -5 $T/time_cfg4.log; exit 1; }
cat $T/time_cfg4.log
bash tools/gpu_cfg_aged.sh $(basename $T) "4" 240
